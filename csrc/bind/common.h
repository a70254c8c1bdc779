// Shared helpers for the torch-facing binding TUs.
#pragma once
#include <c10/hip/HIPStream.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

namespace py = pybind11;

#define IA_CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define IA_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define IA_CHECK_F32(t) TORCH_CHECK((t).scalar_type() == torch::kFloat32, #t " must be float32")
#define IA_CHECK_GPU_F32(t) \
  IA_CHECK_CUDA(t);         \
  IA_CHECK_CONTIG(t);       \
  IA_CHECK_F32(t)

inline hipStream_t ia_stream() { return c10::hip::getCurrentHIPStream().stream(); }

namespace ia {
struct GatherArgs;
struct ConvReduceMulti;
}
// (kernels.cpp) the checked GatherArgs of a cursor-indexed row gather; *incp: the step counter or nullptr
ia::GatherArgs gather_cursor_args(const std::vector<torch::Tensor>& srcs, const torch::Tensor& perm,
                                  const torch::Tensor& cursor, int64_t n, const std::vector<torch::Tensor>& dst,
                                  const c10::optional<torch::Tensor>& inc, float** incp);

// (conv.cpp) the checked ConvReduceMulti of conv_reduce_multi's arguments
ia::ConvReduceMulti conv_reduce_args(const std::vector<torch::Tensor>& xs, const std::vector<torch::Tensor>& dys,
                                     const std::vector<int64_t>& KHs, const std::vector<int64_t>& KWs,
                                     const std::vector<int64_t>& strides, const std::vector<int64_t>& pads,
                                     const std::vector<torch::Tensor>& slabs, const std::vector<torch::Tensor>& dWs,
                                     const std::vector<torch::Tensor>& dbs);

void register_envs(py::module& m);
void register_kernels(py::module& m);
void register_engine(py::module& m);
void register_disc(py::module& m);
void register_airl(py::module& m);
void register_wide(py::module& m);
void register_conv(py::module& m);
void register_comm(py::module& m);
void register_pref(py::module& m);
