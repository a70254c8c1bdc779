// pybind11 surface of the native batched env runtime (csrc/runtime/vec_env.*).
#include "common.h"
#include "vec_env.h"

namespace {

torch::Tensor obs_tensor(const ia::BatchedEnv& e) {
  auto opts = torch::TensorOptions().dtype(e.is_image() ? torch::kUInt8 : torch::kFloat32);
  if (e.is_image()) return torch::empty({e.num_envs(), ia::kPongH, ia::kPongW, ia::kPongStack}, opts);
  return torch::empty({e.num_envs(), e.obs_dim()}, opts);
}

}  // namespace

void register_envs(py::module& m) {
  m.def("native_env_names", &ia::native_env_names);
  py::class_<ia::BatchedEnv>(m, "BatchedEnv")
      .def(py::init<const std::string&, int, int, uint64_t>(), py::arg("name"), py::arg("num_envs"),
           py::arg("max_steps") = -1, py::arg("seed") = 0)
      .def("num_envs", &ia::BatchedEnv::num_envs)
      .def("obs_dim", &ia::BatchedEnv::obs_dim)
      .def("act_dim", &ia::BatchedEnv::act_dim)
      .def("n_actions", &ia::BatchedEnv::n_actions)
      .def("max_steps", &ia::BatchedEnv::max_steps)
      .def("is_image", &ia::BatchedEnv::is_image)
      .def("state_dim", &ia::BatchedEnv::state_dim)
      .def("name", &ia::BatchedEnv::name)
      .def("seed", &ia::BatchedEnv::seed)
      .def("reset",
           [](ia::BatchedEnv& e) {
             auto obs = obs_tensor(e);
             {
               py::gil_scoped_release rel;
               e.reset(obs.data_ptr());
             }
             return obs;
           })
      .def("step",
           [](ia::BatchedEnv& e, py::array_t<float, py::array::c_style | py::array::forcecast> actions) {
             TORCH_CHECK(actions.ndim() == 2 && actions.shape(0) == e.num_envs() && actions.shape(1) == e.act_dim(),
                         "actions must be [num_envs, act_dim]");
             const int n = e.num_envs();
             auto obs = obs_tensor(e);
             auto tobs = obs_tensor(e);
             auto rew = torch::empty({n}, torch::kFloat32);
             auto term = torch::empty({n}, torch::kUInt8);
             auto trunc = torch::empty({n}, torch::kUInt8);
             auto ep_ret = torch::empty({n}, torch::kFloat64);
             auto ep_len = torch::empty({n}, torch::kInt64);
             const float* a = actions.data();
             {
               py::gil_scoped_release rel;
               e.step(a, obs.data_ptr(), rew.data_ptr<float>(), term.data_ptr<uint8_t>(), trunc.data_ptr<uint8_t>(),
                      tobs.data_ptr(), ep_ret.data_ptr<double>(), ep_len.data_ptr<int64_t>());
             }
             return py::make_tuple(obs, rew, term, trunc, tobs, ep_ret, ep_len);
           })
      .def("get_state",
           [](ia::BatchedEnv& e) {
             py::dict d;
             auto st = torch::from_blob(e.state().data(), {e.num_envs(), e.state_dim()}, torch::kFloat32).clone();
             auto rng = torch::from_blob(e.rng().data(), {e.num_envs()}, torch::kInt64).clone();
             auto t = torch::from_blob(e.elapsed().data(), {e.num_envs()}, torch::kInt64).clone();
             d["state"] = st;
             d["rng"] = rng;
             d["elapsed"] = t;
             if (e.is_image())  // frame stacks [N, 84, 84, 4]
               d["frames"] = torch::from_blob(e.frames().data(), {e.num_envs(), ia::kPongH, ia::kPongW, ia::kPongStack},
                                              torch::kUInt8)
                                 .clone();
             return d;
           })
      .def("set_state", [](ia::BatchedEnv& e, py::dict d) {
        auto st = d["state"].cast<torch::Tensor>().contiguous().to(torch::kFloat32);
        auto rng = d["rng"].cast<torch::Tensor>().contiguous().to(torch::kInt64);
        auto t = d["elapsed"].cast<torch::Tensor>().contiguous().to(torch::kInt64);
        TORCH_CHECK(st.numel() == (int64_t)e.state().size(), "state size mismatch");
        memcpy(e.state().data(), st.data_ptr<float>(), st.numel() * sizeof(float));
        memcpy(e.rng().data(), rng.data_ptr<int64_t>(), rng.numel() * sizeof(int64_t));
        memcpy(e.elapsed().data(), t.data_ptr<int64_t>(), t.numel() * sizeof(int64_t));
        if (e.is_image() && d.contains("frames")) {
          auto fr = d["frames"].cast<torch::Tensor>().contiguous().to(torch::kUInt8);
          TORCH_CHECK(fr.numel() == (int64_t)e.frames().size(), "frames size mismatch");
          memcpy(e.frames().data(), fr.data_ptr<uint8_t>(), fr.numel());
        }
      });
}
