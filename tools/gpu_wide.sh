set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/algorithms/test_bc.py \
  "tests/ops/test_kernels.py::test_wide_mlp_matches_fp32_linear" "tests/ops/test_kernels.py::test_wide_dw_split_reduction_deterministic" \
  > gpurun_out/pytest_wide.log 2>&1 && tail -3 gpurun_out/pytest_wide.log &&
timeout -k 10 200 python tools/multibc_prof.py 4 256 200 > gpurun_out/multibc.log 2>&1 && cat gpurun_out/multibc.log &&
timeout -k 10 200 python tools/multibc_prof.py 4 1024 100 >> gpurun_out/multibc.log 2>&1 && tail -1 gpurun_out/multibc.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_multibc -o run -- python tools/multibc_prof.py 4 256 100 > gpurun_out/prof_multibc.log 2>&1 && echo PROF_OK
