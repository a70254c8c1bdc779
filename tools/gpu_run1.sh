set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --engine host --steps 3 --warmup 1 > gpurun_out/bench_host.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_host -o run -- python bench.py --engine host --steps 1 --warmup 1 > gpurun_out/prof_host.log 2>&1
echo EXIT $?
