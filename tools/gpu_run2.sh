set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; exit 1; }
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python bench.py --engine device --steps 5 --warmup 2 > gpurun_out/bench_device.log 2>&1; echo "bench device rc=$?"
timeout -k 10 300 python bench.py --engine host --steps 2 --warmup 1 > gpurun_out/bench_host.log 2>&1; echo "bench host rc=$?"
