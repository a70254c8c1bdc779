set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dev -o run -- python bench.py --engine device --steps 3 --warmup 1 > gpurun_out/prof_dev.log 2>&1; echo "prof rc=$?"
