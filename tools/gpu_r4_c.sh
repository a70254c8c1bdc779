# round-4: every BASELINE config at its recipe (1 GPU) + wide-MLP roofline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarking/bench_configs.py --configs all --steps ${STEPS:-2} --warmup 1 --eval-episodes 5 --out gpurun_out/r4c_configs.jsonl > gpurun_out/r4c_configs.log 2>&1 || { echo "configs failed rc=$?"; grep -v Saving gpurun_out/r4c_configs.log | tail -30; exit 1; }
cut -c1-400 gpurun_out/r4c_configs.jsonl
timeout -k 10 200 python -u tools/wlin_roofline.py > gpurun_out/r4c_wlin.md 2> gpurun_out/r4c_wlin.err || { echo "wlin roofline failed"; tail -20 gpurun_out/r4c_wlin.err; exit 1; }
cat gpurun_out/r4c_wlin.md
