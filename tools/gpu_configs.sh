set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cfg}
CFGS=${CFGS:-all}
timeout -k 10 900 python -u benchmarking/bench_configs.py --configs $CFGS --steps ${STEPS:-2} --warmup 1 --eval-episodes 5 --out gpurun_out/configs_$TAG.jsonl > gpurun_out/configs_$TAG.log 2>&1 || { echo "configs failed rc=$?"; grep -v Saving gpurun_out/configs_$TAG.log | tail -30; exit 1; }
cat gpurun_out/configs_$TAG.jsonl
