"""bench.py's driver contract: the JSON line's keys, and the timed region pinned byte for byte.

The imitation-quality phase (expert demonstrations, untimed imitation to a budget, 50
deterministic evaluation episodes) was added around the throughput measurement; the timed
region itself must stay exactly the round-5 code so the headline stays comparable.
"""

import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")

# sha256 of the text between the "timed region" markers (the round-5 timed code, unchanged)
TIMED_REGION_SHA256 = "c80fc8f7dea3d08bae9288a3d1d41a3c6042625eec66875e842b83af7b0ba9f0"

QUALITY_KEYS = ("final_eval_return", "expert_return", "random_return", "normalized_score")
CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config")


def _timed_region(src: str) -> str:
    a = src.index("# --- timed region")
    a = src.index("\n", a) + 1
    b = src.index("    # --- end of timed region ---")
    return src[a:b]


def test_timed_region_is_pinned():
    with open(BENCH) as f:
        region = _timed_region(f.read())
    assert "time.perf_counter()" in region and "trainer.train(steps_per_round * args.steps)" in region
    assert hashlib.sha256(region.encode()).hexdigest() == TIMED_REGION_SHA256, (
        "bench.py's timed region changed: the headline would no longer be comparable with earlier rounds")


def test_timed_region_has_no_quality_work():
    with open(BENCH) as f:
        region = _timed_region(f.read())
    for name in ("expert_demonstrations", "device_evaluate", "quality_steps", "evaluate_policy"):
        assert name not in region


def _run(args, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = env.get("CUDA_VISIBLE_DEVICES", "") if "gpu" in args else ""
    p = subprocess.run([sys.executable, BENCH] + [a for a in args if a != "gpu"], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_json_has_contract_and_quality_keys_on_cpu():
    rec = _run(["--steps", "1", "--warmup", "0", "--eval-episodes", "2", "--engine", "host"])
    for k in CONTRACT_KEYS + QUALITY_KEYS:
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 1 and rec["warmup"] == 0
    # no GPU: the expert phase is skipped, the data field says the demos are random-policy rollouts
    assert rec["normalized_score"] is None and "random-policy demos" in rec["data"]
    assert rec["final_eval_return"] is not None


@pytest.mark.gpu
def test_bench_quality_phase_on_gpu(tmp_path):
    """Short budgets: the expert phase runs, then a second run reuses the cached demonstrations."""
    args = ["gpu", "--steps", "2", "--warmup", "1", "--expert-steps", "300000", "--quality-steps", "200000",
            "--eval-episodes", "10", "--expert-cache", str(tmp_path)]
    a = _run(args)
    for k in QUALITY_KEYS:
        assert isinstance(a[k], float), (k, a[k])
    assert a["expert_cached"] is False and a["imitation_env_steps_per_rank"] >= 200_000
    assert a["config"]["engine"] == "device" and "expert" in a["data"]
    b = _run(args)
    assert b["expert_cached"] is True
    assert b["expert_return"] == a["expert_return"] and b["random_return"] == a["random_return"]
