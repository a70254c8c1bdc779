"""bench.py's own multi-rank launch (``--gpus N`` without torchrun), rehearsed on gloo."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _run(args, env_extra=None, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_spawns_ranks_and_reports_world():
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--eval-episodes", "0", "--engine", "host"],
             {"IMITATION_AMD_DIST_BACKEND": "gloo", "CUDA_VISIBLE_DEVICES": ""})
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 2 * 4096
    assert len(rec["per_rank_ms_per_step"]) == 2
    assert rec["ms_per_step"] == pytest.approx(max(rec["per_rank_ms_per_step"]), rel=1e-3)


def test_bench_refuses_missing_gpus():
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"CUDA_VISIBLE_DEVICES": ""}, timeout=120)
    assert p.returncode != 0
    assert "needs 2 visible GPUs" in p.stderr
