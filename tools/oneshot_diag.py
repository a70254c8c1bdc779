"""Determinism / equivalence diagnostic of the DP GAIL round with and without the one-shot path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from imitation_amd.testing import dist_workers as W
from imitation_amd.testing.distributed import run_ranks

if __name__ == "__main__":
    os.environ["IMITATION_AMD_DIST_BACKEND"] = "gloo"
    runs = {}
    for mode in ("0", "0", "1", "1"):
        os.environ["IMITATION_AMD_ONESHOT"] = mode
        runs.setdefault(mode, []).append(run_ranks(W.gail_round_worker, 2, 5, timeout=300))
    def md(a, b, key):
        return [float(np.abs(x - y).max()) for x, y in zip(a[0][key], b[0][key])]
    for key in ("reward", "policy"):
        print(key, "gloo vs gloo", md(runs["0"][0], runs["0"][1], key))
        print(key, "oneshot vs oneshot", md(runs["1"][0], runs["1"][1], key))
        print(key, "gloo vs oneshot", md(runs["0"][0], runs["1"][0], key))
        print(key, "rank0 vs rank1 oneshot", md(runs["1"][0], [runs["1"][0][1]], key))
    print("calls", runs["1"][0][0]["oneshot_calls"])
