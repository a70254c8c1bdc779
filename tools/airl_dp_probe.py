"""2-rank one-card AIRL rehearsal: per-round time split into generator (train_gen) and the
rest (discriminator updates + logging), eager gloo DP disc vs graphed one-shot DP disc."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def worker(rank, world, rounds):
    import torch as th

    from imitation_amd.models import recipes

    b = recipes.airl_hopper(device=th.device("cuda", 0), seed=0, rank=rank)
    tr = b.trainer
    gen_t = []
    orig = tr.train_gen

    def timed(*a, **k):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        out = orig(*a, **k)
        th.cuda.synchronize()
        gen_t.append(time.perf_counter() - t0)
        return out

    tr.train_gen = timed
    tr.train(tr.gen_train_timesteps)  # warm-up (graph capture)
    th.cuda.synchronize()
    gen_t.clear()
    t0 = time.perf_counter()
    tr.train(rounds * tr.gen_train_timesteps)
    th.cuda.synchronize()
    tot = (time.perf_counter() - t0) / rounds
    return {"round_ms": tot * 1e3, "gen_ms": float(np.mean(gen_t)) * 1e3, "graphed": tr._graphed_disc_ok()}


if __name__ == "__main__":
    from imitation_amd.testing.distributed import run_ranks

    os.environ["IMITATION_AMD_DIST_BACKEND"] = "gloo"
    for mode in sys.argv[1:] or ["0", "1"]:
        os.environ["IMITATION_AMD_ONESHOT"] = mode
        out = run_ranks(worker, 2, 3, timeout=400)
        print("oneshot", mode, out, flush=True)
