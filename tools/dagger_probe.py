"""Phase timing of one device DAgger-Pong round: collect (chunks / host copies) vs BC."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def main():
    from imitation_amd import models

    b = models.build("dagger_pong", device=th.device("cuda"), seed=0)
    tr = b.trainer
    col = tr._device_collector
    kw = dict(n_epochs=1, log_interval=10**9, progress_bar=False)
    for r in range(3):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        trajs = tr._collect_round(1, 2048)
        th.cuda.synchronize()
        t1 = time.perf_counter()
        steps = sum(len(t) for t in trajs)
        tr._aggregate_current_round()
        th.cuda.synchronize()
        t2 = time.perf_counter()
        tr.bc_trainer.train(**kw)
        th.cuda.synchronize()
        t3 = time.perf_counter()
        tr.round_num += 1
        n_b = len(tr._device_agg) // tr.batch_size
        print(f"round {r}: collect {1e3*(t1-t0):.1f} ms ({col.steps_collected} env steps, {steps} kept, "
              f"{1e6*(t1-t0)/max(1,col.steps_collected/col.N):.1f} us/step) aggregate {1e3*(t2-t1):.1f} ms "
              f"bc {1e3*(t3-t2):.1f} ms ({n_b} batches, {1e3*(t3-t2)/max(1,n_b):.3f} ms/batch) graph={col._sets[0]['graph'] is not None}",
              flush=True)
    tr._writer.flush()
    # the bench step (SimpleDAggerTrainer.train, one round), profiled by cProfile on the host
    import cProfile
    import pstats
    for r in range(2):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        pr = cProfile.Profile()
        pr.enable()
        tr.train(2048, rollout_round_min_episodes=1, rollout_round_min_timesteps=2048, bc_train_kwargs=kw)
        th.cuda.synchronize()
        pr.disable()
        dt = time.perf_counter() - t0
        print(f"train step {r}: {1e3*dt:.1f} ms, {tr.last_train_timesteps_local} steps -> {tr.last_train_timesteps_local/dt:.0f} env-steps/s", flush=True)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
    # chunk replay alone
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        col._run_chunk(col._sets[0])
    th.cuda.synchronize()
    print(f"chunk replay: {1e3*(time.perf_counter()-t0)/20:.3f} ms per {col.chunk} steps", flush=True)


if __name__ == "__main__":
    main()
