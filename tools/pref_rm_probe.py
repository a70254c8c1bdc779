"""DRLHP warm-up reward training in isolation: BasicRewardTrainer (batch 32, AdamW) on a
synthetic Walker2d-shaped preference dataset (500 pairs of 100-step fragments, obs 17,
act 6), 200 epochs as the recipe's initial_epoch_multiplier; prints seconds and the
per-minibatch cost. Run under rocprofv3 for the kernel split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch as th


def main(n_pairs=500, L=100, epochs=200):
    from imitation_amd.algorithms import preference_comparisons as pc
    from imitation_amd.data import types
    from imitation_amd.envs import spaces
    from imitation_amd.rewards.reward_nets import BasicRewardNet
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.networks import RunningNorm

    rng = np.random.default_rng(0)

    def frag():
        return types.TrajectoryWithRew(obs=rng.standard_normal((L + 1, 17)).astype(np.float32),
                                       acts=rng.uniform(-1, 1, (L, 6)).astype(np.float32), infos=None, terminal=False,
                                       rews=rng.standard_normal(L).astype(np.float32))

    pairs = [(frag(), frag()) for _ in range(n_pairs)]
    prefs = rng.integers(0, 2, n_pairs).astype(np.float32)
    th.manual_seed(0)
    rn = BasicRewardNet(spaces.Box(-np.inf, np.inf, (17,)), spaces.Box(-1, 1, (6,)), normalize_input_layer=RunningNorm).cuda()
    trainer = pc.BasicRewardTrainer(pc.PreferenceModel(rn), pc.CrossEntropyRewardLoss(), rng=np.random.default_rng(1),
                                    batch_size=32, epochs=3, custom_logger=imit_logger.configure(format_strs=[]))
    ds = pc.PreferenceDataset()
    ds.push(pairs, prefs)
    import cProfile
    import pstats

    prof = cProfile.Profile() if os.environ.get("PROBE_CPROFILE") else None
    th.cuda.synchronize()
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    trainer.train(ds, epoch_multiplier=epochs / 3)  # cold: packing, store, plan, capture
    th.cuda.synchronize()
    if prof:
        prof.disable()
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)
    print(f"cold call: {time.perf_counter() - t0:.3f} s", flush=True)
    t0 = time.perf_counter()
    trainer.train(ds, epoch_multiplier=epochs / 3)
    th.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_mb = epochs * ((n_pairs + 31) // 32)
    fused = getattr(getattr(trainer, "_mb_graph", None), "fused", None) is not None
    print(f"reward training: {epochs} epochs x {n_pairs} pairs (L={L}): {dt:.3f} s, {1e6 * dt / n_mb:.1f} us / minibatch "
          f"(fused={fused})", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
