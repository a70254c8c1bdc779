"""BC minibatch steps only (NatureCNN ActorCriticCnnPolicy, B=32, graphed), for a kernel trace.
``--sep-gather`` / ``--sep-reduce``: the minibatch gather / the conv weight-gradient reductions as a
launch of their own (A/B of the folded launches); ``--sep-fwd``: the default (not split-K) conv forward."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def main():
    from imitation_amd.algorithms import bc
    from imitation_amd.engine.dagger import DeviceDemoAggregate, DeviceTransitionsLoader
    from imitation_amd.envs.vec_env import native_spaces
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util import logger

    if "--sep-gather" in sys.argv:
        bc._DeviceEpochRunner.fuse_gather = False
    if "--sep-fwd" in sys.argv:
        from imitation_amd.ops import bc_cnn

        bc_cnn.FusedCnnBCStep.splitk_fwd = False
    if "--sep-reduce" in sys.argv:
        bc._DeviceEpochRunner.fuse_reduce = False
    obs_space, act_space = native_spaces("PongNoFrameskip-v4")
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: 1e-3).cuda()
    agg = DeviceDemoAggregate("cuda")
    agg.append(th.randint(0, 255, (4096, 84, 84, 4), dtype=th.uint8, device="cuda"), th.randint(0, 6, (4096,), device="cuda"))
    bct = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(0), policy=pol,
                batch_size=32, device="cuda", custom_logger=logger.configure("/tmp/ia_probe_bc", format_strs=[]))
    bct.set_demonstrations(DeviceTransitionsLoader(agg, 32, 0))
    kw = dict(n_batches=100, log_interval=10**9, progress_bar=False)
    bct.train(**kw)
    th.cuda.synchronize()
    t0 = time.perf_counter()
    bct.train(**kw)
    th.cuda.synchronize()
    tag = "".join(f" ({a[2:]})" for a in sys.argv[1:] if a.startswith("--sep"))
    print(f"BC step B=32{tag}: {1e3 * (time.perf_counter() - t0) / 100:.3f} ms/batch", flush=True)


if __name__ == "__main__":
    main()
