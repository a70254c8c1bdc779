"""Time the NatureCNN pieces of DAgger-Pong on the GPU: policy inference at B=8 and one BC
minibatch step (B=32) -- eager vs graphed -- to see where a DAgger round goes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    th.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main():
    from imitation_amd.algorithms import bc
    from imitation_amd.engine.dagger import DeviceDemoAggregate, DeviceTransitionsLoader, policy_actions
    from imitation_amd.envs.vec_env import native_spaces
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util import logger

    obs_space, act_space = native_spaces("PongNoFrameskip-v4")
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: 1e-3).cuda()
    for B in (8, 32):
        x = th.randint(0, 255, (B, 84, 84, 4), dtype=th.uint8, device="cuda")
        with th.no_grad():
            ms = timeit(lambda: policy_actions(pol, x, False))
        print(f"policy_actions B={B}: {ms:.3f} ms", flush=True)
    agg = DeviceDemoAggregate("cuda")
    agg.append(th.randint(0, 255, (4096, 84, 84, 4), dtype=th.uint8, device="cuda"),
               th.randint(0, 6, (4096,), device="cuda"))
    bct = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(0), policy=pol,
                batch_size=32, device="cuda", custom_logger=logger.configure("/tmp/ia_probe_bc", format_strs=[]))
    bct.set_demonstrations(DeviceTransitionsLoader(agg, 32, 0))
    kw = dict(n_batches=64, log_interval=10**9, progress_bar=False)
    ms = timeit(lambda: bct.train(**kw), n=3) / 64
    print(f"BC step B=32 (graphed={bct._graphed_step() is not None}): {ms:.3f} ms/batch", flush=True)
    os.environ["IMITATION_AMD_BC_GRAPH"] = "0"
    bct._graph_step = None
    ms = timeit(lambda: bct.train(**kw), n=3) / 64
    print(f"BC step B=32 eager: {ms:.3f} ms/batch", flush=True)


if __name__ == "__main__":
    main()
