"""MultiBC on the fork's HomogenousFeedForward32Policy ([256, 256, 128], wide MFMA kernels):
ms per graphed minibatch step. Run under rocprofv3 for the kernel trace."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch as th


def main(n_agents=4, batch=256, steps=200):
    from imitation_amd.algorithms import bc
    from imitation_amd.data import types
    from imitation_amd.envs import spaces
    from imitation_amd.util import logger

    rng = np.random.default_rng(0)
    d, N = 12, 8192
    obs = rng.standard_normal((N, d * n_agents)).astype(np.float32)
    acts = np.stack([(obs[:, d * i] > 0).astype(np.int64) for i in range(n_agents)], axis=1)
    demos = types.TransitionsMinimal(obs=obs, acts=acts, infos=np.array([{}] * N))
    th.manual_seed(0)
    tr = bc.MultiBC(single_agent_observation_space=spaces.Box(-10, 10, (d,)), single_agent_action_space=spaces.Discrete(2),
                    observation_overide=lambda i, o: o[:, d * i: d * i + d], action_overide=lambda i, a: a[:, i],
                    num_agents=n_agents, rng=np.random.default_rng(0), demonstrations=demos, batch_size=batch, device="cuda",
                    optimizer_kwargs=dict(lr=1e-3), custom_logger=logger.configure(format_strs=[]))
    from imitation_amd.ops import mlp as mlp_ops

    mlp_ops.set_wide_bf16(tr.policy)  # the benchmarked config opts in to the bf16 wide kernels
    tr.train(n_batches=10, progress_bar=False, log_interval=10**9)
    th.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train(n_batches=steps, progress_bar=False, log_interval=10**9)
    th.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    g = getattr(tr, "_graph_step", None)
    print(f"multibc agents={n_agents} batch={batch} rows/step={batch * n_agents} ms/step={dt * 1e3:.3f} "
          f"samples/s={batch / dt:.0f} graph_replays={g.n_replays if g else 0}", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
