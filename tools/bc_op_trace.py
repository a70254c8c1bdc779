"""List the torch ops (and their kernel launches) of one eager BC minibatch step on NatureCNN."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def main():
    from imitation_amd.algorithms import bc
    from imitation_amd.engine.dagger import DeviceDemoAggregate, DeviceTransitionsLoader
    from imitation_amd.envs.vec_env import native_spaces
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util import logger

    os.environ["IMITATION_AMD_BC_GRAPH"] = "0"
    obs_space, act_space = native_spaces("PongNoFrameskip-v4")
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: 1e-3).cuda()
    agg = DeviceDemoAggregate("cuda")
    agg.append(th.randint(0, 255, (256, 84, 84, 4), dtype=th.uint8, device="cuda"), th.randint(0, 6, (256,), device="cuda"))
    bct = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(0), policy=pol,
                batch_size=32, device="cuda", custom_logger=logger.configure("/tmp/ia_probe_bc", format_strs=[]))
    bct.set_demonstrations(DeviceTransitionsLoader(agg, 32, 0))
    kw = dict(n_batches=2, log_interval=10**9, progress_bar=False)
    bct.train(**kw)
    th.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        bct.train(n_batches=1, log_interval=10**9, progress_bar=False)
        th.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=60), flush=True)


if __name__ == "__main__":
    main()
