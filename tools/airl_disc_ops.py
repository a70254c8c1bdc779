"""Torch ops / kernels of one eager AIRL discriminator update (airl_hopper recipe)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402


def main():
    from imitation_amd import models
    from imitation_amd.util import networks

    os.environ["IMITATION_AMD_DISC_GRAPH"] = "0"
    b = models.build("airl_hopper", device=th.device("cuda"), seed=0)
    tr = b.trainer
    tr.train_gen(tr.gen_train_timesteps)
    print("disc opt:", type(tr._disc_opt).__name__, "minibatch", tr.demo_minibatch_size, "batch", tr.demo_batch_size, flush=True)
    from torch.profiler import ProfilerActivity, profile

    def one():
        ex = tr._next_expert_batch()
        g_idx = th.randint(0, tr._gen_dev.size(), (tr.demo_batch_size,), device=tr._dev)
        tr._disc_opt.zero_grad()
        with networks.training(tr.reward_train):
            tr._generic_disc_fn(ex["obs"], ex["acts"], ex["next_obs"], ex["dones"], g_idx)

    one()
    th.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        one()
        th.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=70, max_name_column_width=70), flush=True)


if __name__ == "__main__":
    main()
