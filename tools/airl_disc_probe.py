"""Phase cycle counters of the fused AIRL discriminator fwd/bwd kernel (block 0) on the
tuned AIRL-Hopper config (demo batch 2048 x 2 rows, 16 updates per round)."""
import os
import sys

import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd.models import recipes

    b = recipes.build("airl_hopper", device="cuda")
    tr = b.trainer
    assert tr._fused_disc, tr._fused_disc_why
    tr.train(tr.gen_train_timesteps)
    th.cuda.synchronize()
    prof = th.zeros(8, dtype=th.int64, device="cuda")
    tr._disc_plan.set_prof(prof)
    from imitation_amd.util import networks

    with networks.training(tr.reward_train):
        for i in range(16):
            tr._fused_disc_update(0)
    th.cuda.synchronize()
    p = prof.cpu().tolist()
    n = max(1, p[6])
    names = ["zero+stage", "policy fwd+logpi", "reward fwds", "loss", "base+pot(s') bwd", "pot(s) bwd"]
    print("airl_fwd_bwd block-0 cycles per call: " + ", ".join(f"{k} {p[i] / n:.0f}" for i, k in enumerate(names)),
          f"(total {sum(p[:6]) / n:.0f}, lds {tr._disc_plan.lds_bytes} B)", flush=True)
    tr._disc_plan.set_prof(None)


if __name__ == "__main__":
    main()
