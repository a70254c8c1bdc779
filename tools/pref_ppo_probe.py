"""Device-engine PPO update per kernel geometry (rc_gmax = cooperating workgroups per
minibatch): the DRLHP agent (MlpPolicy 64x64 ReLU, batch 128, 20 epochs, 8192 rows) or, with
RECIPE=airl_hopper, the AIRL-Hopper generator (batch 512)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402


def main():
    from imitation_amd import models

    recipe = os.environ.get("RECIPE", "preference_walker2d")
    b = models.build(recipe, device=th.device("cuda"), seed=0)
    ag = b.trainer.trajectory_generator if recipe == "preference_walker2d" else b.trainer
    ag._rollout()
    for g in [int(x) for x in os.environ.get("GMAX", "1,2,4,8,16").split(",")]:
        ag._ppo_static["rc_gmax"] = g
        ag._ppo_static["rc_cw"] = int(os.environ.get("RC_CW", "0"))
        path = ag._C.engine_ppo_path(ag._ppo_static)
        ag._ppo_update()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ag._ppo_update()
        th.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        n_mb = ag._last_ppo_info[1]
        print(f"rc_gmax={g} path={path}: ppo update {1e3 * dt:.2f} ms ({1e6 * dt / n_mb:.1f} us/minibatch)", flush=True)


if __name__ == "__main__":
    main()
