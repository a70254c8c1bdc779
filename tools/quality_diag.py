"""Diagnose imitation quality: device PPO on the env reward, host-loop GAIL vs device GAIL on
the tutorial CartPole config (imitation_amd/testing/imitation_quality.py)."""
import os
import sys
import time

import numpy as np
import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd.algorithms.adversarial.gail import GAIL
    from imitation_amd.rewards.reward_nets import BasicRewardNet
    from imitation_amd.rl.evaluation import evaluate_policy
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.testing import imitation_quality as iq
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    what = sys.argv[1:] or ["gt", "device", "host"]
    demos = iq.cartpole_expert_demos()
    for mode in what:
        th.manual_seed(0)
        np.random.seed(0)
        venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(0), n_envs=8)
        learner = PPO(ActorCriticPolicy, venv, batch_size=64, ent_coef=0.0, learning_rate=4e-4, gamma=0.95, n_epochs=5,
                      seed=0, device="cuda")
        rn = BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
        log = imit_logger.configure(f"/tmp/ia_diag_{mode}", format_strs=["csv"])
        if mode == "host":
            tr = GAIL(demonstrations=demos, demo_batch_size=1024, gen_replay_buffer_capacity=512, n_disc_updates_per_round=8,
                      venv=venv, gen_algo=learner, reward_net=rn, custom_logger=log)
        else:
            from imitation_amd.engine.gail import DeviceGAIL

            tr = DeviceGAIL(demonstrations=demos, demo_batch_size=1024, gen_replay_buffer_capacity=512,
                            n_disc_updates_per_round=8, venv=venv, gen_algo=learner, reward_net=rn, custom_logger=log,
                            debug_use_ground_truth=(mode == "gt"))
        t0 = time.perf_counter()
        for r in range(12):
            tr.train(tr.gen_train_timesteps)
            if hasattr(tr, "sync_env_to_host"):
                tr.sync_env_to_host()
            if hasattr(tr, "device_evaluate"):
                rets, _ = tr.device_evaluate(16, seed=7)
                ret = float(np.mean(rets))
            else:
                ev = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(7), n_envs=8)
                ret, _ = evaluate_policy(learner.policy, ev, n_eval_episodes=16)
            print(f"{mode} round {r}: eval return {ret:.1f} ({time.perf_counter() - t0:.1f} s)", flush=True)
        import csv
        with open(f"/tmp/ia_diag_{mode}/progress.csv") as f:
            rows = list(csv.DictReader(f))
        keys = [k for k in rows[-1] if "disc_acc" in k or "ep_rew" in k or "approx_kl" in k or "entropy" in k]
        for row in rows[-3:]:
            print(mode, {k: row[k] for k in keys}, flush=True)


if __name__ == "__main__":
    main()
