"""Sweep device GAIL / AIRL CartPole (tutorial configs) over budgets / replay capacity /
disc updates: eval return per checkpoint. Args: specs "algo:rounds:cap:ndisc:seed"."""
import os
import sys

import numpy as np
import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd.engine.airl import DeviceAIRL
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.rewards.reward_nets import BasicRewardNet, BasicShapedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.testing import imitation_quality as iq
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    demos = iq.cartpole_expert_demos()
    for spec in sys.argv[1:]:
        algo, rounds, cap, ndisc, seed = spec.split(":")
        rounds, cap, ndisc, seed = int(rounds), int(cap), int(ndisc), int(seed)
        th.manual_seed(seed)
        np.random.seed(seed)
        venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(seed), n_envs=8)
        log = imit_logger.configure(f"/tmp/ia_sweep", format_strs=[])
        if algo == "gail":
            learner = PPO(ActorCriticPolicy, venv, batch_size=64, ent_coef=0.0, learning_rate=4e-4, gamma=0.95,
                          n_epochs=5, seed=seed, device="cuda")
            rn = BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
            tr = DeviceGAIL(demonstrations=demos, demo_batch_size=1024, gen_replay_buffer_capacity=cap,
                            n_disc_updates_per_round=ndisc, venv=venv, gen_algo=learner, reward_net=rn, custom_logger=log)
        else:
            learner = PPO(ActorCriticPolicy, venv, batch_size=64, ent_coef=0.0, learning_rate=5e-4, gamma=0.95,
                          clip_range=0.1, vf_coef=0.1, n_epochs=5, seed=seed, device="cuda")
            rn = BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
            tr = DeviceAIRL(demonstrations=demos, demo_batch_size=2048, gen_replay_buffer_capacity=cap,
                            n_disc_updates_per_round=ndisc, venv=venv, gen_algo=learner, reward_net=rn, custom_logger=log)
        out = []
        every = max(1, rounds // 10)
        for r in range(0, rounds, every):
            tr.train(every * tr.gen_train_timesteps)
            rets, _ = tr.device_evaluate(16, seed=7)
            out.append(round(float(np.mean(rets)), 1))
        print(spec, "steps/round", tr.gen_train_timesteps, "eval:", out, flush=True)


if __name__ == "__main__":
    main()
