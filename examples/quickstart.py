"""Clone the behaviour of an expert with BC -- the reference's examples/quickstart.py on this
framework. The expert comes from the local hub (``experts/``, no network on training nodes)
or is trained here with the in-house PPO; pass ``--fast`` for a seconds-long smoke run.

    python examples/quickstart.py [--fast] [--device cuda]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from imitation_amd.algorithms import bc  # noqa: E402
from imitation_amd.data import rollout  # noqa: E402
from imitation_amd.data.wrappers import RolloutInfoWrapper  # noqa: E402
from imitation_amd.policies.serialize import load_policy  # noqa: E402
from imitation_amd.rl.evaluation import evaluate_policy  # noqa: E402
from imitation_amd.rl.policies import MlpPolicy  # noqa: E402
from imitation_amd.rl.ppo import PPO  # noqa: E402
from imitation_amd.util.util import make_vec_env  # noqa: E402


def get_expert(env, fast: bool, device: str):
    try:
        print("Loading the pretrained expert from the local hub.")
        return load_policy("ppo-huggingface", organization="HumanCompatibleAI", env_name="seals-CartPole-v0", venv=env)
    except FileNotFoundError:
        print("No local hub copy: training an expert.")
        expert = PPO(policy=MlpPolicy, env=env, seed=0, batch_size=64, ent_coef=0.0, learning_rate=3e-4, n_epochs=10,
                     n_steps=64, device=device)
        expert.learn(1_000 if fast else 100_000)
        return expert.policy


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--fast", action="store_true")
    p.add_argument("--device", default="auto")
    a = p.parse_args(argv)
    rng = np.random.default_rng(0)
    env = make_vec_env("seals/CartPole-v0", rng=rng, post_wrappers=[lambda e, _: RolloutInfoWrapper(e)])
    expert = get_expert(env, a.fast, a.device)
    print("Sampling expert transitions.")
    rollouts = rollout.rollout(expert, env, rollout.make_sample_until(min_timesteps=None, min_episodes=4 if a.fast else 50),
                               rng=rng)
    transitions = rollout.flatten_trajectories(rollouts)
    bc_trainer = bc.BC(observation_space=env.observation_space, action_space=env.action_space, demonstrations=transitions,
                       rng=rng, device=a.device)
    n_eval = 2 if a.fast else 10
    before, _ = evaluate_policy(bc_trainer.policy, env, n_eval)
    print(f"Reward before training: {before}")
    print("Training a policy using Behavior Cloning")
    bc_trainer.train(n_epochs=1, progress_bar=False)
    after, _ = evaluate_policy(bc_trainer.policy, env, n_eval)
    print(f"Reward after training: {after}")
    return before, after


if __name__ == "__main__":
    main()
