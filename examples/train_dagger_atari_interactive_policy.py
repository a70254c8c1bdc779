"""DAgger with a human at the keyboard on (synthetic) Pong -- the reference's
examples/train_dagger_atari_interactive_policy.py. The expert is an
:class:`~imitation_amd.policies.interactive.AtariInteractivePolicy` (renders the newest
frame, reads NOOP/FIRE/UP/DOWN keys); the learner is a NatureCNN policy trained by BC.

    python examples/train_dagger_atari_interactive_policy.py
"""

import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from imitation_amd.algorithms import bc, dagger  # noqa: E402
from imitation_amd.policies import interactive  # noqa: E402
from imitation_amd.rl.policies import ActorCriticCnnPolicy  # noqa: E402
from imitation_amd.util.util import make_vec_env  # noqa: E402


def main(total_timesteps: int = 20):
    rng = np.random.default_rng(0)
    env = make_vec_env("PongNoFrameskip-v4", rng=rng, n_envs=1)
    expert = interactive.AtariInteractivePolicy(env)
    learner = ActorCriticCnnPolicy(env.observation_space, env.action_space, lambda _: 1e-3)
    bc_trainer = bc.BC(observation_space=env.observation_space, action_space=env.action_space, rng=rng, policy=learner)
    with tempfile.TemporaryDirectory(prefix="dagger_example_") as tmpdir:
        trainer = dagger.SimpleDAggerTrainer(venv=env, scratch_dir=tmpdir, expert_policy=expert, bc_trainer=bc_trainer,
                                             rng=rng, device_collector=False)  # a human answers every step
        trainer.train(total_timesteps=total_timesteps, rollout_round_min_episodes=1,
                      rollout_round_min_timesteps=total_timesteps)


if __name__ == "__main__":
    main()
