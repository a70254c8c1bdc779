"""Config for ``eval_policy`` (reference: scripts/config/eval_policy.py)."""

from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.scripts.ingredients import environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient

eval_policy_ex = Experiment("eval_policy", ingredients=[logging_ingredient.logging_ingredient,
                                                        environment.environment_ingredient, expert.expert_ingredient])


@eval_policy_ex.config
def replay_defaults():
    eval_n_timesteps = int(1e4)  # Min timesteps to evaluate, optional.
    eval_n_episodes = None  # Num episodes to evaluate, optional.
    videos = False  # save videos (frame stacks; see util.video_wrapper)
    video_kwargs = {}
    render = False
    render_fps = 60
    reward_type = None  # Optional: override with reward of this type
    reward_path = None
    rollout_save_path = None  # where to save rollouts (None: don't)
    explore_kwargs = None  # ExplorationWrapper kwargs (None: don't wrap)


@eval_policy_ex.named_config
def explore_eps_greedy():
    explore_kwargs = dict(switch_prob=1.0, random_prob=0.1)


@eval_policy_ex.named_config
def render():
    environment = dict(num_vec=1, parallel=False)
    render = True


@eval_policy_ex.named_config
def seals_cartpole():
    environment = dict(gym_id="seals/CartPole-v0")


@eval_policy_ex.named_config
def pendulum():
    environment = dict(gym_id="Pendulum-v1")


@eval_policy_ex.named_config
def seals_half_cheetah():
    environment = dict(gym_id="seals/HalfCheetah-v1")


@eval_policy_ex.named_config
def fast():
    environment = dict(gym_id="seals/CartPole-v0", num_vec=1)
    eval_n_timesteps = 1
