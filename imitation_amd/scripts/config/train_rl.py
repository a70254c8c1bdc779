"""Config for ``train_rl`` (reference: scripts/config/train_rl.py)."""

from torch import nn

from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.scripts.ingredients import environment
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, rl

train_rl_ex = Experiment("train_rl", ingredients=[logging_ingredient.logging_ingredient, environment.environment_ingredient,
                                                  rl.rl_ingredient, policy_evaluation.policy_evaluation_ingredient])


@train_rl_ex.config
def train_rl_defaults():
    total_timesteps = int(1e6)
    normalize_reward = True  # VecNormalize on rewards
    normalize_kwargs = dict()
    reward_type = None  # override reward with a learned one (see rewards.serialize)
    reward_path = None
    load_reward_kwargs = {}
    rollout_save_final = True
    rollout_save_n_timesteps = None
    rollout_save_n_episodes = None
    policy_save_interval = 10000  # timesteps between policy saves (<=0 disables)
    policy_save_final = True
    agent_path = None


@train_rl_ex.config
def default_end_cond(rollout_save_n_timesteps, rollout_save_n_episodes):
    if rollout_save_n_timesteps is None and rollout_save_n_episodes is None:
        rollout_save_n_timesteps = 2000


@train_rl_ex.named_config
def acrobot():
    environment = dict(gym_id="Acrobot-v1")


@train_rl_ex.named_config
def cartpole():
    environment = dict(gym_id="CartPole-v1")
    total_timesteps = int(1e5)


@train_rl_ex.named_config
def seals_cartpole():
    environment = dict(gym_id="seals/CartPole-v0", num_vec=8)
    total_timesteps = int(1e5)
    policy = dict(policy_cls="MlpPolicy", policy_kwargs=dict(activation_fn=nn.ReLU, net_arch=[dict(pi=[64, 64], vf=[64, 64])]))
    normalize_reward = False
    rl = dict(batch_size=4096, rl_kwargs=dict(batch_size=256, clip_range=0.4, ent_coef=0.008508727919228772, gae_lambda=0.9,
                                              gamma=0.9999, learning_rate=0.0012403278189645594, max_grad_norm=0.8,
                                              n_epochs=10, vf_coef=0.489343896591493))


@train_rl_ex.named_config
def half_cheetah():
    environment = dict(gym_id="HalfCheetah-v4")
    total_timesteps = int(5e6)


@train_rl_ex.named_config
def seals_half_cheetah():
    environment = dict(gym_id="seals/HalfCheetah-v1", num_vec=1)
    total_timesteps = int(1e6)
    rl = dict(batch_size=512, rl_kwargs=dict(batch_size=64))


@train_rl_ex.named_config
def seals_hopper():
    environment = dict(gym_id="seals/Hopper-v1", num_vec=1)
    total_timesteps = int(1e6)
    rl = dict(batch_size=2048, rl_kwargs=dict(batch_size=512))


@train_rl_ex.named_config
def seals_ant():
    environment = dict(gym_id="seals/Ant-v1", num_vec=1)
    total_timesteps = int(1e6)
    rl = dict(batch_size=2048, rl_kwargs=dict(batch_size=16))


@train_rl_ex.named_config
def seals_swimmer():
    environment = dict(gym_id="seals/Swimmer-v1", num_vec=1)
    total_timesteps = int(1e6)
    rl = dict(batch_size=2048, rl_kwargs=dict(batch_size=64))


@train_rl_ex.named_config
def seals_walker():
    environment = dict(gym_id="seals/Walker2d-v1", num_vec=1)
    total_timesteps = int(1e6)
    rl = dict(batch_size=8192, rl_kwargs=dict(batch_size=128))


@train_rl_ex.named_config
def mountain_car():
    environment = dict(gym_id="MountainCar-v0")


@train_rl_ex.named_config
def seals_mountain_car():
    environment = dict(gym_id="seals/MountainCar-v0")


@train_rl_ex.named_config
def pendulum():
    environment = dict(gym_id="Pendulum-v1")
    rl = dict(batch_size=4096, rl_kwargs=dict(gamma=0.9, learning_rate=1e-3, use_sde=False))
    total_timesteps = int(2e5)


@train_rl_ex.named_config
def fast():
    total_timesteps = int(4)
    policy_save_interval = 2
