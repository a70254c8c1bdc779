"""Config for ``train_preference_comparisons`` (reference: scripts/config/train_preference_comparisons.py)."""

from imitation_amd.algorithms import preference_comparisons
from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.scripts.ingredients import environment
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, reward, rl

train_preference_comparisons_ex = Experiment("train_preference_comparisons", ingredients=[
    logging_ingredient.logging_ingredient, environment.environment_ingredient, reward.reward_ingredient,
    rl.rl_ingredient, policy_evaluation.policy_evaluation_ingredient])

MUJOCO_SHARED_LOCALS = dict(rl=dict(rl_kwargs=dict(ent_coef=0.1)))


@train_preference_comparisons_ex.config
def train_defaults():
    engine = "auto"  # "device": agent rollouts + PPO on the GPU (engine/preference.py); "host": AgentTrainer
    fragment_length = 100  # timesteps per fragment used for comparisons
    total_timesteps = int(1e6)
    total_comparisons = 5000
    num_iterations = 5
    comparison_queue_size = None
    transition_oversampling = 1
    initial_comparison_frac = 0.1
    exploration_frac = 0.0
    preference_model_kwargs = {}
    reward_trainer_kwargs = {"epochs": 3}
    save_preferences = False
    agent_path = None
    gatherer_cls = preference_comparisons.SyntheticGatherer
    gatherer_kwargs = {}
    active_selection = False
    active_selection_oversampling = 2
    uncertainty_on = "logit"
    fragmenter_kwargs = {"warning_threshold": 0}
    trajectory_path = None  # train on a fixed trajectory dataset instead of an agent
    trajectory_generator_kwargs = {}
    allow_variable_horizon = False
    checkpoint_interval = 0
    full_checkpoint_interval = 0  # iterations between FULL trainer checkpoints for exact resume (0 disables)
    full_checkpoint_keep = 3  # newest full checkpoints kept
    resume_from = None  # directory of full checkpoints (a previous run's log_dir/full_checkpoints) to resume from
    query_schedule = "hyperbolic"


@train_preference_comparisons_ex.named_config
def cartpole():
    environment = dict(gym_id="CartPole-v1")
    allow_variable_horizon = True


@train_preference_comparisons_ex.named_config
def seals_cartpole():
    environment = dict(gym_id="seals/CartPole-v0")


@train_preference_comparisons_ex.named_config
def pendulum():
    environment = dict(gym_id="Pendulum-v1")


@train_preference_comparisons_ex.named_config
def mountain_car():
    environment = dict(gym_id="MountainCar-v0")
    allow_variable_horizon = True


@train_preference_comparisons_ex.named_config
def seals_mountain_car():
    environment = dict(gym_id="seals/MountainCar-v0")


@train_preference_comparisons_ex.named_config
def half_cheetah():
    locals().update(**MUJOCO_SHARED_LOCALS)
    environment = dict(gym_id="HalfCheetah-v4")
    rl = dict(batch_size=16384, rl_kwargs=dict(batch_size=1024))


@train_preference_comparisons_ex.named_config
def seals_half_cheetah():
    environment = dict(gym_id="seals/HalfCheetah-v1")
    rl = dict(batch_size=512, rl_kwargs=dict(batch_size=64, clip_range=0.1, ent_coef=3.794797423594763e-06,
                                             gae_lambda=0.95, gamma=0.95, learning_rate=0.0003286871805949382,
                                             max_grad_norm=0.8, n_epochs=5, vf_coef=0.11483689492120866))
    num_iterations = 50
    total_timesteps = 20000000


@train_preference_comparisons_ex.named_config
def seals_ant():
    environment = dict(gym_id="seals/Ant-v1")
    rl = dict(batch_size=2048, rl_kwargs=dict(batch_size=16, clip_range=0.3, ent_coef=3.1441389214159857e-06,
                                              gae_lambda=0.8, gamma=0.995, learning_rate=0.00017959211641976886,
                                              max_grad_norm=0.9, n_epochs=10, vf_coef=0.4351450387648799))


@train_preference_comparisons_ex.named_config
def fast():
    total_timesteps = 50
    total_comparisons = 5
    initial_comparison_frac = 0.2
    num_iterations = 1
    fragment_length = 2
    reward_trainer_kwargs = {"epochs": 1}
