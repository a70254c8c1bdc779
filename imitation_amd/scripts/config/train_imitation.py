"""Config for ``train_imitation`` (bc / dagger / sqil; reference: scripts/config/train_imitation.py)."""

from imitation_amd.scripts.config import register_tuned, tuned_hps
from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.scripts.ingredients import bc
from imitation_amd.scripts.ingredients import demonstrations as demos_common
from imitation_amd.scripts.ingredients import environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, sqil

train_imitation_ex = Experiment("train_imitation", ingredients=[
    logging_ingredient.logging_ingredient, demos_common.demonstrations_ingredient, expert.expert_ingredient,
    environment.environment_ingredient, policy_evaluation.policy_evaluation_ingredient, bc.bc_ingredient,
    sqil.sqil_ingredient])


@train_imitation_ex.config
def config():
    dagger = dict(use_offline_rollouts=False, total_timesteps=1e5, beta_schedule=None,
                  # rounds between FULL trainer checkpoints ({log_dir}/full_checkpoints; 0 disables), newest kept,
                  # and a previous run's full_checkpoints dir to resume from (its scratch dir is reused)
                  full_checkpoint_interval=0, full_checkpoint_keep=3, resume_from=None)


@train_imitation_ex.named_config
def mountain_car():
    environment = dict(gym_id="MountainCar-v0")
    bc = dict(l2_weight=0.0)
    dagger = dict(total_timesteps=20000)


@train_imitation_ex.named_config
def seals_mountain_car():
    environment = dict(gym_id="seals/MountainCar-v0")
    bc = dict(l2_weight=0.0)
    dagger = dict(total_timesteps=20000)


@train_imitation_ex.named_config
def cartpole():
    environment = dict(gym_id="CartPole-v1")
    dagger = dict(total_timesteps=20000)


@train_imitation_ex.named_config
def seals_cartpole():
    environment = dict(gym_id="seals/CartPole-v0")
    dagger = dict(total_timesteps=20000)


@train_imitation_ex.named_config
def pendulum():
    environment = dict(gym_id="Pendulum-v1")


@train_imitation_ex.named_config
def half_cheetah():
    environment = dict(gym_id="HalfCheetah-v4")
    bc = dict(l2_weight=0.0)
    dagger = dict(total_timesteps=60000)


@train_imitation_ex.named_config
def fast():
    dagger = dict(total_timesteps=50)
    bc = dict(train_kwargs=dict(n_batches=50))
    sqil = dict(total_timesteps=50)


register_tuned(train_imitation_ex, [f"{a}_seals_{e}" for a in ("bc", "dagger")
                                    for e in ("ant", "half_cheetah", "hopper", "swimmer", "walker")])
register_tuned(train_imitation_ex, ["fast_dagger_seals_cartpole"])
