"""Config for ``train_adversarial`` (reference: scripts/config/train_adversarial.py)."""

from imitation_amd.rewards import reward_nets
from imitation_amd.scripts.config import register_tuned
from imitation_amd.scripts.config_engine import Experiment
from imitation_amd.scripts.ingredients import demonstrations, environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, reward, rl

train_adversarial_ex = Experiment(
    "train_adversarial",
    ingredients=[logging_ingredient.logging_ingredient, demonstrations.demonstrations_ingredient,
                 reward.reward_ingredient, rl.rl_ingredient, expert.expert_ingredient,
                 environment.environment_ingredient, policy_evaluation.policy_evaluation_ingredient],
)


@train_adversarial_ex.config
def defaults():
    show_config = False
    total_timesteps = int(1e6)  # environment transitions to sample
    algorithm_kwargs = dict(
        demo_batch_size=1024,  # expert samples per discriminator update
        n_disc_updates_per_round=4,
    )
    algorithm_specific = {}  # algorithm_specific[<command>] is merged into the config
    checkpoint_interval = 0  # rounds between checkpoints (<0 disables)
    full_checkpoint_interval = 0  # rounds between FULL trainer checkpoints for exact resume (0 disables)
    full_checkpoint_keep = 3  # newest full checkpoints kept
    resume_from = None  # directory of full checkpoints (a previous run's log_dir/full_checkpoints) to resume from
    agent_path = None  # warm-start generator from this model
    engine = "auto"  # "device": whole GAIL / AIRL round on the GPU (engine/{gail,airl}.py); "host": reference loop


@train_adversarial_ex.config
def aliases_default_gen_batch_size(algorithm_kwargs, rl):
    # replay capacity == generator batch: equivalent to no replay buffer (reference default)
    algorithm_kwargs["gen_replay_buffer_capacity"] = rl["batch_size"]


MUJOCO_SHARED_LOCALS = dict(rl=dict(rl_kwargs=dict(ent_coef=0.1)))


@train_adversarial_ex.named_config
def acrobot():
    environment = dict(gym_id="Acrobot-v1")
    algorithm_kwargs = {"allow_variable_horizon": True}


@train_adversarial_ex.named_config
def cartpole():
    environment = dict(gym_id="CartPole-v1")
    algorithm_kwargs = {"allow_variable_horizon": True}


@train_adversarial_ex.named_config
def seals_cartpole():
    environment = dict(gym_id="seals/CartPole-v0")
    total_timesteps = int(1.4e6)


@train_adversarial_ex.named_config
def mountain_car():
    environment = dict(gym_id="MountainCar-v0")
    algorithm_kwargs = {"allow_variable_horizon": True}


@train_adversarial_ex.named_config
def seals_mountain_car():
    environment = dict(gym_id="seals/MountainCar-v0")


@train_adversarial_ex.named_config
def pendulum():
    environment = dict(gym_id="Pendulum-v1")


CHEETAH_SHARED_LOCALS = dict(
    MUJOCO_SHARED_LOCALS,
    rl=dict(batch_size=16384, rl_kwargs=dict(batch_size=1024)),
    algorithm_specific=dict(airl=dict(total_timesteps=int(5e6)), gail=dict(total_timesteps=int(8e6))),
    reward=dict(algorithm_specific=dict(airl=dict(net_cls=reward_nets.BasicShapedRewardNet,
                                                  net_kwargs=dict(reward_hid_sizes=(32,), potential_hid_sizes=(32,))))),
    algorithm_kwargs=dict(n_disc_updates_per_round=16, gen_replay_buffer_capacity=16384, demo_batch_size=8192),
)


@train_adversarial_ex.named_config
def half_cheetah():
    locals().update(**CHEETAH_SHARED_LOCALS)
    environment = dict(gym_id="HalfCheetah-v4")


@train_adversarial_ex.named_config
def seals_half_cheetah():
    locals().update(**CHEETAH_SHARED_LOCALS)
    environment = dict(gym_id="seals/HalfCheetah-v1")


@train_adversarial_ex.named_config
def seals_hopper():
    locals().update(**MUJOCO_SHARED_LOCALS)
    environment = dict(gym_id="seals/Hopper-v1")


@train_adversarial_ex.named_config
def seals_walker():
    locals().update(**MUJOCO_SHARED_LOCALS)
    environment = dict(gym_id="seals/Walker2d-v1")


@train_adversarial_ex.named_config
def seals_swimmer():
    locals().update(**MUJOCO_SHARED_LOCALS)
    environment = dict(gym_id="seals/Swimmer-v1")


@train_adversarial_ex.named_config
def seals_ant():
    locals().update(**MUJOCO_SHARED_LOCALS)
    environment = dict(gym_id="seals/Ant-v1")
    total_timesteps = int(3e7)
    algorithm_kwargs = dict(shared=dict(demo_batch_size=8192))
    rl = dict(batch_size=16384)


@train_adversarial_ex.named_config
def fast():
    # Minimal compute for tests: >=10 timesteps so at least one round happens.
    total_timesteps = 10
    algorithm_kwargs = dict(demo_batch_size=1, n_disc_updates_per_round=4)


register_tuned(train_adversarial_ex, [f"{a}_seals_{e}" for a in ("airl", "gail")
                                      for e in ("ant", "half_cheetah", "hopper", "swimmer", "walker")])
