"""RL algorithm ingredient (reference: scripts/ingredients/rl.py)."""

import logging
import warnings
from typing import Any, Dict, Mapping, Optional, Type

from imitation_amd.policies import serialize
from imitation_amd.policies.replay_buffer_wrapper import ReplayBufferRewardWrapper
from imitation_amd.rl import base as rl_base
from imitation_amd.rl import buffers
from imitation_amd.rl.off_policy import OffPolicyAlgorithm
from imitation_amd.rl.ppo import PPO
from imitation_amd.rl.sac import SAC
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients.policy import policy_ingredient

rl_ingredient = Ingredient("rl", ingredients=[policy_ingredient, logging_ingredient.logging_ingredient])
logger = logging.getLogger(__name__)


@rl_ingredient.config
def config():
    rl_cls = None
    batch_size = None
    rl_kwargs = dict()
    locals()


@rl_ingredient.config_hook
def config_hook(config, command_name, logger):
    res = {}
    if config["rl"]["rl_cls"] is None and command_name != "sqil":
        res["rl_cls"] = PPO
        res["batch_size"] = 2048  # n_steps = batch_size // num_vec
        res["rl_kwargs"] = dict(learning_rate=3e-4, batch_size=64, n_epochs=10, ent_coef=0.0)
    return res


@rl_ingredient.named_config
def fast():
    batch_size = 2
    rl_kwargs = dict(batch_size=2, n_epochs=1)
    locals()


@rl_ingredient.named_config
def sac():
    rl_cls = SAC
    warnings.warn("SAC currently only supports continuous action spaces.", category=RuntimeWarning)
    batch_size = 256
    rl_kwargs = dict(batch_size=None)
    locals()


def _maybe_add_relabel_buffer(rl_kwargs: Dict[str, Any], relabel_reward_fn=None) -> Dict[str, Any]:
    rl_kwargs = dict(rl_kwargs)
    if relabel_reward_fn:
        bk = dict(reward_fn=relabel_reward_fn)
        bk["replay_buffer_class"] = rl_kwargs.get("replay_buffer_class", buffers.ReplayBuffer)
        rl_kwargs["replay_buffer_class"] = ReplayBufferRewardWrapper
        if "replay_buffer_kwargs" in rl_kwargs:
            bk.update(rl_kwargs["replay_buffer_kwargs"])
        rl_kwargs["replay_buffer_kwargs"] = bk
    return rl_kwargs


@rl_ingredient.capture
def make_rl_algo(venv, rl_cls: Type[rl_base.BaseAlgorithm], batch_size: int, rl_kwargs: Mapping[str, Any],
                 policy: Mapping[str, Any], _seed: int, relabel_reward_fn=None) -> rl_base.BaseAlgorithm:
    if batch_size % venv.num_envs != 0:
        raise ValueError(f"num_envs={venv.num_envs} must evenly divide batch_size={batch_size}.")
    rl_kwargs = dict(rl_kwargs)
    if rl_cls is SAC:
        rl_kwargs.pop("n_epochs", None)
    if issubclass(rl_cls, rl_base.OnPolicyAlgorithm):
        assert "n_steps" not in rl_kwargs, "set 'n_steps' at top-level using 'batch_size'. n_steps = batch_size // num_vec"
        rl_kwargs["n_steps"] = batch_size // venv.num_envs
    elif issubclass(rl_cls, OffPolicyAlgorithm):
        if rl_kwargs.get("batch_size") is not None:
            raise ValueError("set 'batch_size' at top-level")
        rl_kwargs["batch_size"] = batch_size
        rl_kwargs = _maybe_add_relabel_buffer(rl_kwargs, relabel_reward_fn)
    else:
        raise TypeError(f"Unsupported RL algorithm '{rl_cls}'")
    algo = rl_cls(policy=policy["policy_cls"], policy_kwargs=dict(policy["policy_kwargs"]), env=venv, seed=_seed,
                  **rl_kwargs)
    logger.info(f"RL algorithm: {type(algo)}")
    return algo


@rl_ingredient.capture
def load_rl_algo_from_path(_seed: int, agent_path: str, venv, rl_cls: Type[rl_base.BaseAlgorithm],
                           rl_kwargs: Mapping[str, Any], relabel_reward_fn=None) -> rl_base.BaseAlgorithm:
    rl_kwargs = dict(rl_kwargs)
    if rl_cls is SAC:
        rl_kwargs.pop("n_epochs", None)
    if issubclass(rl_cls, OffPolicyAlgorithm):
        rl_kwargs = _maybe_add_relabel_buffer(rl_kwargs, relabel_reward_fn)
    agent = serialize.load_stable_baselines_model(cls=rl_cls, path=agent_path, venv=venv, seed=_seed, **rl_kwargs)
    logger.info(f"Warm starting agent from '{agent_path}'")
    return agent
