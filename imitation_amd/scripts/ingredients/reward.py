"""Reward-net ingredient (reference: scripts/ingredients/reward.py)."""

import logging
from typing import Any, Mapping, Optional, Type

from imitation_amd.rewards import reward_nets
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.util import networks

reward_ingredient = Ingredient("reward")
logger = logging.getLogger(__name__)


@reward_ingredient.config
def config():
    net_cls = None  # defaults to BasicRewardNet (BasicShapedRewardNet for airl), see config_hook
    net_kwargs = {}
    normalize_output_layer = networks.RunningNorm
    add_std_alpha = None
    ensemble_size = None
    ensemble_member_config = {}
    locals()


@reward_ingredient.named_config
def normalize_input_disable():
    net_kwargs = {"normalize_input_layer": None}


@reward_ingredient.named_config
def normalize_input_running():
    net_kwargs = {"normalize_input_layer": networks.RunningNorm}


@reward_ingredient.named_config
def normalize_output_disable():
    normalize_output_layer = None


@reward_ingredient.named_config
def normalize_output_running():
    normalize_output_layer = networks.RunningNorm


@reward_ingredient.named_config
def normalize_output_ema():
    normalize_output_layer = networks.EMANorm


@reward_ingredient.named_config
def reward_ensemble():
    net_cls = reward_nets.RewardEnsemble
    add_std_alpha = 0
    ensemble_size = 5
    normalize_output_layer = None
    ensemble_member_config = {"net_cls": reward_nets.BasicRewardNet, "net_kwargs": {},
                              "normalize_output_layer": networks.RunningNorm}
    locals()


@reward_ingredient.config_hook
def config_hook(config, command_name, logger):
    res = {}
    if config["reward"]["net_cls"] is None:
        res["net_cls"] = reward_nets.BasicShapedRewardNet if command_name == "airl" else reward_nets.BasicRewardNet
    if "normalize_input_layer" not in config["reward"]["net_kwargs"]:
        res["net_kwargs"] = {"normalize_input_layer": networks.RunningNorm}
    if "net_cls" in res and issubclass(res["net_cls"], reward_nets.RewardEnsemble):
        del res["net_kwargs"]["normalize_input_layer"]
    return res


def _make_reward_net(venv, net_cls: Type[reward_nets.RewardNet], net_kwargs: Mapping[str, Any],
                     normalize_output_layer: Optional[Type[networks.BaseNorm]]):
    net = net_cls(venv.observation_space, venv.action_space, **net_kwargs)
    if normalize_output_layer is not None:
        net = reward_nets.NormalizedRewardNet(net, normalize_output_layer)
    return net


@reward_ingredient.capture
def make_reward_net(venv, net_cls: Type[reward_nets.RewardNet], net_kwargs: Mapping[str, Any],
                    normalize_output_layer: Optional[Type[networks.BaseNorm]], add_std_alpha: Optional[float],
                    ensemble_size: Optional[int], ensemble_member_config: Optional[Mapping[str, Any]]) -> reward_nets.RewardNet:
    if issubclass(net_cls, reward_nets.RewardEnsemble):
        if ensemble_member_config is None:
            raise ValueError("Must specify ensemble_member_config.")
        if ensemble_size is None:
            raise ValueError("Must specify ensemble_size.")
        members = [_make_reward_net(venv, **ensemble_member_config) for _ in range(ensemble_size)]
        net: reward_nets.RewardNet = net_cls(venv.observation_space, venv.action_space, members)
        if add_std_alpha is not None:
            net = reward_nets.AddSTDRewardWrapper(net, default_alpha=add_std_alpha)
        if normalize_output_layer is not None:
            raise ValueError("Output normalization not supported on RewardEnsembles.")
        return net
    return _make_reward_net(venv, net_cls, net_kwargs, normalize_output_layer)
