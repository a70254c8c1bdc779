"""Reward ingredient: ensembles, the AddSTD wrapper and the configuration errors
(upstream tests/scripts/ingredients/test_rewards.py)."""

import numpy as np
import pytest

from imitation_amd.rewards import reward_nets
from imitation_amd.scripts.ingredients import reward
from imitation_amd.util import networks
from imitation_amd.util.util import make_vec_env

MEMBER = {"net_cls": reward_nets.BasicRewardNet, "net_kwargs": {}, "normalize_output_layer": None}


@pytest.fixture
def venv():
    return make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(0), n_envs=1)


def _make(venv, **kw):
    args = dict(venv=venv, net_cls=reward_nets.RewardEnsemble, add_std_alpha=None, net_kwargs={},
                normalize_output_layer=None, ensemble_size=3, ensemble_member_config=MEMBER)
    args.update(kw)
    return reward.make_reward_net(**args)


def test_ensemble_and_std_wrapper(venv):
    net = _make(venv)
    assert isinstance(net, reward_nets.RewardEnsemble) and net.num_members == 3
    wrapped = _make(venv, add_std_alpha=0.0)
    assert isinstance(wrapped, reward_nets.AddSTDRewardWrapper)


def test_plain_net_with_output_norm(venv):
    net = _make(venv, net_cls=reward_nets.BasicRewardNet, normalize_output_layer=networks.RunningNorm)
    assert isinstance(net, reward_nets.NormalizedRewardNet)


@pytest.mark.parametrize("kw, msg", [
    (dict(ensemble_size=None), "Must specify ensemble_size"),
    (dict(ensemble_member_config=None, ensemble_size=5), "Must specify ensemble_member_config"),
    (dict(normalize_output_layer=networks.RunningNorm, ensemble_size=5), "Output normalization not supported on RewardEnsembles"),
])
def test_configuration_errors(venv, kw, msg):
    with pytest.raises(ValueError, match=msg):
        _make(venv, **kw)
