"""Reward nets, wrappers and serialization (reference: tests/rewards/test_reward_nets.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.envs import spaces
from imitation_amd.rewards import reward_nets, serialize
from imitation_amd.testing import reward_nets as testing_reward_nets
from imitation_amd.util import networks

OBS = spaces.Box(-1, 1, (4,))
ACT = spaces.Discrete(3)


def _batch(n=10, seed=0):
    r = np.random.default_rng(seed)
    obs = r.uniform(-1, 1, (n, 4)).astype(np.float32)
    return obs, r.integers(0, 3, n), r.uniform(-1, 1, (n, 4)).astype(np.float32), r.random(n) < 0.2


MAKERS = {
    "basic": lambda: reward_nets.BasicRewardNet(OBS, ACT),
    "basic_norm": lambda: reward_nets.BasicRewardNet(OBS, ACT, normalize_input_layer=networks.RunningNorm),
    "shaped": lambda: reward_nets.BasicShapedRewardNet(OBS, ACT),
    "normalized": lambda: reward_nets.NormalizedRewardNet(reward_nets.BasicRewardNet(OBS, ACT), networks.RunningNorm),
    "normalized_shaped": lambda: reward_nets.NormalizedRewardNet(reward_nets.BasicShapedRewardNet(OBS, ACT), networks.RunningNorm),
    "ensemble_std": lambda: reward_nets.AddSTDRewardWrapper(testing_reward_nets.make_ensemble(OBS, ACT, 3), default_alpha=0.1),
    "normalized_ensemble_std": lambda: reward_nets.NormalizedRewardNet(
        reward_nets.AddSTDRewardWrapper(testing_reward_nets.make_ensemble(OBS, ACT, 2)), networks.RunningNorm),
}


@pytest.mark.parametrize("name", list(MAKERS))
def test_serialize_identity(name, tmp_path):
    net = MAKERS[name]()
    b = _batch()
    path = tmp_path / "net.pt"
    serialize.save_reward_net(net, path)
    loaded = serialize.load_reward_net(path)
    assert type(loaded) is type(net)
    np.testing.assert_allclose(net.predict(*b), loaded.predict(*b), rtol=1e-6)


@pytest.mark.parametrize(
    "name,key",
    [("shaped", "RewardNet_shaped"), ("shaped", "RewardNet_unshaped"), ("normalized", "RewardNet_normalized"),
     ("normalized", "RewardNet_unnormalized"), ("ensemble_std", "RewardNet_std_added"),
     ("normalized_ensemble_std", "RewardNet_std_added"), ("basic", "zero")],
)
def test_load_reward_registry(name, key, tmp_path):
    net = MAKERS[name]()
    path = tmp_path / "net.pt"
    serialize.save_reward_net(net, path)
    fn = serialize.load_reward(key, str(path), None)
    b = _batch()
    out = fn(*b)
    assert out.shape == (10,)
    if key == "RewardNet_unshaped":
        np.testing.assert_allclose(out, net.base.predict(*b), rtol=1e-6)
    if key == "RewardNet_unnormalized":
        np.testing.assert_allclose(out, net.base.predict(*b), rtol=1e-6)
    if key == "zero":
        assert np.all(out == 0)


def test_wrong_wrapper_structure_raises(tmp_path):
    serialize.save_reward_net(MAKERS["basic"](), tmp_path / "n.pt")
    with pytest.raises(TypeError, match="Wrapper structure should match"):
        serialize.load_reward("RewardNet_shaped", str(tmp_path / "n.pt"), None)


def test_shaping_formula():
    base = reward_nets.BasicRewardNet(OBS, ACT)
    pot = reward_nets.BasicPotentialMLP(OBS, hid_sizes=[8])
    shaped = reward_nets.ShapedRewardNet(base, pot, discount_factor=0.9)
    s, a, ns, d = shaped.preprocess(*_batch())
    expect = base(s, a, ns, d) + 0.9 * (1 - d) * pot(ns).flatten() - pot(s).flatten()
    th.testing.assert_close(shaped(s, a, ns, d), expect)


def test_normalized_reward_net_stats():
    net = MAKERS["normalized"]()
    b = _batch(200)
    for _ in range(20):
        net.predict_processed(*b)
    out = net.predict_processed(*b, update_stats=False)
    assert abs(out.mean()) < 0.1 and abs(out.std() - 1) < 0.2


def test_ensemble_moments():
    ens = testing_reward_nets.make_ensemble(OBS, ACT, 4)
    b = _batch()
    all_r = ens.predict_processed_all(*b)
    mean, var = ens.predict_reward_moments(*b)
    np.testing.assert_allclose(mean, all_r.mean(-1), rtol=1e-6)
    np.testing.assert_allclose(var, all_r.var(-1, ddof=1), rtol=1e-5)
    with pytest.raises(ValueError):
        reward_nets.RewardEnsemble(OBS, ACT, [reward_nets.BasicRewardNet(OBS, ACT)])


def test_add_std_requires_variance():
    with pytest.raises(TypeError):
        reward_nets.AddSTDRewardWrapper(reward_nets.BasicRewardNet(OBS, ACT))


def test_forward_wrapper_on_predict_processed_raises():
    with pytest.raises(ValueError):
        reward_nets.ShapedRewardNet(MAKERS["normalized"](), lambda x: x.sum(1), 0.9)


def test_mock_reward_net():
    m = testing_reward_nets.MockRewardNet(OBS, ACT, value=2.5)
    np.testing.assert_allclose(m.predict(*_batch()), 2.5)


def test_cnn_reward_net_shapes():
    img = spaces.Box(0, 255, (16, 16, 3), dtype=np.uint8)
    for kw in (dict(use_action=True, use_done=False), dict(use_action=True, use_done=True), dict(use_action=False, use_done=True)):
        net = reward_nets.CnnRewardNet(img, ACT, hid_channels=(4, 4), **kw)
        obs = np.random.randint(0, 255, (5, 16, 16, 3), dtype=np.uint8)
        out = net.predict(obs, np.array([0, 1, 2, 0, 1]), obs, np.array([0, 1, 0, 0, 1], bool))
        assert out.shape == (5,)
    with pytest.raises(ValueError):
        reward_nets.CnnRewardNet(OBS, ACT)


def _potential(x):
    return th.zeros(x.shape[0], device=x.device)


def _frozen_lake_venv(rng):
    from imitation_amd.util import util

    return util.make_vec_env("FrozenLake-v1", n_envs=1, rng=rng)


def test_strip_wrappers_basic(rng):
    """Reference ``test_strip_wrappers_basic``: a matching outer wrapper is removed, a
    non-matching one is a no-op."""
    from imitation_amd.rewards import serialize as rserialize
    from imitation_amd.util import networks

    venv = _frozen_lake_venv(rng)
    net = reward_nets.NormalizedRewardNet(reward_nets.BasicRewardNet(venv.observation_space, venv.action_space),
                                          networks.RunningNorm)
    net = rserialize._strip_wrappers(net, wrapper_types=[reward_nets.NormalizedRewardNet])
    assert isinstance(net, reward_nets.BasicRewardNet)
    net = rserialize._strip_wrappers(net, wrapper_types=[reward_nets.ShapedRewardNet])
    assert isinstance(net, reward_nets.BasicRewardNet)


def test_strip_wrappers_complex(rng):
    """Wrappers are stripped outside-in only: the wrong order removes nothing."""
    from imitation_amd.rewards import serialize as rserialize
    from imitation_amd.util import networks

    venv = _frozen_lake_venv(rng)
    net = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space)
    net = reward_nets.ShapedRewardNet(net, _potential, discount_factor=0.99)
    net = reward_nets.NormalizedRewardNet(net, networks.RunningNorm)
    net = rserialize._strip_wrappers(net, wrapper_types=[reward_nets.ShapedRewardNet, reward_nets.NormalizedRewardNet])
    assert isinstance(net, reward_nets.NormalizedRewardNet) and isinstance(net.base, reward_nets.ShapedRewardNet)
    net = rserialize._strip_wrappers(net, wrapper_types=[reward_nets.NormalizedRewardNet, reward_nets.ShapedRewardNet])
    assert isinstance(net, reward_nets.BasicRewardNet)


def test_strip_wrappers_image(rng):
    """The same on a CNN reward net over Atari-shaped frames."""
    from imitation_amd.rewards import serialize as rserialize
    from imitation_amd.util import networks, util

    venv = util.make_vec_env("PongNoFrameskip-v4", n_envs=1, rng=rng)
    net = reward_nets.CnnRewardNet(venv.observation_space, venv.action_space)
    net = reward_nets.ShapedRewardNet(net, _potential, discount_factor=0.99)
    net = reward_nets.NormalizedRewardNet(net, networks.RunningNorm)
    net = rserialize._strip_wrappers(net, wrapper_types=[reward_nets.NormalizedRewardNet, reward_nets.ShapedRewardNet])
    assert isinstance(net, reward_nets.CnnRewardNet)


def test_predict_processed_wrappers_pass_on_kwargs():
    """``NormalizedRewardNet`` / ``AddSTDRewardWrapper``-style wrappers forward extra keyword
    arguments of ``predict_processed`` to the base (reference test of the same name)."""
    from unittest import mock

    from imitation_amd.envs import spaces
    from imitation_amd.testing import reward_nets as testing_reward_nets

    obs_space, act_space = spaces.Box(-1, 1, (2,)), spaces.Box(-1, 1, (1,))
    base = testing_reward_nets.MockRewardNet(obs_space, act_space)
    base.predict_processed = mock.Mock(return_value=np.zeros((10,)))
    from imitation_amd.util import networks

    wrapped = reward_nets.NormalizedRewardNet(base, networks.RunningNorm)  # the reference's concrete wrapper
    args = (np.zeros((10, 2)), np.zeros((10, 1)), np.zeros((10, 2)), np.zeros(10, dtype=bool))
    wrapped.predict_processed(*args, foobar=42)
    base.predict_processed.assert_called_once_with(*args, foobar=42)


def test_predict_processed_wrappers_pass_method_calls_to_base():
    """forward / predict_th / predict / predict_processed / preprocess and the device / dtype
    properties of a PredictProcessedWrapper go to the wrapped net."""
    from unittest import mock

    from imitation_amd.envs import spaces
    from imitation_amd.testing import reward_nets as testing_reward_nets

    obs_space, act_space = spaces.Box(-1, 1, (2,)), spaces.Box(-1, 1, (1,))
    from imitation_amd.util import networks

    base = testing_reward_nets.MockRewardNet(obs_space, act_space)
    wrapper = reward_nets.NormalizedRewardNet(base, networks.RunningNorm)
    np_args = (np.zeros((10, 2), np.float32), np.zeros((10, 1), np.float32), np.zeros((10, 2), np.float32),
               np.zeros(10, dtype=bool))
    th_args = tuple(th.as_tensor(a) for a in np_args)
    for attr, call_with, ret in [("forward", th_args, th.zeros(10)), ("predict_th", np_args, th.zeros(10)),
                                 ("predict", np_args, np.zeros(10)), ("predict_processed", np_args, np.zeros(10)),
                                 ("preprocess", np_args, th_args)]:
        m = mock.MagicMock(return_value=ret)
        object.__setattr__(base, attr, m)
        getattr(wrapper, attr)(*call_with)
        m.assert_called_once_with(*call_with)
    assert wrapper.device == base.device and wrapper.dtype == base.dtype


def test_load_reward_passes_along_alpha_to_add_std_predict_processed(tmp_path):
    """Keyword arguments of load_reward reach AddSTDRewardWrapper.predict_processed: the
    loaded reward function is mean + alpha * std of the members (reference
    test_reward_nets.py:838)."""
    ens = testing_reward_nets.make_ensemble(OBS, ACT, 2)
    net = reward_nets.AddSTDRewardWrapper(ens, default_alpha=0.0)
    path = tmp_path / "net.pt"
    serialize.save_reward_net(net, path)
    b = _batch()
    mean, var = ens.predict_reward_moments(*b)
    for alpha in (-0.5, 0.0, 2.0):
        out = serialize.load_reward("RewardNet_std_added", str(path), None, alpha=alpha)(*b)
        np.testing.assert_allclose(out, mean + alpha * np.sqrt(var), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("wrapper", ["normalized", "std_added"])
def test_predict_processed_wrappers_pass_method_calls_to_base(wrapper):
    """A PredictProcessedWrapper forwards forward / predict_th / predict / preprocess to its
    base and exposes the base's device and dtype (reference test_reward_nets.py:808)."""
    from unittest import mock

    if wrapper == "normalized":
        w = reward_nets.NormalizedRewardNet(reward_nets.BasicRewardNet(OBS, ACT), networks.RunningNorm)
    else:
        w = reward_nets.AddSTDRewardWrapper(testing_reward_nets.make_ensemble(OBS, ACT, 2))
    base = mock.create_autospec(testing_reward_nets.MockRewardNet)
    base.device = th.device("cpu")
    base.dtype = th.float32
    w._base = base
    np_b = _batch()
    th_b = tuple(th.as_tensor(x) for x in np_b)
    for attr, args, ret in [("forward", th_b, th.zeros(10)), ("predict_th", np_b, th.zeros(10)),
                            ("predict", np_b, np.zeros(10)), ("preprocess", np_b, th_b)]:
        setattr(base, attr, mock.MagicMock(return_value=ret))
        getattr(w, attr)(*args)
        getattr(base, attr).assert_called_once_with(*args)
    assert w.device is base.device and w.dtype is base.dtype
