"""Reward-net behaviours of the reference test-suite (``tests/rewards/test_reward_nets.py``):
the construction matrix over env kinds / input selections / normalisers, CNN input
validation, wrapper stripping and structure validation, the serialization identity matrix,
ensembles, AddSTD, shaping, wrapper pass-through, parameterless devices and a training
regression."""

import numpy as np
import pytest
import torch as th

from imitation_amd.envs import make as make_env
from imitation_amd.envs import spaces
from imitation_amd.rewards import reward_nets, serialize
from imitation_amd.testing import reward_nets as testing_reward_nets
from imitation_amd.util import networks

ENVS = ["FrozenLake-v1", "CartPole-v1", "Pendulum-v1"]
IMAGE_ENVS = ["PongNoFrameskip-v4"]
REWARD_NET_KWARGS = [
    {},
    {"normalize_input_layer": networks.RunningNorm},
    {"use_state": True, "use_action": True, "use_next_state": True, "use_done": True},
    {"use_state": False, "use_action": True, "use_next_state": True, "use_done": False},
]
MAKE_REWARD_NET = [reward_nets.BasicRewardNet, reward_nets.BasicShapedRewardNet]
NORMALIZE_OUTPUT = [None, networks.RunningNorm]


def _spaces(env_name):
    env = make_env(env_name)
    return env.observation_space, env.action_space


def _batch(obs_space, act_space, n=6, seed=0):
    obs_space.seed(seed)
    act_space.seed(seed)
    obs = np.stack([obs_space.sample() for _ in range(n)])
    nxt = np.stack([obs_space.sample() for _ in range(n)])
    acts = np.stack([act_space.sample() for _ in range(n)])
    dones = np.zeros(n, dtype=bool)
    dones[-1] = True
    return obs, acts, nxt, dones


def _make(cls, obs_space, act_space, kwargs, normalize_output):
    net = cls(obs_space, act_space, **kwargs)
    if normalize_output is not None:
        net = reward_nets.NormalizedRewardNet(net, normalize_output)
    return net


@pytest.mark.parametrize("env_name", ENVS)
@pytest.mark.parametrize("cls", MAKE_REWARD_NET)
@pytest.mark.parametrize("kwargs", REWARD_NET_KWARGS)
@pytest.mark.parametrize("normalize_output", NORMALIZE_OUTPUT)
def test_init_no_crash_and_predict(env_name, cls, kwargs, normalize_output):
    obs_space, act_space = _spaces(env_name)
    net = _make(cls, obs_space, act_space, kwargs, normalize_output)
    b = _batch(obs_space, act_space)
    out = net.predict(*b)
    assert out.shape == (6,) and np.all(np.isfinite(out))
    proc = net.predict_processed(*b)
    assert proc.shape == (6,) and np.all(np.isfinite(proc))


@pytest.mark.parametrize("env_name", IMAGE_ENVS)
@pytest.mark.parametrize("kwargs", [{}, {"use_action": False}, {"use_state": False, "use_next_state": True},
                                    {"use_done": True}])
@pytest.mark.parametrize("normalize_output", NORMALIZE_OUTPUT)
def test_image_init_no_crash(env_name, kwargs, normalize_output):
    obs_space, act_space = _spaces(env_name)
    net = _make(reward_nets.CnnRewardNet, obs_space, act_space, kwargs, normalize_output)
    b = _batch(obs_space, act_space, n=2)
    assert net.predict(*b).shape == (2,)


NOT_QUITE_IMAGE_SPACES = (
    spaces.Box(0, 255, shape=(84, 84, 3), dtype=np.float32),
    spaces.Box(0, 254, shape=(84, 84, 3), dtype=np.uint8),
    spaces.Box(1, 255, shape=(84, 84, 3), dtype=np.uint8),
    spaces.Box(0, 255, shape=(84, 84), dtype=np.uint8),
)
ATARI_OBS = spaces.Box(0, 255, shape=(84, 84, 3), dtype=np.uint8)


def test_cnn_reward_net_input_validation():
    with pytest.raises(ValueError, match="must take current or next state"):
        reward_nets.CnnRewardNet(ATARI_OBS, spaces.Discrete(14), use_state=False, use_next_state=False)
    for obs_space in NOT_QUITE_IMAGE_SPACES:
        with pytest.raises(ValueError, match="requires observations to be images"):
            reward_nets.CnnRewardNet(obs_space, spaces.Discrete(14))
    with pytest.raises(ValueError, match="can only use Discrete action spaces"):
        reward_nets.CnnRewardNet(ATARI_OBS, spaces.MultiDiscrete((2, 2)))
    reward_nets.CnnRewardNet(ATARI_OBS, spaces.MultiDiscrete((2, 2)), use_action=False)


def test_cnn_potential_input_validation():
    for obs_space in NOT_QUITE_IMAGE_SPACES:
        with pytest.raises(ValueError, match="must be given image inputs"):
            reward_nets.BasicPotentialCNN(obs_space, hid_sizes=(32,))


@pytest.mark.parametrize("dimensions", (1, 3, 4, 5))
def test_cnn_transpose_input_validation(dimensions):
    tens = th.zeros((2,) * dimensions)
    if dimensions == 4:
        assert reward_nets.cnn_transpose(tens).shape == (2, 2, 2, 2)
    else:
        with pytest.raises(ValueError, match="Invalid input: "):
            reward_nets.cnn_transpose(tens)


def _potential(x):
    return th.zeros(len(x), device=x.device)


@pytest.mark.parametrize("image", [False, True])
def test_strip_wrappers(image):
    obs_space, act_space = _spaces(IMAGE_ENVS[0] if image else "FrozenLake-v1")
    base_cls = reward_nets.CnnRewardNet if image else reward_nets.BasicRewardNet
    net = reward_nets.NormalizedRewardNet(base_cls(obs_space, act_space), networks.RunningNorm)
    net = serialize._strip_wrappers(net, wrapper_types=[reward_nets.NormalizedRewardNet])
    assert isinstance(net, base_cls)
    net = serialize._strip_wrappers(net, wrapper_types=[reward_nets.ShapedRewardNet])  # not wrapped: no-op
    assert isinstance(net, base_cls)
    net = reward_nets.ShapedRewardNet(base_cls(obs_space, act_space), _potential, discount_factor=0.99)
    net = reward_nets.NormalizedRewardNet(net, networks.RunningNorm)
    out = serialize._strip_wrappers(net, wrapper_types=[reward_nets.ShapedRewardNet, reward_nets.NormalizedRewardNet])
    assert isinstance(out, reward_nets.NormalizedRewardNet) and isinstance(out.base, reward_nets.ShapedRewardNet)
    out = serialize._strip_wrappers(net, wrapper_types=[reward_nets.NormalizedRewardNet, reward_nets.ShapedRewardNet])
    assert isinstance(out, base_cls)


def test_validate_wrapper_structure():
    obs_space, act_space = _spaces("FrozenLake-v1")

    class RewardNetA(reward_nets.RewardNet):
        def forward(self, *args):  # pragma: no cover
            ...

    class WrapperB(reward_nets.RewardNetWrapper):
        def forward(self, *args):  # pragma: no cover
            ...

    net = WrapperB(RewardNetA(obs_space, act_space))
    assert isinstance(net.base, RewardNetA)
    serialize._validate_wrapper_structure(net, {(WrapperB, RewardNetA)})
    err = pytest.raises(TypeError, match=r"Wrapper structure should match \[.*\] but found \[.*\]")
    with err:
        serialize._validate_wrapper_structure(net, {(RewardNetA,)})
    with pytest.raises(TypeError, match=r"Wrapper structure should match"):
        serialize._validate_wrapper_structure(RewardNetA(obs_space, act_space), {(WrapperB,)})
    with pytest.raises(TypeError, match=r"Wrapper structure should match"):
        serialize._validate_wrapper_structure(net, {(WrapperB, RewardNetA, WrapperB)})
    serialize._validate_wrapper_structure(net, {(WrapperB, RewardNetA), (RewardNetA,)})
    with pytest.raises(TypeError, match=r"Wrapper structure should match"):
        serialize._validate_wrapper_structure(net, {(RewardNetA, WrapperB)})


@pytest.mark.parametrize("env_name", ENVS)
def test_cant_load_unnorm_as_norm(env_name, tmp_path):
    obs_space, act_space = _spaces(env_name)
    path = tmp_path / "net.pt"
    serialize.save_reward_net(reward_nets.BasicRewardNet(obs_space, act_space), path)
    with pytest.raises(TypeError):
        serialize.load_reward("RewardNet_normalized", str(path), None)


@pytest.mark.parametrize("env_name", ENVS)
@pytest.mark.parametrize("cls", MAKE_REWARD_NET)
@pytest.mark.parametrize("kwargs", REWARD_NET_KWARGS)
@pytest.mark.parametrize("normalize_output", NORMALIZE_OUTPUT)
def test_serialize_identity(env_name, cls, kwargs, normalize_output, tmp_path):
    """Save / load (weights_only) gives the same predictions; the normalised wrapper also after
    its statistics moved (train-mode processed predictions)."""
    obs_space, act_space = _spaces(env_name)
    net = _make(cls, obs_space, act_space, kwargs, normalize_output)
    b = _batch(obs_space, act_space)
    if normalize_output is not None:
        for seed in range(3):  # move the output normaliser's statistics
            net.predict_processed(*_batch(obs_space, act_space, seed=seed + 1), update_stats=True)
    path = tmp_path / "net.pt"
    serialize.save_reward_net(net, path)
    loaded = serialize.load_reward_net(path)
    assert type(loaded) is type(net)
    np.testing.assert_allclose(loaded.predict(*b), net.predict(*b), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(loaded.predict_processed(*b, update_stats=False),
                               net.predict_processed(*b, update_stats=False), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("normalize_output", NORMALIZE_OUTPUT)
def test_serialize_identity_images(normalize_output, tmp_path):
    obs_space, act_space = _spaces(IMAGE_ENVS[0])
    net = _make(reward_nets.CnnRewardNet, obs_space, act_space, {}, normalize_output)
    b = _batch(obs_space, act_space, n=2)
    path = tmp_path / "net.pt"
    serialize.save_reward_net(net, path)
    np.testing.assert_allclose(serialize.load_reward_net(path).predict(*b), net.predict(*b), rtol=1e-5, atol=1e-6)


def test_potential_net_2d_obs():
    """Shaping works with 2-D (matrix) observations: flattened by the potential MLP."""
    obs_space = spaces.Box(-1, 1, (3, 4))
    act_space = spaces.Discrete(2)
    net = reward_nets.BasicShapedRewardNet(obs_space, act_space)
    b = _batch(obs_space, act_space)
    assert net.predict(*b).shape == (6,)


@pytest.fixture
def env_2d():
    return spaces.Box(-1, 1, (2,)), spaces.Discrete(2)


def test_ensemble_errors_if_there_are_too_few_members(env_2d):
    obs, act = env_2d
    for n in (0, 1):
        with pytest.raises(ValueError, match="at least 2"):
            reward_nets.RewardEnsemble(obs, act, members=[reward_nets.BasicRewardNet(obs, act) for _ in range(n)])


def test_reward_ensemble_predict_reward_moments(env_2d):
    obs_space, act_space = env_2d
    members = [testing_reward_nets.MockRewardNet(obs_space, act_space, value=v) for v in (1.0, 3.0, 8.0)]
    ens = reward_nets.RewardEnsemble(obs_space, act_space, members=members)
    b = _batch(obs_space, act_space)
    mean, var = ens.predict_reward_moments(*b)
    np.testing.assert_allclose(mean, 4.0)
    np.testing.assert_allclose(var, np.var([1.0, 3.0, 8.0], ddof=1), rtol=1e-6)
    np.testing.assert_allclose(ens.predict(*b), 4.0)


def test_ensemble_members_have_different_parameters(env_2d):
    ens = testing_reward_nets.make_ensemble(*env_2d, num_members=3)
    p = [next(m.parameters()).detach() for m in ens.members]
    assert not th.equal(p[0], p[1]) and not th.equal(p[1], p[2])


def test_add_std_wrapper_raises_error_when_wrapping_wrong_type(env_2d):
    with pytest.raises(TypeError, match="not an instance of RewardNetWithVariance"):
        reward_nets.AddSTDRewardWrapper(reward_nets.BasicRewardNet(*env_2d))


@pytest.mark.parametrize("alpha", [0.0, 0.5, 2.0])
def test_add_std_reward_wrapper(env_2d, alpha):
    obs_space, act_space = env_2d
    members = [testing_reward_nets.MockRewardNet(obs_space, act_space, value=v) for v in (2.0, 4.0)]
    ens = reward_nets.RewardEnsemble(obs_space, act_space, members=members)
    wrapped = reward_nets.AddSTDRewardWrapper(ens, default_alpha=alpha)
    b = _batch(obs_space, act_space)
    np.testing.assert_allclose(wrapped.predict_processed(*b), 3.0 + alpha * np.sqrt(2.0), rtol=1e-6)
    np.testing.assert_allclose(wrapped.predict_processed(*b, alpha=1.0), 3.0 + np.sqrt(2.0), rtol=1e-6)


def test_shaped_reward_net(env_2d):
    obs_space, act_space = env_2d
    base = testing_reward_nets.MockRewardNet(obs_space, act_space, value=1.5)

    def pot(x):
        return x.sum(dim=1)

    net = reward_nets.ShapedRewardNet(base, pot, discount_factor=0.9)
    obs, acts, nxt, dones = _batch(obs_space, act_space)
    exp = 1.5 + 0.9 * (1 - dones) * nxt.sum(1) - obs.sum(1)
    np.testing.assert_allclose(net.predict(obs, acts, nxt, dones), exp, rtol=1e-5, atol=1e-6)


def test_forward_wrapper_cannot_be_applied_predict_processed_wrapper(env_2d):
    norm = reward_nets.NormalizedRewardNet(reward_nets.BasicRewardNet(*env_2d), networks.RunningNorm)
    with pytest.raises(ValueError):
        reward_nets.ShapedRewardNet(norm, _potential, discount_factor=0.99)


def test_predict_processed_wrappers_pass_on_kwargs_and_calls(env_2d):
    """AddSTD -> Normalized chain: kwargs reach the inner predict_processed; unknown
    attributes resolve on the base net."""
    obs_space, act_space = env_2d
    members = [testing_reward_nets.MockRewardNet(obs_space, act_space, value=v) for v in (1.0, 5.0)]
    ens = reward_nets.RewardEnsemble(obs_space, act_space, members=members)
    net = reward_nets.NormalizedRewardNet(reward_nets.AddSTDRewardWrapper(ens), networks.RunningNorm)
    b = _batch(obs_space, act_space)
    low = net.predict_processed(*b, alpha=0.0, update_stats=False)
    high = net.predict_processed(*b, alpha=3.0, update_stats=False)
    assert np.all(high > low)
    assert net.base.base.num_members == 2


def test_load_reward_passes_along_alpha_to_add_std(env_2d, tmp_path):
    obs_space, act_space = env_2d
    members = [testing_reward_nets.MockRewardNet(obs_space, act_space, value=v) for v in (0.0, 2.0)]
    ens = reward_nets.RewardEnsemble(obs_space, act_space, members=members)
    path = tmp_path / "net.pt"
    serialize.save_reward_net(reward_nets.AddSTDRewardWrapper(ens, default_alpha=0.0), path)
    b = _batch(obs_space, act_space)
    fn0 = serialize.load_reward("RewardNet_std_added", str(path), None)
    fn2 = serialize.load_reward("RewardNet_std_added", str(path), None, alpha=2.0)
    np.testing.assert_allclose(fn2(*b) - fn0(*b), 2.0 * np.sqrt(2.0), rtol=1e-5)


@pytest.mark.parametrize("env_name", ENVS)
def test_device_for_parameterless_model(env_name):
    obs_space, act_space = _spaces(env_name)
    net = testing_reward_nets.MockRewardNet(obs_space, act_space)
    assert net.device == th.device("cpu")


@pytest.mark.parametrize("normalize_input_layer", [None, networks.RunningNorm])
def test_training_regression(normalize_input_layer):
    """A BasicRewardNet regresses a smooth function of (s, a) with Adam."""
    obs_space, act_space = spaces.Box(-1, 1, (3,)), spaces.Box(-1, 1, (2,))
    th.manual_seed(0)
    net = reward_nets.BasicRewardNet(obs_space, act_space, normalize_input_layer=normalize_input_layer)
    opt = th.optim.Adam(net.parameters(), lr=1e-2)
    rng = np.random.default_rng(0)
    losses = []
    for _ in range(300):
        s = rng.uniform(-1, 1, (64, 3)).astype(np.float32)
        a = rng.uniform(-1, 1, (64, 2)).astype(np.float32)
        target = th.as_tensor(np.sin(s[:, 0]) + a[:, 1] ** 2)
        st, at, nt, dt = net.preprocess(s, a, s, np.zeros(64, dtype=bool))
        loss = ((net(st, at, nt, dt) - target) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert np.mean(losses[-20:]) < 0.1 * np.mean(losses[:20])


DESERIALIZATION_TYPES = ["zero", "RewardNet_normalized", "RewardNet_unnormalized", "RewardNet_shaped", "RewardNet_unshaped"]


def _saved_reward(env_name, reward_type, tmp_path, is_image):
    """A saved reward net of the shape the reward type's loader expects (reference
    _make_env_and_save_reward_net)."""
    obs_space, act_space = _spaces(env_name)
    if is_image:
        net = reward_nets.CnnRewardNet(obs_space, act_space)
    else:
        net = reward_nets.BasicRewardNet(obs_space, act_space)
    if reward_type == "RewardNet_normalized":
        net = reward_nets.NormalizedRewardNet(net, networks.RunningNorm)
    elif reward_type == "RewardNet_shaped":
        pot_cls = reward_nets.BasicPotentialCNN if is_image else reward_nets.BasicPotentialMLP
        net = reward_nets.ShapedRewardNet(net, pot_cls(obs_space, [8, 8]), discount_factor=0.99)
    path = tmp_path / "reward.pt"
    serialize.save_reward_net(net, path)
    return obs_space, act_space, path


def _assert_reward_valid(env_name, reward_type, tmp_path, is_image):
    obs_space, act_space, path = _saved_reward(env_name, reward_type, tmp_path, is_image)
    n = 10
    obs, acts, next_obs, _ = _batch(obs_space, act_space, n=n)
    fn = serialize.load_reward(reward_type, str(path), None)
    rew = fn(obs, acts, next_obs, np.arange(n))
    assert isinstance(rew, np.ndarray)
    assert rew.shape == (n,)
    assert np.issubdtype(rew.dtype, np.number)


@pytest.mark.parametrize("env_name", ENVS)
@pytest.mark.parametrize("reward_type", DESERIALIZATION_TYPES)
def test_reward_valid(env_name, reward_type, tmp_path):
    """Every registered reward loader returns a numeric [n] array (reference test_reward_valid)."""
    _assert_reward_valid(env_name, reward_type, tmp_path, is_image=False)


@pytest.mark.parametrize("env_name", IMAGE_ENVS)
@pytest.mark.parametrize("reward_type", DESERIALIZATION_TYPES)
def test_reward_valid_image(env_name, reward_type, tmp_path):
    _assert_reward_valid(env_name, reward_type, tmp_path, is_image=True)
