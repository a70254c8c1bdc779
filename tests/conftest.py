"""Shared fixtures; registers the ``gpu`` marker (GPU tests run on the MI355X box)."""

import os
import sys

import numpy as np
import pytest
import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "expensive: long-running test")


def pytest_collection_modifyitems(config, items):
    if th.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def torch_single_threaded():
    """Mirror the reference's single-threaded torch fixture (tests/conftest.py:26-39)."""
    n = th.get_num_threads()
    th.set_num_threads(1)
    yield
    th.set_num_threads(n)


@pytest.fixture
def rng():
    return np.random.default_rng(seed=0)


@pytest.fixture
def device():
    return th.device("cuda" if th.cuda.is_available() else "cpu")


@pytest.fixture(params=[1, 4])
def cartpole_venv(request, rng):
    from imitation_amd.data.wrappers import RolloutInfoWrapper
    from imitation_amd.util.util import make_vec_env

    return make_vec_env("seals/CartPole-v0", rng=rng, n_envs=request.param,
                        post_wrappers=[lambda e, _: RolloutInfoWrapper(e)])


@pytest.fixture
def custom_logger(tmp_path):
    from imitation_amd.util import logger

    return logger.configure(str(tmp_path))


TESTDATA = os.path.join(ROOT, "tests", "testdata")
CARTPOLE_EXPERT_ZIP = os.path.join(TESTDATA, "expert_models", "cartpole_0", "policies", "final", "model.zip")


@pytest.fixture(scope="session", autouse=True)
def local_expert_hub(tmp_path_factory):
    """A local stand-in for the HF hub holding the checked-in CartPole expert
    (the reference pulls ``HumanCompatibleAI/ppo-<env>`` from the network)."""
    hub = tmp_path_factory.mktemp("hub")
    for env_name in ("seals-CartPole-v0", "CartPole-v1", "CartPole-v0"):
        d = hub / "HumanCompatibleAI" / f"ppo-{env_name}"
        d.mkdir(parents=True)
        os.symlink(CARTPOLE_EXPERT_ZIP, d / "model.zip")
    old = os.environ.get("IMITATION_AMD_HUB")
    os.environ["IMITATION_AMD_HUB"] = str(hub)
    yield hub
    if old is None:
        os.environ.pop("IMITATION_AMD_HUB", None)
    else:
        os.environ["IMITATION_AMD_HUB"] = old


@pytest.fixture(scope="session")
def expert_cache_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("experts")


@pytest.fixture
def cartpole_expert_trajectories(expert_cache_dir):
    from imitation_amd.testing.expert_trajectories import lazy_generate_expert_trajectories

    return lazy_generate_expert_trajectories(expert_cache_dir, "seals/CartPole-v0", 60, np.random.default_rng(0))


@pytest.fixture
def cartpole_expert_policy(cartpole_venv):
    from imitation_amd.policies import serialize

    return serialize.load_policy("ppo-huggingface", cartpole_venv, env_name="seals/CartPole-v0")


@pytest.fixture
def pendulum_expert_trajectories():
    from imitation_amd.data import serialize

    return serialize.load_with_rewards(os.path.join(TESTDATA, "expert_models", "pendulum_0", "rollouts", "final.npz"))


@pytest.fixture
def pendulum_venv(rng):
    from imitation_amd.data.wrappers import RolloutInfoWrapper
    from imitation_amd.util.util import make_vec_env

    return make_vec_env("Pendulum-v1", rng=rng, n_envs=4, post_wrappers=[lambda e, _: RolloutInfoWrapper(e)])
