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
    from imitation_amd.util.util import make_vec_env

    return make_vec_env("CartPole-v1", rng=rng, n_envs=request.param)


@pytest.fixture
def custom_logger(tmp_path):
    from imitation_amd.util import logger

    return logger.configure(str(tmp_path))
