"""Regularizers and λ updaters (reference: tests/test_regularization.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.regularization import regularizers, updaters
from imitation_amd.util import logger as imit_logger


@pytest.fixture
def logger(tmp_path):
    return imit_logger.configure(str(tmp_path), ["stdout"])


@pytest.mark.parametrize("f,interval", [(0.5, (0.9, 1.1)), (0.1, (0.0, 10.0))])
def test_interval_param_scaler(f, interval):
    s = updaters.IntervalParamScaler(f, interval)
    lam = 1.0
    train = th.tensor(1.0)
    assert s(lam, train, th.tensor(interval[1] * 2)) == pytest.approx(lam * (1 + f))
    if interval[0] > 0:
        assert s(lam, train, th.tensor(interval[0] / 2)) == pytest.approx(lam * (1 - f))
    assert s(lam, train, th.tensor((interval[0] + interval[1]) / 2)) == lam
    assert s(lam, 0.0, 0.0) == lam
    assert s(lam, 0.0, 1.0) == pytest.approx(lam * (1 + f))


@pytest.mark.parametrize("bad", [dict(scaling_factor=0.0, tolerable_interval=(0, 1)),
                                 dict(scaling_factor=1.0, tolerable_interval=(0, 1)),
                                 dict(scaling_factor=0.5, tolerable_interval=(1, 0)),
                                 dict(scaling_factor=0.5, tolerable_interval=(-1, 1)),
                                 dict(scaling_factor=0.5, tolerable_interval=(0, 1, 2))])
def test_interval_param_scaler_raises(bad):
    with pytest.raises(ValueError):
        updaters.IntervalParamScaler(**bad)


def test_scaler_argument_validation():
    s = updaters.IntervalParamScaler(0.5, (0.9, 1.1))
    with pytest.raises(ValueError):
        s(0.0, 1.0, 1.0)
    with pytest.raises(ValueError):
        s(1, 1.0, 1.0)
    with pytest.raises(ValueError):
        s(1.0, th.ones(2), 1.0)
    with pytest.raises(ValueError):
        s(1.0, -1.0, 1.0)


def test_regularizer_validation(logger):
    opt = th.optim.SGD([th.nn.Parameter(th.ones(2))], lr=0.1)
    with pytest.raises(ValueError):
        regularizers.LpRegularizer(opt, 0.0, None, logger, p=2)
    with pytest.raises(ValueError):
        regularizers.LpRegularizer(opt, 1.0, None, logger, p=2, val_split=0.5)
    with pytest.raises(ValueError):
        regularizers.LpRegularizer(opt, 1.0, updaters.IntervalParamScaler(0.5, (0.9, 1.1)), logger, p=2)
    with pytest.raises(ValueError):
        regularizers.LpRegularizer(opt, 1.0, None, logger, p=0)


@pytest.mark.parametrize("p", [1, 2, 3])
def test_lp_regularizer(p, logger):
    w = th.nn.Parameter(th.tensor([1.0, -2.0, 3.0]))
    b = th.nn.Parameter(th.tensor([0.5]))
    opt = th.optim.SGD([w, b], lr=0.1)
    reg = regularizers.LpRegularizer.create(initial_lambda=0.25, p=p)(optimizer=opt, logger=logger)
    loss = (w.sum() + b.sum()) * 0.0
    out = reg.regularize_and_backward(loss)
    expect = 0.25 * (np.sum(np.abs([1.0, -2.0, 3.0]) ** p) + 0.5 ** p)
    assert float(out) == pytest.approx(expect, rel=1e-5)
    np.testing.assert_allclose(w.grad.numpy(), 0.25 * p * np.sign([1, -2, 3]) * np.abs([1, -2, 3]) ** (p - 1), rtol=1e-5)


def test_weight_decay_regularizer(logger):
    w = th.nn.Parameter(th.tensor([1.0, -2.0]))
    opt = th.optim.SGD([w], lr=0.1)
    reg = regularizers.WeightDecayRegularizer.create(initial_lambda=0.5)(optimizer=opt, logger=logger)
    reg.regularize_and_backward((w * 3).sum())
    np.testing.assert_allclose(w.detach().numpy(), np.array([1.0, -2.0]) * (1 - 0.5 * 0.1), rtol=1e-6)
    np.testing.assert_allclose(w.grad.numpy(), [3.0, 3.0])


def test_update_params(logger):
    opt = th.optim.SGD([th.nn.Parameter(th.ones(2))], lr=0.1)
    reg = regularizers.LpRegularizer(opt, 1.0, updaters.IntervalParamScaler(0.5, (0.9, 1.1)), logger, p=2, val_split=0.1)
    reg.update_params(1.0, 2.0)
    assert reg.lambda_ == pytest.approx(1.5)
