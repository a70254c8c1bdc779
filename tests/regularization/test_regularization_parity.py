"""Regularizer behaviours of the reference's tests/test_regularization.py, expressed against this
package: logged lambda / regularized loss, custom loss and weight penalties, lambda updates over
a grid of loss ratios, validation of constructor arguments, Lp norms over multi-parameter /
multi-group optimizers and per-group-lr weight decay (CPU)."""

import itertools

import numpy as np
import pytest
import torch as th

from imitation_amd.regularization import regularizers, updaters
from imitation_amd.util import logger as imit_logger

LAMBDAS = [0.1, 1.0, 10.0]
BASES = [10.0, 1.0, 0.1, 0.01]


@pytest.fixture
def log(tmp_path):
    return imit_logger.configure(str(tmp_path), ["stdout"])


def _value(log, key):
    return log.default_logger.name_to_value[key]


class _ScaleLoss(regularizers.LossRegularizer):
    """Regularized loss = (1 + lambda) * loss."""

    def _loss_penalty(self, loss):
        return loss * self.lambda_


class _ScaleWeights(regularizers.WeightRegularizer):
    """After backward every weight becomes (1 + lambda) * weight."""

    def _weight_penalty(self, weight, group):
        return weight * self.lambda_


class _Noop(regularizers.Regularizer):
    def regularize_and_backward(self, loss):
        loss.backward()


def _opt(values=(1.0,), lr=0.1):
    return th.optim.SGD([th.nn.Parameter(th.tensor([v])) for v in values], lr=lr)


@pytest.mark.parametrize("lam", LAMBDAS)
def test_initial_lambda_is_logged(lam, log):
    reg = _Noop(_opt(), lam, None, log)
    assert reg.lambda_ == lam and _value(log, "regularization_lambda") == lam


@pytest.mark.parametrize("lam,base", list(itertools.product(LAMBDAS, BASES)))
def test_update_params_moves_lambda_and_logs_it(lam, base, log):
    scaler = updaters.IntervalParamScaler(0.25, (0.9, 1.1))
    reg = _Noop(_opt(), lam, scaler, log, val_split=0.1)
    train = th.tensor(base)
    val = train * scaler.tolerable_interval[1] * 2  # overfitting: lambda grows
    want = scaler(lam, train, val)
    reg.update_params(train, val)
    assert want == pytest.approx(lam * 1.25) and reg.lambda_ == want
    assert _value(log, "regularization_lambda") == want
    reg.update_params(train, train * 0.5)  # val / train below the interval: lambda shrinks
    assert reg.lambda_ == pytest.approx(want * 0.75)


def test_update_params_without_updater_keeps_lambda(log):
    reg = _Noop(_opt(), 0.5, None, log)
    reg.update_params(1.0, 100.0)
    assert reg.lambda_ == 0.5


@pytest.mark.parametrize("lam,base", list(itertools.product(LAMBDAS, BASES)))
def test_loss_regularizer_scales_loss_and_gradient(lam, base, log):
    opt = _opt((2.0,))
    (w,) = opt.param_groups[0]["params"]
    reg = _ScaleLoss(opt, lam, None, log)
    opt.zero_grad()
    loss = base * w.sum()
    out = reg.regularize_and_backward(loss)
    assert th.allclose(out.detach(), loss.detach() * (1 + lam))
    assert _value(log, "regularized_loss") == pytest.approx(float(out.detach()))
    assert th.allclose(w.grad, th.tensor([base * (1 + lam)]))


@pytest.mark.parametrize("lam,base", list(itertools.product(LAMBDAS, BASES)))
def test_weight_regularizer_applies_penalty_after_backward(lam, base, log):
    opt = _opt((3.0,))
    (w,) = opt.param_groups[0]["params"]
    w0 = w.detach().clone()
    reg = _ScaleWeights(opt, lam, None, log)
    opt.zero_grad()
    reg.regularize_and_backward(base * w.pow(2).sum() / 2)
    # the gradient is taken at the weight BEFORE the penalty, the weight afterwards
    assert th.allclose(w.grad, base * w0)
    assert th.allclose(w.detach(), w0 * (1 + lam))


@pytest.mark.parametrize("val_split", [0.0, 1.0, -0.5, 1.5, 1, "0.1"])
def test_bad_val_split_raises(val_split, log):
    with pytest.raises(ValueError, match="val_split"):
        _Noop(_opt(), 1.0, updaters.IntervalParamScaler(0.5, (0.9, 1.1)), log, val_split=val_split)


def test_constructor_argument_combinations(log):
    scaler = updaters.IntervalParamScaler(0.5, (0.9, 1.1))
    with pytest.raises(ValueError, match="non-zero"):
        _Noop(_opt(), 0.0, None, log)
    with pytest.raises(ValueError, match="validation split"):
        _Noop(_opt(), 1.0, scaler, log)
    with pytest.raises(ValueError, match="updater"):
        _Noop(_opt(), 1.0, None, log, val_split=0.2)
    # a zero initial lambda is fine when an updater can raise it
    reg = _Noop(_opt(), 0.0, scaler, log, val_split=0.2)
    assert reg.lambda_ == 0.0


@pytest.mark.parametrize("p", [0.5, 1.5, -1, 0, "random value"])
def test_lp_regularizer_rejects_non_positive_integer_p(p, log):
    with pytest.raises(ValueError):
        regularizers.LpRegularizer(_opt(), 1.0, None, log, p=p)


@pytest.mark.parametrize("p,lam", list(itertools.product([1, 2, 3], [0.1, 1.0])))
def test_lp_regularizer_over_parameter_groups(p, lam, log):
    g = th.Generator().manual_seed(p)
    a = th.nn.Parameter(th.randn(3, 2, generator=g))
    b = th.nn.Parameter(th.randn(4, generator=g))
    c = th.nn.Parameter(th.randn(2, 2, generator=g))
    opt = th.optim.SGD([{"params": [a, b], "lr": 0.1}, {"params": [c], "lr": 0.01}])
    reg = regularizers.LpRegularizer(opt, lam, None, log, p=p)
    opt.zero_grad()
    loss = (a * 0).sum() + (b * 0).sum() + (c * 0).sum()
    out = reg.regularize_and_backward(loss)
    ps = [x.detach().numpy() for x in (a, b, c)]
    want = lam * sum(np.sum(np.abs(x) ** p) for x in ps)
    assert float(out) == pytest.approx(want, rel=1e-5)
    for x, xd in zip((a, b, c), ps):
        np.testing.assert_allclose(x.grad.numpy(), lam * p * np.sign(xd) * np.abs(xd) ** (p - 1), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("lam", [0.1, 1.0, 5.0])
def test_weight_decay_uses_each_group_lr(lam, log):
    a = th.nn.Parameter(th.tensor([1.0, -2.0]))
    c = th.nn.Parameter(th.tensor([4.0]))
    opt = th.optim.SGD([{"params": [a], "lr": 0.1}, {"params": [c], "lr": 0.02}])
    reg = regularizers.WeightDecayRegularizer(opt, lam, None, log)
    opt.zero_grad()
    reg.regularize_and_backward((a * 2).sum() + (c * 3).sum())
    np.testing.assert_allclose(a.detach().numpy(), np.array([1.0, -2.0]) * (1 - lam * 0.1), rtol=1e-6)
    np.testing.assert_allclose(c.detach().numpy(), np.array([4.0]) * (1 - lam * 0.02), rtol=1e-6)
    np.testing.assert_allclose(a.grad.numpy(), [2.0, 2.0])
    np.testing.assert_allclose(c.grad.numpy(), [3.0])


def test_factory_passes_arguments_through(log):
    scaler = updaters.IntervalParamScaler(0.5, (0.9, 1.1))
    make = regularizers.LpRegularizer.create(initial_lambda=0.3, lambda_updater=scaler, val_split=0.2, p=2)
    reg = make(optimizer=_opt(), logger=log)
    assert isinstance(reg, regularizers.LpRegularizer)
    assert (reg.lambda_, reg.lambda_updater, reg.val_split, reg.p) == (0.3, scaler, 0.2, 2)


@pytest.mark.parametrize("lam,ratio", list(itertools.product([0.5, 2.0], [0.5, 0.95, 1.0, 1.05, 3.0])))
def test_interval_scaler_direction(lam, ratio):
    s = updaters.IntervalParamScaler(0.2, (0.9, 1.1))
    new = s(lam, th.tensor(2.0), th.tensor(2.0 * ratio))
    if ratio > 1.1:
        assert new == pytest.approx(lam * 1.2)
    elif ratio < 0.9:
        assert new == pytest.approx(lam * 0.8)
    else:
        assert new == lam
