"""λ updaters (reference: src/imitation/regularization/updaters.py).

:class:`IntervalParamScaler` scales λ up by ``1 + f`` when ``val/train`` loss exceeds
the tolerable interval and down by ``1 - f`` when below it.
"""

from __future__ import annotations

from typing import Protocol, Tuple, Union

import numpy as np
import torch as th

LossType = Union[th.Tensor, float]


class LambdaUpdater(Protocol):
    """``(lambda_, train_loss, val_loss) -> new lambda``; must be side-effect free."""

    def __call__(self, lambda_, train_loss: LossType, val_loss: LossType) -> float:
        ...


def _is_scalar(x) -> bool:
    return isinstance(x, float) or (isinstance(x, th.Tensor) and x.dim() == 0)


class IntervalParamScaler(LambdaUpdater):
    def __init__(self, scaling_factor: float, tolerable_interval: Tuple[float, float]):
        eps = np.finfo(float).eps
        if not (eps < scaling_factor < 1 - eps):
            raise ValueError("scaling_factor must be in (0, 1) within machine precision.")
        if len(tolerable_interval) != 2:
            raise ValueError("tolerable_interval must be a tuple of length 2")
        lo, hi = tolerable_interval
        if not (0 <= lo < hi):
            raise ValueError("tolerable_interval must be a tuple whose first element is at least 0 and the "
                             "second element is greater than the first")
        self.scaling_factor = scaling_factor
        self.tolerable_interval = tolerable_interval

    def __call__(self, lambda_: float, train_loss: LossType, val_loss: LossType) -> float:
        if not _is_scalar(val_loss):
            raise ValueError("val_loss must be a scalar")
        if not _is_scalar(train_loss):
            raise ValueError("train_loss must be a scalar")
        eps = np.finfo(float).eps
        if abs(lambda_) < eps:
            raise ValueError("lambda_ must not be zero. Make sure that you're not scaling the value of lambda down "
                             "too quickly or passing an initial value of zero to the lambda parameter.")
        if lambda_ < 0:
            raise ValueError("lambda_ must be non-negative")
        if not isinstance(lambda_, float):
            raise ValueError("lambda_ must be a float")
        train = float(train_loss)
        val = float(val_loss)
        if train < 0 or val < 0:
            raise ValueError("losses must be non-negative for this updater")
        if train < eps and val < eps:
            return lambda_
        if train < eps <= val:
            return lambda_ * (1 + self.scaling_factor)
        ratio = val / train
        if ratio > self.tolerable_interval[1]:
            return lambda_ * (1 + self.scaling_factor)
        if ratio < self.tolerable_interval[0]:
            return lambda_ * (1 - self.scaling_factor)
        return lambda_
