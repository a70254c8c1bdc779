"""Loss- and weight-space regularizers (reference: src/imitation/regularization/regularizers.py).

Built in two steps like the reference: ``SomeRegularizer.create(...)`` returns a
factory; the trainer calls it with its optimizer and logger. The Lp penalty and the
decoupled weight decay run as multi-tensor ops (``torch._foreach_*``), i.e. one
fused launch over all parameters instead of one kernel per tensor.
"""

from __future__ import annotations

import abc
from typing import Generic, Optional, Protocol, Type, TypeVar, Union

import numpy as np
import torch as th
from torch import optim

from imitation_amd.regularization import updaters
from imitation_amd.util import logger as imit_logger

Scalar = Union[th.Tensor, float]
R = TypeVar("R")
Self = TypeVar("Self", bound="Regularizer")
T_Regularizer_co = TypeVar("T_Regularizer_co", covariant=True)


class RegularizerFactory(Protocol[T_Regularizer_co]):
    def __call__(self, *, optimizer: optim.Optimizer, logger: imit_logger.HierarchicalLogger) -> T_Regularizer_co:
        ...


def _params(optimizer: optim.Optimizer):
    return [p for g in optimizer.param_groups for p in g["params"]]


class Regularizer(abc.ABC, Generic[R]):
    optimizer: optim.Optimizer
    lambda_: float
    lambda_updater: Optional[updaters.LambdaUpdater]
    logger: imit_logger.HierarchicalLogger
    val_split: Optional[float]

    def __init__(self, optimizer: optim.Optimizer, initial_lambda: float, lambda_updater: Optional[updaters.LambdaUpdater],
                 logger: imit_logger.HierarchicalLogger, val_split: Optional[float] = None) -> None:
        if lambda_updater is None and np.allclose(initial_lambda, 0.0):
            raise ValueError("If you do not pass a regularizer parameter updater your regularization strength must "
                             "be non-zero, as this would result in no regularization.")
        if val_split is not None and (not isinstance(val_split, float) or np.allclose(val_split, 0.0)
                                      or val_split <= 0 or val_split >= 1):
            raise ValueError(f"val_split = {val_split} must be a float strictly between 0 and 1.")
        if lambda_updater is not None and val_split is None:
            raise ValueError("If you pass a regularizer parameter updater, you must also specify a validation split. "
                             "Otherwise the updater won't have any validation data to use for updating.")
        if lambda_updater is None and val_split is not None:
            raise ValueError("If you pass a validation split, you must also pass a regularizer parameter updater. "
                             "Otherwise you are wasting data into the validation split that will not be used.")
        self.optimizer = optimizer
        self.lambda_ = initial_lambda
        self.lambda_updater = lambda_updater
        self.logger = logger
        self.val_split = val_split
        self.logger.record("regularization_lambda", self.lambda_)

    @classmethod
    def create(cls: Type[Self], initial_lambda: float, lambda_updater: Optional[updaters.LambdaUpdater] = None,
               val_split: Optional[float] = None, **kwargs) -> RegularizerFactory[Self]:
        def factory(*, optimizer: optim.Optimizer, logger: imit_logger.HierarchicalLogger) -> Self:
            return cls(initial_lambda=initial_lambda, optimizer=optimizer, lambda_updater=lambda_updater, logger=logger,
                       val_split=val_split, **kwargs)

        return factory

    @abc.abstractmethod
    def regularize_and_backward(self, loss: th.Tensor) -> R:
        """Apply the regularization and call ``backward`` on the (regularized) loss."""

    def update_params(self, train_loss: Scalar, val_loss: Scalar) -> None:
        if self.lambda_updater is not None:
            self.lambda_ = self.lambda_updater(self.lambda_, train_loss, val_loss)
            self.logger.record("regularization_lambda", self.lambda_)


class LossRegularizer(Regularizer[Scalar]):
    @abc.abstractmethod
    def _loss_penalty(self, loss: Scalar) -> Scalar:
        """Term added to the loss."""

    def regularize_and_backward(self, loss: th.Tensor) -> Scalar:
        regularized_loss = th.add(loss, self._loss_penalty(loss))
        regularized_loss.backward()
        self.logger.record("regularized_loss", regularized_loss.item())
        return regularized_loss


class WeightRegularizer(Regularizer):
    @abc.abstractmethod
    def _weight_penalty(self, weight: th.Tensor, group: dict) -> Scalar:
        """Term added to each weight after backward."""

    def regularize_and_backward(self, loss: th.Tensor) -> None:
        loss.backward()
        with th.no_grad():
            for group in self.optimizer.param_groups:
                for param in group["params"]:
                    param.data = th.add(param.data, self._weight_penalty(param, group))


class LpRegularizer(LossRegularizer):
    """``λ Σ_params ||θ||_p^p``."""

    p: int

    def __init__(self, optimizer: optim.Optimizer, initial_lambda: float, lambda_updater: Optional[updaters.LambdaUpdater],
                 logger: imit_logger.HierarchicalLogger, p: int, val_split: Optional[float] = None) -> None:
        super().__init__(optimizer, initial_lambda, lambda_updater, logger, val_split)
        if not isinstance(p, int) or p < 1:
            raise ValueError("p must be a positive integer")
        self.p = p

    def _loss_penalty(self, loss: Scalar) -> Scalar:
        del loss
        params = _params(self.optimizer)
        norms = th._foreach_norm(params, self.p)  # one multi-tensor launch
        return self.lambda_ * th.stack(norms).pow(self.p).sum()


class WeightDecayRegularizer(WeightRegularizer):
    """Decoupled decay ``θ <- θ - λ lr θ`` (per param group lr)."""

    def _weight_penalty(self, weight, group) -> Scalar:
        return -self.lambda_ * group["lr"] * weight.data

    def regularize_and_backward(self, loss: th.Tensor) -> None:
        loss.backward()
        with th.no_grad():
            for group in self.optimizer.param_groups:
                th._foreach_mul_(list(group["params"]), 1.0 - self.lambda_ * group["lr"])
