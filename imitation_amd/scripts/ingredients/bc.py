"""BC ingredient (reference: scripts/ingredients/bc.py).

Fixes a reference bug: ``make_or_load_policy`` dropped the freshly built policy
(``bc.py:75-76``), so BC always fell back to its default policy regardless of the
``policy`` ingredient; here the configured policy is returned and used.
"""

import warnings
from typing import Optional, Sequence

import torch as th

from imitation_amd.algorithms import bc
from imitation_amd.data import types
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.scripts.ingredients import policy

bc_ingredient = Ingredient("bc", ingredients=[policy.policy_ingredient])


@bc_ingredient.config
def config():
    batch_size = 32
    l2_weight = 3e-5
    optimizer_cls = th.optim.Adam
    optimizer_kwargs = dict(lr=4e-4)
    train_kwargs = dict(n_epochs=None, n_batches=None, log_interval=500)
    agent_path = None  # serialized policy to start from
    locals()


@bc_ingredient.capture
def make_bc(venv, expert_trajs: Sequence[types.Trajectory], custom_logger, batch_size: int, l2_weight: float,
            optimizer_cls, optimizer_kwargs, _rnd) -> bc.BC:
    return bc.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                 policy=make_or_load_policy(venv), demonstrations=expert_trajs, custom_logger=custom_logger, rng=_rnd,
                 batch_size=batch_size, l2_weight=l2_weight, optimizer_cls=optimizer_cls,
                 optimizer_kwargs=optimizer_kwargs)


@bc_ingredient.capture
def make_or_load_policy(venv, agent_path: Optional[str]):
    if agent_path is None:
        return policy.make_policy(venv)
    warnings.warn("When agent_path is specified, policy.policy_cls and policy.policy_kwargs are ignored.", RuntimeWarning)
    return bc.reconstruct_policy(agent_path)
