"""Final policy evaluation ingredient (reference: scripts/ingredients/policy_evaluation.py)."""

from typing import Mapping

import numpy as np

from imitation_amd.data import rollout
from imitation_amd.rl import base as rl_base
from imitation_amd.scripts.config_engine import Ingredient

policy_evaluation_ingredient = Ingredient("policy_evaluation")


@policy_evaluation_ingredient.config
def config():
    n_episodes_eval = 50  # episodes for the final mean ground-truth return
    locals()


@policy_evaluation_ingredient.named_config
def fast():
    n_episodes_eval = 1


@policy_evaluation_ingredient.capture
def eval_policy(rl_algo, venv, n_episodes_eval: int, _rnd: np.random.Generator) -> Mapping[str, float]:
    """``rollout_stats`` of ``n_episodes_eval`` episodes (sets ``rl_algo``'s env to ``venv``)."""
    sample_until = rollout.make_min_episodes(n_episodes_eval)
    if isinstance(rl_algo, rl_base.BaseAlgorithm):
        rl_algo.set_env(venv)
        train_env = rl_algo.get_env()
    else:
        train_env = venv
    trajs = rollout.generate_trajectories(rl_algo, train_env, sample_until=sample_until, rng=_rnd)
    return rollout.rollout_stats(trajs)


@policy_evaluation_ingredient.capture
def eval_trainer(trainer, venv, n_episodes_eval: int, _rnd: np.random.Generator) -> Mapping[str, float]:
    """:func:`eval_policy` of ``trainer.policy`` on ``venv``, run on the GPU by a device engine
    (``device_rollout_stats``: the same ``rollout_stats`` keys and stopping rule, stochastic actions,
    learned-reward returns; no host round trip per env step) when it offers it for this
    configuration, else on the host."""
    dev = getattr(trainer, "device_rollout_stats", None)
    if dev is not None:
        stats = dev(n_episodes_eval)
        if stats is not None:
            return stats
    return eval_policy(trainer.policy, venv)
