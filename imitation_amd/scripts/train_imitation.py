"""Train BC, DAgger or SQIL (reference: src/imitation/scripts/train_imitation.py).

    python -m imitation_amd.scripts.train_imitation bc with seals_cartpole demonstrations.n_expert_demos=50
"""

from __future__ import annotations

import logging
import os.path as osp
import pathlib
from typing import Any, Dict, Mapping, Optional, Sequence

import numpy as np

from imitation_amd.algorithms import dagger as dagger_algorithm
from imitation_amd.algorithms import sqil as sqil_algorithm
from imitation_amd.data import rollout, types
from imitation_amd.scripts.config.train_imitation import train_imitation_ex
from imitation_amd.scripts.config_engine import FileStorageObserver
from imitation_amd.scripts.ingredients import bc as bc_ingredient
from imitation_amd.scripts.ingredients import demonstrations, environment, expert
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation
from imitation_amd.util import util

logger = logging.getLogger(__name__)


def _collect_stats(imit_stats: Mapping[str, float], expert_trajs: Sequence[types.Trajectory]) -> Dict[str, Any]:
    stats: Dict[str, Any] = {"imit_stats": imit_stats}
    if all(isinstance(t, types.TrajectoryWithRew) for t in expert_trajs):
        stats["expert_stats"] = rollout.rollout_stats(expert_trajs)
    else:
        logger.warning("Expert trajectories do not have reward information, so expert statistics cannot be computed.")
    return stats


@train_imitation_ex.command
def bc(bc: Dict[str, Any], _run, _rnd: np.random.Generator) -> Mapping[str, Mapping[str, float]]:
    """Behavioral cloning; the final policy is saved to ``{log_dir}/final.th``."""
    custom_logger, log_dir = logging_ingredient.setup_logging()
    expert_trajs = demonstrations.get_expert_trajectories()
    with environment.make_venv() as venv:
        trainer = bc_ingredient.make_bc(venv, expert_trajs, custom_logger)
        kwargs = dict(log_rollouts_venv=venv, **bc["train_kwargs"])
        if kwargs["n_epochs"] is None and kwargs["n_batches"] is None:
            kwargs["n_batches"] = 50_000
        trainer.train(**kwargs)
        util.save_policy(trainer.policy, policy_path=osp.join(log_dir, "final.th"))
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    return _collect_stats(imit_stats, expert_trajs)


@train_imitation_ex.command
def dagger(bc: Dict[str, Any], dagger: Mapping[str, Any], _run, _rnd: np.random.Generator) -> Mapping[str, Mapping[str, float]]:
    """DAgger with the expert ingredient's policy as the synthetic teacher."""
    custom_logger, log_dir = logging_ingredient.setup_logging()
    expert_trajs: Optional[Sequence[types.Trajectory]] = None
    if dagger["use_offline_rollouts"]:
        expert_trajs = demonstrations.get_expert_trajectories()
    with environment.make_venv() as venv:
        trainer = bc_ingredient.make_bc(venv, expert_trajs, custom_logger)
        kwargs = dict(log_rollouts_venv=venv, **bc["train_kwargs"])
        if kwargs["n_epochs"] is None and kwargs["n_batches"] is None:
            kwargs["n_epochs"] = 4
        expert_policy = expert.get_expert_policy(venv)
        dagger_trainer = dagger_algorithm.SimpleDAggerTrainer(
            venv=venv, scratch_dir=osp.join(log_dir, "scratch"), expert_trajs=expert_trajs, expert_policy=expert_policy,
            custom_logger=custom_logger, bc_trainer=trainer, beta_schedule=dagger["beta_schedule"], rng=_rnd)
        dagger_trainer.train(total_timesteps=int(dagger["total_timesteps"]), bc_train_kwargs=kwargs)
        print(f"Model saved to {dagger_trainer.save_trainer()}")
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    return _collect_stats(imit_stats, dagger_trainer._all_demos)


@train_imitation_ex.command
def sqil(sqil: Mapping[str, Any], policy: Mapping[str, Any], rl: Mapping[str, Any], _run,
         _rnd: np.random.Generator) -> Mapping[str, Mapping[str, float]]:
    """Soft Q imitation learning (DQN by default)."""
    custom_logger, log_dir = logging_ingredient.setup_logging()
    expert_trajs = demonstrations.get_expert_trajectories()
    with environment.make_venv() as venv:
        trainer = sqil_algorithm.SQIL(venv=venv, demonstrations=expert_trajs, policy=policy["policy_cls"],
                                      custom_logger=custom_logger, rl_algo_class=rl["rl_cls"], rl_kwargs=rl["rl_kwargs"])
        trainer.train(total_timesteps=int(sqil["total_timesteps"]), **sqil["train_kwargs"])
        util.save_policy(trainer.policy, policy_path=osp.join(log_dir, "final.th"))
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    return _collect_stats(imit_stats, expert_trajs)


def main_console(argv=None):
    train_imitation_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "train_imitation"))
    return train_imitation_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
