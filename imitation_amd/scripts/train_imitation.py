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
from imitation_amd.utils import watchdog

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
        with watchdog.cli_watchdog("train_imitation") as wd:
            if kwargs.get("on_epoch_end") is None:  # (per epoch: the graphed device epochs call nothing per batch)
                kwargs["on_epoch_end"] = wd.beat
            trainer.train(**kwargs)
        util.save_policy(trainer.policy, policy_path=osp.join(log_dir, "final.th"))
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    return _collect_stats(imit_stats, expert_trajs)


@train_imitation_ex.command
def dagger(bc: Dict[str, Any], dagger: Mapping[str, Any], _run, _rnd: np.random.Generator) -> Mapping[str, Mapping[str, float]]:
    """DAgger with the expert ingredient's policy as the synthetic teacher.

    ``dagger.full_checkpoint_interval`` > 0 writes the whole trainer state every that many rounds
    to ``{log_dir}/full_checkpoints`` (:func:`imitation_amd.utils.checkpoint.dagger_state`);
    ``dagger.resume_from=<dir>`` restores the newest one, reuses that run's scratch dir (the round
    files the host path re-reads) and collects only the remaining timesteps."""
    import json

    from imitation_amd.utils.checkpoint import META_FILE, CheckpointManager

    custom_logger, log_dir = logging_ingredient.setup_logging()
    resume_from = dagger.get("resume_from")
    interval = int(dagger.get("full_checkpoint_interval", 0) or 0)
    keep = int(dagger.get("full_checkpoint_keep", 3))
    scratch = osp.join(log_dir, "scratch")
    resume_meta = None
    if resume_from:
        mgr_in = CheckpointManager(resume_from, keep=keep)
        step = mgr_in.agreed_step()
        if step is None:
            raise ValueError(f"resume_from={resume_from!r} holds no full checkpoint")
        with open(osp.join(mgr_in._rank_dir(step), META_FILE)) as f:
            resume_meta = json.load(f)
        scratch = resume_meta["scratch_dir"]
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
            venv=venv, scratch_dir=scratch, expert_trajs=None if resume_meta else expert_trajs,
            expert_policy=expert_policy, custom_logger=custom_logger, bc_trainer=trainer,
            beta_schedule=dagger["beta_schedule"], rng=_rnd)
        total = int(dagger["total_timesteps"])
        done = 0
        if resume_meta is not None:
            mgr_in.restore_latest(dagger_trainer)
            done = int(resume_meta["collected"])
            logger.info(f"Resumed from {resume_from} at round {dagger_trainer.round_num} ({done} timesteps collected)")
        mgr = CheckpointManager(str(log_dir / "full_checkpoints"), keep=keep) if interval > 0 else None

        def round_callback(round_num: int, collected: int) -> None:
            if mgr is not None and round_num % interval == 0:
                mgr.save(dagger_trainer, round_num, meta=dict(collected=done + collected, total_timesteps=total,
                                                              scratch_dir=str(dagger_trainer.base_scratch_dir)))

        with watchdog.cli_watchdog("train_imitation") as wd:
            def beat(round_num: int, collected: int) -> None:
                wd.beat()
                round_callback(round_num, collected)

            if total - done > 0:
                dagger_trainer.train(total_timesteps=total - done, bc_train_kwargs=kwargs, round_callback=beat)
            wd.beat()
        print(f"Model saved to {dagger_trainer.save_trainer()}")
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    out = _collect_stats(imit_stats, dagger_trainer._all_demos)
    if resume_meta is not None:
        out["resumed_round"] = int(resume_meta["step"])
    return out


@train_imitation_ex.command
def sqil(sqil: Mapping[str, Any], policy: Mapping[str, Any], rl: Mapping[str, Any], _run,
         _rnd: np.random.Generator) -> Mapping[str, Mapping[str, float]]:
    """Soft Q imitation learning (DQN by default)."""
    custom_logger, log_dir = logging_ingredient.setup_logging()
    expert_trajs = demonstrations.get_expert_trajectories()
    with environment.make_venv() as venv:
        trainer = sqil_algorithm.SQIL(venv=venv, demonstrations=expert_trajs, policy=policy["policy_cls"],
                                      custom_logger=custom_logger, rl_algo_class=rl["rl_cls"], rl_kwargs=rl["rl_kwargs"])
        with watchdog.cli_watchdog("train_imitation") as wd:
            train_kwargs = dict(sqil["train_kwargs"])
            if "callback" not in train_kwargs:
                train_kwargs["callback"] = watchdog.rl_beat_callback(wd)
            trainer.train(total_timesteps=int(sqil["total_timesteps"]), **train_kwargs)
        util.save_policy(trainer.policy, policy_path=osp.join(log_dir, "final.th"))
        imit_stats = policy_evaluation.eval_policy(trainer.policy, venv)
    return _collect_stats(imit_stats, expert_trajs)


def main_console(argv=None):
    train_imitation_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "train_imitation"))
    return train_imitation_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
