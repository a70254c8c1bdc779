"""Train a reward model from preference comparisons (reference:
src/imitation/scripts/train_preference_comparisons.py).

Checkpoints: ``{log_dir}/checkpoints/{iter|final}/reward_net.pt`` (pickle-free) and
``policy/model.zip``; ``save_preferences`` writes ``{log_dir}/preferences.npz``.
"""

from __future__ import annotations

import functools
import logging
import pathlib
from typing import Any, Mapping, Optional, Type, Union

import numpy as np

from imitation_amd.utils import watchdog
from imitation_amd.algorithms import preference_comparisons
from imitation_amd.data import serialize as data_serialize
from imitation_amd.policies import serialize as policies_serialize
from imitation_amd.rewards import serialize as reward_serialize
from imitation_amd.scripts.config.train_preference_comparisons import train_preference_comparisons_ex
from imitation_amd.scripts.config_engine import FileStorageObserver
from imitation_amd.scripts.ingredients import environment
from imitation_amd.scripts.ingredients import logging as logging_ingredient
from imitation_amd.scripts.ingredients import policy_evaluation, reward
from imitation_amd.scripts.ingredients import rl as rl_common


logger = logging.getLogger(__name__)


def save_model(agent_trainer: preference_comparisons.AgentTrainer, save_path: pathlib.Path) -> None:
    policies_serialize.save_stable_model(output_dir=save_path / "policy", model=agent_trainer.algorithm)


def save_checkpoint(trainer: preference_comparisons.PreferenceComparisons, save_path: pathlib.Path,
                    allow_save_policy: Optional[bool]) -> None:
    save_path.mkdir(parents=True, exist_ok=True)
    reward_serialize.save_reward_net(trainer.model, save_path / "reward_net.pt")
    if allow_save_policy:
        assert isinstance(trainer.trajectory_generator, preference_comparisons.AgentTrainer)
        save_model(trainer.trajectory_generator, save_path)
    else:
        trainer.logger.warn("trainer.trajectory_generator doesn't contain a policy to save.")


def _make_agent_trainer(engine: str, **kwargs) -> preference_comparisons.AgentTrainer:
    """:class:`~imitation_amd.engine.preference.DeviceAgentTrainer` (rollouts, learned reward,
    exploration wrapper and PPO on the GPU) when ``engine`` allows and the agent is eligible,
    else the host :class:`AgentTrainer`; ``engine=device`` fails loudly when not eligible."""
    why = "engine=host"
    if engine in ("auto", "device"):
        from imitation_amd.engine import preference as device_pref

        ok, why = device_pref.supports(kwargs["venv"], kwargs["algorithm"], kwargs["reward_fn"])
        if ok:
            trainer = device_pref.DeviceAgentTrainer(**kwargs)
            trainer.engine_kind = "device"
            logger.info("Using the device agent (DeviceAgentTrainer)")
            return trainer
    if engine == "device":
        raise ValueError(f"engine=device requested but unsupported: {why}")
    trainer = preference_comparisons.AgentTrainer(**kwargs)
    trainer.engine_kind = "host"
    return trainer


@train_preference_comparisons_ex.main
def train_preference_comparisons(total_timesteps: int, total_comparisons: int, num_iterations: int,
                                 comparison_queue_size: Optional[int], fragment_length: int,
                                 transition_oversampling: float, initial_comparison_frac: float,
                                 exploration_frac: float, trajectory_path: Optional[str],
                                 trajectory_generator_kwargs: Mapping[str, Any], save_preferences: bool,
                                 agent_path: Optional[str], preference_model_kwargs: Mapping[str, Any],
                                 reward_trainer_kwargs: Mapping[str, Any],
                                 gatherer_cls: Type[preference_comparisons.PreferenceGatherer],
                                 gatherer_kwargs: Mapping[str, Any], active_selection: bool,
                                 active_selection_oversampling: int, uncertainty_on: str,
                                 fragmenter_kwargs: Mapping[str, Any], allow_variable_horizon: bool,
                                 checkpoint_interval: int, query_schedule: Union[str, Any],
                                 _rnd: np.random.Generator, engine: str = "auto", full_checkpoint_interval: int = 0,
                                 full_checkpoint_keep: int = 3, resume_from: Optional[str] = None) -> Mapping[str, Any]:
    """Reward learning from synthetic (or dataset) preferences; returns final reward loss/accuracy
    and, when an agent is trained, its rollout statistics. ``full_checkpoint_interval`` > 0 writes
    the whole trainer state every that many iterations to ``{log_dir}/full_checkpoints``
    (:class:`~imitation_amd.utils.checkpoint.CheckpointManager`); ``resume_from=<dir>`` restores the
    newest one and runs only the remaining iterations of the schedule."""
    total_timesteps, total_comparisons, num_iterations = int(total_timesteps), int(total_comparisons), int(num_iterations)
    comparison_queue_size = int(comparison_queue_size) if comparison_queue_size is not None else None
    fragment_length = int(fragment_length)
    checkpoint_interval = int(checkpoint_interval)
    custom_logger, log_dir = logging_ingredient.setup_logging()
    with environment.make_venv() as venv:
        reward_net = reward.make_reward_net(venv)
        relabel = functools.partial(reward_net.predict_processed, update_stats=False)
        agent = (rl_common.make_rl_algo(venv, relabel_reward_fn=relabel) if agent_path is None else
                 rl_common.load_rl_algo_from_path(agent_path=agent_path, venv=venv, relabel_reward_fn=relabel))
        if trajectory_path is None:
            reward_net = reward_net.to(agent.device)
            trajectory_generator = _make_agent_trainer(engine, algorithm=agent, reward_fn=reward_net, venv=venv,
                                                       exploration_frac=exploration_frac, rng=_rnd,
                                                       custom_logger=custom_logger, **trajectory_generator_kwargs)
        else:
            if exploration_frac > 0:
                raise ValueError("exploration_frac can't be set when a trajectory dataset is used")
            trajectory_generator = preference_comparisons.TrajectoryDataset(
                trajectories=data_serialize.load_with_rewards(trajectory_path), rng=_rnd, custom_logger=custom_logger,
                **trajectory_generator_kwargs)
        fragmenter: preference_comparisons.Fragmenter = preference_comparisons.RandomFragmenter(
            **fragmenter_kwargs, rng=_rnd, custom_logger=custom_logger)
        preference_model = preference_comparisons.PreferenceModel(**preference_model_kwargs, model=reward_net)
        if active_selection:
            fragmenter = preference_comparisons.ActiveSelectionFragmenter(
                preference_model=preference_model, base_fragmenter=fragmenter,
                fragment_sample_factor=int(active_selection_oversampling), uncertainty_on=uncertainty_on,
                custom_logger=custom_logger)
        gatherer = gatherer_cls(**gatherer_kwargs, rng=_rnd, custom_logger=custom_logger)
        reward_trainer = preference_comparisons._make_reward_trainer(
            preference_model, preference_comparisons.CrossEntropyRewardLoss(), _rnd, reward_trainer_kwargs)
        main_trainer = preference_comparisons.PreferenceComparisons(
            trajectory_generator, reward_net, num_iterations=num_iterations, fragmenter=fragmenter,
            preference_gatherer=gatherer, reward_trainer=reward_trainer, comparison_queue_size=comparison_queue_size,
            fragment_length=fragment_length, transition_oversampling=transition_oversampling,
            initial_comparison_frac=initial_comparison_frac, custom_logger=custom_logger,
            allow_variable_horizon=allow_variable_horizon, query_schedule=query_schedule)

        from imitation_amd.utils.checkpoint import CheckpointManager

        full_checkpoint_interval = int(full_checkpoint_interval)
        resumed = None
        if resume_from:
            resumed = CheckpointManager(resume_from, keep=int(full_checkpoint_keep)).restore_latest(main_trainer)
            logger.info(f"Resumed from {resume_from} after {resumed} iterations")
        full_mgr = (CheckpointManager(str(log_dir / "full_checkpoints"), keep=int(full_checkpoint_keep))
                    if full_checkpoint_interval > 0 else None)

        with watchdog.cli_watchdog("train_preference_comparisons") as wd:
            def save_callback(iteration_num):
                wd.beat()
                if checkpoint_interval > 0 and iteration_num % checkpoint_interval == 0:
                    save_checkpoint(main_trainer, log_dir / "checkpoints" / f"{iteration_num:04d}",
                                    allow_save_policy=trajectory_path is None)
                done = main_trainer._completed_iterations
                if full_mgr is not None and done % full_checkpoint_interval == 0:
                    full_mgr.save(main_trainer, done)

            results = dict(main_trainer.train(total_timesteps, total_comparisons, callback=save_callback))
            wd.beat()
            results["engine"] = getattr(trajectory_generator, "engine_kind", "dataset")
            if resumed is not None:
                results["resumed_iterations"] = resumed
            if trajectory_path is None:
                results["imit_stats"] = policy_evaluation.eval_policy(agent, venv)
    if save_preferences:
        main_trainer.dataset.save(log_dir / "preferences.npz")
    if checkpoint_interval >= 0:
        save_checkpoint(main_trainer, log_dir / "checkpoints" / "final", allow_save_policy=trajectory_path is None)
    return results


def main_console(argv=None):
    train_preference_comparisons_ex.observers.append(
        FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "train_preference_comparisons"))
    return train_preference_comparisons_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
