"""DAgger: dataset aggregation with a β-mixture of expert and learner control.

Reference: ``src/imitation/algorithms/dagger.py`` -- beta schedules
(``:28-96``), ``InteractiveTrajectoryCollector`` (``:151-287``), ``DAggerTrainer``
(``:294-552``) and ``SimpleDAggerTrainer`` (``:555-697``). Public API and the on-disk
demo layout are the reference's; the internals are organised around three pieces:

* :class:`RoundDemoStore` owns every round's demonstrations: the files
  (``<scratch>/demos/round-XYZ/[prefix-]dagger-demo-<i>-<uuid>.npz``, one HF-dataset
  dir per trajectory, readable by the reference) and an in-memory aggregate that grows
  by the NEW rounds only (the reference re-flattens every demo each round). Under data
  parallelism every rank writes into its own scratch tree (``<scratch>/rank-RR``) and
  the newly loaded rounds are all-gathered, so all replicas train BC on the identical
  union in (round, rank, file) order; the "no demos yet" decision is rank-agreed.
* the collectors: :class:`InteractiveTrajectoryCollector` (host VecEnv wrapper, the
  human-in-the-loop API) or, for native image envs on a GPU,
  :class:`imitation_amd.engine.dagger.DeviceDAggerCollector` (env stepping, frame
  rendering, both CNN policies and the β-mix on the device; see that module).
* :class:`DAggerTrainer` rounds: collect -> ingest -> BC (the BC step all-reduces its
  gradient bucket under DP, ``algorithms/bc.py``) -> advance the round counter.

Checkpoints are tensor/JSON-only (``torch.load(weights_only=True)``).
"""

from __future__ import annotations

import abc
import json
import logging
import os
import pathlib
import uuid
from typing import Any, Callable, Dict, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np
import torch as th

from imitation_amd.utils import gcfreeze, profiling

from imitation_amd.algorithms import base, bc
from imitation_amd.data import rollout, serialize, types
from imitation_amd.envs import spaces as spaces_mod
from imitation_amd.envs.vec_env import VecEnvWrapper
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl import save_util
from imitation_amd.rl.base import check_for_correct_spaces
from imitation_amd.rl.policies import get_device
from imitation_amd.util import logger as imit_logger
from imitation_amd.util import util

log = logging.getLogger(__name__)


# ----------------------------------------------------------------------------- β schedules
class BetaSchedule(abc.ABC):
    """β(round): probability that the expert's (rather than the learner's) action is executed."""

    @abc.abstractmethod
    def __call__(self, round_num: int) -> float:
        """β for round ``round_num``."""

    def to_json(self) -> Dict[str, Any]:
        return {"type": "default"}


class LinearBetaSchedule(BetaSchedule):
    """β ramps linearly from 1 down to 0 over ``rampdown_rounds`` rounds."""

    def __init__(self, rampdown_rounds: int) -> None:
        self.rampdown_rounds = rampdown_rounds

    def __call__(self, round_num: int) -> float:
        assert round_num >= 0
        return float(np.clip(1.0 - round_num / self.rampdown_rounds, 0.0, 1.0))

    def to_json(self) -> Dict[str, Any]:
        return {"type": "linear", "rampdown_rounds": self.rampdown_rounds}


class ExponentialBetaSchedule(BetaSchedule):
    """β = ``decay_probability`` ** round."""

    def __init__(self, decay_probability: float):
        if not 0 < decay_probability <= 1:
            raise ValueError("decay_probability lies outside the range (0, 1].")
        self.decay_probability = decay_probability

    def __call__(self, round_num: int) -> float:
        assert round_num >= 0
        return self.decay_probability**round_num

    def to_json(self) -> Dict[str, Any]:
        return {"type": "exponential", "decay_probability": self.decay_probability}


def _schedule_from_json(d: Mapping[str, Any]) -> Optional[BetaSchedule]:
    kind = d.get("type")
    if kind == "linear":
        return LinearBetaSchedule(d["rampdown_rounds"])
    if kind == "exponential":
        return ExponentialBetaSchedule(d["decay_probability"])
    return None


def _schedule_json(schedule) -> Dict[str, Any]:
    if isinstance(schedule, BetaSchedule):
        return schedule.to_json()
    log.warning("beta schedule %r is not serializable; a reloaded trainer uses the default", schedule)
    return {"type": "default"}


# ----------------------------------------------------------------------------- demo store
def _demo_filename(index: int, rng: np.random.Generator, prefix: str = "") -> str:
    tag = uuid.UUID(int=int.from_bytes(rng.bytes(16), "big"), version=4).hex
    return f"{prefix + '-' if prefix else ''}dagger-demo-{index}-{tag}.npz"


def _save_dagger_demo(trajectory: types.Trajectory, trajectory_index: int, save_dir: types.AnyPath,
                      rng: np.random.Generator, prefix: str = "") -> pathlib.Path:
    """Write one trajectory as ``save_dir/[prefix-]dagger-demo-<index>-<uuid>.npz``."""
    if not isinstance(trajectory, types.Trajectory):
        raise TypeError(f"expected a Trajectory, got {type(trajectory)}")
    path = util.parse_path(save_dir) / _demo_filename(trajectory_index, rng, prefix)
    if path.exists():
        raise FileExistsError(f"DAgger demonstration path already exists: {path}")
    serialize.save(path, [trajectory])
    log.info("saved demo at %s", path)
    return path


class RoundDemoStore:
    """All demonstrations of a DAgger run, per round, on disk and aggregated in memory.

    ``root`` is this rank's scratch tree. :meth:`ingest` reads rounds that have not been
    read yet, all-gathers them across DP ranks and extends the flat aggregate handed to
    BC (one concatenation of the new transitions)."""

    def __init__(self, root: pathlib.Path):
        self.root = root
        self.trajectories: List[types.Trajectory] = []
        self.loaded_through = -1  # last round already in memory
        self._flat: Optional[types.Transitions] = None

    def round_dir(self, round_num: int) -> pathlib.Path:
        return self.root / "demos" / f"round-{round_num:03d}"

    def files(self, round_num: int) -> List[pathlib.Path]:
        d = self.round_dir(round_num)
        if not d.is_dir():
            return []
        return [d / name for name in sorted(p.name for p in d.iterdir()) if name.endswith(".npz")]

    def write(self, trajectory: types.Trajectory, index: int, round_num: int, rng: np.random.Generator,
              prefix: str = "") -> pathlib.Path:
        return _save_dagger_demo(trajectory, index, self.round_dir(round_num), rng, prefix)

    def demos_everywhere(self, round_num: int) -> bool:
        """True iff EVERY rank has at least one demo file for ``round_num`` (rank-agreed)."""
        have = float(len(self.files(round_num)) > 0)
        if pdist.world_size() > 1:
            have = pdist.allreduce_scalars([have], op="min")[0]
        return have > 0

    def ingest(self, through_round: int) -> Tuple[types.Transitions, List[int]]:
        """Load rounds ``loaded_through+1 .. through_round`` (all ranks' files, rank order);
        returns the aggregate transitions and the per-round counts of new demos."""
        new: List[types.Trajectory] = []
        counts: List[int] = []
        for r in range(self.loaded_through + 1, through_round + 1):
            local = [serialize.load(p)[0] for p in self.files(r)]
            parts = pdist.all_gather_object(local) if pdist.world_size() > 1 else [local]
            counts.append(sum(len(p) for p in parts))
            for part in parts:
                new.extend(part)
        self.loaded_through = max(self.loaded_through, through_round)
        self.trajectories.extend(new)
        if new:
            fresh = rollout.flatten_trajectories(new)
            self._flat = fresh if self._flat is None else _concat_transitions(self._flat, fresh)
        log.info("aggregate now holds %d demos (%d new)", len(self.trajectories), len(new))
        assert self._flat is not None, "ingest() found no demonstrations"
        return self._flat, counts


def _concat_transitions(a: types.Transitions, b: types.Transitions) -> types.Transitions:
    cat = lambda x, y: types.DictObs.concatenate([x, y]) if isinstance(x, types.DictObs) else np.concatenate([x, y])  # noqa: E731
    return types.Transitions(obs=cat(a.obs, b.obs), acts=np.concatenate([a.acts, b.acts]),
                             infos=np.concatenate([a.infos, b.infos]), next_obs=cat(a.next_obs, b.next_obs),
                             dones=np.concatenate([a.dones, b.dones]))


# ----------------------------------------------------------------------------- host collector
class InteractiveTrajectoryCollector(VecEnvWrapper):
    """VecEnv wrapper for DAgger data collection (reference ``dagger.py:151-287``).

    ``step(actions)`` takes the EXPERT's intended actions. Per env and step, independently,
    the expert action is executed with probability β and the learner's
    (``get_robot_acts(obs)``) otherwise; the recorded action is always the expert's.
    Every finished episode is written to ``save_dir`` as a demo file."""

    def __init__(self, venv, get_robot_acts: Callable[[np.ndarray], np.ndarray], beta: float, save_dir: types.AnyPath,
                 rng: np.random.Generator) -> None:
        super().__init__(venv)
        if not 0 <= beta <= 1:
            raise ValueError(f"beta={beta} outside [0, 1]")
        self.get_robot_acts = get_robot_acts
        self.beta = beta
        self.save_dir = save_dir
        self.rng = rng
        self.traj_accum: Optional[rollout.TrajectoryAccumulator] = None
        self._obs: Optional[np.ndarray] = None
        self._expert_acts: Optional[np.ndarray] = None

    def seed(self, seed: Optional[int] = None) -> List[Optional[int]]:
        """Reseed the β-mixing RNG and the wrapped envs."""
        self.rng = np.random.default_rng(seed=seed)
        return list(self.venv.seed(seed))

    def reset(self) -> np.ndarray:
        obs = self.venv.reset()
        if not isinstance(obs, np.ndarray):
            raise TypeError("DAgger collection needs array observations")
        self.traj_accum = rollout.TrajectoryAccumulator()
        for env_idx in range(len(obs)):
            self.traj_accum.add_step({"obs": obs[env_idx]}, key=env_idx)
        self._obs, self._expert_acts = obs, None
        return obs

    def _executed_actions(self, expert: np.ndarray) -> np.ndarray:
        learner_turn = self.rng.uniform(0, 1, size=(self.num_envs,)) > self.beta
        executed = np.array(expert)
        if learner_turn.any():
            executed[learner_turn] = self.get_robot_acts(self._obs[learner_turn])
        return executed

    def step_async(self, actions: np.ndarray) -> None:
        if self.traj_accum is None or self._obs is None:
            raise RuntimeError("call .reset() before .step()")
        executed = self._executed_actions(actions)
        self._expert_acts = actions
        self.venv.step_async(executed)

    def step_wait(self):
        obs, rews, dones, infos = self.venv.step_wait()
        if self._expert_acts is None or self.traj_accum is None:
            raise RuntimeError("step_wait() without step_async()")
        self._obs = obs
        finished = self.traj_accum.add_steps_and_auto_finish(obs=obs, acts=self._expert_acts, rews=rews, infos=infos,
                                                             dones=dones)
        for k, traj in enumerate(finished):
            _save_dagger_demo(traj, k, self.save_dir, self.rng)
        return obs, rews, dones, infos


class NeedsDemosException(Exception):
    """Signals demos need to be collected for current round before continuing."""


# ----------------------------------------------------------------------------- trainers
class DAggerTrainer(base.BaseImitationAlgorithm):
    """DAgger rounds with a low-level API suitable for interactive (human) feedback.

    ``create_trajectory_collector`` -> collect episodes with it -> ``extend_and_update``
    (aggregate + BC + next round)."""

    DEFAULT_N_EPOCHS: int = 4

    def __init__(self, *, venv, scratch_dir: types.AnyPath, rng: np.random.Generator,
                 beta_schedule: Optional[Callable[[int], float]] = None, bc_trainer: bc.BC,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        super().__init__(custom_logger=custom_logger)
        self.beta_schedule = beta_schedule if beta_schedule is not None else LinearBetaSchedule(15)
        self.base_scratch_dir = util.parse_path(scratch_dir)
        world = pdist.world_size()
        self.scratch_dir = self.base_scratch_dir / f"rank-{pdist.rank():02d}" if world > 1 else self.base_scratch_dir
        self.venv = venv
        self.rng = rng
        self.round_num = 0
        self._store = RoundDemoStore(self.scratch_dir)
        try:
            check_for_correct_spaces(self.venv, bc_trainer.observation_space, bc_trainer.action_space)
        except ValueError as e:
            log.warning("%s", e)
        self.bc_trainer = bc_trainer
        self.bc_trainer.logger = self.logger

    def __getstate__(self):
        d = dict(self.__dict__)
        d.pop("venv", None)
        d.pop("_logger", None)
        return d

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return super().logger

    @logger.setter
    def logger(self, value: imit_logger.HierarchicalLogger) -> None:
        self._logger = value
        self.bc_trainer.logger = value

    @property
    def policy(self):
        return self.bc_trainer.policy

    @property
    def batch_size(self) -> int:
        return self.bc_trainer.batch_size

    @property
    def _all_demos(self) -> List[types.Trajectory]:
        """Every demonstration trajectory aggregated so far (all ranks, round order)."""
        return self._store.trajectories

    def _demo_dir_path_for_round(self, round_num: Optional[int] = None) -> pathlib.Path:
        return self._store.round_dir(self.round_num if round_num is None else round_num)

    def _aggregate_current_round(self) -> None:
        """Make BC see the union of all rounds up to the current one (rank-agreed)."""
        if not self._store.demos_everywhere(self.round_num):
            raise NeedsDemosException(
                f"No demos found for round {self.round_num} in dir '{self._demo_dir_path_for_round()}'"
                + (" on every rank" if pdist.world_size() > 1 else "")
                + ". Maybe you need to collect some demos? See .create_trajectory_collector()")
        if self._store.loaded_through >= self.round_num:
            return
        transitions, counts = self._store.ingest(self.round_num)
        log.info("loaded %d new demos from %d rounds", sum(counts), len(counts))
        if len(transitions) < self.batch_size:
            raise ValueError(f"Not enough transitions to form a single batch: self.batch_size={self.batch_size} > "
                             f"len(transitions)={len(transitions)}")
        seed = int(self.rng.integers(0, 2**31 - 1)) + 7919 * pdist.rank()
        self.bc_trainer.set_demonstrations(base.TransitionsBatchLoader(transitions, self.batch_size, shuffle=True,
                                                                       drop_last=True, seed=seed))

    def _log_rollouts_venv(self):
        """Where BC's rollout statistics run by default (the reference: ``self.venv``)."""
        return self.venv

    def extend_and_update(self, bc_train_kwargs: Optional[Mapping[str, Any]] = None) -> int:
        """Aggregate the new demos, train BC on everything collected so far, advance the round."""
        kwargs = dict(bc_train_kwargs or {})
        kwargs.setdefault("log_rollouts_venv", self._log_rollouts_venv())
        if "n_epochs" not in kwargs and "n_batches" not in kwargs:
            kwargs["n_epochs"] = self.DEFAULT_N_EPOCHS
        if pdist.world_size() > 1:
            lo, neg_hi = pdist.allreduce_scalars([self.round_num, -self.round_num], op="min")
            if lo != -neg_hi:
                raise RuntimeError(f"DAgger ranks disagree on the round number ({int(lo)}..{int(-neg_hi)})")
        self._aggregate_current_round()
        log.info("training BC at round %d", self.round_num)
        self.bc_trainer.train(**kwargs)
        self.round_num += 1
        return self.round_num

    def _robot_actions(self, obs: np.ndarray) -> np.ndarray:
        return self.bc_trainer.policy.predict(obs)[0]

    def create_trajectory_collector(self) -> InteractiveTrajectoryCollector:
        """Host collector for the current round (β from the schedule, demos into the round dir)."""
        return InteractiveTrajectoryCollector(venv=self.venv, get_robot_acts=self._robot_actions,
                                              beta=self.beta_schedule(self.round_num),
                                              save_dir=self._demo_dir_path_for_round(), rng=self.rng)

    def _checkpoint_meta(self) -> Dict[str, Any]:
        bct = self.bc_trainer
        opt_cls = type(bct.optimizer)
        return {
            "class": type(self).__name__,
            "round_num": self.round_num,
            "beta_schedule": _schedule_json(self.beta_schedule),
            "rng_state": self.rng.bit_generator.state,
            "bc": {
                "batch_size": bct.batch_size,
                "minibatch_size": bct.minibatch_size,
                "optimizer_cls": f"{opt_cls.__module__}:{opt_cls.__qualname__}",
                "optimizer_kwargs": {k: v for k, v in bct.optimizer.defaults.items()
                                     if k in ("lr", "eps", "amsgrad", "momentum", "alpha")},
                "ent_weight": bct.loss_calculator.ent_weight,
                "l2_weight": bct.loss_calculator.l2_weight,
            },
        }

    def save_trainer(self) -> Tuple[pathlib.Path, pathlib.Path]:
        """Write ``checkpoint-{round}.pt`` / ``checkpoint-latest.pt`` (JSON metadata + optimizer
        state) and ``policy-{round}.pt`` / ``policy-latest.pt`` into this rank's scratch dir."""
        self.scratch_dir.mkdir(parents=True, exist_ok=True)
        ckpt = {"format": "imitation_amd.dagger.v1", "meta": json.dumps(self._checkpoint_meta()),
                "optimizer": self.bc_trainer.optimizer.state_dict()}
        tags = (f"{self.round_num:03d}", "latest")
        ckpt_paths = [self.scratch_dir / f"checkpoint-{t}.pt" for t in tags]
        pol_paths = [self.scratch_dir / f"policy-{t}.pt" for t in tags]
        for cp, pp in zip(ckpt_paths, pol_paths):
            th.save(ckpt, cp)
            util.save_policy(self.policy, pp)
        expert = getattr(self, "expert_policy", None)
        if expert is not None and hasattr(expert, "save"):
            expert.save(self.scratch_dir / "expert-policy.pt")
        return ckpt_paths[0], pol_paths[0]


def reconstruct_trainer(scratch_dir: types.AnyPath, venv, custom_logger: Optional[imit_logger.HierarchicalLogger] = None,
                        device: Union[th.device, str] = "auto") -> DAggerTrainer:
    """Rebuild a trainer saved by :meth:`DAggerTrainer.save_trainer` (reference
    ``dagger.py:99-127``). Demonstrations are re-read from the scratch dir on the next
    update. Under DP each rank reads its own ``rank-RR`` subtree."""
    from imitation_amd.rl.policies import load_policy_file

    custom_logger = custom_logger or imit_logger.configure()
    root = util.parse_path(scratch_dir)
    own = root / f"rank-{pdist.rank():02d}" if pdist.world_size() > 1 else root
    ckpt = th.load(own / "checkpoint-latest.pt", map_location=get_device(device), weights_only=True)
    meta = json.loads(ckpt["meta"])
    policy = load_policy_file(own / "policy-latest.pt", device=device)
    b = meta["bc"]
    bc_trainer = bc.BC(observation_space=policy.observation_space, action_space=policy.action_space,
                       rng=np.random.default_rng(), policy=policy, demonstrations=None, batch_size=b["batch_size"],
                       minibatch_size=b["minibatch_size"], optimizer_cls=save_util._resolve_class(b["optimizer_cls"]),
                       optimizer_kwargs=b["optimizer_kwargs"], ent_weight=b["ent_weight"], l2_weight=b["l2_weight"],
                       custom_logger=custom_logger)
    bc_trainer.optimizer.load_state_dict(ckpt["optimizer"])
    rng = np.random.default_rng()
    rng.bit_generator.state = meta["rng_state"]
    common = dict(venv=venv, scratch_dir=root, rng=rng, beta_schedule=_schedule_from_json(meta["beta_schedule"]),
                  bc_trainer=bc_trainer, custom_logger=custom_logger)
    if meta["class"] == "SimpleDAggerTrainer":
        trainer: DAggerTrainer = SimpleDAggerTrainer(expert_policy=load_policy_file(own / "expert-policy.pt", device=device),
                                                     **common)
    else:
        trainer = DAggerTrainer(**common)
    trainer.round_num = meta["round_num"]
    return trainer


class SimpleDAggerTrainer(DAggerTrainer):
    """DAgger with a synthetic (policy) expert: ``train`` runs whole rounds by itself.

    Each round collects at least ``max(rollout_round_min_timesteps, batch_size)`` steps
    and ``rollout_round_min_episodes`` episodes PER RANK (weak scaling; the expert acts
    deterministically), then aggregates and trains. ``total_timesteps`` counts the env
    steps of all ranks. Native image envs on a GPU collect with the device collector
    (``device_collector='auto'``)."""

    def __init__(self, *, venv, scratch_dir: types.AnyPath, expert_policy, rng: np.random.Generator,
                 expert_trajs: Optional[Sequence[types.Trajectory]] = None, device_collector: Union[str, bool] = "auto",
                 **dagger_trainer_kwargs):
        super().__init__(venv=venv, scratch_dir=scratch_dir, rng=rng, **dagger_trainer_kwargs)
        for what in ("observation_space", "action_space"):
            if getattr(expert_policy, what) != getattr(self.venv, what):
                raise ValueError(f"Mismatched {what.split('_')[0]} space between expert_policy and venv")
        self.expert_policy = expert_policy
        for k, traj in enumerate(expert_trajs or ()):
            self._store.write(traj, k, self.round_num, self.rng, prefix="initial_data")
        self._device_collector = None
        self._writer = None
        if device_collector:
            from imitation_amd.engine import dagger as dagger_engine

            ok, why = dagger_engine.supports(self.venv, self.expert_policy, self.bc_trainer.policy)
            if ok:
                self._device_collector = dagger_engine.DeviceDAggerCollector(self.venv, self.expert_policy,
                                                                             self.bc_trainer.policy, self.rng)
                # the round's frames land on the host in the writer thread (before its files are
                # written) or at the end of train(), not on the collect -> BC path
                self._device_collector.async_frames = os.environ.get("IMITATION_AMD_DAGGER_ASYNC_FRAMES", "1") != "0"
                self._landings: List[Any] = []
                self._device_agg = dagger_engine.DeviceDemoAggregate(self.bc_trainer.policy.device)
                self._device_counts: Dict[int, int] = {}
                # demo files are persisted in the background (flushed by save_trainer /
                # flush_demos and at interpreter exit); BC trains from the device aggregate
                self._writer = dagger_engine.AsyncDemoWriter()
                import atexit

                atexit.register(self._writer.close)
                if expert_trajs:
                    self._device_append(list(expert_trajs), self.round_num)
            elif device_collector is True:
                raise ValueError(f"device DAgger collector not applicable: {why}")

    def _device_append(self, trajs: Sequence[types.Trajectory], round_num: int, obs=None, acts=None) -> None:
        """Add demos to the device aggregate (all-gathered under DP); host arrays are uploaded."""
        if obs is None:
            flat = rollout.flatten_trajectories(list(trajs))
            dev = self._device_agg.device
            obs = th.as_tensor(np.asarray(flat.obs), device=dev)
            acts = th.as_tensor(np.asarray(flat.acts), device=dev)
            if isinstance(self.venv.action_space, spaces_mod.Discrete):
                acts = acts.long()
        self._device_agg.append(obs, acts)
        self._device_counts[round_num] = self._device_counts.get(round_num, 0) + len(trajs)
        self._store.trajectories.extend(trajs)

    def _log_rollouts_venv(self):
        """With the device collector, BC's rollout statistics run on the device as well
        (same stopping rule and keys as the host rollouts over ``self.venv``)."""
        if self._device_collector is not None:
            from imitation_amd.engine import dagger as dagger_engine

            return dagger_engine.DeviceStatsVenv(self._device_collector)
        return self.venv

    @property
    def collector_kind(self) -> str:
        return "device" if self._device_collector is not None else "host"

    def _collect_round(self, min_episodes: int, min_timesteps: int) -> List[types.TrajectoryWithRew]:
        beta = self.beta_schedule(self.round_num)
        if self._device_collector is not None:
            col = self._device_collector
            trajs = col.collect(beta, min_timesteps=min_timesteps, min_episodes=min_episodes)
            if col.last_landing is not None:
                self._landings.append(col.last_landing)
                self._writer.submit(col.last_landing.land)  # (the writer is FIFO: before the files)
            for k, traj in enumerate(trajs):  # reference-format demo files, off the critical path
                self._writer.submit(self._store.write, traj, k, self.round_num, np.random.default_rng(self.rng.integers(2**63)))
            self._device_append(trajs, self.round_num, col.last_obs, col.last_acts)
            return trajs
        collector = self.create_trajectory_collector()
        sample_until = rollout.make_sample_until(min_timesteps=min_timesteps, min_episodes=min_episodes)
        return rollout.generate_trajectories(policy=self.expert_policy, venv=collector, sample_until=sample_until,
                                             deterministic_policy=True, rng=collector.rng)

    def _aggregate_current_round(self) -> None:
        if self._device_collector is None:
            return super()._aggregate_current_round()
        have = float(self._device_counts.get(self.round_num, 0) > 0)
        if pdist.world_size() > 1:
            have = pdist.allreduce_scalars([have], op="min")[0]
        if not have:
            raise NeedsDemosException(f"No demos collected for round {self.round_num}")
        if self._store.loaded_through >= self.round_num:
            return
        self._store.loaded_through = self.round_num
        if len(self._device_agg) < self.batch_size:
            raise ValueError(f"Not enough transitions to form a single batch: self.batch_size={self.batch_size} > "
                             f"len(transitions)={len(self._device_agg)}")
        from imitation_amd.engine import dagger as dagger_engine

        seed = int(self.rng.integers(0, 2**31 - 1)) + 7919 * pdist.rank()
        self.bc_trainer.set_demonstrations(dagger_engine.DeviceTransitionsLoader(self._device_agg, self.batch_size, seed))

    def land_frames(self) -> None:
        """Block until the host observation arrays of every collected trajectory are filled
        (device collector: the frames' D2H copies run asynchronously)."""
        pending = getattr(self, "_landings", None)
        while pending:
            pending.pop(0).land()

    def flush_demos(self) -> None:
        """Block until every collected demonstration is on disk (device collector only)."""
        if self._writer is not None:
            self._writer.flush()
        self.land_frames()

    def save_trainer(self) -> Tuple[pathlib.Path, pathlib.Path]:
        if self._writer is not None:
            self._writer.flush()  # every demo file of the finished rounds is on disk
        return super().save_trainer()

    @gcfreeze.during
    def train(self, total_timesteps: int, *, rollout_round_min_episodes: int = 3, rollout_round_min_timesteps: int = 500,
              bc_train_kwargs: Optional[dict] = None,
              round_callback: Optional[Callable[[int, int], None]] = None) -> None:
        """Run rounds until ``total_timesteps`` env steps (all ranks) have been collected.
        ``round_callback(round_num, collected)`` runs after every round (``round_num`` = rounds
        done, ``collected`` = env steps of this call so far): the CLI's full checkpoints."""
        try:
            self._train_rounds(total_timesteps, rollout_round_min_episodes, rollout_round_min_timesteps, bc_train_kwargs,
                               round_callback)
        finally:
            self.land_frames()  # the trajectories handed out are complete when train() returns (or raises)

    def _train_rounds(self, total_timesteps: int, rollout_round_min_episodes: int, rollout_round_min_timesteps: int,
                      bc_train_kwargs: Optional[dict], round_callback=None) -> None:
        collected = 0
        local = 0
        rounds = 0
        min_steps = max(rollout_round_min_timesteps, self.batch_size)
        while collected < total_timesteps:
            with profiling.range("dagger/collect"):
                trajs = self._collect_round(rollout_round_min_episodes, min_steps)
            lens = [len(t) for t in trajs]
            n_eps, n_steps = len(trajs), sum(lens)
            local += n_steps
            if pdist.world_size() > 1:
                n_eps, n_steps = (int(v) for v in pdist.allreduce_scalars([n_eps, n_steps], op="sum"))
            collected += n_steps
            for t in trajs:
                self._logger.record_mean("dagger/mean_episode_reward", float(np.sum(t.rews)))
            lg = self._logger
            lg.record("dagger/total_timesteps", collected)
            lg.record("dagger/round_num", rounds)
            lg.record("dagger/round_episode_count", n_eps)
            lg.record("dagger/round_timestep_count", n_steps)
            with profiling.range("dagger/bc_update"):
                self.extend_and_update(bc_train_kwargs)
            rounds += 1
            if round_callback is not None:
                round_callback(self.round_num, collected)
        self.last_train_timesteps = collected  # all ranks
        self.last_train_timesteps_local = local
