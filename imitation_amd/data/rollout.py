"""Rollout engine (reference: ``src/imitation/data/rollout.py``).

* :class:`TrajectoryAccumulator` (``rollout.py:58-188``) -- per-env partial
  trajectories, auto-finished on ``done`` using ``info["terminal_observation"]``;
* sample-until conditions (``:194-272``);
* :func:`policy_to_callable` (``:289-380``) and the fork's
  :func:`homogenous_policy_to_callable` (``:382-423``);
* :func:`generate_trajectories` (``:426-554``) with unbiased stopping: once the
  condition holds, envs are deactivated only as their episodes finish;
* :func:`rollout_stats` (``:557-608``), :func:`flatten_trajectories[_with_rew]`
  (``:611-669``), :func:`generate_transitions`, :func:`rollout`,
  :func:`discounted_sum` (``:776-805``), :func:`unwrap_traj` (``:31-55``).

The hot loop keeps the reference's semantics; its cost on this framework is
dominated by the native batched env step (``NativeVecEnv``) and one fused
policy launch per step.
"""

from __future__ import annotations

import collections
import dataclasses
import functools
import logging
from typing import Any, Callable, Dict, Hashable, Iterable, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np

from imitation_amd.data import types
from imitation_amd.envs import spaces
from imitation_amd.envs.vec_env import VecEnv


def unwrap_traj(traj: types.TrajectoryWithRew) -> types.TrajectoryWithRew:
    """Replace ``obs``/``rews`` with the ``RolloutInfoWrapper``-captured originals."""
    if traj.infos is None:
        raise ValueError("Trajectory must have infos to unwrap")
    ep_info = traj.infos[-1]["rollout"]
    res = dataclasses.replace(traj, obs=ep_info["obs"], rews=ep_info["rews"])
    assert len(res.obs) == len(res.acts) + 1
    assert len(res.rews) == len(res.acts)
    return res


class TrajectoryAccumulator:
    """Accumulates per-key partial trajectories step by step."""

    def __init__(self):
        self.partial_trajectories = collections.defaultdict(list)

    def add_step(self, step_dict: Mapping[str, Any], key: Hashable = None) -> None:
        self.partial_trajectories[key].append(step_dict)

    def finish_trajectory(self, key: Hashable, terminal: bool) -> types.TrajectoryWithRew:
        part_dicts = self.partial_trajectories.pop(key)
        cols: Dict[str, List[Any]] = collections.defaultdict(list)
        for part in part_dicts:
            for k, v in part.items():
                cols[k].append(v)
        stacked = {k: types.stack_maybe_dictobs(v) for k, v in cols.items()}
        traj = types.TrajectoryWithRew(**stacked, terminal=terminal)
        assert traj.rews.shape[0] == traj.acts.shape[0] == len(traj.obs) - 1
        return traj

    def add_steps_and_auto_finish(self, acts, obs, rews: np.ndarray, dones: np.ndarray, infos: List[dict]) -> List[types.TrajectoryWithRew]:
        trajs: List[types.TrajectoryWithRew] = []
        wrapped_obs = types.maybe_wrap_in_dictobs(obs)
        for env_idx in range(len(wrapped_obs)):
            assert env_idx in self.partial_trajectories
            assert list(self.partial_trajectories[env_idx][0].keys()) == ["obs"], (
                "Need to first initialize partial trajectory using self._traj_accum.add_step({'obs': ob}, key=env_idx)"
            )
        for env_idx, (act, ob, rew, done, info) in enumerate(zip(acts, wrapped_obs, rews, dones, infos)):
            real_ob = types.maybe_wrap_in_dictobs(info["terminal_observation"]) if done else ob
            self.add_step(dict(acts=act, rews=rew, obs=real_ob, infos=info), env_idx)
            if done:
                trajs.append(self.finish_trajectory(env_idx, terminal=True))
                self.add_step(dict(obs=ob), env_idx)
        return trajs


GenTrajTerminationFn = Callable[[Sequence[types.TrajectoryWithRew]], bool]


def make_min_episodes(n: int) -> GenTrajTerminationFn:
    assert n >= 1
    return lambda trajectories: len(trajectories) >= n


def make_min_timesteps(n: int) -> GenTrajTerminationFn:
    assert n >= 1

    def f(trajectories: Sequence[types.TrajectoryWithRew]):
        return sum(len(t.obs) - 1 for t in trajectories) >= n

    return f


def make_sample_until(min_timesteps: Optional[int] = None, min_episodes: Optional[int] = None) -> GenTrajTerminationFn:
    if min_timesteps is None and min_episodes is None:
        raise ValueError("At least one of min_timesteps and min_episodes needs to be non-None")
    conditions = []
    if min_timesteps is not None:
        if min_timesteps <= 0:
            raise ValueError(f"min_timesteps={min_timesteps} if provided must be positive")
        conditions.append(make_min_timesteps(min_timesteps))
    if min_episodes is not None:
        if min_episodes <= 0:
            raise ValueError(f"min_episodes={min_episodes} if provided must be positive")
        conditions.append(make_min_episodes(min_episodes))

    def sample_until(trajs: Sequence[types.TrajectoryWithRew]) -> bool:
        return all(cond(trajs) for cond in conditions)

    return sample_until


PolicyCallable = Callable[[Any, Optional[Tuple[np.ndarray, ...]], Optional[np.ndarray]], Tuple[np.ndarray, Optional[Tuple[np.ndarray, ...]]]]
AnyPolicy = Any


def _is_sb_like(policy) -> bool:
    from imitation_amd.rl.base import BaseAlgorithm
    from imitation_amd.rl.policies import BasePolicy

    return isinstance(policy, (BaseAlgorithm, BasePolicy))


def policy_to_callable(policy: AnyPolicy, venv: VecEnv, deterministic_policy: bool = False) -> PolicyCallable:
    """Any policy-like object -> ``(obs, states, episode_starts) -> (acts, states)``."""
    from imitation_amd.rl.base import BaseAlgorithm, check_for_correct_spaces

    if policy is None:

        def get_actions(observations, states, episode_starts):
            acts = [venv.action_space.sample() for _ in range(len(observations))]
            return np.stack(acts, axis=0), None

    elif _is_sb_like(policy):

        def get_actions(observations, states, episode_starts):
            return policy.predict(observations, state=states, episode_start=episode_starts, deterministic=deterministic_policy)

    elif callable(policy):
        if deterministic_policy:
            raise ValueError(
                "Cannot set deterministic_policy=True when policy is a callable, since deterministic_policy argument is ignored."
            )
        get_actions = policy
    else:
        raise TypeError(f"Policy must be None, a stable-baselines policy or algorithm, or a Callable, got {type(policy)} instead")

    if isinstance(policy, BaseAlgorithm):
        try:
            check_for_correct_spaces(venv, policy.observation_space, policy.action_space)
        except ValueError as e:
            venv_shape = venv.observation_space.shape
            pol_shape = policy.observation_space.shape
            if len(venv_shape) != 3 or len(pol_shape) != 3:
                raise e
            if (venv_shape[2], venv_shape[0], venv_shape[1]) != pol_shape:
                raise e
            raise ValueError(
                "Policy and environment observation shape mismatch. This is likely caused by "
                "https://github.com/HumanCompatibleAI/imitation/issues/599. If encountering this from rollout.rollout, "
                "try calling:\nrollout.rollout(expert, expert.get_env(), ...) instead of\nrollout.rollout(expert, env, ...)\n\n"
                f"Policy observation shape: {pol_shape} \nEnvironment observation shape: {venv_shape}"
            )
    return get_actions


def homogenous_policy_to_callable(policy, venv: VecEnv, deterministic_policy: bool = False) -> PolicyCallable:
    """Callable for a parameter-shared multi-agent policy (fork addition, ``rollout.py:382-423``).

    The agents' sub-observations are evaluated as ONE batched forward (agents folded
    into the batch axis) inside :class:`HomogenousActorCriticPolicy`.
    """
    if policy is None:

        def get_actions(observations, states, episode_starts):
            acts = [venv.action_space.sample() for _ in range(len(observations))]
            return np.stack(acts, axis=0), None

    elif _is_sb_like(policy):

        def get_actions(observations, states, episode_starts):
            return policy.predict(observations, state=states, episode_start=episode_starts, deterministic=deterministic_policy)

    else:
        raise TypeError(f"Policy must be None, a stable-baselines policy or algorithm, or a Callable, got {type(policy)} instead")
    return get_actions


def generate_trajectories(
    policy: AnyPolicy,
    venv: VecEnv,
    sample_until: GenTrajTerminationFn,
    rng: np.random.Generator,
    num_homogenous_agents: int = 1,
    *,
    deterministic_policy: bool = False,
) -> Sequence[types.TrajectoryWithRew]:
    """Roll out ``policy`` in ``venv`` until ``sample_until`` holds (unbiased stopping)."""
    from imitation_amd.policies.base import HomogenousActorCriticPolicy

    if isinstance(policy, HomogenousActorCriticPolicy):
        get_actions = homogenous_policy_to_callable(policy, venv, deterministic_policy)
    else:
        get_actions = policy_to_callable(policy, venv, deterministic_policy)
    trajectories: List[types.TrajectoryWithRew] = []
    accum = TrajectoryAccumulator()
    obs = venv.reset()
    assert isinstance(obs, (np.ndarray, dict)), "Tuple observations are not supported."
    wrapped = types.maybe_wrap_in_dictobs(obs)
    for env_idx, ob in enumerate(wrapped):
        accum.add_step(dict(obs=ob), env_idx)
    active = np.ones(venv.num_envs, dtype=bool)
    state = None
    dones = np.zeros(venv.num_envs, dtype=bool)
    while np.any(active):
        acts, state = get_actions(obs, state, dones)
        obs, rews, dones, infos = venv.step(acts)
        assert isinstance(obs, (np.ndarray, dict)), "Tuple observations are not supported."
        wrapped = types.maybe_wrap_in_dictobs(obs)
        dones &= active
        trajectories.extend(accum.add_steps_and_auto_finish(acts, wrapped, rews, dones, infos))
        if sample_until(trajectories):
            active &= ~dones
    rng.shuffle(trajectories)  # type: ignore[arg-type]
    for traj in trajectories:
        n = len(traj.acts)
        if isinstance(venv.observation_space, spaces.Dict):
            exp_obs = {k: (n + 1,) + v.shape for k, v in venv.observation_space.items()}
        else:
            exp_obs = (n + 1,) + venv.observation_space.shape
        assert traj.obs.shape == exp_obs, f"expected shape {exp_obs}, got {traj.obs.shape}"
        exp_act = (n,) + venv.action_space.shape
        assert traj.acts.shape == exp_act, f"expected shape {exp_act}, got {traj.acts.shape}"
        assert traj.rews.shape == (n,), f"expected shape {(n,)}, got {traj.rews.shape}"
    return trajectories


def rollout_stats(trajectories: Sequence[types.TrajectoryWithRew]) -> Mapping[str, float]:
    """``n_traj`` + ``{return,len,monitor_return}_{min,mean,std,max}`` (+ ``monitor_return_len``)."""
    assert len(trajectories) > 0
    out: Dict[str, float] = {"n_traj": len(trajectories)}
    desc = {
        "return": np.asarray([sum(t.rews) for t in trajectories]),
        "len": np.asarray([len(t.rews) for t in trajectories]),
    }
    mon = []
    for t in trajectories:
        if t.infos is not None:
            r = t.infos[-1].get("episode", {}).get("r")
            if r is not None:
                mon.append(r)
    if mon:
        desc["monitor_return"] = np.asarray(mon)
        out["monitor_return_len"] = len(desc["monitor_return"])
    for name, vals in desc.items():
        for stat in ("min", "mean", "std", "max"):
            out[f"{name}_{stat}"] = getattr(np, stat)(vals).item()
    for v in out.values():
        assert isinstance(v, (int, float))
    return out


def flatten_trajectories(trajectories: Iterable[types.Trajectory]) -> types.Transitions:
    trajectories = list(trajectories)

    def all_of_type(key, t):
        return all(isinstance(getattr(tr, key), t) for tr in trajectories)

    assert all_of_type("obs", types.DictObs) or all_of_type("obs", np.ndarray)
    assert all_of_type("acts", np.ndarray)
    parts: Dict[str, List[Any]] = {k: [] for k in ("obs", "next_obs", "acts", "dones", "infos")}
    for traj in trajectories:
        parts["acts"].append(traj.acts)
        parts["obs"].append(traj.obs[:-1])
        parts["next_obs"].append(traj.obs[1:])
        dones = np.zeros(len(traj.acts), dtype=bool)
        dones[-1] = traj.terminal
        parts["dones"].append(dones)
        parts["infos"].append(np.array([{}] * len(traj)) if traj.infos is None else traj.infos)
    cat = {k: types.concatenate_maybe_dictobs(v) for k, v in parts.items()}
    lengths = set(map(len, cat.values()))
    assert len(lengths) == 1, f"expected one length, got {lengths}"
    return types.Transitions(**cat)


def flatten_trajectories_with_rew(trajectories: Sequence[types.TrajectoryWithRew]) -> types.TransitionsWithRew:
    transitions = flatten_trajectories(trajectories)
    rews = np.concatenate([t.rews for t in trajectories])
    return types.TransitionsWithRew(**types.dataclass_quick_asdict(transitions), rews=rews)


def generate_transitions(policy: AnyPolicy, venv: VecEnv, n_timesteps: int, rng: np.random.Generator, *,
                         truncate: bool = True, **kwargs: Any) -> types.TransitionsWithRew:
    traj = generate_trajectories(policy, venv, sample_until=make_min_timesteps(n_timesteps), rng=rng, **kwargs)
    transitions = flatten_trajectories_with_rew(traj)
    if truncate and n_timesteps is not None:
        d = types.dataclass_quick_asdict(transitions)
        transitions = types.TransitionsWithRew(**{k: v[:n_timesteps] for k, v in d.items()})
    return transitions


def rollout(policy: AnyPolicy, venv: VecEnv, sample_until: GenTrajTerminationFn, rng: np.random.Generator, *,
            unwrap: bool = True, exclude_infos: bool = True, verbose: bool = True, **kwargs: Any) -> Sequence[types.TrajectoryWithRew]:
    trajs = generate_trajectories(policy, venv, sample_until, rng=rng, **kwargs)
    if unwrap:
        trajs = [unwrap_traj(t) for t in trajs]
    if exclude_infos:
        trajs = [dataclasses.replace(t, infos=None) for t in trajs]
    if verbose:
        logging.info(f"Rollout stats: {rollout_stats(trajs)}")
    return trajs


def discounted_sum(arr: np.ndarray, gamma: float) -> Union[np.ndarray, float]:
    """Discounted sum over the time axis (first axis), first step undiscounted."""
    assert arr.ndim in (1, 2)
    if gamma == 1.0:
        return arr.sum(axis=0)
    return np.polynomial.polynomial.polyval(gamma, arr)
