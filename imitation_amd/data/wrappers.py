"""Environment wrappers for collecting rollouts (reference: ``src/imitation/data/wrappers.py``).

* :class:`BufferingWrapper` (``wrappers.py:13-169``) records every transition
  of the wrapped VecEnv; ``pop_trajectories`` / ``pop_finished_trajectories`` /
  ``pop_transitions`` with the reference's premature-reset error (``:45-51``).
* :class:`RolloutInfoWrapper` (``:172-208``) stashes the raw episode obs/rews in
  the final step's ``info["rollout"]``.
* :class:`VecRolloutInfoWrapper` -- the same contract for a whole VecEnv at once
  (needed for the native batched envs, which have no per-env Python object).
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from imitation_amd.data import rollout, types
from imitation_amd.envs import core
from imitation_amd.envs.vec_env import VecEnv, VecEnvWrapper


class BufferingWrapper(VecEnvWrapper):
    """Saves transitions of the underlying VecEnv (retrieve with ``pop_transitions``)."""

    def __init__(self, venv: VecEnv, error_on_premature_reset: bool = True):
        super().__init__(venv)
        self.error_on_premature_reset = error_on_premature_reset
        self._trajectories: List[types.TrajectoryWithRew] = []
        self._ep_lens: List[int] = []
        self._init_reset = False
        self._traj_accum: Optional[rollout.TrajectoryAccumulator] = None
        self._saved_acts = None
        self._timesteps: Optional[np.ndarray] = None
        self.n_transitions: Optional[int] = None

    def reset(self, **kwargs):
        if self._init_reset and self.error_on_premature_reset and self.n_transitions > 0:
            raise RuntimeError("BufferingWrapper reset() before samples were accessed")
        self._init_reset = True
        self.n_transitions = 0
        obs = self.venv.reset(**kwargs)
        self._traj_accum = rollout.TrajectoryAccumulator()
        wrapped = types.maybe_wrap_in_dictobs(obs)
        for i, ob in enumerate(wrapped):
            self._traj_accum.add_step({"obs": ob}, key=i)
        self._timesteps = np.zeros((len(wrapped),), dtype=int)
        return types.maybe_unwrap_dictobs(wrapped)

    def step_async(self, actions):
        assert self._init_reset
        assert self._saved_acts is None
        self.venv.step_async(actions)
        self._saved_acts = actions

    def step_wait(self):
        assert self._init_reset
        assert self._saved_acts is not None
        acts, self._saved_acts = self._saved_acts, None
        obs, rews, dones, infos = self.venv.step_wait()
        self.n_transitions += self.num_envs
        self._timesteps += 1
        ep_lens = self._timesteps[dones]
        if len(ep_lens) > 0:
            self._ep_lens += list(ep_lens)
        self._timesteps[dones] = 0
        self._trajectories.extend(self._traj_accum.add_steps_and_auto_finish(acts, obs, rews, dones, infos))
        return obs, rews, dones, infos

    def _finish_partial_trajectories(self) -> Sequence[types.TrajectoryWithRew]:
        assert self._traj_accum is not None
        trajs = []
        for i in range(self.num_envs):
            n_transitions = len(self._traj_accum.partial_trajectories[i]) - 1
            assert n_transitions >= 0, "Invalid TrajectoryAccumulator state"
            if n_transitions >= 1:
                traj = self._traj_accum.finish_trajectory(i, terminal=False)
                trajs.append(traj)
                self._traj_accum.add_step({"obs": traj.obs[-1]}, key=i)
        return trajs

    def pop_finished_trajectories(self) -> Tuple[Sequence[types.TrajectoryWithRew], Sequence[int]]:
        trajectories, ep_lens = self._trajectories, self._ep_lens
        self._trajectories, self._ep_lens = [], []
        self.n_transitions = 0
        return trajectories, ep_lens

    def pop_trajectories(self) -> Tuple[Sequence[types.TrajectoryWithRew], Sequence[int]]:
        if self.n_transitions == 0:
            return [], []
        self._trajectories.extend(self._finish_partial_trajectories())
        return self.pop_finished_trajectories()

    def pop_transitions(self) -> types.TransitionsWithRew:
        if self.n_transitions == 0:
            raise RuntimeError("Called pop_transitions on an empty BufferingWrapper")
        n = self.n_transitions
        trajectories, _ = self.pop_trajectories()
        transitions = rollout.flatten_trajectories_with_rew(trajectories)
        assert len(transitions.obs) == n
        return transitions


class RolloutInfoWrapper(core.Wrapper):
    """Adds the whole episode's raw obs/rews to ``info["rollout"]`` at episode end."""

    def __init__(self, env: core.Env):
        super().__init__(env)
        self._obs = None
        self._rews = None

    def reset(self, **kwargs):
        new_obs, info = super().reset(**kwargs)
        self._obs = [types.maybe_wrap_in_dictobs(new_obs)]
        self._rews = []
        return new_obs, info

    def step(self, action):
        obs, rew, terminated, truncated, info = self.env.step(action)
        self._obs.append(types.maybe_wrap_in_dictobs(obs))
        self._rews.append(rew)
        if terminated or truncated:
            assert "rollout" not in info
            info["rollout"] = {"obs": types.stack_maybe_dictobs(self._obs), "rews": np.stack(self._rews)}
        return obs, rew, terminated, truncated, info


class VecRolloutInfoWrapper(VecEnvWrapper):
    """:class:`RolloutInfoWrapper` semantics for every env of a VecEnv (auto-reset aware)."""

    def reset(self, **kwargs):
        obs = self.venv.reset(**kwargs)
        self._obs = [[np.array(o)] for o in obs]
        self._rews = [[] for _ in range(self.num_envs)]
        return obs

    def step_wait(self):
        obs, rews, dones, infos = self.venv.step_wait()
        for i in range(self.num_envs):
            self._rews[i].append(rews[i])
            if dones[i]:
                self._obs[i].append(np.array(infos[i]["terminal_observation"]))
                assert "rollout" not in infos[i]
                infos[i]["rollout"] = {"obs": np.stack(self._obs[i]), "rews": np.stack(self._rews[i])}
                self._obs[i] = [np.array(obs[i])]
                self._rews[i] = []
            else:
                self._obs[i].append(np.array(obs[i]))
        return obs, rews, dones, infos
