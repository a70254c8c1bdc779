"""Tabular (finite-state) MDP / POMDP environments.

The reference's MCE-IRL (``src/imitation/algorithms/mce_irl.py:27, 38-41``)
consumes seals ``base_envs.TabularModelPOMDP`` and its tests use seals
``RandomTransitionEnv`` / ``CliffWorld`` (``tests/algorithms/test_mce_irl.py:45-55``).
seals is not installed, so the same model-based env family lives here:
explicit ``transition_matrix[S, A, S']``, ``reward_matrix`` (state, state-action or
state-action-state), ``observation_matrix[S, O]``, ``initial_state_dist`` and a
fixed ``horizon``.
"""

from __future__ import annotations

from typing import Optional

import numpy as np

from imitation_amd.envs import core, spaces


class TabularModelPOMDP(core.Env):
    """Finite-horizon tabular POMDP with an explicit model."""

    def __init__(
        self,
        *,
        transition_matrix: np.ndarray,
        observation_matrix: np.ndarray,
        reward_matrix: np.ndarray,
        horizon: int,
        initial_state_dist: Optional[np.ndarray] = None,
    ):
        self.transition_matrix = np.asarray(transition_matrix, dtype=np.float64)
        self.observation_matrix = np.asarray(observation_matrix)
        self.reward_matrix = np.asarray(reward_matrix, dtype=np.float64)
        self._horizon = int(horizon)
        n_states = self.transition_matrix.shape[0]
        if initial_state_dist is None:
            initial_state_dist = np.ones(n_states) / n_states
        self.initial_state_dist = np.asarray(initial_state_dist, dtype=np.float64)
        assert self.transition_matrix.shape[0] == self.transition_matrix.shape[2]
        assert self.observation_matrix.shape[0] == n_states
        assert np.allclose(self.transition_matrix.sum(-1), 1.0)
        assert np.isclose(self.initial_state_dist.sum(), 1.0)
        self.observation_space = spaces.Box(
            low=float(self.observation_matrix.min()),
            high=float(self.observation_matrix.max()),
            shape=(self.observation_matrix.shape[1],),
            dtype=self.observation_matrix.dtype if self.observation_matrix.dtype != np.float64 else np.float32,
        )
        self.action_space = spaces.Discrete(self.transition_matrix.shape[1])
        self.state_space = spaces.Discrete(n_states)
        self._cur_state: Optional[int] = None
        self._n_actions_taken: Optional[int] = None

    @property
    def horizon(self) -> Optional[int]:
        return self._horizon

    @horizon.setter
    def horizon(self, h: Optional[int]) -> None:
        self._horizon = None if h is None else int(h)

    @property
    def n_states(self) -> int:
        return self.transition_matrix.shape[0]

    @property
    def n_actions(self) -> int:
        return self.transition_matrix.shape[1]

    @property
    def state_dim(self) -> int:
        return self.n_states

    @property
    def action_dim(self) -> int:
        return self.n_actions

    @property
    def obs_dim(self) -> int:
        return self.observation_matrix.shape[1]

    @property
    def feature_matrix(self) -> np.ndarray:
        return self.observation_matrix

    @property
    def state(self) -> int:
        return self._cur_state

    @state.setter
    def state(self, s: int) -> None:
        self._cur_state = int(s)

    def obs_from_state(self, state: int) -> np.ndarray:
        return self.observation_matrix[state].astype(self.observation_space.dtype)

    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        self._cur_state = int(self.np_random.choice(self.n_states, p=self.initial_state_dist))
        self._n_actions_taken = 0
        return self.obs_from_state(self._cur_state), {}

    def reward_fn(self, state, action, new_state) -> float:
        r = self.reward_matrix
        if r.ndim == 1:
            return float(r[state])
        if r.ndim == 2:
            return float(r[state, action])
        return float(r[state, action, new_state])

    def step(self, action):
        if self._cur_state is None:
            raise RuntimeError("need to call reset() before step()")
        old = self._cur_state
        probs = self.transition_matrix[old, int(action)]
        new = int(self.np_random.choice(self.n_states, p=probs))
        self._cur_state = new
        rew = self.reward_fn(old, int(action), new)
        self._n_actions_taken += 1
        done = self._horizon is not None and self._n_actions_taken >= self._horizon
        return self.obs_from_state(new), rew, False, done, {"old_state": old, "new_state": new}


class TabularModelMDP(TabularModelPOMDP):
    """Fully observed variant: observation = one-hot state."""

    def __init__(self, *, transition_matrix, reward_matrix, horizon, initial_state_dist=None):
        n = np.asarray(transition_matrix).shape[0]
        super().__init__(
            transition_matrix=transition_matrix,
            observation_matrix=np.eye(n, dtype=np.float32),
            reward_matrix=reward_matrix,
            horizon=horizon,
            initial_state_dist=initial_state_dist,
        )


def make_random_trans_mat(n_states: int, n_actions: int, max_branch_factor: int, rand_state: np.random.Generator) -> np.ndarray:
    out = np.zeros((n_states, n_actions, n_states), dtype=np.float64)
    for s in range(n_states):
        for a in range(n_actions):
            succ = rand_state.choice(n_states, size=(max_branch_factor,), replace=False)
            probs = rand_state.dirichlet(np.ones(max_branch_factor))
            out[s, a, succ] = probs
    return out / out.sum(-1, keepdims=True)


def make_random_state_dist(n_avail: int, n_states: int, rand_state: np.random.Generator) -> np.ndarray:
    assert 0 < n_avail <= n_states
    init = np.zeros((n_states,))
    idx = rand_state.choice(n_states, size=(n_avail,), replace=False)
    init[idx] = rand_state.dirichlet(np.ones(n_avail))
    return init / init.sum()


def make_obs_mat(n_states: int, is_random: bool, obs_dim: Optional[int], rand_state: np.random.Generator) -> np.ndarray:
    if not is_random:
        assert obs_dim is None
        return np.identity(n_states, dtype=np.float32)
    assert obs_dim is not None and obs_dim > 0
    return rand_state.normal(0, 1, (n_states, obs_dim)).astype(np.float32)


class RandomTransitionEnv(TabularModelPOMDP):
    """Random MDP with a random linear reward and sparse random transitions."""

    def __init__(
        self,
        *,
        n_states: int,
        n_actions: int,
        branch_factor: int,
        horizon: int,
        random_obs: bool,
        obs_dim: Optional[int] = None,
        generator_seed: Optional[int] = None,
    ):
        if obs_dim is None:
            obs_dim = n_states if random_obs else None
        rng = np.random.default_rng(generator_seed)
        obs_mat = make_obs_mat(n_states, random_obs, obs_dim, rng)
        trans = make_random_trans_mat(n_states, n_actions, branch_factor, rng)
        init = make_random_state_dist(branch_factor, n_states, rng)
        weights = rng.normal(0, 1, (obs_mat.shape[-1],))
        reward = obs_mat @ weights
        super().__init__(
            transition_matrix=trans,
            observation_matrix=obs_mat,
            reward_matrix=reward,
            horizon=horizon,
            initial_state_dist=init,
        )


class CliffWorld(TabularModelPOMDP):
    """Grid world with a cliff along the bottom row (seals ``CliffWorld``)."""

    def __init__(
        self,
        *,
        width: int = 7,
        height: int = 4,
        horizon: int = 9,
        use_xy_obs: bool = True,
        rew_default: float = -1.0,
        rew_goal: float = 10.0,
        rew_cliff: float = -10.0,
        fail_p: float = 0.3,
    ):
        n_states = width * height
        O = np.zeros((n_states, 2 if use_xy_obs else n_states), dtype=np.float32)
        R = np.zeros((n_states,))
        T = np.zeros((n_states, 4, n_states))

        def to_id(r, c):
            return width * r + c

        for row in range(height):
            for col in range(width):
                s = to_id(row, col)
                if use_xy_obs:
                    O[s] = [col / (width - 1), row / (height - 1)]
                else:
                    O[s, s] = 1
                if row == height - 1 and col == width - 1:
                    R[s] = rew_goal
                elif row == height - 1 and col > 0:
                    R[s] = rew_cliff
                else:
                    R[s] = rew_default
                if row == height - 1 and col > 0:
                    T[s, :, s] = 1  # absorbing
                    continue
                for a, (dr, dc) in enumerate([(-1, 0), (1, 0), (0, -1), (0, 1)]):
                    nr = min(max(row + dr, 0), height - 1)
                    nc = min(max(col + dc, 0), width - 1)
                    T[s, a, to_id(nr, nc)] += 1 - fail_p
                    T[s, a, s] += fail_p
        init = np.zeros(n_states)
        init[to_id(height - 1, 0)] = 1.0
        super().__init__(transition_matrix=T, observation_matrix=O, reward_matrix=R, horizon=horizon, initial_state_dist=init)
        self.width, self.height = width, height


class ExposePOMDPStateWrapper(core.Wrapper):
    """Observe the latent state index instead of the observation vector (seals ``ExposePOMDPStateWrapper``)."""

    def __init__(self, env: TabularModelPOMDP):
        super().__init__(env)
        self.observation_space = env.unwrapped.state_space

    def reset(self, *, seed=None, options=None):
        _, info = self.env.reset(seed=seed, options=options)
        return self.env.unwrapped.state, info

    def step(self, action):
        _, rew, term, trunc, info = self.env.step(action)
        return self.env.unwrapped.state, rew, term, trunc, info
