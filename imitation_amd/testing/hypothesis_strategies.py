"""Hypothesis strategies for spaces, infos and trajectories
(reference: src/imitation/testing/hypothesis_strategies.py)."""

from __future__ import annotations

import hypothesis.extra.numpy as hnp
import hypothesis.strategies as st
import numpy as np

from imitation_amd.data import types
from imitation_amd.envs import spaces

gym_spaces = st.sampled_from(
    [
        spaces.Discrete(3),
        spaces.MultiDiscrete([3, 4]),
        spaces.Box(-1, 1, shape=(1,)),
        spaces.Box(-1, 1, shape=(2,)),
        spaces.Box(-np.inf, np.inf, shape=(2,)),
    ]
)

info_dict_contents = st.dictionaries(
    st.text(),
    st.one_of(
        st.integers(),
        st.floats(allow_nan=False),
        st.text(),
        st.lists(st.integers(), max_size=3),
    ),
    max_size=3,
)

trajectory_length = st.integers(min_value=1, max_value=10)


def _samples(space, n):
    """n+1 observations or n actions sampled from ``space`` with a fixed seed."""
    space.seed(0)
    return np.array([space.sample() for _ in range(n)])


@st.composite
def _trajectory(draw, obs_space, act_space, with_rew: bool):
    length = draw(trajectory_length)
    obs = _samples(obs_space, length + 1)
    acts = _samples(act_space, length)
    infos = np.array([draw(info_dict_contents) for _ in range(length)], dtype=object)
    terminal = draw(st.booleans())
    if with_rew:
        rews = draw(hnp.arrays(np.float32, (length,), elements=st.floats(-10, 10, width=32)))
        return types.TrajectoryWithRew(obs=obs, acts=acts, infos=infos, terminal=terminal, rews=rews)
    return types.Trajectory(obs=obs, acts=acts, infos=infos, terminal=terminal)


_shared_obs_space = st.shared(gym_spaces, key="obs_space")
_shared_act_space = st.shared(gym_spaces, key="act_space")

trajectory = st.one_of(
    gym_spaces.flatmap(lambda o: gym_spaces.flatmap(lambda a: _trajectory(o, a, False))),
    gym_spaces.flatmap(lambda o: gym_spaces.flatmap(lambda a: _trajectory(o, a, True))),
)

trajectories_without_reward_list = st.lists(
    st.tuples(_shared_obs_space, _shared_act_space).flatmap(lambda oa: _trajectory(oa[0], oa[1], False)),
    min_size=1, max_size=10,
)
trajectories_with_reward_list = st.lists(
    st.tuples(_shared_obs_space, _shared_act_space).flatmap(lambda oa: _trajectory(oa[0], oa[1], True)),
    min_size=1, max_size=10,
)
trajectories_list = st.one_of(trajectories_without_reward_list, trajectories_with_reward_list)
