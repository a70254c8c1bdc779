"""Host-side episode cutting of the device DRLHP agent (engine/preference.py), on CPU:
staged rollout rounds -> TrajectoryWithRew objects with BufferingWrapper semantics
(episodes spanning rounds, terminal obs appended, end-step-then-env order)."""

import collections

import numpy as np
import torch as th

from imitation_amd.engine.preference import DeviceAgentTrainer


def _bare(N=3, D=2, A=1, T=4):
    tr = object.__new__(DeviceAgentTrainer)
    tr.N, tr.T, tr.D, tr.A, tr.discrete = N, T, D, A, False
    tr._stage_cols = (D, D, A, 1, 1, 1)
    tr._stage_host = th.zeros(T, N, sum(tr._stage_cols))
    tr._finished = []
    tr._n_since_pop = 0
    tr._wrapped_ret = np.zeros(N)

    class _RW:
        episode_rewards = collections.deque(maxlen=100)

    tr.reward_venv_wrapper = _RW()
    tr._reset_accumulator()
    return tr


def _fill(tr, t0, dones):
    """Stage one round: obs = (global step, env), next_obs = obs + 0.5, act = step, rew = step."""
    T, N, D = tr.T, tr.N, tr.D
    st = tr._stage_host.numpy()
    for t in range(T):
        for n in range(N):
            g = t0 + t
            st[t, n, :D] = [g, n]
            st[t, n, D : 2 * D] = [g + 0.5, n]
            st[t, n, 2 * D] = g
            st[t, n, 2 * D + 1] = g
            st[t, n, 2 * D + 2] = float(dones[t][n])
            st[t, n, 2 * D + 3] = 1.0


def test_accumulate_cuts_episodes_across_rounds():
    tr = _bare()
    d1 = [[0, 0, 0], [0, 1, 0], [0, 0, 0], [1, 0, 0]]  # env1 ends at t=1, env0 at t=3
    _fill(tr, 0, d1)
    added = tr._accumulate(track_wrapped=True)
    assert added == 2 + 4
    e1, e0 = tr._finished  # end-step order: env1 (t=1) before env0 (t=3)
    np.testing.assert_array_equal(e1.obs[:, 0], [0, 1, 1.5])
    np.testing.assert_array_equal(e1.obs[:, 1], [1, 1, 1])
    np.testing.assert_array_equal(e0.acts.reshape(-1), [0, 1, 2, 3])
    np.testing.assert_array_equal(e0.rews, [0, 1, 2, 3])
    assert e0.terminal and e0.rews.dtype == np.float32
    assert list(tr.reward_venv_wrapper.episode_rewards) == [2.0, 4.0]
    d2 = [[0, 0, 1], [0, 0, 0], [0, 1, 0], [0, 0, 0]]  # env2 ends at t=0 of round 2 (5 steps), env1 at t=2
    _fill(tr, 4, d2)
    tr._accumulate(track_wrapped=False)
    e2, e1b = tr._finished[2:]
    np.testing.assert_array_equal(e2.obs[:, 0], [0, 1, 2, 3, 4, 4.5])
    np.testing.assert_array_equal(e1b.obs[:, 0], [2, 3, 4, 5, 6, 6.5])
    assert tr._n_since_pop == 24
    popped = tr._pop_finished()
    assert len(popped) == 4 and tr._finished == [] and tr._n_since_pop == 0
    # env0's open episode started at global step 4 and is still partial
    assert sum(len(p[1]) for p in tr._partial[0]) == 4
