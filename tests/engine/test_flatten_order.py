"""The vectorised replay order of a device round (engine/gail.py flatten_order) == the
per-step loop of BufferingWrapper -> flatten -> FIFO store it replaces (CPU)."""

import numpy as np

from imitation_amd.engine.gail import flatten_order


def _loop_reference(dones, running):
    running = running.copy()
    T, N = dones.shape
    finished, partial, ep_lens = [], [], []
    seg_start = np.zeros(N, dtype=np.int64)
    for t in range(T):
        for n in np.flatnonzero(dones[t]):
            finished.append((t, n, int(seg_start[n])))
            ep_lens.append(int(running[n] + t - seg_start[n] + 1))
            running[n] = 0
            seg_start[n] = t + 1
    for n in range(N):
        if seg_start[n] < T:
            partial.append((n, int(seg_start[n])))
            running[n] += T - seg_start[n]
    order = []
    for (t, n, s) in finished:
        order.extend((np.arange(s, t + 1) * N + n).tolist())
    for (n, s) in partial:
        order.extend((np.arange(s, T) * N + n).tolist())
    return np.asarray(order, dtype=np.int64), [f[0] for f in finished], [f[1] for f in finished], ep_lens, running


def test_flatten_order_matches_loop():
    rng = np.random.default_rng(0)
    for trial in range(300):
        T, N = int(rng.integers(1, 40)), int(rng.integers(1, 9))
        d = rng.random((T, N)) < rng.choice([0.0, 0.02, 0.2, 0.9, 1.0])
        if trial % 7 == 0:
            d[-1, :] = True  # fixed-horizon envs: every env done at the round end
        run = rng.integers(0, 100, N)
        got, want = flatten_order(d, run), _loop_reference(d, run)
        np.testing.assert_array_equal(got[0], want[0])
        assert list(got[1]) == want[1] and list(got[2]) == want[2] and got[3] == want[3]
        np.testing.assert_array_equal(got[4], want[4])
