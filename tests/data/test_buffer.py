"""Ring buffers (reference: tests/data/test_buffer.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.data import buffer, types


def test_buffer_store_sample_wraparound():
    b = buffer.Buffer(4, sample_shapes={"a": (2,)}, dtypes={"a": np.float32})
    b.store({"a": np.arange(6, dtype=np.float32).reshape(3, 2)})
    assert b.size() == 3
    b.store({"a": np.arange(100, 106, dtype=np.float32).reshape(3, 2)})
    assert b.size() == 4
    s = b.sample(50, rng=np.random.default_rng(0))["a"]
    assert s.shape == (50, 2)
    # only the 4 newest rows survive
    assert set(s[:, 0].tolist()) <= {4.0, 100.0, 102.0, 104.0}


def test_buffer_truncate():
    b = buffer.Buffer(2, sample_shapes={"a": ()}, dtypes={"a": np.int64})
    with pytest.raises(ValueError):
        b.store({"a": np.arange(5)}, truncate_ok=False)
    b.store({"a": np.arange(5)}, truncate_ok=True)
    assert sorted(b.sample(20, rng=np.random.default_rng(0))["a"].tolist())[0] >= 3


def test_replay_buffer_transitions():
    n = 10
    tr = types.Transitions(obs=np.random.rand(n, 3).astype(np.float32), acts=np.random.rand(n, 2).astype(np.float32),
                           infos=np.array([{}] * n), next_obs=np.random.rand(n, 3).astype(np.float32),
                           dones=np.zeros(n, bool))
    rb = buffer.ReplayBuffer.from_data(tr, capacity=20)
    assert rb.size() == n
    s = rb.sample(7, rng=np.random.default_rng(0))
    assert isinstance(s, types.Transitions) and s.obs.shape == (7, 3) and s.acts.shape == (7, 2)


def test_device_buffer():
    db = buffer.DeviceBuffer(8, {"x": (3,)}, {"x": th.float32}, device="cpu")
    db.store({"x": th.arange(30, dtype=th.float32).reshape(10, 3)})
    assert db.size() == 8
    s = db.sample(16, generator=th.Generator().manual_seed(0))["x"]
    assert s.shape == (16, 3)
    assert s[:, 0].min() >= 6  # oldest two rows overwritten
