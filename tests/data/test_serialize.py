"""Trajectory serialization: HF dataset dir, legacy npz, pickle refusal
(reference: tests/data/test_serialize.py, tests/data/test_huggingface_utils.py)."""

import os

import numpy as np
import pytest
from hypothesis import given, settings

from imitation_amd.data import huggingface_utils, serialize, types
from imitation_amd.testing import hypothesis_strategies as h_strats

from tests.conftest import TESTDATA


@settings(deadline=None, max_examples=15)
@given(trajectories=h_strats.trajectories_list)
def test_save_load_roundtrip(tmp_path_factory, trajectories):
    path = tmp_path_factory.mktemp("trajs") / "t"
    serialize.save(path, trajectories)
    loaded = serialize.load(path)
    assert len(loaded) == len(trajectories)
    for a, b in zip(trajectories, loaded):
        assert a == b


@settings(deadline=None, max_examples=15)
@given(trajectories=h_strats.trajectories_list)
def test_hf_dataset_sequence_slicing(trajectories):
    ds = huggingface_utils.trajectories_to_dataset(trajectories)
    seq = huggingface_utils.TrajectoryDatasetSequence(ds)
    assert len(seq) == len(trajectories)
    for a, b in zip(trajectories, seq):
        assert a == b
    assert list(seq[::2]) == list(trajectories[::2])


def test_info_encoding_roundtrip():
    info = {"a": 1, "b": [1, 2], "c": {"d": "x"}, "e": np.float32(2.5)}
    dec = huggingface_utils.decode_info(huggingface_utils.encode_info(info))
    assert dec["a"] == 1 and dec["b"] == [1, 2] and dec["c"] == {"d": "x"} and float(dec["e"]) == 2.5


def test_load_reference_npz_rollouts():
    trajs = serialize.load_with_rewards(os.path.join(TESTDATA, "expert_models", "cartpole_0", "rollouts", "final.npz"))
    assert len(trajs) > 10
    assert all(isinstance(t, types.TrajectoryWithRew) for t in trajs)
    assert trajs[0].obs.shape[1] == 4
    assert np.mean([t.rews.sum() for t in trajs]) > 400


def test_pickle_refused(tmp_path):
    p = tmp_path / "x.pkl"
    p.write_bytes(b"\x80\x04N.")
    with pytest.raises(Exception):
        serialize.load(p)


def test_arrow_native_dataset_equals_from_dict(tmp_path):
    """The zero-copy nested-Arrow build has from_dict's exact features and content."""
    import datasets

    from imitation_amd.data import huggingface_utils as hu

    rng = np.random.default_rng(0)
    for obs_shape, act_shape, with_rew in [((84, 84, 4), (), True), ((5,), (3,), False), ((2, 3), (), True)]:
        trajs = []
        for L in (7, 3):
            obs = (rng.integers(0, 255, (L + 1,) + obs_shape, dtype=np.uint8) if len(obs_shape) == 3
                   else rng.standard_normal((L + 1,) + obs_shape).astype(np.float32))
            acts = rng.integers(0, 6, L) if act_shape == () else rng.standard_normal((L,) + act_shape).astype(np.float32)
            kw = dict(obs=obs, acts=acts, infos=[{"k": i} for i in range(L)], terminal=bool(L % 2))
            trajs.append(types.TrajectoryWithRew(rews=rng.standard_normal(L).astype(np.float32), **kw) if with_rew
                         else types.Trajectory(**kw))
        fast = hu._fast_dataset(trajs, None)
        slow = datasets.Dataset.from_dict(hu.trajectories_to_dict(trajs))
        assert fast is not None and fast.features == slow.features
        assert fast.data.table.equals(slow.data.table.cast(fast.data.table.schema))
