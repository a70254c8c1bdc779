"""TrajectoryDatasetSequence: wrapped save/load round trip, slicing and lazily decoded info
dicts (upstream tests/data/test_huggingface_utils.py)."""

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from imitation_amd.data import huggingface_utils, serialize
from imitation_amd.testing import hypothesis_strategies as h_strats


def _wrap(trajs):
    return huggingface_utils.TrajectoryDatasetSequence(huggingface_utils.trajectories_to_dataset(trajs))


@given(trajectories=h_strats.trajectories_list)
@settings(suppress_health_check=[HealthCheck.function_scoped_fixture], deadline=None, max_examples=15)
def test_wrapped_sequence_save_load(tmp_path_factory, trajectories):
    path = tmp_path_factory.mktemp("hf")
    serialize.save(path, _wrap(trajectories))
    loaded = serialize.load(path)
    assert len(loaded) == len(trajectories)
    for a, b in zip(trajectories, loaded):
        assert a == b


@given(st.data(), h_strats.trajectory)
@settings(deadline=None, max_examples=25)
def test_sliced_info_dicts(data, trajectory):
    wrapped = _wrap([trajectory])[0]
    if trajectory.infos is None:
        assert wrapped.infos is None
        return
    sl = data.draw(st.slices(len(trajectory.infos)))
    assert list(wrapped.infos[sl]) == list(trajectory.infos[sl])
    for i in range(len(trajectory.infos)):
        assert wrapped.infos[i] == trajectory.infos[i]


@given(st.data(), h_strats.trajectories_list)
@settings(deadline=None, max_examples=10)
def test_sliced_trajectory_access(data, trajectories):
    """Reference test_sliced_access: a slice of the dataset sequence yields the same trajectories
    as the same slice of the list (10 slices per dataset: building the dataset dominates)."""
    wrapped = _wrap(trajectories)
    for _ in range(10):
        sl = data.draw(st.slices(len(trajectories)))
        idx = list(range(*sl.indices(len(trajectories))))
        got = list(wrapped[sl])
        assert len(got) == len(idx)
        for i, t in zip(idx, got):
            assert t == trajectories[i]
