"""CPU checks of the host twins of the RL kernels (csrc/kernels/rl.hip)."""

import numpy as np
import pytest

from imitation_amd.ops import rl as rl_ops


@pytest.mark.parametrize("n", [1, 2, 5, 64, 1000, 4096])
def test_feistel_rows_are_permutations(n):
    p = rl_ops.random_permutations_reference(4, n, 1234)
    assert p.shape == (4, n) and p.dtype == np.int32
    for row in p:
        assert np.array_equal(np.sort(row), np.arange(n))
    if n >= 64:
        assert not np.array_equal(p[0], p[1])  # epochs draw different orders


def test_feistel_keyed_and_roughly_uniform():
    a = rl_ops.random_permutations_reference(1, 4096, 1)
    b = rl_ops.random_permutations_reference(1, 4096, 2)
    assert not np.array_equal(a, b)
    np.testing.assert_array_equal(a, rl_ops.random_permutations_reference(1, 4096, 1))
    # where index 0 lands over many keys: ~uniform over 16 buckets
    pos = np.array([int(np.flatnonzero(rl_ops.random_permutations_reference(1, 256, s)[0] == 0)[0]) for s in range(800)])
    counts = np.bincount(pos // 16, minlength=16)
    assert counts.min() > 20 and counts.max() < 80
    # displacement is not concentrated near the identity
    assert np.mean(np.abs(a[0] - np.arange(4096))) > 1000


def test_categorical_eval_reference_matches_distribution():
    import torch as th

    from imitation_amd.rl.distributions import CategoricalDistribution

    z = th.randn(50, 6)
    a = th.randint(0, 6, (50,))
    d = CategoricalDistribution(6).proba_distribution(z)
    lp, ent = d.log_prob_entropy(a)
    th.testing.assert_close(lp, d.log_prob(a))
    th.testing.assert_close(ent, d.entropy())


def test_gather_rows_cpu_and_hbm_capacity():
    import torch as th

    from imitation_amd.data.buffer import hbm_capacity

    a, b = th.arange(12).reshape(6, 2), th.arange(6.0)
    got = rl_ops.gather_rows([a, b], th.tensor([1, 0]), th.tensor([1, 2]), 3)
    assert th.equal(got[0], a[[4, 2]]) and th.equal(got[1], b[[4, 2]])
    # 288 GB free, half of it minus the 4 GiB reserve, Pong transitions (84*84*4 + 8 bytes)
    cap = hbm_capacity(84 * 84 * 4 + 8, free_bytes=288 * 10**9)
    assert cap == (144 * 10**9 - (4 << 30)) // (84 * 84 * 4 + 8) and cap > 4_900_000
    with pytest.raises(ValueError):
        hbm_capacity(0, free_bytes=10)


def test_wide_mlp_path_is_opt_in(monkeypatch):
    """The bf16-operand wide kernels (wlin.hip) are opt-in: a generic wide MLP stays on the
    fp32 path unless the module or the process asks for them (advisor round 3)."""
    from imitation_amd.ops import mlp as mlp_ops
    from imitation_amd.util import networks

    dims = [17, 256, 256, 6]
    monkeypatch.delenv("IMITATION_AMD_WIDE_MLP", raising=False)
    assert mlp_ops.fusable([17, 64, 64, 6]) and not mlp_ops.fusable(dims)
    assert mlp_ops.fusable(dims, True) and not mlp_ops.fusable(dims, False)
    monkeypatch.setenv("IMITATION_AMD_WIDE_MLP", "1")
    assert mlp_ops.fusable(dims)
    monkeypatch.delenv("IMITATION_AMD_WIDE_MLP")
    net = networks.build_mlp(in_size=17, hid_sizes=[256, 256], out_size=6)
    assert not net._fusion_plan()
    mlp_ops.set_wide_bf16(net)
    assert net._fusion_plan() and net._fusion_plan()["wide"] is True
    mlp_ops.set_wide_bf16(net, False)
    assert not net._fusion_plan()
