"""Data-parallel correctness on CPU with gloo, world_size 2 (N ranks x mb == 1 rank x N*mb)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.testing import dist_workers as W
from imitation_amd.testing.distributed import run_ranks


def test_allreduce_moments():
    rng = np.random.default_rng(0)
    data = [rng.normal(size=(5, 3)).astype(np.float32), rng.normal(size=(9, 3)).astype(np.float32) + 2]
    out = run_ranks(W.moments_worker, 2, data)
    full = np.concatenate(data)
    for mean, var, count in out:
        np.testing.assert_allclose(mean, full.mean(0), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(var, full.var(0), rtol=1e-4, atol=1e-6)
        assert count == 14


def test_running_norm_synchronised():
    """DP RunningNorm == one process seeing the concatenation of the ranks' batches."""
    from imitation_amd.util import networks

    rng = np.random.default_rng(1)
    shards = [[rng.normal(size=(4, 2)).astype(np.float32) * (r + 1) for _ in range(3)] for r in range(2)]
    out = run_ranks(W.running_norm_worker, 2, shards)
    ref = networks.RunningNorm(2)
    with th.no_grad():
        for step in range(3):
            ref.update_stats(th.as_tensor(np.concatenate([shards[0][step], shards[1][step]])))
    for mean, var, count in out:
        np.testing.assert_allclose(mean, ref.running_mean.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(var, ref.running_var.numpy(), rtol=1e-4, atol=1e-6)
        assert count == int(ref.count.item())


def test_grad_bucket_mean_and_broadcast():
    out = run_ranks(W.grad_bucket_worker, 2)
    (g0, p0), (g1, p1) = out
    for a, b in zip(p0, p1):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(g0, g1):
        np.testing.assert_allclose(a, b)
    # d/dW sum(W x + b) over 4 rows of value (r+1): mean over ranks of 4*(r+1) = 6
    np.testing.assert_allclose(g0[0], np.full((2, 3), 6.0))
    np.testing.assert_allclose(g0[1], np.full(2, 4.0))


def test_all_gather_rows_uneven():
    out = run_ranks(W.gather_rows_worker, 2)
    exp = np.concatenate([np.arange(2, dtype=np.float32).reshape(1, 2), np.arange(4, dtype=np.float32).reshape(2, 2) + 100])
    for o in out:
        np.testing.assert_array_equal(o, exp)


def test_bc_data_parallel_equals_large_batch():
    rng = np.random.default_rng(0)
    batch, steps = 16, 5
    obs = rng.normal(size=(2 * batch * steps, 4)).astype(np.float32)
    acts = (obs[:, 0] > 0).astype(np.int64)
    dp = run_ranks(W.bc_dp_worker, 2, obs, acts, batch, steps, 0)
    for a, b in zip(dp[0], dp[1]):
        np.testing.assert_array_equal(a, b)
    single = run_ranks(W.bc_dp_worker, 1, obs, acts, 2 * batch, steps, 0)[0]
    for a, b in zip(dp[0], single):
        np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


def test_ppo_ranks_stay_in_sync():
    out = run_ranks(W.ppo_dp_worker, 2, 3)
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_device_gail_replicated_dp_matches_large_batch(world, monkeypatch):
    """world ranks share one GPU over gloo: after one device PPO round every rank holds the
    bit-identical model, equal to the fp32 reference over the gathered rows (minibatch world x 64)."""
    monkeypatch.setenv("IMITATION_AMD_DIST_BACKEND", "gloo")
    out = run_ranks(W.device_gail_dp_worker, world, 5, 64, timeout=240)
    for r in range(1, world):
        for a, b in zip(out[0]["params"], out[r]["params"]):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(out[0]["norm"][0], out[r]["norm"][0])
    assert out[0]["max_dev"] < 2e-3 * max(1.0, out[0]["max_ref"]), out[0]["max_dev"]


def test_preference_reward_dp_equals_large_minibatch():
    """2 ranks x minibatch mb == 1 rank x minibatch 2*mb (replicated dataset, averaged grads,
    all-reduced RunningNorm moments); the replicas are bit-identical."""
    P, L, mb, epochs, seed = 40, 6, 4, 2, 3
    dp = run_ranks(W.pref_reward_dp_worker, 2, P, L, mb, epochs, seed)
    for a, b in zip(dp[0], dp[1]):
        np.testing.assert_array_equal(a, b)
    ref = W.pref_reward_dp_worker(0, 1, P, L, 2 * mb, epochs, seed)
    # index 5 = the output bias: the Bradley-Terry loss depends on reward DIFFERENCES only, so
    # its gradient is rounding noise that Adam normalises into full-size steps -- excluded
    for i, (a, b) in enumerate(zip(dp[0], ref)):
        if i != 5:
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


def test_preference_pairs_all_gathered_in_rank_order():
    out = run_ranks(W.pref_gather_worker, 2, 11)
    assert out[0] == out[1]
    sums, prefs = out[0]
    assert len(sums) == 3 + 4 and len(prefs) == 7


def test_dagger_data_parallel(tmp_path):
    """Per-rank scratch dirs, rank-agreed rounds, the all-gathered demo union on every rank
    and bit-identical BC replicas (grads averaged over the gloo group)."""
    out = run_ranks(W.dagger_dp_worker, 2, str(tmp_path), 5)
    a, b = out
    assert a["scratch"] != b["scratch"] and a["scratch"].endswith("rank-00") and b["scratch"].endswith("rank-01")
    assert a["round_num"] == b["round_num"] >= 1
    assert a["n_demos"] == b["n_demos"] == a["local_files"] + b["local_files"]
    assert a["last"] == b["last"] == a["local"] + b["local"]
    for p, q in zip(a["params"], b["params"]):
        np.testing.assert_array_equal(p, q)


@pytest.mark.parametrize("mode", ["auto", "1", "0"])
def test_oneshot_off_without_gpu(mode, monkeypatch):
    monkeypatch.setenv("IMITATION_AMD_ONESHOT", mode)
    out = run_ranks(W.oneshot_cpu_worker, 2)
    for o in out:
        assert not o["comm"] and not o["active"] and not o["moments_device"]
        assert o["sum"] == [3.0] * 5
