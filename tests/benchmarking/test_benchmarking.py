"""Benchmark tooling (reference: tests/test_benchmarking.py + benchmarking/*)."""

import json
import pathlib

import numpy as np
import pytest

from imitation_amd.benchmarking import probability_of_improvement as poi
from imitation_amd.benchmarking import stats, summary, util


def test_iqm_and_mean():
    x = np.arange(1, 9, dtype=float).reshape(4, 2)
    assert stats.aggregate_mean(x) == 4.5
    assert stats.aggregate_iqm(x) == pytest.approx(np.mean([3, 4, 5, 6]))


def test_probability_of_improvement_bounds():
    a = np.ones((5, 3))
    assert stats.probability_of_improvement(a + 1, a) == 1.0
    assert stats.probability_of_improvement(a, a) == 0.5
    point, ci = stats.get_interval_estimates({"k": (a + np.random.rand(5, 3), a)}, stats.probability_of_improvement, reps=50)
    assert 0 <= ci["k"][0][0] <= point["k"][0] <= ci["k"][1][0] <= 1


def _fake_runs(root: pathlib.Path, algo: str, env: str, scores, expert=10.0):
    for i, s in enumerate(scores):
        d = root / f"{algo}-{env}-{i}" / "sacred" / "1"
        d.mkdir(parents=True)
        (d / "config.json").write_text(json.dumps({"environment": {"gym_id": env}, "seed": i}))
        (d / "run.json").write_text(json.dumps({"command": algo, "status": "COMPLETED", "result": {
            "imit_stats": {"monitor_return_mean": s, "return_mean": s},
            "expert_stats": {"monitor_return_mean": expert, "return_mean": expert}}}))


def test_summary_and_poi(tmp_path):
    _fake_runs(tmp_path / "a", "gail", "envA", [5, 6, 7])
    _fake_runs(tmp_path / "a", "gail", "envB", [8, 9, 10])
    _fake_runs(tmp_path / "b", "bc", "envA", [1, 2, 3])
    _fake_runs(tmp_path / "b", "bc", "envB", [1, 2, 3])
    lines = list(summary.print_markdown_summary(tmp_path / "a", random_score_fn=lambda env: 0.0))
    text = "\n".join(lines)
    assert "### GAIL" in text and "IQM" in text and "envA | 6.000" in text
    res = poi.main([str(tmp_path / "a"), str(tmp_path / "b"), "--bootstrap-reps", "50"])
    assert res.probability_of_improvement == 1.0
    n = util.sacred_output_to_csv(tmp_path / "a", tmp_path / "out.csv")
    assert n == 6


def test_benchmark_commands():
    cmds = util.benchmark_commands()
    assert len(cmds) == 200
    assert cmds[0].startswith("python -m imitation_amd.scripts.train_imitation bc with bc_seals_ant seed=1")


def test_benchmark_configs_resolve():
    """Every tuned benchmark config resolves (reference validates them via print_config)."""
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    for cmd in util.benchmark_commands(seeds=(1,)):
        parts = cmd.split()
        algo, named = parts[3], parts[5]
        ex = train_imitation_ex if "train_imitation" in parts[2] else train_adversarial_ex
        cfg = ex.resolve_config([named], {"seed": 1}, algo)
        assert cfg["environment"]["gym_id"].startswith("seals/")


def test_clean_config_file(tmp_path):
    src = tmp_path / "config.json"
    src.write_text(json.dumps({"seed": 1, "agent_path": None, "demonstrations": {"path": "x", "n": 1}, "empty": {}}))
    util.clean_config_file(src, tmp_path / "clean.json")
    assert json.loads((tmp_path / "clean.json").read_text()) == {"demonstrations": {"n": 1}}
