"""Sacred run-directory discovery / grouping (upstream tests/util/test_sacred_file_parsing.py)."""

import json

from imitation_amd.util import sacred_file_parsing as sfp


def _run_dir(path, command, env, status="COMPLETED"):
    path.mkdir(parents=True, exist_ok=True)
    (path / "config.json").write_text(json.dumps({"environment": {"gym_id": env}}))
    (path / "run.json").write_text(json.dumps({"status": status, "command": command}))


def test_find_runs_recursively(tmp_path):
    _run_dir(tmp_path / "a", "ppo", "CartPole-v1")
    _run_dir(tmp_path / "nested" / "b", "ppo", "CartPole-v1")
    _run_dir(tmp_path / "nested" / "deeper" / "c", "gail", "Pendulum-v1")
    runs = list(sfp.find_sacred_runs(tmp_path))
    assert len(runs) == 3
    assert sorted(r["command"] for _, r in runs) == ["gail", "ppo", "ppo"]
    assert {c["environment"]["gym_id"] for c, _ in runs} == {"CartPole-v1", "Pendulum-v1"}


def test_only_completed_runs(tmp_path):
    for i, status in enumerate(["COMPLETED", "FAILED", "RUNNING", "COMPLETED"]):
        _run_dir(tmp_path / f"r{i}", "airl", "CartPole-v1", status=status)
    assert len(list(sfp.find_sacred_runs(tmp_path))) == 4
    done = list(sfp.find_sacred_runs(tmp_path, only_completed_runs=True))
    assert len(done) == 2 and all(r["status"] == "COMPLETED" for _, r in done)


def test_group_by_algo_and_env(tmp_path):
    spec = [("ppo", "CartPole-v1"), ("airl", "CartPole-v1"), ("ppo", "CartPole-v1"), ("gail", "CartPole-v1"),
            ("ppo", "LunarLander-v2"), ("airl", "LunarLander-v2")]
    for i, (algo, env) in enumerate(spec):
        _run_dir(tmp_path / f"run{i}", algo, env)
    grouped = sfp.group_runs_by_algo_and_env(tmp_path)
    assert set(grouped) == {"ppo", "airl", "gail"}
    assert set(grouped["ppo"]) == {"CartPole-v1", "LunarLander-v2"}
    assert set(grouped["gail"]) == {"CartPole-v1"}
    assert len(grouped["ppo"]["CartPole-v1"]) == 2
