"""The legacy experiment sweeps (experiments/sweeps.py) in --fast mode."""

import importlib.util
import pathlib

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _sweeps():
    spec = importlib.util.spec_from_file_location("sweeps", ROOT / "experiments" / "sweeps.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("cmd", ["bc", "dagger", "rollouts_from_policies"])
def test_fast_sweeps_complete(tmp_path, monkeypatch, cmd):
    monkeypatch.chdir(tmp_path)
    rows = _sweeps().main([cmd, "--fast", "--gpus", "0", "--log-root", str(tmp_path / "out")])
    assert rows and all(r["status"] == "COMPLETED" for r in rows)


def test_fast_transfer_learning_sweep(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rows = _sweeps().main(["transfer_learn", "--fast", "--algo", "airl", "--gpus", "0", "--log-root", str(tmp_path / "out")])
    assert rows and all(r["status"] == "COMPLETED" for r in rows)


def test_convert_traj_to_baselines_npz(tmp_path):
    from imitation_amd.data import serialize, types

    rng = np.random.default_rng(0)
    trajs = [types.TrajectoryWithRew(obs=rng.standard_normal((L + 1, 3)).astype(np.float32), acts=rng.integers(0, 2, L),
                                     infos=None, terminal=True, rews=np.ones(L, np.float32)) for L in (4, 6)]
    serialize.save(tmp_path / "src", trajs)
    dst = _sweeps().main(["convert_traj", str(tmp_path / "src"), str(tmp_path / "b" / "gail.npz")])
    d = np.load(dst)
    assert d["obs"].shape == (10, 3) and d["acs"].shape == (10,) and np.allclose(d["ep_rets"], [4, 6])


def test_quickstart_example_fast(monkeypatch, tmp_path):
    monkeypatch.chdir(tmp_path)
    spec = importlib.util.spec_from_file_location("quickstart", ROOT / "examples" / "quickstart.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    before, after = mod.main(["--fast", "--device", "cpu"])
    assert np.isfinite(before) and np.isfinite(after)


def test_quickstart_shell_example_runs_twice(tmp_path):
    """Reference tests/test_examples.py: the CLI quickstart (RL expert, then GAIL and AIRL from its
    rollouts) runs to completion, twice in the same directory."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, PYTHONPATH=str(ROOT) + os.pathsep + os.environ.get("PYTHONPATH", ""))
    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "python").symlink_to(sys.executable)
    env["PATH"] = str(bindir) + os.pathsep + env["PATH"]
    for _ in range(2):
        r = subprocess.run(["bash", "-e", str(ROOT / "examples" / "quickstart.sh")], cwd=tmp_path, env=env,
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "quickstart" / "rl" / "rollouts" / "final.npz").exists()
