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


# ---------------------------------------------------------------- experiments/commands.py
COMMANDS_PY = ROOT / "experiments" / "commands.py"


def _commands(*flags, cwd=None):
    import subprocess
    import sys

    out = subprocess.run([sys.executable, str(COMMANDS_PY), *flags], capture_output=True, check=True, cwd=cwd,
                         stdin=subprocess.DEVNULL)
    return out.stdout.decode().strip().split("\n")


@pytest.fixture
def hps_dir(tmp_path):
    _commands("--export_tuned_hps", str(tmp_path / "hps"))
    return tmp_path / "hps"


def test_commands_local_config(hps_dir):
    """One (config file, seed) -> one command in the reference's format (reference
    test_commands_local_config; the run id ends with the adler32 of the file name)."""
    cfg = hps_dir / "fast_dagger_seals_cartpole.json"
    cmds = _commands("--name=run0", f"--cfg_pattern={cfg}", "--output_dir=output")
    assert cmds == [f"python -m imitation_amd.scripts.train_imitation dagger --capture=sys --name=run0 "
                    f"--file_storage=output/sacred/$USER-cmd-run0-dagger-0-c9420c90 with {cfg} seed=0 "
                    f"logging.log_root=output"]


def test_commands_local_config_runs(hps_dir, tmp_path):
    """The printed command runs to completion (reference test_commands_local_config_runs)."""
    import os
    import subprocess

    cfg = hps_dir / "fast_dagger_seals_cartpole.json"
    out = tmp_path / "out"
    (cmd,) = _commands("--name=run0", f"--cfg_pattern={cfg}", f"--output_dir={out}")
    env = dict(os.environ, USER=os.environ.get("USER", "user"), PYTHONPATH=str(ROOT))
    done = subprocess.run(cmd + " environment.fast policy_evaluation.fast", shell=True, cwd=tmp_path, env=env,
                          capture_output=True, stdin=subprocess.DEVNULL, timeout=600)
    assert done.returncode == 0, done.stderr.decode()[-2000:]
    assert list((out / "sacred").glob("*-cmd-run0-dagger-0-c9420c90/*/run.json"))


def test_commands_multiple_configs_multiple_seeds(hps_dir):
    cmds = _commands("--name=run0", f"--cfg_pattern={hps_dir}/*ai*_seals_walker*.json", "--output_dir=output",
                     "--seeds", "0", "1", "2")
    assert len(cmds) == 6
    assert sum("train_adversarial airl" in c for c in cmds) == 3 and sum("train_adversarial gail" in c for c in cmds) == 3
    assert {c.split(" seed=")[1].split(" ")[0] for c in cmds} == {"0", "1", "2"}


def test_commands_remote_config(hps_dir):
    """--remote: each command as a containerised cluster job reading the config from
    --remote_cfg_dir (reference test_commands_hofvarpnir_config)."""
    cfg = hps_dir / "fast_dagger_seals_cartpole.json"
    (cmd,) = _commands("--name=run0", f"--cfg_pattern={cfg}", "--output_dir=/data/output", "--remote",
                       "--remote_cfg_dir=/data/hps", "--container=img:tag")
    assert cmd.startswith("ctl job run --name $USER-cmd-run0-dagger-0-c9420c90 --command \"python -m ")
    assert "with /data/hps/fast_dagger_seals_cartpole.json seed=0 logging.log_root=/data/output\"" in cmd
    assert "--container img:tag" in cmd


def test_commands_named_config_mode():
    cmds = _commands("--name=x", "--cfg", "gail_seals_hopper", "--seeds", "3", "--gpus-per-run", "8")
    assert len(cmds) == 1 and cmds[0].startswith("torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 ")
    assert " with gail_seals_hopper seed=3 " in cmds[0]
