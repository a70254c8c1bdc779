"""CLI smoke tests with the ``fast`` named configs (reference: tests/scripts/test_scripts.py)."""

import json
import os
import pathlib

import numpy as np
import pytest

from imitation_amd.scripts import config_engine as ce

FAST_ENV = ["environment.fast", "policy_evaluation.fast"]


@pytest.fixture(autouse=True)
def _chdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)


def _updates(tmp_path, **kw):
    return {"logging": {"log_root": str(tmp_path / "out")}, **kw}


# ---------------------------------------------------------------- config engine
def test_config_precedence_and_fixed_values():
    ing = ce.Ingredient("ing")

    @ing.config
    def cfg():
        a = 1
        b = a * 10
        d = dict(x=1, y=2)

    @ing.named_config
    def big():
        a = 5

    ex = ce.Experiment("ex", ingredients=[ing])

    @ex.config
    def top(ing):
        c = ing["b"] + 1

    @ex.main
    def main(_config):
        return _config

    c = ex.resolve_config([], {})
    assert c["ing"] == {"a": 1, "b": 10, "d": {"x": 1, "y": 2}} and c["c"] == 11
    c = ex.resolve_config(["ing.big"], {})
    assert c["ing"]["a"] == 5 and c["ing"]["b"] == 50  # named config values are fixed for later scopes
    c = ex.resolve_config(["ing.big"], {"ing": {"a": 7, "d": {"y": 9}}})
    assert c["ing"]["a"] == 7 and c["ing"]["b"] == 70 and c["ing"]["d"] == {"x": 1, "y": 9}  # CLI wins
    assert ex.run(config_updates={"seed": 3}).result["seed"] == 3


def test_config_hooks_rank_below_updates():
    ing = ce.Ingredient("r")

    @ing.config
    def cfg():
        k = None

    @ing.config_hook
    def hook(config, command_name, logger):
        return {"k": "from_hook", "cmd": command_name}

    ex = ce.Experiment("e", ingredients=[ing])

    @ex.command
    def go(r):
        return r

    assert ex.run("go").result == {"k": "from_hook", "cmd": "go"}
    assert ex.run("go", config_updates={"r": {"k": "cli"}}).result["k"] == "cli"


def test_parse_command_line():
    cmd, named, upd, opts = ce.parse_command_line(
        ["gail", "with", "fast", "rl.batch_size=64", "x='s'", "y=[1,2]", "-F", "dir"], {"gail", "airl"})
    assert cmd == "gail" and named == ["fast"] and opts["file_storage"] == "dir"
    assert upd == {"rl": {"batch_size": 64}, "x": "s", "y": [1, 2]}


def test_file_storage_observer(tmp_path):
    ex = ce.Experiment("obs")

    @ex.main
    def main():
        print("hello")
        return {"v": 1}

    ex.observers.append(ce.FileStorageObserver(tmp_path / "runs"))
    ex.run()
    d = tmp_path / "runs" / "1"
    run = json.loads((d / "run.json").read_text())
    assert run["status"] == "COMPLETED" and run["result"] == {"v": 1}
    assert "hello" in (d / "cout.txt").read_text()
    assert "seed" in json.loads((d / "config.json").read_text())


# ---------------------------------------------------------------- scripts
def test_print_config(capsys):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    train_adversarial_ex.run("print_config", named_configs=["gail_seals_half_cheetah"])
    out = capsys.readouterr().out
    assert "seals/HalfCheetah-v1" in out and "demo_batch_size = 8192" in out


@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial(tmp_path, command):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    run = train_adversarial_ex.run(command, named_configs=["fast", "demonstrations.fast", "rl.fast", *FAST_ENV],
                                   config_updates=_updates(tmp_path, checkpoint_interval=1))
    assert run.status == "COMPLETED"
    assert "imit_stats" in run.result and "expert_stats" in run.result
    ckpts = list((tmp_path / "out").rglob("checkpoints/final"))
    assert ckpts and (ckpts[0] / "reward_train.pt").exists() and (ckpts[0] / "gen_policy" / "model.zip").exists()


def test_engine_device_fails_loudly_without_a_gpu(tmp_path):
    """``engine=device`` never silently falls back to the host loop."""
    import torch as th

    from imitation_amd.scripts.train_adversarial import train_adversarial_ex
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    if th.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(ValueError, match="engine=device"):
        train_adversarial_ex.run("airl", named_configs=["fast", "demonstrations.fast", "rl.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path, engine="device"))
    with pytest.raises(ValueError, match="engine=device"):
        train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV],
                                            config_updates=_updates(tmp_path, engine="device"))
    run = train_adversarial_ex.run("gail", named_configs=["fast", "demonstrations.fast", "rl.fast", *FAST_ENV],
                                   config_updates=_updates(tmp_path))
    assert run.result["engine"] == "host"


def _device_cli_updates(tmp_path, **kw):
    # random-policy "expert" demos: no hub model is needed on the box
    return _updates(tmp_path, environment=dict(gym_id="seals/Hopper-v1", num_vec=8, parallel=False),
                    expert=dict(policy_type="random", loader_kwargs={}),
                    rl=dict(batch_size=1024, rl_kwargs=dict(batch_size=64, n_epochs=1)), engine="device",
                    checkpoint_interval=-1, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial_routes_to_device_engine(tmp_path, command):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    run = train_adversarial_ex.run(command, named_configs=["demonstrations.fast", "policy_evaluation.fast"],
                                   config_updates=_device_cli_updates(
                                       tmp_path, total_timesteps=2048,
                                       algorithm_kwargs=dict(demo_batch_size=256, n_disc_updates_per_round=2)))
    assert run.status == "COMPLETED" and run.result["engine"] == "device"


@pytest.mark.gpu
def test_train_preference_comparisons_routes_to_device_agent(tmp_path):
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    run = train_preference_comparisons_ex.run(named_configs=["policy_evaluation.fast"], config_updates=_device_cli_updates(
        tmp_path, total_timesteps=4096, total_comparisons=16, num_iterations=2, fragment_length=20,
        reward_trainer_kwargs=dict(epochs=1)))
    assert run.status == "COMPLETED" and run.result["engine"] == "device"


def test_train_adversarial_algorithm_specific_merge():
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    c = train_adversarial_ex.resolve_config(["seals_half_cheetah"], {}, "airl")
    assert c["total_timesteps"] == int(5e6) and c["reward"]["net_kwargs"]["reward_hid_sizes"] == (32,)
    c = train_adversarial_ex.resolve_config(["seals_half_cheetah"], {}, "gail")
    assert c["total_timesteps"] == int(8e6)


def test_transfer_learning(tmp_path):
    """train_adversarial -> reward_test.pt -> train_rl on that reward (reference transfer test)."""
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex
    from imitation_amd.scripts.train_rl import train_rl_ex

    train_adversarial_ex.run("airl", named_configs=["fast", "demonstrations.fast", "rl.fast", *FAST_ENV],
                             config_updates=_updates(tmp_path))
    reward_path = next((tmp_path / "out").rglob("checkpoints/final/reward_test.pt"))
    run = train_rl_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV],
                          config_updates=_updates(tmp_path, reward_type="RewardNet_unshaped", reward_path=str(reward_path)))
    assert run.status == "COMPLETED" and "return_mean" in run.result


@pytest.mark.parametrize("command", ["bc", "dagger", "sqil"])
def test_train_imitation(tmp_path, command):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    run = train_imitation_ex.run(command, named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path))
    assert run.status == "COMPLETED" and "imit_stats" in run.result


def test_train_bc_warm_start(tmp_path):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    train_imitation_ex.run("bc", named_configs=["fast", "demonstrations.fast", *FAST_ENV], config_updates=_updates(tmp_path))
    policy = next((tmp_path / "out").rglob("final.th"))
    run = train_imitation_ex.run("bc", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path, bc={"agent_path": str(policy)}))
    assert run.status == "COMPLETED"


def test_train_dagger_offline_rollouts(tmp_path):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    run = train_imitation_ex.run("dagger", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path, dagger={"use_offline_rollouts": True}))
    assert run.status == "COMPLETED"


def test_train_rl_and_eval_policy(tmp_path):
    from imitation_amd.scripts.eval_policy import eval_policy_ex
    from imitation_amd.scripts.train_rl import train_rl_ex

    run = train_rl_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV], config_updates=_updates(tmp_path))
    assert run.status == "COMPLETED"
    policy_dir = next((tmp_path / "out").rglob("policies/final"))
    assert (policy_dir / "model.zip").exists()
    assert next((tmp_path / "out").rglob("rollouts/final.npz")).exists()
    ev = eval_policy_ex.run(named_configs=["fast"], config_updates=_updates(
        tmp_path, expert={"policy_type": "ppo", "loader_kwargs": {"path": str(policy_dir / "model.zip")}},
        rollout_save_path="rollouts.npz", explore_kwargs={"switch_prob": 1.0, "random_prob": 0.1}))
    assert ev.status == "COMPLETED" and ev.result["n_traj"] >= 1


@pytest.mark.parametrize("extra", [[], ["reward.reward_ensemble"]])
def test_train_preference_comparisons(tmp_path, extra):
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    upd = _updates(tmp_path, save_preferences=True)
    if extra:
        upd["active_selection"] = True
    run = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV, *extra], config_updates=upd)
    assert run.status == "COMPLETED" and "reward_loss" in run.result
    assert next((tmp_path / "out").rglob("preferences.npz")).exists()
    assert next((tmp_path / "out").rglob("checkpoints/final/reward_net.pt")).exists()


def test_analyze_and_parallel(tmp_path, capsys):
    from imitation_amd.scripts.analyze import analysis_ex
    from imitation_amd.scripts.parallel import parallel_ex

    run = parallel_ex.run(named_configs=["generate_test_data"],
                          config_updates={"base_config_updates": _updates(tmp_path), "local_dir": str(tmp_path / "par")})
    assert len(run.result) == 2 and all(r["status"] == "COMPLETED" for r in run.result)
    table = analysis_ex.run("analyze_imitation", config_updates={"source_dir_str": str(tmp_path / "par"),
                                                                 "table_verbosity": 3}).result
    assert len(table) == 2
    tb = analysis_ex.run("gather_tb_directories", config_updates={"source_dir_str": str(tmp_path / "par")}).result
    assert tb["n_tb_dirs"] >= 0


def test_tuning_fast(tmp_path):
    from imitation_amd.scripts.tuning import tuning_ex

    run = tuning_ex.run(named_configs=["fast_rl"], config_updates={"parallel_run_config": {
        "base_config_updates": _updates(tmp_path), "tune_run_kwargs": {"local_dir": str(tmp_path / "tune")}}})
    assert "best_sample" in run.result and len(run.result["eval_metrics"]) == 2


def test_search_space_generation():
    from imitation_amd.scripts import tune

    trials = tune.generate_trials({"a": tune.grid_search([1, 2]), "b": {"c": tune.choice([5])}, "d": 3}, 2,
                                  np.random.default_rng(0))
    assert len(trials) == 4 and sorted(t["a"] for t in trials) == [1, 1, 2, 2]
    assert all(t["b"]["c"] == 5 and t["d"] == 3 for t in trials)


def test_convert_trajs(tmp_path):
    import shutil

    from imitation_amd.data import serialize
    from imitation_amd.scripts import convert_trajs
    from tests.conftest import TESTDATA

    src = tmp_path / "final.npz"
    shutil.copy(os.path.join(TESTDATA, "expert_models", "cartpole_0", "rollouts", "final.npz"), src)
    out = convert_trajs.update_traj_file_in_place(src)
    assert out == tmp_path / "final" and len(serialize.load(out)) == len(serialize.load(src))


def test_unknown_option_before_with_raises():
    """an unknown ``--option`` (e.g. the typo ``--print-config``) fails like Sacred
    instead of being ignored; Sacred's run options are still accepted."""
    import pytest

    from imitation_amd.scripts.config_engine import parse_command_line

    cmd, named, upd, opts = parse_command_line(["--name=run0", "--capture=sys", "--unobserved", "gail", "with", "x=1"],
                                               ["gail"])
    assert cmd == "gail" and upd == {"x": 1} and opts == {"name": "run0", "capture": "sys", "unobserved": True}
    with pytest.raises(ValueError, match="print-config"):
        parse_command_line(["--print-config", "gail"], ["gail"])
