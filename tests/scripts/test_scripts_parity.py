"""CLI behaviours of the reference test-suite not covered by ``test_scripts.py``
(reference: ``tests/scripts/test_scripts.py`` -- SAC variants :186/:211/:614, SQIL :428,
adversarial warm start :585 and the algorithm value error :635, train_rl double
normalisation :768 and CNN policy :799, analyze gather_tb :1008)."""

import os
import pathlib
import numpy as np
import pytest
import torch as th

FAST_ENV = ["environment.fast", "policy_evaluation.fast"]
RANDOM_EXPERT = {"policy_type": "random", "loader_kwargs": {}}


@pytest.fixture(autouse=True)
def _chdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)


def _updates(tmp_path, **kw):
    return {"logging": {"log_root": str(tmp_path / "out")}, **kw}


def _check_imit_result(result):
    assert "imit_stats" in result and "expert_stats" in result
    assert np.isfinite(result["imit_stats"]["monitor_return_mean"])


@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial_sac(tmp_path, command):
    """rl.sac after rl.fast (so the SAC batch size stays at the top level) on Pendulum."""
    from imitation_amd.rl.sac import SAC
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    run = train_adversarial_ex.run(command, named_configs=["pendulum", "fast", "demonstrations.fast", "rl.fast", "rl.sac", "policy.sac",
                                                           *FAST_ENV],
                                   config_updates=_updates(tmp_path, expert=RANDOM_EXPERT))
    assert run.config["rl"]["rl_cls"] is SAC
    assert run.status == "COMPLETED"
    _check_imit_result(run.result)


def test_train_preference_comparisons_sac(tmp_path):
    from imitation_amd.rl.sac import SAC
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    upd = _updates(tmp_path, environment={"gym_id": "Pendulum-v1"})
    run = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", "rl.sac", "policy.sac", *FAST_ENV], config_updates=upd)
    assert run.config["rl"]["rl_cls"] is SAC
    assert run.status == "COMPLETED" and "reward_loss" in run.result
    # rl.sac BEFORE rl.fast: rl.fast sets rl_kwargs.batch_size again, which SAC rejects
    with pytest.raises(Exception, match="set 'batch_size' at top-level"):
        train_preference_comparisons_ex.run(named_configs=["rl.sac", "policy.sac", "fast", "rl.fast", *FAST_ENV],
                                            config_updates=_updates(tmp_path, environment={"gym_id": "Pendulum-v1"}))


def test_train_preference_comparisons_sac_reward_relabel(tmp_path):
    """SAC with a relabelling replay buffer (``ReplayBufferRewardWrapper`` around the chosen
    buffer class), reference test_scripts.py:211."""
    from imitation_amd.rl import buffers
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    upd = _updates(tmp_path, environment={"gym_id": "Pendulum-v1"},
                   rl={"rl_kwargs": {"replay_buffer_class": buffers.ReplayBuffer,
                                     "replay_buffer_kwargs": {"handle_timeout_termination": True}}})
    run = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", "rl.sac", "policy.sac", *FAST_ENV], config_updates=upd)
    assert run.status == "COMPLETED"


def test_train_sqil_cartpole(tmp_path):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    run = train_imitation_ex.run("sqil", named_configs=["seals_cartpole", "fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path))
    assert run.status == "COMPLETED"
    _check_imit_result(run.result)


def test_train_sqil_local_demonstrations(tmp_path):
    """SQIL from a local rollout file (the reference loads the same demos from the hub)."""
    from imitation_amd.scripts.train_imitation import train_imitation_ex
    from tests.conftest import TESTDATA

    path = os.path.join(TESTDATA, "expert_models", "cartpole_0", "rollouts", "final.npz")
    run = train_imitation_ex.run("sqil", named_configs=["cartpole", "fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path, demonstrations={"source": "local", "path": path}))
    assert run.status == "COMPLETED"


@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial_warmstart(tmp_path, command):
    """The final generator checkpoint warm-starts a second run (``agent_path``)."""
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    named = ["cartpole", "fast", "demonstrations.fast", "rl.fast", *FAST_ENV]
    run = train_adversarial_ex.run(command, named_configs=named, config_updates=_updates(tmp_path))
    policy_path = next((tmp_path / "out").rglob("checkpoints/final/gen_policy"))
    assert (policy_path / "model.zip").exists()
    run2 = train_adversarial_ex.run(command, named_configs=named,
                                    config_updates=_updates(tmp_path, agent_path=str(policy_path)))
    assert run2.status == "COMPLETED"
    _check_imit_result(run2.result)


def test_train_adversarial_algorithm_value_error(tmp_path):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    named = ["cartpole", "fast", "demonstrations.fast", "rl.fast", *FAST_ENV]
    with pytest.raises(TypeError, match="BAD_VALUE"):
        train_adversarial_ex.run("gail", named_configs=named,
                                 config_updates=_updates(tmp_path, algorithm_kwargs={"BAD_VALUE": "bar"}))
    with pytest.raises(TypeError, match="BAD_VALUE"):
        train_adversarial_ex.run("gail", named_configs=named,
                                 config_updates=_updates(tmp_path, reward={"net_kwargs": {"BAD_VALUE": "bar"}}))
    with pytest.raises(TypeError, match="BAD_VALUE"):
        train_adversarial_ex.run("gail", named_configs=named,
                                 config_updates=_updates(tmp_path, rl={"rl_kwargs": {"BAD_VALUE": "bar"}}))


def test_train_rl_double_normalization(tmp_path):
    """A reward net that is already a NormalizedRewardNet plus ``normalize_reward=True``
    warns (reference test_scripts.py:768)."""
    from imitation_amd.envs import make as make_env
    from imitation_amd.rewards import reward_nets
    from imitation_amd.rewards import serialize as reward_serialize
    from imitation_amd.scripts.train_rl import train_rl_ex
    from imitation_amd.util import networks

    env = make_env("CartPole-v1")
    net = reward_nets.NormalizedRewardNet(reward_nets.BasicRewardNet(env.observation_space, env.action_space),
                                          networks.RunningNorm)
    path = str(tmp_path / "reward.pt")
    reward_serialize.save_reward_net(net, path)  # spec + state dict (loaded weights_only)
    with pytest.warns(RuntimeWarning, match="Applying normalization to already normalized reward function"):
        run = train_rl_ex.run(named_configs=["cartpole", "fast", "rl.fast", *FAST_ENV],
                              config_updates=_updates(tmp_path, reward_type="RewardNet_normalized", normalize_reward=True,
                                                      reward_path=path))
    assert run.status == "COMPLETED"


def test_train_rl_cnn_policy(tmp_path):
    """train_rl on an Atari-shaped image env with a CNN reward net and the cnn_policy config
    (reference test_scripts.py:799 uses Asteroids; the image-shaped env here is Pong)."""
    from imitation_amd.envs import make as make_env
    from imitation_amd.rewards import reward_nets
    from imitation_amd.rewards import serialize as reward_serialize
    from imitation_amd.scripts.train_rl import train_rl_ex

    env = make_env("PongNoFrameskip-v4")
    net = reward_nets.CnnRewardNet(env.observation_space, env.action_space)
    path = str(tmp_path / "reward.pt")
    reward_serialize.save_reward_net(net, path)
    run = train_rl_ex.run(named_configs=["fast", "rl.fast", "policy.cnn_policy", *FAST_ENV],
                          config_updates=_updates(tmp_path, environment={"gym_id": "PongNoFrameskip-v4", "num_vec": 1},
                                                  reward_type="RewardNet_unnormalized", reward_path=path,
                                                  total_timesteps=16, rl={"batch_size": 8, "rl_kwargs": {"batch_size": 8,
                                                                                                      "n_epochs": 1}}))
    assert run.status == "COMPLETED" and "return_mean" in run.result


def test_analyze_gather_tb(tmp_path):
    """gather_tb_directories over the runs of a parallel sweep: one symlinked TB dir per run
    that logged one (reference test_scripts.py:1008)."""
    from imitation_amd.scripts.analyze import analysis_ex
    from imitation_amd.scripts.parallel import parallel_ex

    par = parallel_ex.run(named_configs=["generate_test_data"],
                          config_updates={"base_config_updates": _updates(tmp_path), "local_dir": str(tmp_path / "par"),
                                          "num_samples": 2, "run_name": "test"})
    assert all(r["status"] == "COMPLETED" for r in par.result)
    run = analysis_ex.run("gather_tb_directories", config_updates={"source_dirs": [str(tmp_path / "par")]})
    assert run.status == "COMPLETED"
    res = run.result
    assert res["n_tb_dirs"] >= 1
    out = pathlib.Path(res["gather_dir"])
    assert out.is_dir() and any(out.rglob("*"))


SCRIPT_MODS = ["analyze", "eval_policy", "parallel", "train_adversarial", "train_imitation",
               "train_preference_comparisons", "train_rl", "tuning"]


@pytest.mark.parametrize("mod_name", SCRIPT_MODS)
def test_main_console(mod_name, monkeypatch):
    """Every script's console entry point runs (print_config) -- reference test_main_console."""
    import importlib
    import sys

    mod = importlib.import_module(f"imitation_amd.scripts.{mod_name}")
    monkeypatch.setattr(sys, "argv", ["sacred-pytest-stub", "print_config"])
    mod.main_console()


def test_train_bc_main_with_none_demonstrations_raises_value_error(tmp_path):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    with pytest.raises(ValueError, match="n_expert_demos must be specified"):
        train_imitation_ex.run("bc", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                               config_updates=_updates(tmp_path, demonstrations={"n_expert_demos": None}))


def test_train_dagger_warmstart(tmp_path):
    """A DAgger run warm-started from the previous run's latest scratch policy (reference
    test_train_dagger_warmstart)."""
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    run = train_imitation_ex.run("dagger", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates=_updates(tmp_path))
    assert run.status == "COMPLETED"
    policy_path = pathlib.Path(run.config["logging"]["log_dir"]) / "scratch" / "policy-latest.pt"
    assert policy_path.exists()
    warm = train_imitation_ex.run("dagger", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                  config_updates=_updates(tmp_path, bc={"agent_path": str(policy_path)}))
    assert warm.status == "COMPLETED" and isinstance(warm.result, dict)


@pytest.mark.parametrize("named_configs", [[], ["reward.normalize_output_running"], ["reward.normalize_output_disable"]])
def test_train_preference_comparisons_reward_named_config(tmp_path, named_configs):
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex
    from imitation_amd.util import networks

    run = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV, *named_configs],
                                              config_updates=_updates(tmp_path))
    expect = None if "reward.normalize_output_disable" in named_configs else networks.RunningNorm
    assert run.config["reward"]["normalize_output_layer"] is expect
    assert run.status == "COMPLETED" and isinstance(run.result, dict)


def test_parallel_arg_errors(tmp_path):
    """Bad base / search-space argument types raise (reference test_parallel_arg_errors)."""
    from imitation_amd.scripts.parallel import parallel_ex

    base = {"base_config_updates": _updates(tmp_path), "local_dir": str(tmp_path / "par")}
    cases = [({"base_named_configs": {}}, "Sequence"), ({"base_config_updates": ()}, "Mapping"),
             ({"search_space": {"named_configs": {}}}, "Sequence"), ({"search_space": {"config_updates": ()}}, "Mapping")]
    for upd, match in cases:
        with pytest.raises(TypeError, match=match):
            parallel_ex.run(named_configs=["generate_test_data"], config_updates={**base, **upd})


@pytest.mark.parametrize("env_name", ["seals_cartpole", "mountain_car", "seals_mountain_car"])
def test_train_preference_comparisons_envs_no_crash(tmp_path, env_name):
    """The env named configs of train_preference_comparisons run end to end (reference
    test_scripts.py:171)."""
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    run = train_preference_comparisons_ex.run(named_configs=[env_name, "fast", "rl.fast", *FAST_ENV],
                                              config_updates=_updates(tmp_path))
    assert run.status == "COMPLETED" and isinstance(run.result, dict)


def test_train_rl_sac(tmp_path):
    """rl.sac after rl.fast on Pendulum (reference test_scripts.py:486)."""
    from imitation_amd.rl.sac import SAC
    from imitation_amd.scripts.train_rl import train_rl_ex

    run = train_rl_ex.run(named_configs=["pendulum", "environment.fast", "rl.fast", "fast", "rl.sac", "policy.sac"],
                          config_updates=_updates(tmp_path))
    assert run.config["rl"]["rl_cls"] is SAC
    assert run.status == "COMPLETED" and isinstance(run.result, dict)


@pytest.mark.parametrize("config", [
    {"reward_type": "zero", "reward_path": "foobar"},
    {"explore_kwargs": {"switch_prob": 1.0, "random_prob": 0.1}},
    {"rollout_save_path": "{log_dir}/rollouts.npz"},
])
def test_eval_policy_configs(tmp_path, config):
    """eval_policy's reward wrapping, exploration and rollout saving (reference
    test_scripts.py:518): a wrapped reward makes return_mean differ from the monitor's."""
    from imitation_amd.scripts.eval_policy import eval_policy_ex

    run = eval_policy_ex.run(named_configs=["environment.fast", "fast"], config_updates=_updates(tmp_path, **config))
    assert run.status == "COMPLETED"
    stats = run.result
    assert "return_mean" in stats and "monitor_return_mean" in stats
    if "reward_type" in config:
        assert stats["return_mean"] != stats["monitor_return_mean"]
    else:
        assert stats["return_mean"] == stats["monitor_return_mean"]
    if "rollout_save_path" in config:
        assert next((tmp_path / "out").rglob("rollouts.npz")).exists()


def test_converted_trajectories_equal_original(tmp_path):
    """convert_trajs turns a legacy npz file into the current format with equal trajectories
    (reference test_scripts.py:1070)."""
    import shutil

    from imitation_amd.data import serialize
    from imitation_amd.scripts import convert_trajs
    from tests.conftest import TESTDATA

    src = tmp_path / "final.npz"
    shutil.copy(os.path.join(TESTDATA, "expert_models", "cartpole_0", "rollouts", "final.npz"), src)
    old = serialize.load(src)
    converted = serialize.load(convert_trajs.update_traj_file_in_place(src))
    assert len(old) == len(converted)
    for a, b in zip(old, converted):
        assert a == b


def test_convert_trajs_from_current_format_is_idempotent(tmp_path):
    """Converting a file that is already in the current format leaves it unchanged (reference
    test_scripts.py:1085)."""
    import filecmp
    import shutil

    from imitation_amd.scripts import convert_trajs
    from tests.conftest import TESTDATA

    src = tmp_path / "final.npz"
    shutil.copy(os.path.join(TESTDATA, "expert_models", "cartpole_0", "rollouts", "final.npz"), src)
    current = convert_trajs.update_traj_file_in_place(src)
    orig = current.with_suffix(".orig")
    shutil.copytree(current, orig)
    again = convert_trajs.update_traj_file_in_place(current)
    cmp = filecmp.dircmp(again, orig)
    assert cmp.diff_files == [] and cmp.left_only == [] and cmp.right_only == [], "convert_trajs not idempotent"


def test_parallel_train_adversarial_custom_env(tmp_path):
    """A parallel sweep of train_adversarial on Pendulum with demonstrations from a train_rl run, two
    repeats of a one-choice search space (reference test_scripts.py:912)."""
    from imitation_amd.scripts import tune
    from imitation_amd.scripts.parallel import parallel_ex
    from imitation_amd.scripts.train_rl import train_rl_ex

    rl_dir = tmp_path / "rl"
    train_rl_ex.run(named_configs=["pendulum", "environment.fast", "rl.fast", "fast"],
                    config_updates={"logging": {"log_dir": str(rl_dir)}})
    demo_path = rl_dir / "rollouts" / "final.npz"
    assert demo_path.exists()
    run = parallel_ex.run(config_updates={
        "sacred_ex_name": "train_adversarial", "repeat": 2, "local_dir": str(tmp_path / "par"),
        "base_named_configs": ["pendulum", "environment.fast", "demonstrations.fast", "rl.fast", "fast"],
        "base_config_updates": _updates(tmp_path, demonstrations={"source": "local", "path": str(demo_path),
                                                                         "n_expert_demos": 1}),
        "search_space": {"command_name": tune.choice(["gail"])}})
    assert run.status == "COMPLETED"
    assert len(run.result) == 2 and all(r["status"] == "COMPLETED" for r in run.result)
