"""Exact resume from the CLIs (VERDICT r5 missing #2).

Run N rounds with full checkpoints, stop ("kill"), run again with ``resume_from`` for 2N rounds
in total: the final reward net, generator and evaluation equal those of 2N uninterrupted
rounds -- exactly on the host loop (CPU) and bitwise on the device engine (GPU). The reference
only snapshots the reward net / policy (``src/imitation/scripts/train_adversarial.py:25-35,157``),
so a crashed run restarts from zero there.
"""

import glob
import os

import pytest
import torch as th

FAST_ENV = ["environment.fast", "policy_evaluation.fast"]


@pytest.fixture(autouse=True)
def _chdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)


def _final_params(log_root):
    from imitation_amd.rewards import serialize as reward_serialize
    from imitation_amd.rl.save_util import load_from_zip_file

    (rew,) = glob.glob(os.path.join(log_root, "**", "checkpoints", "final", "reward_train.pt"), recursive=True)
    net = reward_serialize.load_reward_net(rew, device="cpu")
    out = {f"reward.{k}": v.detach().cpu() for k, v in net.state_dict().items()}
    (zp,) = glob.glob(os.path.join(log_root, "**", "checkpoints", "final", "gen_policy", "model.zip"), recursive=True)
    _, params, _ = load_from_zip_file(zp, device="cpu")

    def flat(prefix, x):
        if isinstance(x, th.Tensor):
            out[prefix] = x.detach().cpu()
        elif isinstance(x, dict):
            for n, v in x.items():
                flat(f"{prefix}.{n}", v)
        elif isinstance(x, (list, tuple)):
            for i, v in enumerate(x):
                flat(f"{prefix}.{i}", v)

    flat("gen", params)  # policy weights and optimizer moments
    return out


def _full_ckpts(log_root):
    return sorted(glob.glob(os.path.join(log_root, "**", "full_checkpoints", "ckpt-*"), recursive=True))


def _adversarial(tmp_path, name, command, named, updates):
    from imitation_amd.scripts.train_adversarial import train_adversarial_ex

    root = str(tmp_path / name)
    run = train_adversarial_ex.run(command, named_configs=named,
                                   config_updates={"logging": {"log_root": root}, "seed": 0, **updates})
    assert run.status == "COMPLETED"
    return root, run.result


def _check_resume(tmp_path, command, named, updates, per_round, n):
    full, res_full = _adversarial(tmp_path, "full", command, named, dict(updates, total_timesteps=2 * n * per_round))
    first, _ = _adversarial(tmp_path, "first", command, named,
                            dict(updates, total_timesteps=n * per_round, full_checkpoint_interval=2))
    ck = _full_ckpts(first)
    assert [os.path.basename(c) for c in ck][-1] == f"ckpt-{n:010d}"
    resumed, res_resumed = _adversarial(tmp_path, "resumed", command, named,
                                        dict(updates, total_timesteps=2 * n * per_round, full_checkpoint_interval=2,
                                             resume_from=os.path.dirname(ck[-1])))
    assert res_resumed["resumed_rounds"] == n  # restored, not re-run from scratch
    a, b = _final_params(full), _final_params(resumed)
    assert a.keys() == b.keys()
    for k in a:
        assert th.equal(a[k], b[k]), f"{k} differs after resume"
    assert res_full["imit_stats"] == res_resumed["imit_stats"]
    return res_full


@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial_resume_is_exact_on_host(tmp_path, command):
    named = ["fast", "demonstrations.fast", "rl.fast", *FAST_ENV]
    # rl.fast: 2 envs x 1 step = 2 env steps per round; 4 rounds, then 4 more after the restart
    _check_resume(tmp_path, command, named, dict(engine="host"), per_round=2, n=4)


def test_full_checkpoints_keep_newest(tmp_path):
    named = ["fast", "demonstrations.fast", "rl.fast", *FAST_ENV]
    root, _ = _adversarial(tmp_path, "keep", "gail", named,
                           dict(engine="host", total_timesteps=2 * 10, full_checkpoint_interval=2, full_checkpoint_keep=2))
    assert [os.path.basename(c) for c in _full_ckpts(root)] == ["ckpt-0000000008", "ckpt-0000000010"]


@pytest.mark.gpu
@pytest.mark.parametrize("command", ["gail", "airl"])
def test_train_adversarial_resume_is_bitwise_on_device(tmp_path, command):
    named = ["demonstrations.fast", "policy_evaluation.fast"]
    updates = dict(environment=dict(gym_id="seals/Hopper-v1", num_vec=8, parallel=False),
                   # ZeroPolicy demos: a RandomPolicy expert samples from an unseeded action space (as the
                   # reference's does), so its demonstrations -- and the run -- differ run to run
                   expert=dict(policy_type="zero", loader_kwargs={}),
                   rl=dict(batch_size=1024, rl_kwargs=dict(batch_size=64, n_epochs=1)), engine="device",
                   algorithm_kwargs=dict(demo_batch_size=256, n_disc_updates_per_round=2), checkpoint_interval=0)
    _check_resume(tmp_path, command, named, updates, per_round=1024, n=4)


def _preference(tmp_path, name, updates):
    from imitation_amd.scripts.train_preference_comparisons import train_preference_comparisons_ex

    root = str(tmp_path / name)
    run = train_preference_comparisons_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV],
                                              config_updates={"logging": {"log_root": root}, "seed": 0, **updates})
    assert run.status == "COMPLETED"
    return root, run.result


def _pref_final(root):
    from imitation_amd.rewards import serialize as reward_serialize

    (rew,) = glob.glob(os.path.join(root, "**", "checkpoints", "final", "reward_net.pt"), recursive=True)
    return {k: v.detach().cpu() for k, v in reward_serialize.load_reward_net(rew, device="cpu").state_dict().items()}


def _check_pref_resume(tmp_path, updates, kill_after):
    import shutil

    full, res_full = _preference(tmp_path, "full", dict(updates, full_checkpoint_interval=1, full_checkpoint_keep=10))
    ck = [c for c in _full_ckpts(full) if c.endswith(f"ckpt-{kill_after:010d}")]
    assert len(ck) == 1
    killed = tmp_path / "killed_run"  # the run "died" after `kill_after` iterations: only that checkpoint exists
    shutil.copytree(ck[0], killed / os.path.basename(ck[0]))
    resumed, res_resumed = _preference(tmp_path, "resumed", dict(updates, resume_from=str(killed)))
    assert res_resumed["resumed_iterations"] == kill_after  # restored, not re-run from scratch
    a, b = _pref_final(full), _pref_final(resumed)
    for k in a:
        assert th.equal(a[k], b[k]), f"{k} differs after resume"
    assert res_full["reward_loss"] == res_resumed["reward_loss"]
    assert res_full["reward_accuracy"] == res_resumed["reward_accuracy"]
    if "imit_stats" in res_full:
        assert res_full["imit_stats"] == res_resumed["imit_stats"]


@pytest.mark.parametrize("kill_after", [1, 2])
def test_train_preference_comparisons_resume_is_exact_on_host(tmp_path, kill_after):
    # 3 iterations + the initial one: iterations 0..3; the agent's trajectories in flight (finished
    # but not sampled, partial episodes) are part of the checkpoint
    _check_pref_resume(tmp_path, dict(engine="host", num_iterations=3, total_timesteps=60, total_comparisons=8),
                       kill_after)


@pytest.mark.gpu
def test_train_preference_comparisons_resume_is_bitwise_on_device(tmp_path):
    updates = dict(environment=dict(gym_id="seals/Hopper-v1", num_vec=8, parallel=False),
                   rl=dict(batch_size=1024, rl_kwargs=dict(batch_size=64, n_epochs=1)), engine="device",
                   total_timesteps=4 * 1024, total_comparisons=16, num_iterations=3, fragment_length=4,
                   reward_trainer_kwargs=dict(epochs=1), checkpoint_interval=0)
    _check_pref_resume(tmp_path, updates, 2)


def _dagger(tmp_path, name, dagger_cfg):
    from imitation_amd.scripts.train_imitation import train_imitation_ex

    root = str(tmp_path / name)
    run = train_imitation_ex.run("dagger", named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                 config_updates={"logging": {"log_root": root}, "seed": 0,
                                                 "bc": {"train_kwargs": {"n_batches": 8}},
                                                 "dagger": dict(total_timesteps=1500, **dagger_cfg)})
    assert run.status == "COMPLETED"
    return root, run.result


def _dagger_policy(root):
    (p,) = glob.glob(os.path.join(root, "**", "scratch", "policy-latest.pt"), recursive=True)
    out = {}

    def flat(prefix, x):
        if isinstance(x, th.Tensor):
            out[prefix] = x.clone()
        elif isinstance(x, dict):
            for k, v in x.items():
                flat(f"{prefix}.{k}", v)

    flat("policy", th.load(p, map_location="cpu", weights_only=True))
    return out


def test_train_imitation_dagger_resume_is_exact_on_host(tmp_path):
    """3 DAgger rounds (>= 500 steps each) with a full checkpoint per round; a run that "died"
    after round 1 resumes from it (reusing its scratch dir's round files) and ends where the
    uninterrupted run did."""
    import shutil

    full, res_full = _dagger(tmp_path, "full", dict(full_checkpoint_interval=1, full_checkpoint_keep=10))
    want = _dagger_policy(full)
    (ck,) = [c for c in _full_ckpts(full) if c.endswith("ckpt-0000000001")]
    killed = tmp_path / "killed_run"
    shutil.copytree(ck, killed / os.path.basename(ck))
    resumed, res_resumed = _dagger(tmp_path, "resumed", dict(resume_from=str(killed)))
    assert res_resumed["resumed_round"] == 1
    got = _dagger_policy(full)  # the resumed run trains on in the original run's scratch dir
    assert want and want.keys() == got.keys()
    for k in want:
        assert th.equal(want[k], got[k]), f"{k} differs after resume"
    assert res_full["imit_stats"] == res_resumed["imit_stats"]


def test_every_training_cli_runs_under_the_hang_watchdog(tmp_path, monkeypatch):
    """train_imitation (bc / dagger / sqil), train_rl and eval_policy run
    inside ``cli_watchdog`` (train_adversarial / train_preference_comparisons already did)."""
    from imitation_amd.utils import watchdog

    used = []
    real = watchdog.cli_watchdog

    def spy(name):
        used.append(name)
        return real(name)

    monkeypatch.setattr(watchdog, "cli_watchdog", spy)
    from imitation_amd.scripts.eval_policy import eval_policy_ex
    from imitation_amd.scripts.train_imitation import train_imitation_ex
    from imitation_amd.scripts.train_rl import train_rl_ex

    upd = {"logging": {"log_root": str(tmp_path / "o")}}
    for cmd in ("bc", "dagger", "sqil"):
        assert train_imitation_ex.run(cmd, named_configs=["fast", "demonstrations.fast", *FAST_ENV],
                                      config_updates=upd).status == "COMPLETED"
    assert train_rl_ex.run(named_configs=["fast", "rl.fast", *FAST_ENV], config_updates=upd).status == "COMPLETED"
    assert eval_policy_ex.run(named_configs=["fast"], config_updates=upd).status == "COMPLETED"
    assert used.count("train_imitation") == 3 and "train_rl" in used and "eval_policy" in used
