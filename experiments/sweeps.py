"""Seed x env sweeps of the reference's legacy experiment scripts, as one Python launcher.

Reference: ``experiments/{bc,dagger,transfer_learn}_benchmark.sh``,
``rollouts_from_policies.sh`` (+ ``rollouts_from_policies_config.csv``) and
``convert_traj.py`` -- bash + GNU ``parallel`` driving Sacred CLIs. Here every trial goes
through :func:`imitation_amd.scripts.parallel.run_trials` (a spawn process pool; one trial
per GPU slot on a GPU node, ``HIP_VISIBLE_DEVICES`` set per slot), and the summary of
each sweep is printed / returned:

    python experiments/sweeps.py bc [--fast] [--paper] [--seeds 0 1 2]
    python experiments/sweeps.py dagger [--fast]
    python experiments/sweeps.py transfer_learn --algo airl [--fast]   # adversarial -> RL on the learned reward
    python experiments/sweeps.py rollouts_from_policies [--fast]       # expert rollouts per env config
    python experiments/sweeps.py convert_traj SRC DST.npz               # -> openai/baselines GAIL npz
"""

from __future__ import annotations

import argparse
import csv
import pathlib
import sys
from typing import Any, Dict, List, Sequence

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))

from imitation_amd.scripts.parallel import run_trials  # noqa: E402
from imitation_amd.util.util import make_unique_timestamp  # noqa: E402

FAST = ["environment.fast", "demonstrations.fast", "policy_evaluation.fast", "fast"]
HERE = pathlib.Path(__file__).resolve().parent


def _trials(command: str, envs: Sequence[str], seeds: Sequence[int], extra: Sequence[str], log_root: str,
            updates: Dict[str, Any] = None) -> List[Dict[str, Any]]:
    out = []
    for env in envs:
        for s in seeds:
            upd = {"seed": s, "logging": {"log_root": log_root}, **(updates or {})}
            out.append({"command_name": command, "named_configs": [env, *extra], "config_updates": upd})
    return out


def _report(trials, recs) -> List[Dict[str, Any]]:
    rows = []
    for t, r in zip(trials, recs):
        rows.append(dict(env=t["named_configs"][0], seed=t["config_updates"]["seed"], status=r["status"],
                         metric=r["metric"]))
        print(f"{rows[-1]['env']:28s} seed={rows[-1]['seed']:<3d} {r['status']:10s} {r['metric']}")
    return rows


def sweep_bc(a) -> List[Dict[str, Any]]:
    """``bc_benchmark.sh``: BC experts on seals CartPole (``--paper``: + MountainCar, HalfCheetah)."""
    envs = ["seals_cartpole", "seals_mountain_car", "seals_half_cheetah"] if a.paper else ["seals_cartpole"]
    seeds, extra = ([0], FAST) if a.fast else (a.seeds, [])
    trials = _trials("bc", envs, seeds, extra, a.log_root)
    return _report(trials, run_trials("train_imitation", trials, f"{a.log_root}/sacred", "bc_benchmark", {"gpu": a.gpus}))


def sweep_dagger(a) -> List[Dict[str, Any]]:
    """``dagger_benchmark.sh``: DAgger on the same env list as the BC sweep."""
    envs = ["seals_cartpole", "seals_mountain_car", "seals_half_cheetah"] if a.paper else ["seals_cartpole"]
    seeds, extra = ([0], FAST) if a.fast else (a.seeds, [])
    trials = _trials("dagger", envs, seeds, extra, a.log_root)
    return _report(trials, run_trials("train_imitation", trials, f"{a.log_root}/sacred", "dagger_benchmark",
                                      {"gpu": a.gpus}))


def sweep_transfer_learn(a) -> List[Dict[str, Any]]:
    """``transfer_learn_benchmark.sh``: train GAIL/AIRL per imitation-benchmark row, then train
    RL from scratch on each learned ``reward_test.pt`` (RewardNet_unshaped)."""
    rows = list(csv.DictReader(open(HERE / "imit_benchmark_config.csv")))
    seeds = [0] if a.fast else a.seeds
    if a.fast:
        rows = rows[:1]
    adv_extra = FAST + ["rl.fast"] if a.fast else []
    rl_extra = ["rl.fast", "environment.fast", "policy_evaluation.fast", "fast"] if a.fast else []
    stage1 = []
    for r in rows:  # one log root per (env, seed): stage 2 finds that trial's own reward
        for s in seeds:
            root = f"{a.log_root}/adversarial/{r['env_config_name']}_{s}"
            stage1 += _trials(a.algo, [r["env_config_name"]], [s], adv_extra, root)
    recs1 = run_trials("train_adversarial", stage1, f"{a.log_root}/adversarial/sacred", f"transfer_{a.algo}", {"gpu": a.gpus})
    _report(stage1, recs1)
    stage2 = []
    for t, r in zip(stage1, recs1):
        root = pathlib.Path(t["config_updates"]["logging"]["log_root"])
        reward = next(root.rglob("checkpoints/final/reward_test.pt"), None) if r["status"] == "COMPLETED" else None
        if reward is None:
            continue
        upd = {"seed": t["config_updates"]["seed"], "logging": {"log_root": f"{a.log_root}/rl"},
               "reward_type": "RewardNet_unshaped", "reward_path": str(reward)}
        stage2.append({"command_name": None, "named_configs": [t["named_configs"][0], *rl_extra], "config_updates": upd})
    recs2 = run_trials("train_rl", stage2, f"{a.log_root}/rl/sacred", "transfer_rl", {"gpu": a.gpus}) if stage2 else []
    return _report(stage2, recs2)


def sweep_rollouts_from_policies(a) -> List[Dict[str, Any]]:
    """``rollouts_from_policies.sh``: roll out the hub expert of each config row and save the
    trajectories (``eval_policy`` with ``rollout_save_path``)."""
    rows = list(csv.DictReader(open(HERE / "rollouts_from_policies_config.csv")))
    if a.fast:
        rows = rows[:1]
    trials = []
    for r in rows:
        n = 1 if a.fast else int(r["n_demonstrations"])
        upd = {"seed": 0, "logging": {"log_root": a.log_root}, "eval_n_episodes": n,
               "rollout_save_path": f"{a.log_root}/{r['env_config_name']}/rollouts.npz"}
        if a.fast:
            upd["expert"] = {"policy_type": "random", "loader_kwargs": {}}
        trials.append({"command_name": None, "named_configs": [r["env_config_name"]] + (["fast"] if a.fast else []),
                       "config_updates": upd})
    return _report(trials, run_trials("eval_policy", trials, f"{a.log_root}/sacred", "rollouts_from_policies", {"gpu": a.gpus}))


def convert_trajs_to_baselines(trajs) -> Dict[str, np.ndarray]:
    """openai/baselines GAIL dict (``acs``, ``rews``, ``obs``, ``ep_rets``) of rewarded trajectories."""
    from imitation_amd.data import rollout

    flat = rollout.flatten_trajectories_with_rew(trajs)
    return dict(acs=flat.acts, rews=flat.rews, obs=flat.obs, ep_rets=np.array([np.sum(t.rews) for t in trajs]))


def convert_traj(a) -> pathlib.Path:
    """``convert_traj.py``: imitation trajectories (HF dir / npz) -> baselines GAIL npz."""
    from imitation_amd.data import serialize

    src, dst = pathlib.Path(a.src), pathlib.Path(a.dst)
    out = convert_trajs_to_baselines(serialize.load_with_rewards(src))
    dst.parent.mkdir(parents=True, exist_ok=True)
    with open(dst, "wb") as f:
        np.savez_compressed(f, **out)
    print(f"Dumped rollouts to {dst}")
    return dst


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    for name in ("bc", "dagger", "transfer_learn", "rollouts_from_policies"):
        s = sub.add_parser(name)
        s.add_argument("--fast", action="store_true")
        s.add_argument("--paper", action="store_true")
        s.add_argument("--seeds", nargs="+", type=int, default=[0, 1, 2])
        s.add_argument("--algo", default="gail", choices=["gail", "airl"])
        s.add_argument("--gpus", type=int, default=1, help="GPUs per trial (trials spread over the node's GPUs)")
        s.add_argument("--log-root", default=f"output/{name}/{make_unique_timestamp()}")
    c = sub.add_parser("convert_traj")
    c.add_argument("src")
    c.add_argument("dst")
    a = p.parse_args(argv)
    fn = {"bc": sweep_bc, "dagger": sweep_dagger, "transfer_learn": sweep_transfer_learn,
          "rollouts_from_policies": sweep_rollouts_from_policies, "convert_traj": convert_traj}[a.cmd]
    return fn(a)


if __name__ == "__main__":
    main()
