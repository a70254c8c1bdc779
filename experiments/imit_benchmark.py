"""Imitation benchmark sweep over a CSV of (env_config_name, gen_batch_size, n_expert_demos)
(reference: experiments/imit_benchmark.sh, which drives GNU parallel). Trials run through
``scripts.parallel.run_trials`` (local process pool; on a GPU node one trial per GPU).

    python experiments/imit_benchmark.py --algo gail [--fast] [--seeds 0 1 2 3 4]
"""

from __future__ import annotations

import argparse
import csv
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))

from imitation_amd.scripts.parallel import run_trials  # noqa: E402
from imitation_amd.util.util import make_unique_timestamp  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--algo", default="gail", choices=["gail", "airl"])
    p.add_argument("--csv", default=str(pathlib.Path(__file__).with_name("imit_benchmark_config.csv")))
    p.add_argument("--seeds", nargs="+", type=int, default=[0, 1, 2, 3, 4])
    p.add_argument("--fast", action="store_true")
    p.add_argument("--log-root", default=f"output/imit_benchmark/{make_unique_timestamp()}")
    p.add_argument("--gpus-per-trial", type=int, default=1)
    a = p.parse_args(argv)
    rows = list(csv.DictReader(open(a.csv)))
    base = []
    seeds = a.seeds
    if a.fast:
        rows, seeds = rows[:1], [0]
        base = ["environment.fast", "demonstrations.fast", "rl.fast", "policy_evaluation.fast", "fast"]
    trials = []
    for r in rows:
        for s in seeds:
            upd = {"seed": s, "demonstrations": {"n_expert_demos": int(r["n_expert_demos"])},
                   "logging": {"log_root": a.log_root}}
            if not a.fast:
                upd["rl"] = {"batch_size": int(r["gen_batch_size"])}
            trials.append({"command_name": a.algo, "named_configs": [r["env_config_name"], *base], "config_updates": upd})
    recs = run_trials("train_adversarial", trials, f"{a.log_root}/sacred", f"imit_benchmark_{a.algo}",
                      {"gpu": a.gpus_per_trial})
    for t, r in zip(trials, recs):
        print(t["named_configs"][0], t["config_updates"]["seed"], r["status"], r["metric"])
    return recs


if __name__ == "__main__":
    main()
