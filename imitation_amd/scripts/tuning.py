"""Two-phase hyper-parameter tuning (reference: src/imitation/scripts/tuning.py):
(1) ``parallel`` search over ``parallel_run_config.search_space`` (TPE, ``tune.TPESearch``:
the reference's OptunaSearch; each sample repeated ``repeat`` times with fresh seeds), (2) re-evaluation of the best
configuration (highest mean return over its repeats) on ``num_eval_seeds`` new seeds.
"""

from __future__ import annotations

import copy
import json
import pathlib
from typing import Any, Dict, List

import numpy as np

from imitation_amd.scripts import tune
from imitation_amd.scripts.parallel import parallel_ex
from imitation_amd.scripts.config.tuning import tuning_ex
from imitation_amd.scripts.config_engine import FileStorageObserver


def find_best_trial(records: List[Dict[str, Any]], print_return: bool = False) -> Dict[str, Any]:
    """Group trials by sampled config (ignoring seeds); pick the best mean metric."""
    groups: Dict[str, List[Dict[str, Any]]] = {}
    for r in records:
        key = json.dumps(r["sample"], sort_keys=True, default=str)
        groups.setdefault(key, []).append(r)
    best_key = max(groups, key=lambda k: np.nanmean([r["metric"] for r in groups[k]]))
    best = groups[best_key]
    if print_return:
        rets = np.array([r["metric"] for r in best])
        print("All returns:", rets)
        print("Mean return:", np.nanmean(rets))
        print("Std return:", np.nanstd(rets))
        print("Total seeds:", len(rets))
    return best[0]


def evaluate_trial(trial: Dict[str, Any], num_eval_seeds: int, run_name: str, parallel_run_config: Dict[str, Any],
                   resources_per_trial: Dict[str, int]) -> List[Dict[str, Any]]:
    space = copy.deepcopy(trial["sample"])
    space.setdefault("config_updates", {})
    space["config_updates"]["seed"] = tune.grid_search(list(range(100, 100 + num_eval_seeds)))
    cfg = copy.deepcopy(parallel_run_config)
    cfg.update(run_name=run_name, num_samples=1, search_space=space, resources_per_trial=resources_per_trial, repeat=1,
               experiment_checkpoint_path="")
    # every evaluation seed exactly once: the grid expansion, not the model-based search
    cfg["tune_run_kwargs"] = dict(cfg.get("tune_run_kwargs") or {}, search_alg="random")
    run = parallel_ex.run(config_updates=cfg)
    rets = np.array([r["metric"] for r in run.result])
    print("Evaluation returns:", rets, "mean", np.nanmean(rets), "std", np.nanstd(rets))
    return run.result


@tuning_ex.main
def tune_main(parallel_run_config, eval_best_trial_resource_multiplier: int = 1, num_eval_seeds: int = 5):
    cfg = copy.deepcopy(parallel_run_config)
    # model-based search, as the reference's tuning (OptunaSearch, scripts/tuning.py:43-46)
    cfg.setdefault("tune_run_kwargs", {}).setdefault("search_alg", "tpe")
    run = parallel_ex.run(config_updates=cfg)
    records = run.result
    if not records:
        raise ValueError("No trials found.")
    best = find_best_trial(records, print_return=True)
    out = {"best_sample": best["sample"], "best_metric": best["metric"]}
    if num_eval_seeds > 0:
        res = dict(cfg.get("resources_per_trial", {}))
        if "cpu" in res:
            res["cpu"] *= eval_best_trial_resource_multiplier
        evals = evaluate_trial(best, num_eval_seeds, f"{cfg['run_name']}_best_hp_eval", cfg, res)
        out["eval_metrics"] = [r["metric"] for r in evals]
    return out


def main_console(argv=None):
    tuning_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "tuning"))
    return tuning_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
