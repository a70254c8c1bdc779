"""Probability that one algorithm's runs beat a baseline's (reference:
benchmarking/compute_probability_of_improvement.py)."""

from __future__ import annotations

import argparse
import dataclasses
import pathlib
import warnings
from typing import Dict, List, Optional

import numpy as np

from imitation_amd.benchmarking import stats
from imitation_amd.util.sacred_file_parsing import SacredRun, group_runs_by_algo_and_env


def make_score_matrix_from_runs_by_env(runs_by_env: Dict[str, List[SacredRun]], envs: Optional[List[str]] = None) -> np.ndarray:
    envs = list(runs_by_env) if envs is None else envs
    counts = {e: len(runs_by_env[e]) for e in envs}
    n = min(counts.values())
    if len(set(counts.values())) > 1:
        warnings.warn(f"The runs for the environments have different sample counts {counts}; truncating to {n}.")
    return np.asarray([[r["result"]["imit_stats"]["monitor_return_mean"] for r in runs_by_env[e][:n]] for e in envs]).T


@dataclasses.dataclass
class ProbabilityOfImprovementResult:
    probability_of_improvement: float
    confidence_interval: np.ndarray
    samples_per_env: int
    baseline_samples_per_env: int


def compute_probability_of_improvement(runs_by_env, baseline_runs_by_env, reps: int) -> ProbabilityOfImprovementResult:
    envs = sorted(set(runs_by_env) & set(baseline_runs_by_env))
    x = make_score_matrix_from_runs_by_env(runs_by_env, envs)
    y = make_score_matrix_from_runs_by_env(baseline_runs_by_env, envs)
    point, cis = stats.get_interval_estimates({"baseline_vs_new": (x, y)}, stats.probability_of_improvement, reps=reps)
    return ProbabilityOfImprovementResult(float(point["baseline_vs_new"][0]), np.squeeze(cis["baseline_vs_new"]),
                                          x.shape[0], y.shape[0])


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("runs_dir", type=pathlib.Path)
    p.add_argument("baseline_runs_dir", nargs="?", default=None, type=pathlib.Path)
    p.add_argument("--algo", type=str)
    p.add_argument("--baseline-algo", type=str)
    p.add_argument("--bootstrap-reps", type=int, default=2000)
    a = p.parse_args(argv)
    base_dir = a.baseline_runs_dir or a.runs_dir
    runs = group_runs_by_algo_and_env(a.runs_dir, only_completed_runs=True)
    base = group_runs_by_algo_and_env(base_dir, only_completed_runs=True)
    algo = a.algo or (list(runs)[0] if len(runs) == 1 else None)
    balgo = a.baseline_algo or (list(base)[0] if len(base) == 1 else algo)
    if algo is None or balgo is None:
        raise ValueError("Several algorithms found; specify --algo / --baseline-algo")
    res = compute_probability_of_improvement(runs[algo], base[balgo], a.bootstrap_reps)
    print(f"P({algo} > {balgo}) = {res.probability_of_improvement:.3f} "
          f"[{res.confidence_interval[0]:.3f}, {res.confidence_interval[1]:.3f}] "
          f"(samples/env {res.samples_per_env} vs {res.baseline_samples_per_env})")
    return res


if __name__ == "__main__":  # pragma: no cover
    main()
