"""Markdown summary of a benchmark directory (reference: benchmarking/sacred_output_to_markdown_summary.py).

Scores are normalised as ``(score - random) / (expert - random)``; the random-agent score
comes from rolling out a uniform-random policy in our env (the reference downloads
``HumanCompatibleAI/random-<env>`` rollouts, unavailable offline).
"""

from __future__ import annotations

import argparse
import pathlib
from collections import Counter
from functools import lru_cache
from typing import Generator

import numpy as np

from imitation_amd.benchmarking import stats
from imitation_amd.util.sacred_file_parsing import find_sacred_runs, group_runs_by_algo_and_env


@lru_cache(maxsize=None)
def get_random_agent_score(env: str, n_episodes: int = 20) -> float:
    from imitation_amd.data import rollout, wrappers
    from imitation_amd.policies.base import RandomPolicy
    from imitation_amd.util import util

    rng = np.random.default_rng(0)
    venv = util.make_vec_env(env, n_envs=4, rng=rng, post_wrappers=[lambda e, _: wrappers.RolloutInfoWrapper(e)])
    trajs = rollout.rollout(RandomPolicy(venv.observation_space, venv.action_space), venv,
                            rollout.make_min_episodes(n_episodes), rng=rng)
    return float(rollout.rollout_stats(trajs)["monitor_return_mean"])


def _score(run, key="imit_stats"):
    st = run["result"][key]
    return st.get("monitor_return_mean", st["return_mean"])


def print_markdown_summary(path: pathlib.Path, random_score_fn=get_random_agent_score) -> Generator[str, None, None]:
    if not path.exists():
        raise NotADirectoryError(f"Path {path} does not exist.")
    yield "# Benchmark Summary"
    yield ""
    yield f"This is a summary of the runs in `{path}`."
    runs = group_runs_by_algo_and_env(path)
    algos = sorted(runs)
    status_counts = Counter(run["status"] for _, run in find_sacred_runs(path))
    statuses = sorted(status_counts)
    if statuses != ["COMPLETED"]:
        yield "## Run status"
        yield "Status | Count"
        yield "--- | ---"
        for s in statuses:
            yield f"{s} | {status_counts[s]}"
        yield ""
    yield "## Scores"
    yield ""
    yield "Normalized score: `(score - random_score) / (expert_score - random_score)`."
    for algo in algos:
        yield f"### {algo.upper()}"
        yield "Environment | Score (mean/std)| Normalized Score (mean/std) | N"
        yield " --- | --- | --- | --- "
        acc = []
        for env in sorted(runs[algo]):
            done = [r for r in runs[algo][env] if r.get("status") == "COMPLETED"]
            scores = [_score(r) for r in done]
            experts = [_score(r, "expert_stats") for r in done]
            rnd = random_score_fn(env)
            norm = [(s - rnd) / (e - rnd) for s, e in zip(scores, experts)]
            acc.append(norm)
            yield f"{env} | {np.mean(scores):.3f} / {np.std(scores):.3f} | {np.mean(norm):.3f} / {np.std(norm):.3f} | {len(scores)}"
        n = min(len(a) for a in acc)
        mat = np.asarray([a[:n] for a in acc]).T
        point, cis = stats.get_interval_estimates({"normalized_score": mat},
                                                  lambda x: np.array([stats.aggregate_mean(x), stats.aggregate_iqm(x)]),
                                                  reps=1000)
        p, c = point["normalized_score"], cis["normalized_score"]
        yield ""
        yield "#### Aggregate Normalized scores"
        yield "Metric | Value | 95% CI"
        yield " --- | --- | --- "
        yield f"Mean | {p[0]:.3f} | [{c[0][0]:.3f}, {c[1][0]:.3f}]"
        yield f"IQM | {p[1]:.3f} | [{c[0][1]:.3f}, {c[1][1]:.3f}]"
        yield ""


def main(argv=None):
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument("path", type=pathlib.Path)
    parser.add_argument("--output", type=pathlib.Path, default="summary.md")
    args = parser.parse_args(argv)
    with open(args.output, "w") as fh:
        for line in print_markdown_summary(args.path):
            fh.write(line + "\n")


if __name__ == "__main__":  # pragma: no cover
    main()
