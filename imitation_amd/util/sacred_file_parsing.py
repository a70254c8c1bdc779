"""Parse experiment-run directories (reference: src/imitation/util/sacred_file_parsing.py)."""

from __future__ import annotations

import json
import pathlib
import warnings
from collections import defaultdict
from typing import Any, Dict, Generator, List, Tuple

SacredRun = Dict[str, Any]
SacredConfAndRun = Tuple[Dict[str, Any], SacredRun]
GroupedRuns = Dict[str, Dict[str, List[SacredRun]]]


def find_sacred_runs(run_path: pathlib.Path, only_completed_runs: bool = False) -> Generator[SacredConfAndRun, None, None]:
    """Yield ``(config, run)`` for every ``config.json`` + ``run.json`` pair below ``run_path``."""
    for config_path in pathlib.Path(run_path).rglob("config.json"):
        run_file = config_path.parent / "run.json"
        if not run_file.exists():
            warnings.warn(f"Run {config_path.parent} has no run.json")
            continue
        run = json.loads(run_file.read_text())
        if only_completed_runs and run.get("status") != "COMPLETED":
            continue
        yield json.loads(config_path.read_text()), run


def group_runs_by_algo_and_env(path: pathlib.Path, only_completed_runs: bool = False) -> GroupedRuns:
    """``runs[algo][env]`` where algo is the run's command and env ``environment.gym_id``."""
    grouped: GroupedRuns = defaultdict(lambda: defaultdict(list))
    for conf, run in find_sacred_runs(path, only_completed_runs):
        grouped[run["command"]][conf["environment"]["gym_id"]].append(run)
    return grouped
