"""Benchmark-run helpers (reference: benchmarking/util.py, sacred_output_to_csv.py)
and the command generator behind ``run_all_benchmarks.sh``."""

from __future__ import annotations

import argparse
import csv
import json
import pathlib
from typing import Dict, List, Sequence

from imitation_amd.util.sacred_file_parsing import find_sacred_runs

ALGOS = {"bc": "train_imitation", "dagger": "train_imitation", "airl": "train_adversarial", "gail": "train_adversarial"}
ENVS = ("seals_ant", "seals_half_cheetah", "seals_hopper", "seals_swimmer", "seals_walker")


def benchmark_commands(seeds: Sequence[int] = tuple(range(1, 11)), algos=tuple(ALGOS), envs=ENVS,
                       extra: str = "") -> List[str]:
    """The 4 algos x 5 envs x 10 seeds benchmark commands (tuned named configs)."""
    return [f"python -m imitation_amd.scripts.{ALGOS[a]} {a} with {a}_{e} seed={s}{(' ' + extra) if extra else ''}"
            for a in algos for e in envs for s in seeds]


def filter_config_files(files: List[str], /) -> List[pathlib.Path]:
    """Keep the last ``config.json`` per experiment (``<exp>/<info>/sacred/<id>/config.json``)."""
    experiments: Dict[pathlib.Path, List[pathlib.Path]] = {}
    for f in map(pathlib.Path, files):
        if f.name == "config.json":
            experiments.setdefault(f.parents[3], []).append(f)
    return [sorted(v, key=lambda p: p.parents[1])[-1] for v in experiments.values()]


def remove_empty_dicts(d: dict) -> None:
    for k, v in list(d.items()):
        if isinstance(v, dict):
            remove_empty_dicts(v)
            if not v:
                d.pop(k)


def clean_config_file(file: pathlib.Path, write_path: pathlib.Path, /) -> None:
    """Strip seeds / paths so only hyper-parameters remain (tuned-HP JSON format)."""
    config = json.loads(pathlib.Path(file).read_text())
    for k in ("agent_path", "seed"):
        config.pop(k, None)
    config.get("demonstrations", {}).pop("path", None)
    config.get("expert", {}).get("loader_kwargs", {}).pop("path", None)
    config.get("logging", {}).pop("log_dir", None)
    config.get("logging", {}).pop("log_root", None)
    remove_empty_dicts(config)
    pathlib.Path(write_path).write_text(json.dumps(config, indent=2, sort_keys=True))


def sacred_output_to_csv(path: pathlib.Path, out: pathlib.Path) -> int:
    rows = []
    for conf, run in find_sacred_runs(path, only_completed_runs=True):
        res = run.get("result") or {}
        rows.append({"algo": run["command"], "env": conf["environment"]["gym_id"], "seed": conf.get("seed"),
                     "return_mean": (res.get("imit_stats") or {}).get("monitor_return_mean"),
                     "expert_return_mean": (res.get("expert_stats") or {}).get("monitor_return_mean")})
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["algo", "env", "seed", "return_mean", "expert_return_mean"])
        w.writeheader()
        w.writerows(rows)
    return len(rows)


def main(argv=None):
    p = argparse.ArgumentParser(description="benchmark helpers")
    sub = p.add_subparsers(dest="cmd", required=True)
    g = sub.add_parser("commands")
    g.add_argument("--extra", default="")
    c = sub.add_parser("csv")
    c.add_argument("path", type=pathlib.Path)
    c.add_argument("out", type=pathlib.Path)
    a = p.parse_args(argv)
    if a.cmd == "commands":
        print("\n".join(benchmark_commands(extra=a.extra)))
    else:
        print(sacred_output_to_csv(a.path, a.out), "rows")


if __name__ == "__main__":  # pragma: no cover
    main()
