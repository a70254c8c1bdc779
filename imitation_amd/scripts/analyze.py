"""Tabulate finished runs and gather TensorBoard dirs (reference: src/imitation/scripts/analyze.py)."""

from __future__ import annotations

import itertools
import json
import logging
import pathlib
import tempfile
import warnings
from typing import Any, Callable, Iterable, List, Mapping, Optional, Sequence, Set

import pandas as pd

from imitation_amd.scripts.config.analyze import analysis_ex
from imitation_amd.scripts.config_engine import FileStorageObserver
from imitation_amd.util import sacred as sacred_util
from imitation_amd.util import util
from imitation_amd.util.sacred import dict_get_nested as get


@analysis_ex.capture
def _gather_sacred_dicts(source_dirs: Sequence[str], run_name: Optional[str], env_name: Optional[str],
                         skip_failed_runs: bool) -> List[sacred_util.SacredDicts]:
    dirs = itertools.chain.from_iterable(sacred_util.filter_subdirs(util.parse_path(d)) for d in source_dirs)
    sds = []
    for d in dirs:
        try:
            sds.append(sacred_util.SacredDicts.load_from_dir(d))
        except json.JSONDecodeError:
            warnings.warn(f"Invalid JSON file in {d}", RuntimeWarning)
    out: Iterable = sds
    if run_name is not None:
        out = [sd for sd in out if get(sd.run, "experiment.name") == run_name]
    if env_name is not None:
        out = [sd for sd in out if get(sd.config, "environment.gym_id") == env_name]
    if skip_failed_runs:
        out = [sd for sd in out if get(sd.run, "status") != "FAILED"]
    return list(out)


@analysis_ex.command
def gather_tb_directories() -> dict:
    """Symlink every run's TensorBoard dirs into one fresh directory under /tmp/analysis_tb."""
    root = pathlib.Path("/tmp/analysis_tb")
    root.mkdir(exist_ok=True)
    tmp_dir = pathlib.Path(tempfile.mkdtemp(dir=root))
    count = 0
    for sd in _gather_sacred_dicts():
        # the run's own log dir (recorded in its config) when it exists, else the directory
        # above the observer's run dir (the reference layout: <log_dir>/sacred/<id>)
        log_dir = (sd.config.get("logging") or {}).get("log_dir")
        run_dir = pathlib.Path(log_dir) if log_dir and pathlib.Path(log_dir).is_dir() else sd.sacred_dir.parent.parent
        for basename in ("log", "rl", "tb", "sb_tb"):
            src = tuple(sacred_util.filter_subdirs(run_dir, lambda p, b=basename: p.name == b))
            if src:
                assert len(src) == 1, "expect at most one TB dir of each type"
                links = tmp_dir / basename
                links.mkdir(exist_ok=True)
                (links / run_dir.name).symlink_to(src[0])
                count += 1
    logging.info(f"Symlinked {count} TensorBoard dirs to {tmp_dir}.")
    return {"n_tb_dirs": count, "gather_dir": str(tmp_dir)}


def _get_exp_command(sd) -> str:
    return str(sd.run.get("command"))


def _get_algo_name(sd) -> str:
    return {"gail": "GAIL", "airl": "AIRL", "bc": "BC", "train_bc": "BC", "dagger": "DAgger", "train_dagger": "DAgger",
            "sqil": "SQIL"}.get(_get_exp_command(sd), f"??exp_command={_get_exp_command(sd)}")


def _make_return_summary(stats: dict, prefix: str = "") -> str:
    return "{:3g} ± {:3g} (n={})".format(stats[f"{prefix}return_mean"], stats[f"{prefix}return_std"], stats["n_traj"])


def _return_summaries(sd) -> dict:
    imit = get(sd.run, "result.imit_stats")
    expert = get(sd.run, "result.expert_stats")
    ratio = None
    if imit is not None and expert is not None and "monitor_return_mean" in imit:
        ratio = imit["monitor_return_mean"] / expert["return_mean"]
    return dict(expert_return_summary=_make_return_summary(expert) if expert else None,
                imit_return_summary=(_make_return_summary(imit, "monitor_") if imit and "monitor_return_mean" in imit
                                     else (_make_return_summary(imit) if imit else None)),
                imit_expert_ratio=ratio)


table_entry_fns: Mapping[str, Callable[[Any], Any]] = {
    "status": lambda sd: get(sd.run, "status"),
    "exp_command": _get_exp_command,
    "algo": _get_algo_name,
    "env_name": lambda sd: get(sd.config, "environment.gym_id"),
    "n_expert_demos": lambda sd: get(sd.config, "demonstrations.n_expert_demos"),
    "run_name": lambda sd: get(sd.run, "experiment.name"),
    "expert_return_summary": lambda sd: _return_summaries(sd)["expert_return_summary"],
    "imit_return_summary": lambda sd: _return_summaries(sd)["imit_return_summary"],
    "imit_expert_ratio": lambda sd: _return_summaries(sd)["imit_expert_ratio"],
}
_V0: Set[str] = {"algo", "env_name", "expert_return_summary", "imit_return_summary"}
table_verbosity_mapping: List[Set[str]] = [_V0, _V0 | {"n_expert_demos"},
                                           _V0 | {"n_expert_demos", "status", "imit_expert_ratio", "exp_command", "run_name"}]


@analysis_ex.command
def analyze_imitation(csv_output_path: Optional[str], tex_output_path: Optional[str], print_table: bool,
                      table_verbosity: int) -> pd.DataFrame:
    """One row per run: algorithm, env, expert and imitation return summaries (verbosity 0-3)."""
    keys = table_verbosity_mapping[min(table_verbosity, 2)]
    fns = {k: v for k, v in table_entry_fns.items() if k in keys}
    rows = []
    for sd in _gather_sacred_dicts():
        row = pd.json_normalize(sd.config) if table_verbosity == 3 else pd.DataFrame(index=[0])
        for col, fn in fns.items():
            row[col] = fn(sd)
        rows.append(row)
    table = pd.concat(rows) if rows else pd.DataFrame()
    if len(table) > 0:
        table = table.sort_values(by=["algo", "env_name"])
    if csv_output_path is not None:
        table.to_csv(csv_output_path, index=False)
        print(f"Wrote CSV file to {csv_output_path}")
    if tex_output_path is not None:
        with open(tex_output_path, "w") as f:
            f.write(table.to_latex(index=False))
        print(f"Wrote TeX file to {tex_output_path}")
    if print_table:
        print(table.to_string(index=False))
    return table


def main_console(argv=None):
    analysis_ex.observers.append(FileStorageObserver(pathlib.Path.cwd() / "output" / "sacred" / "analyze"))
    return analysis_ex.run_commandline(argv)


if __name__ == "__main__":  # pragma: no cover
    main_console()
