"""Helpers for experiment-run directories written by the config engine's
FileStorageObserver (reference: src/imitation/util/sacred.py; same on-disk layout as Sacred)."""

from __future__ import annotations

import json
import os
import pathlib
import warnings
from typing import Any, Callable, NamedTuple, Optional, Sequence

from imitation_amd.data import types
from imitation_amd.util import util


class SacredDicts(NamedTuple):
    """Each dict ``foo`` is loaded from ``f"{sacred_dir}/foo.json"``."""

    sacred_dir: pathlib.Path
    config: dict
    run: dict

    @classmethod
    def load_from_dir(cls, sacred_dir: pathlib.Path) -> "SacredDicts":
        sacred_dir = pathlib.Path(sacred_dir)
        return cls(sacred_dir=sacred_dir, config=json.loads((sacred_dir / "config.json").read_text()),
                   run=json.loads((sacred_dir / "run.json").read_text()))


def dir_contains_sacred_jsons(dir_path: pathlib.Path) -> bool:
    return (dir_path / "run.json").is_file() and (dir_path / "config.json").is_file()


def filter_subdirs(root_dir: pathlib.Path, filter_fn: Callable[[pathlib.Path], bool] = dir_contains_sacred_jsons, *,
                   nested_ok: bool = False) -> Sequence[pathlib.Path]:
    """All subdirectories (symlinks not followed) accepted by ``filter_fn``."""
    found = {pathlib.Path(root) for root, _, _ in os.walk(root_dir, followlinks=False) if filter_fn(pathlib.Path(root))}
    if not nested_ok:
        for a in found:
            for b in found:
                if a != b and b in a.parents:
                    raise ValueError(f"Found nested directories: {a} and {b}")
    return list(found)


def get_sacred_dir_from_run(run) -> Optional[pathlib.Path]:
    from imitation_amd.scripts.config_engine import FileStorageObserver

    for obs in getattr(run, "observers", []):
        if isinstance(obs, FileStorageObserver) and hasattr(obs, "dir"):
            return util.parse_path(obs.dir)
    return None


def build_sacred_symlink(log_dir: types.AnyPath, run) -> None:
    """Symlink ``{log_dir}/sacred`` -> the run's observer directory (relative link)."""
    log_dir = util.parse_path(log_dir)
    sacred_dir = get_sacred_dir_from_run(run)
    if sacred_dir is None:
        warnings.warn(RuntimeWarning("Couldn't find sacred directory."))
        return
    link = log_dir / "sacred"
    if link.is_symlink():
        link.unlink()
    link.symlink_to(pathlib.Path(os.path.relpath(sacred_dir, start=log_dir)), target_is_directory=True)


def dict_get_nested(d: dict, nested_key: str, *, sep: str = ".", default: Any = None) -> Any:
    cur: Any = d
    for key in nested_key.split(sep):
        if isinstance(cur, dict) and key in cur:
            cur = cur[key]
        else:
            return default
    return cur
