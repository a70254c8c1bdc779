"""Hierarchical logger (reference: ``src/imitation/util/logger.py``).

``HierarchicalLogger.accumulate_means(name)`` routes ``record`` calls to a cached
sub-logger under ``<dir>/raw/<prefixes>/<name>`` (key ``raw/.../key``) while
``record_mean``-ing them into the root logger under ``mean/.../key``
(``logger.py:290-315``). Nested contexts raise; ``add_accumulate_prefix`` only
outside, ``add_key_prefix`` only inside the context (``:161-217``).

Distributed runs: only rank 0 writes files/stdout (other ranks get a logger
with no output formats), so metric keys and on-disk layout match the reference.
"""

from __future__ import annotations

import contextlib
import datetime
import os
import pathlib
import sys
import tempfile
from typing import Any, Dict, Generator, List, Optional, Sequence, Tuple

from imitation_amd.rl import logger as sb_logger


def make_output_format(_format: str, log_dir: str, log_suffix: str = "", max_length: int = 50) -> sb_logger.KVWriter:
    os.makedirs(log_dir, exist_ok=True)
    if _format == "stdout":
        return sb_logger.HumanOutputFormat(sys.stdout, max_length=max_length)
    if _format == "log":
        return sb_logger.HumanOutputFormat(os.path.join(log_dir, f"log{log_suffix}.txt"), max_length=max_length)
    return sb_logger.make_output_format(_format, log_dir, log_suffix)


def _build_output_formats(folder: pathlib.Path, format_strs: Sequence[str]) -> Sequence[sb_logger.KVWriter]:
    folder.mkdir(parents=True, exist_ok=True)
    out: List[sb_logger.KVWriter] = []
    for f in format_strs:
        if f == "wandb":
            out.append(WandbOutputFormat())
        else:
            out.append(make_output_format(f, str(folder)))
    return out


class HierarchicalLogger(sb_logger.Logger):
    """Logger with ``accumulate_means`` sub-logger contexts (see module docstring)."""

    def __init__(self, default_logger: sb_logger.Logger, format_strs: Sequence[str] = ("stdout", "log", "csv")):
        self.default_logger = default_logger
        self.current_logger: Optional[sb_logger.Logger] = None
        self._cached_loggers: Dict[str, sb_logger.Logger] = {}
        self._accumulate_prefixes: List[str] = []
        self._key_prefixes: List[str] = []
        self._subdir: Optional[str] = None
        self._name: Optional[str] = None
        self.format_strs = format_strs
        super().__init__(folder=self.default_logger.dir, output_formats=[])

    def _update_name_to_maps(self) -> None:
        self.name_to_value = self._logger.name_to_value
        self.name_to_count = self._logger.name_to_count
        self.name_to_excluded = self._logger.name_to_excluded

    @contextlib.contextmanager
    def add_accumulate_prefix(self, prefix: str) -> Generator[None, None, None]:
        if self.current_logger is not None:
            raise RuntimeError("Cannot add prefix when accumulate_means context is already active.")
        try:
            self._accumulate_prefixes.append(prefix)
            yield
        finally:
            self._accumulate_prefixes.pop()

    def get_accumulate_prefixes(self) -> str:
        prefixes = "/".join(self._accumulate_prefixes)
        return prefixes + "/" if prefixes else ""

    @contextlib.contextmanager
    def add_key_prefix(self, prefix: str) -> Generator[None, None, None]:
        if self.current_logger is None:
            raise RuntimeError("Cannot add key prefix when accumulate_means context is not active.")
        try:
            self._key_prefixes.append(prefix)
            yield
        finally:
            self._key_prefixes.pop()

    @contextlib.contextmanager
    def accumulate_means(self, name: str) -> Generator[None, None, None]:
        if self.current_logger is not None:
            raise RuntimeError("Nested `accumulate_means` context")
        subdir = os.path.join(*self._accumulate_prefixes, name)
        if subdir in self._cached_loggers:
            logger = self._cached_loggers[subdir]
        else:
            assert self.default_logger.dir is not None
            folder = pathlib.Path(self.default_logger.dir) / "raw" / subdir
            folder.mkdir(exist_ok=True, parents=True)
            fmts = _build_output_formats(folder, self.format_strs)
            logger = sb_logger.Logger(str(folder), list(fmts))
            self._cached_loggers[subdir] = logger
        try:
            self.current_logger = logger
            self._subdir = subdir
            self._name = name
            self._update_name_to_maps()
            yield
        finally:
            self.current_logger = None
            self._subdir = None
            self._name = None
            self._update_name_to_maps()

    def record(self, key, val, exclude=None):
        if self.current_logger is not None:
            assert self._subdir is not None
            raw_key = "/".join(["raw", *self._accumulate_prefixes, self._name, *self._key_prefixes, key])
            self.current_logger.record(raw_key, val, exclude)
            mean_key = "/".join(["mean", *self._accumulate_prefixes, self._name, *self._key_prefixes, key])
            self.default_logger.record_mean(mean_key, val, exclude)
        else:
            self.default_logger.record(key, val, exclude)

    @property
    def _logger(self):
        return self.current_logger if self.current_logger is not None else self.default_logger

    def dump(self, step=0):
        self._logger.dump(step)

    def get_dir(self) -> str:
        return self._logger.get_dir()

    def log(self, *args, **kwargs):
        self.default_logger.log(*args, **kwargs)

    def set_level(self, level: int) -> None:
        self.default_logger.set_level(level)

    def record_mean(self, key, val, exclude=None):
        self.default_logger.record_mean(key, val, exclude)

    def close(self):
        self.default_logger.close()
        for logger in self._cached_loggers.values():
            logger.close()


class WandbOutputFormat(sb_logger.KVWriter):
    """Weights & Biases writer (requires ``wandb``, which is optional)."""

    def __init__(self):
        try:
            import wandb
        except ModuleNotFoundError as e:  # pragma: no cover
            raise ModuleNotFoundError(
                "Trying to log data with `WandbOutputFormat` but `wandb` not installed: try `pip install wandb`."
            ) from e
        self.wandb_module = wandb

    def write(self, key_values, key_excluded, step=0):  # pragma: no cover - needs wandb
        for (key, value), (key_ex, excluded) in zip(sorted(key_values.items()), sorted(key_excluded.items())):
            assert key == key_ex
            if excluded is not None and "wandb" in excluded:
                continue
            self.wandb_module.log({key: value}, step=step)
        self.wandb_module.log({}, commit=True)

    def close(self) -> None:  # pragma: no cover
        self.wandb_module.finish()


def configure(folder=None, format_strs: Optional[Sequence[str]] = None) -> HierarchicalLogger:
    """Configure a :class:`HierarchicalLogger` (library default formats stdout/log/csv)."""
    if folder is None:
        tempdir = tempfile.gettempdir()
        now = datetime.datetime.now()
        timestamp = now.strftime("imitation-%Y-%m-%d-%H-%M-%S-%f")
        folder = os.path.join(tempdir, timestamp)
    folder = str(folder)
    if format_strs is None:
        format_strs = ["stdout", "log", "csv"]
    from imitation_amd.parallel import dist as pdist

    if pdist.rank() != 0:
        # Non-zero DP ranks keep the API but write nothing.
        default_logger = sb_logger.Logger(folder, [])
        return HierarchicalLogger(default_logger, [])
    output_formats = _build_output_formats(pathlib.Path(folder), format_strs)
    default_logger = sb_logger.Logger(folder, list(output_formats))
    return HierarchicalLogger(default_logger, format_strs)
