"""Hierarchical logger (reference: ``src/imitation/util/logger.py``).

Same observable behaviour as the reference's ``HierarchicalLogger``: inside
``accumulate_means(name)`` every ``record(key, v)`` is written to a per-scope sub-logger
as ``raw/<accumulate prefixes>/<name>/<key prefixes>/<key>`` (output files under
``<dir>/raw/<prefixes>/<name>/``) and averaged into the root logger as
``mean/<...same path...>/<key>``; outside a scope ``record`` goes to the root.
``add_accumulate_prefix`` is only legal outside a scope, ``add_key_prefix`` only inside,
and scopes do not nest.

Organisation here: the active scope is one :class:`_Scope` value (name, sub-logger, key
prefixes) instead of parallel mutable fields, sub-loggers come from a
:class:`_SubLoggerCache` keyed by their directory, and key paths are built by one helper.
Data parallel runs: only rank 0 writes (other ranks get loggers without output formats),
so metric keys and the on-disk layout are independent of the world size.
"""

from __future__ import annotations

import contextlib
import dataclasses
import datetime
import os
import pathlib
import sys
import tempfile
from typing import Dict, Iterator, List, Optional, Sequence

from imitation_amd.rl import logger as sb_logger

DEFAULT_FORMATS = ("stdout", "log", "csv")


def make_output_format(_format: str, log_dir: str, log_suffix: str = "", max_length: int = 50) -> sb_logger.KVWriter:
    """One SB3-style writer; ``stdout`` / ``log`` use a wider key column than SB3's default."""
    os.makedirs(log_dir, exist_ok=True)
    if _format in ("stdout", "log"):
        target = sys.stdout if _format == "stdout" else os.path.join(log_dir, f"log{log_suffix}.txt")
        return sb_logger.HumanOutputFormat(target, max_length=max_length)
    return sb_logger.make_output_format(_format, log_dir, log_suffix)


def _build_output_formats(folder: pathlib.Path, format_strs: Sequence[str]) -> List[sb_logger.KVWriter]:
    folder.mkdir(parents=True, exist_ok=True)
    return [WandbOutputFormat() if f == "wandb" else make_output_format(f, str(folder)) for f in format_strs]


def _key(kind: str, accumulate: Sequence[str], name: str, key_prefixes: Sequence[str], key: str) -> str:
    return "/".join([kind, *accumulate, name, *key_prefixes, key])


@dataclasses.dataclass
class _Scope:
    """The active ``accumulate_means`` context."""

    name: str
    subdir: str
    logger: sb_logger.Logger
    key_prefixes: List[str] = dataclasses.field(default_factory=list)


class _SubLoggerCache:
    """Sub-loggers of the ``raw/...`` scopes, created on first use and kept for reuse."""

    def __init__(self, root_dir: Optional[str], format_strs: Sequence[str], async_writes: bool = False):
        self.root_dir = root_dir
        self.format_strs = list(format_strs)
        self.async_writes = async_writes
        self.loggers: Dict[str, sb_logger.Logger] = {}

    def get(self, subdir: str) -> sb_logger.Logger:
        lg = self.loggers.get(subdir)
        if lg is None:
            assert self.root_dir is not None
            folder = pathlib.Path(self.root_dir) / "raw" / subdir
            folder.mkdir(exist_ok=True, parents=True)
            lg = sb_logger.Logger(str(folder), _build_output_formats(folder, self.format_strs), async_writes=self.async_writes)
            self.loggers[subdir] = lg
        return lg

    def close(self) -> None:
        for lg in self.loggers.values():
            lg.close()


class HierarchicalLogger(sb_logger.Logger):
    """SB3 logger with ``accumulate_means`` scopes (module docstring)."""

    def __init__(self, default_logger: sb_logger.Logger, format_strs: Sequence[str] = DEFAULT_FORMATS):
        self.default_logger = default_logger
        self.format_strs = format_strs
        self._subloggers = _SubLoggerCache(default_logger.dir, format_strs, getattr(default_logger, "async_writes", False))
        self._accumulate_prefixes: List[str] = []
        self._scope: Optional[_Scope] = None
        super().__init__(folder=default_logger.dir, output_formats=[], async_writes=getattr(default_logger, "async_writes", False))
        self._sync_maps()

    # ------------------------------------------------------------------ scope state
    @property
    def current_logger(self) -> Optional[sb_logger.Logger]:
        return self._scope.logger if self._scope is not None else None

    @property
    def _logger(self) -> sb_logger.Logger:
        return self._scope.logger if self._scope is not None else self.default_logger

    def _sync_maps(self) -> None:
        """``name_to_*`` are those of whichever logger is active (as in the reference)."""
        lg = self._logger
        self.name_to_value, self.name_to_count, self.name_to_excluded = lg.name_to_value, lg.name_to_count, lg.name_to_excluded

    # ------------------------------------------------------------------ prefixes / scopes
    @contextlib.contextmanager
    def add_accumulate_prefix(self, prefix: str) -> Iterator[None]:
        """Prefix the scope path of every ``accumulate_means`` opened inside (outside scopes only)."""
        if self._scope is not None:
            raise RuntimeError("Cannot add prefix when accumulate_means context is already active.")
        self._accumulate_prefixes.append(prefix)
        try:
            yield
        finally:
            self._accumulate_prefixes.pop()

    def get_accumulate_prefixes(self) -> str:
        joined = "/".join(self._accumulate_prefixes)
        return joined + "/" if joined else ""

    @contextlib.contextmanager
    def add_key_prefix(self, prefix: str) -> Iterator[None]:
        """Prefix the keys recorded inside the active scope."""
        if self._scope is None:
            raise RuntimeError("Cannot add key prefix when accumulate_means context is not active.")
        self._scope.key_prefixes.append(prefix)
        try:
            yield
        finally:
            self._scope.key_prefixes.pop()

    @contextlib.contextmanager
    def accumulate_means(self, name: str) -> Iterator[None]:
        """Route records to the ``raw/.../name`` sub-logger and their means to the root."""
        if self._scope is not None:
            raise RuntimeError("Nested `accumulate_means` context")
        subdir = os.path.join(*self._accumulate_prefixes, name)
        self._scope = _Scope(name=name, subdir=subdir, logger=self._subloggers.get(subdir))
        self._sync_maps()
        try:
            yield
        finally:
            self._scope = None
            self._sync_maps()

    # ------------------------------------------------------------------ recording
    def record(self, key, val, exclude=None):
        scope = self._scope
        if scope is None:
            self.default_logger.record(key, val, exclude)
            return
        scope.logger.record(_key("raw", self._accumulate_prefixes, scope.name, scope.key_prefixes, key), val, exclude)
        self.default_logger.record_mean(_key("mean", self._accumulate_prefixes, scope.name, scope.key_prefixes, key), val,
                                        exclude)

    def record_mean(self, key, val, exclude=None):
        self.default_logger.record_mean(key, val, exclude)

    def dump(self, step=0):
        self._logger.dump(step)

    def get_dir(self) -> str:
        return self._logger.get_dir()

    def log(self, *args, **kwargs):
        self.default_logger.log(*args, **kwargs)

    def set_level(self, level: int) -> None:
        self.default_logger.set_level(level)

    def flush(self) -> None:
        self.default_logger.flush()

    def close(self):
        self.default_logger.close()
        self._subloggers.close()

    @property
    def _cached_loggers(self) -> Dict[str, sb_logger.Logger]:
        return self._subloggers.loggers


class WandbOutputFormat(sb_logger.KVWriter):
    """Weights & Biases writer (``wandb`` is optional and not installed here)."""

    def __init__(self):
        try:
            import wandb
        except ModuleNotFoundError as e:  # pragma: no cover
            raise ModuleNotFoundError(
                "Trying to log data with `WandbOutputFormat` but `wandb` not installed: try `pip install wandb`."
            ) from e
        self.wandb_module = wandb

    def write(self, key_values, key_excluded, step=0):  # pragma: no cover - needs wandb
        payload = {k: v for k, v in sorted(key_values.items())
                   if not (key_excluded.get(k) is not None and "wandb" in key_excluded[k])}
        for k, v in payload.items():
            self.wandb_module.log({k: v}, step=step)
        self.wandb_module.log({}, commit=True)

    def close(self) -> None:  # pragma: no cover
        self.wandb_module.finish()


def _default_folder() -> str:
    stamp = datetime.datetime.now().strftime("imitation-%Y-%m-%d-%H-%M-%S-%f")
    return os.path.join(tempfile.gettempdir(), stamp)


def configure(folder=None, format_strs: Optional[Sequence[str]] = None,
              async_writes: Optional[bool] = None) -> HierarchicalLogger:
    """A :class:`HierarchicalLogger` writing to ``folder`` (a fresh temp dir by default) with
    ``format_strs`` (library default stdout/log/csv); DP ranks other than 0 write nothing.
    ``async_writes``: format writes on the shared writer thread (default:
    ``IMITATION_AMD_LOG_ASYNC``; the CLIs turn it on)."""
    from imitation_amd.parallel import dist as pdist

    folder = str(folder) if folder is not None else _default_folder()
    formats = list(DEFAULT_FORMATS if format_strs is None else format_strs)
    if pdist.rank() != 0:
        return HierarchicalLogger(sb_logger.Logger(folder, []), [])
    return HierarchicalLogger(sb_logger.Logger(folder, _build_output_formats(pathlib.Path(folder), formats),
                                               async_writes=async_writes), formats)
