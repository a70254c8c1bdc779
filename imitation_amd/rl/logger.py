"""Key-value logger with stdout / log / csv / json / tensorboard writers.

This is the SB3 ``logger`` surface that the reference's
``HierarchicalLogger`` subclasses (``src/imitation/util/logger.py:17-44``;
SURVEY §5.5). ``tensorboard`` is not installed on this image, so
:class:`TensorBoardOutputFormat` writes TF event files directly (length-prefixed
records with masked CRC32C, hand-encoded ``Event``/``Summary`` protos) -- readable
by any TensorBoard.
"""

from __future__ import annotations

import csv
import json
import os
import struct
import sys
import time
import warnings
from collections import defaultdict
from typing import Any, Dict, List, Mapping, Optional, Sequence, TextIO, Tuple, Union

import numpy as np

DEBUG, INFO, WARN, ERROR, DISABLED = 10, 20, 30, 40, 50


class KVWriter:
    def write(self, key_values: Dict[str, Any], key_excluded: Dict[str, Tuple[str, ...]], step: int = 0) -> None:
        raise NotImplementedError

    def close(self) -> None:
        pass


class SeqWriter:
    def write_sequence(self, sequence: List[str]) -> None:
        raise NotImplementedError


def _is_excluded(excluded, fmt: str) -> bool:
    return excluded is not None and fmt in excluded


class HumanOutputFormat(KVWriter, SeqWriter):
    """Aligned ASCII table; keys with a ``tag/`` prefix are grouped and indented."""

    def __init__(self, filename_or_file: Union[str, TextIO], max_length: int = 36):
        self.max_length = max_length
        if isinstance(filename_or_file, str):
            self.file = open(filename_or_file, "w")
            self.own_file = True
        else:
            assert hasattr(filename_or_file, "write")
            self.file = filename_or_file
            self.own_file = False

    def write(self, key_values, key_excluded, step=0):
        key2str: Dict[Tuple[str, str], str] = {}
        tag = ""
        for (key, value), (_, excluded) in zip(sorted(key_values.items()), sorted(key_excluded.items())):
            if excluded is not None and ("stdout" in excluded or "log" in excluded):
                continue
            if isinstance(value, (float, np.floating)):
                value_str = f"{value:<8.3g}"
            else:
                value_str = str(value)
            if key.find("/") > 0:
                tag = key[: key.find("/") + 1]
                key2str[(tag, self._truncate(tag))] = ""
            if len(tag) > 0 and tag in key:
                key = f"{'':3}{key[len(tag):]}"
            truncated_key = self._truncate(key)
            if (tag, truncated_key) in key2str:
                raise ValueError(f"Key '{key}' truncated to '{truncated_key}' that already exists.")
            key2str[(tag, truncated_key)] = self._truncate(value_str)
        if not key2str:
            warnings.warn("Tried to write empty key-value dict")
            return
        key_width = max(len(k[1]) for k in key2str)
        val_width = max(len(v) for v in key2str.values())
        dashes = "-" * (key_width + val_width + 7)
        lines = [dashes]
        for (_, key), value in key2str.items():
            lines.append(f"| {key}{' ' * (key_width - len(key))} | {value}{' ' * (val_width - len(value))} |")
        lines.append(dashes)
        self.file.write("\n".join(lines) + "\n")
        self.file.flush()

    def _truncate(self, string: str) -> str:
        if len(string) > self.max_length:
            string = string[: self.max_length - 3] + "..."
        return string

    def write_sequence(self, sequence: List[str]) -> None:
        for i, elem in enumerate(sequence):
            self.file.write(str(elem))
            if i < len(sequence) - 1:
                self.file.write(" ")
        self.file.write("\n")
        self.file.flush()

    def close(self) -> None:
        if self.own_file:
            self.file.close()


class JSONOutputFormat(KVWriter):
    def __init__(self, filename: str):
        self.file = open(filename, "w")

    def write(self, key_values, key_excluded, step=0):
        def cast(v):
            if hasattr(v, "dtype"):
                if getattr(v, "shape", ()) == () or len(v) == 1:
                    return float(np.asarray(v).item())
                return np.asarray(v).tolist()
            return v

        d = {k: cast(v) for k, v in key_values.items() if not _is_excluded(key_excluded.get(k), "json")}
        self.file.write(json.dumps(d) + "\n")
        self.file.flush()

    def close(self):
        self.file.close()


class CSVOutputFormat(KVWriter):
    """CSV with a growing header (the file is rewritten when new keys appear)."""

    def __init__(self, filename: str):
        self.file = open(filename, "w+")
        self.keys: List[str] = []
        self.separator = ","
        self.quotechar = '"'

    def write(self, key_values, key_excluded, step=0):
        key_values = {k: v for k, v in key_values.items() if not _is_excluded(key_excluded.get(k), "csv")}
        extra_keys = key_values.keys() - set(self.keys)
        if extra_keys:
            self.keys.extend(sorted(extra_keys))
            self.file.seek(0)
            lines = self.file.readlines()
            self.file.seek(0)
            self.file.truncate()
            self.file.write(self.separator.join(self.keys) + "\n")
            for line in lines[1:]:
                self.file.write(line[:-1])
                self.file.write(self.separator * len(extra_keys))
                self.file.write("\n")
        for i, key in enumerate(self.keys):
            if i > 0:
                self.file.write(self.separator)
            value = key_values.get(key)
            if isinstance(value, str):
                value = value.replace(self.quotechar, self.quotechar + self.quotechar)
                self.file.write(self.quotechar + value + self.quotechar)
            elif value is not None:
                self.file.write(str(value))
        self.file.write("\n")
        self.file.flush()

    def close(self):
        self.file.close()


# --------------------------------------------------------------------------- TF event files
def _crc32c_table():
    poly = 0x82F63B78
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_CRC_TABLE = _crc32c_table()


def _crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = _crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _event(wall_time: float, step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None) -> bytes:
    msg = _field(1, 1) + struct.pack("<d", wall_time) + _field(2, 0) + _varint(step)
    if file_version is not None:
        fv = file_version.encode()
        msg += _field(3, 2) + _varint(len(fv)) + fv
    if summary is not None:
        msg += _field(5, 2) + _varint(len(summary)) + summary
    return msg


def _scalar_summary(tag: str, value: float) -> bytes:
    t = tag.encode()
    val = _field(1, 2) + _varint(len(t)) + t + _field(2, 5) + struct.pack("<f", float(value))
    return _field(1, 2) + _varint(len(val)) + val


def _native_tb():
    """``imitation_amd._C`` when it is built (its ``tb_scalar_records`` encodes a whole dump:
    ``csrc/runtime/tb_events.cpp``), else None (pure-Python encoding below)."""
    try:
        from imitation_amd import _native

        C = _native.load(build_if_missing=False)
        return C if hasattr(C, "tb_scalar_records") else None
    except Exception:  # noqa: BLE001 -- not built (e.g. a docs build): Python fallback
        return None


def encode_scalar_records(wall_time: float, step: int, tags: Sequence[str], values: Sequence[float], native=None) -> bytes:
    """Framed TFRecords of one dump's scalars (Python reference of ``tb_scalar_records``)."""
    if native is not None:
        return native.tb_scalar_records(float(wall_time), int(step), list(tags), [float(v) for v in values])
    out = bytearray()
    for tag, value in zip(tags, values):
        data = _event(wall_time, int(step), summary=_scalar_summary(tag, float(value)))
        header = struct.pack("<Q", len(data))
        out += header + struct.pack("<I", _masked_crc(header)) + data + struct.pack("<I", _masked_crc(data))
    return bytes(out)


class TensorBoardOutputFormat(KVWriter):
    """TF event file writer. ``write`` only snapshots the dump's scalars; a background thread
    encodes them (natively when ``imitation_amd._C`` is built) and appends them to the file, so a
    training loop pays ~microseconds per dump instead of the encoding + CRC + flush (the
    reference writes synchronously through torch's SummaryWriter, which also queues to a
    writer thread). ``flush`` / ``close`` drain the queue; every write is on disk after them."""

    def __init__(self, folder: str, background: Optional[bool] = None):
        os.makedirs(folder, exist_ok=True)
        fname = os.path.join(folder, f"events.out.tfevents.{int(time.time())}.{os.uname().nodename}.{os.getpid()}")
        self.file = open(fname, "wb")
        self._native = _native_tb()
        self._write_record(_event(time.time(), 0, file_version="brain.Event:2"))
        self.file.flush()
        if background is None:
            background = os.environ.get("IMITATION_AMD_TB_THREAD", "0") == "1"
        self._queue = None
        self._thread = None
        self._error: Optional[BaseException] = None
        if background:
            import queue
            import threading

            self._queue = queue.Queue()
            self._thread = threading.Thread(target=self._drain, name="tb-writer", daemon=True)
            self._thread.start()

    def _write_record(self, data: bytes) -> None:
        header = struct.pack("<Q", len(data))
        self.file.write(header + struct.pack("<I", _masked_crc(header)) + data + struct.pack("<I", _masked_crc(data)))

    def _encode_and_write(self, item) -> None:
        wall, step, tags, vals = item
        self.file.write(encode_scalar_records(wall, step, tags, vals, self._native))

    def _drain(self) -> None:
        q = self._queue
        while True:
            item = q.get()
            try:
                if item is None:
                    return
                self._encode_and_write(item)
                if q.empty():
                    self.file.flush()
            except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's next write / flush
                self._error = e
            finally:
                q.task_done()

    def _check(self) -> None:
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError("tensorboard writer thread failed") from e

    def write(self, key_values, key_excluded, step=0):
        tags, vals = [], []
        for key, value in sorted(key_values.items()):
            if _is_excluded(key_excluded.get(key), "tensorboard"):
                continue
            if isinstance(value, (int, float, np.integer, np.floating)) and not isinstance(value, bool):
                tags.append(key)
                vals.append(float(value))
        if not tags:
            return
        item = (time.time(), int(step), tags, vals)
        if self._queue is None:
            self._encode_and_write(item)
            self.file.flush()
            return
        self._check()
        self._queue.put(item)

    def flush(self) -> None:
        if self._queue is not None:
            self._queue.join()
            self._check()
        self.file.flush()

    def close(self):
        if self._thread is not None:
            self._queue.put(None)
            self._thread.join()
            self._thread = None
            self._check()
        self.file.close()


def make_output_format(_format: str, log_dir: str, log_suffix: str = "") -> KVWriter:
    os.makedirs(log_dir, exist_ok=True)
    if _format == "stdout":
        return HumanOutputFormat(sys.stdout)
    if _format == "log":
        return HumanOutputFormat(os.path.join(log_dir, f"log{log_suffix}.txt"))
    if _format == "json":
        return JSONOutputFormat(os.path.join(log_dir, f"progress{log_suffix}.json"))
    if _format == "csv":
        return CSVOutputFormat(os.path.join(log_dir, f"progress{log_suffix}.csv"))
    if _format == "tensorboard":
        return TensorBoardOutputFormat(log_dir)
    raise ValueError(f"Unknown format specified: {_format}")


class _WriterThread:
    """ONE daemon thread running the queued format writes of every asynchronous :class:`Logger`
    in submission order (so the stdout / log / csv / tensorboard outputs of all sub-loggers keep
    the order a synchronous run produces). A training loop's dump then costs a dict snapshot;
    the formatting, encoding and file I/O run while the main thread waits on the GPU (event
    synchronisation releases the GIL). An exception in a write is re-raised by the next
    submit / drain."""

    def __init__(self):
        import queue
        import threading

        self._q: "queue.Queue" = queue.Queue()
        self._lock = threading.Lock()
        self._thread = None
        self._error: Optional[BaseException] = None

    def _run(self) -> None:
        while True:
            fn = self._q.get()
            try:
                fn()
            except BaseException as e:  # noqa: BLE001 -- surfaced on the caller's thread
                if self._error is None:
                    self._error = e
            finally:
                self._q.task_done()

    def _raise(self) -> None:
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError("asynchronous logger write failed") from e

    def submit(self, fn) -> None:
        import threading

        self._raise()
        with self._lock:
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name="ia-log-writer", daemon=True)
                self._thread.start()
        self._q.put(fn)

    def drain(self) -> None:
        if self._thread is not None:
            self._q.join()
        self._raise()


_WRITER = _WriterThread()


def flush_async_writes() -> None:
    """Block until every queued asynchronous logger write is done (also run at exit)."""
    _WRITER.drain()


def _drain_at_exit() -> None:
    try:
        _WRITER.drain()
    except Exception as e:  # noqa: BLE001 -- interpreter shutdown: report, do not raise
        print(f"imitation_amd logger: {e!r}", file=sys.stderr)


import atexit  # noqa: E402

atexit.register(_drain_at_exit)


def async_default() -> bool:
    """``IMITATION_AMD_LOG_ASYNC=1``: loggers built without an explicit choice write asynchronously."""
    return os.environ.get("IMITATION_AMD_LOG_ASYNC", "0") == "1"


class Logger:
    """Accumulate ``record``/``record_mean`` key-values and ``dump`` them to writers.

    ``async_writes``: ``dump`` / ``log`` hand a snapshot to the shared writer thread
    (:class:`_WriterThread`) instead of formatting and writing on the caller's thread;
    ``flush`` / ``close`` (and interpreter exit) wait for the writes."""

    def __init__(self, folder: Optional[str], output_formats: List[KVWriter], async_writes: Optional[bool] = None):
        self.name_to_value: Dict[str, float] = defaultdict(float)
        self.name_to_count: Dict[str, int] = defaultdict(int)
        self.name_to_excluded: Dict[str, Tuple[str, ...]] = {}
        self.level = INFO
        self.dir = folder
        self.output_formats = output_formats
        self.async_writes = async_default() if async_writes is None else bool(async_writes)

    @staticmethod
    def to_tuple(string_or_tuple) -> Tuple[str, ...]:
        if string_or_tuple is None:
            return ("",)
        if isinstance(string_or_tuple, tuple):
            return string_or_tuple
        return (string_or_tuple,)

    def record(self, key: str, value: Any, exclude=None) -> None:
        self.name_to_value[key] = value
        self.name_to_excluded[key] = self.to_tuple(exclude)

    def record_mean(self, key: str, value: Any, exclude=None) -> None:
        if value is None:
            return
        old_val, count = self.name_to_value[key], self.name_to_count[key]
        self.name_to_value[key] = old_val * count / (count + 1) + value / (count + 1)
        self.name_to_count[key] = count + 1
        self.name_to_excluded[key] = self.to_tuple(exclude)

    def dump(self, step: int = 0) -> None:
        if self.level == DISABLED:
            return
        kv = [f for f in self.output_formats if isinstance(f, KVWriter)]
        if kv and self.async_writes:
            values, excluded = dict(self.name_to_value), dict(self.name_to_excluded)

            def write_all(kv=kv, values=values, excluded=excluded, step=step):
                for fmt in kv:
                    fmt.write(values, excluded, step)

            _WRITER.submit(write_all)
        else:
            for fmt in kv:
                fmt.write(self.name_to_value, self.name_to_excluded, step)
        self.name_to_value.clear()
        self.name_to_count.clear()
        self.name_to_excluded.clear()

    def log(self, *args, level: int = INFO) -> None:
        if self.level <= level:
            seq = [f for f in self.output_formats if isinstance(f, SeqWriter)]
            if not seq:
                return
            items = list(map(str, args))
            if self.async_writes:
                _WRITER.submit(lambda seq=seq, items=items: [f.write_sequence(items) for f in seq])
            else:
                for fmt in seq:
                    fmt.write_sequence(items)

    def flush(self) -> None:
        """Wait for this process's queued asynchronous writes."""
        _WRITER.drain()

    def debug(self, *args) -> None:
        self.log(*args, level=DEBUG)

    def info(self, *args) -> None:
        self.log(*args, level=INFO)

    def warn(self, *args) -> None:
        self.log(*args, level=WARN)

    def error(self, *args) -> None:
        self.log(*args, level=ERROR)

    def set_level(self, level: int) -> None:
        self.level = level

    def get_dir(self) -> Optional[str]:
        return self.dir

    def close(self) -> None:
        if self.async_writes:
            _WRITER.drain()
        for fmt in self.output_formats:
            fmt.close()


def configure(folder: Optional[str] = None, format_strings: Optional[List[str]] = None) -> Logger:
    if folder is None:
        folder = os.getenv("SB3_LOGDIR")
    if folder is None:
        import datetime
        import tempfile

        folder = os.path.join(tempfile.gettempdir(), datetime.datetime.now().strftime("SB3-%Y-%m-%d-%H-%M-%S-%f"))
    os.makedirs(folder, exist_ok=True)
    if format_strings is None:
        format_strings = os.getenv("SB3_LOG_FORMAT", "stdout,log,csv").split(",")
    format_strings = [f for f in format_strings if f]
    output_formats = [make_output_format(f, folder, "") for f in format_strings]
    return Logger(folder=folder, output_formats=output_formats)
