"""HierarchicalLogger semantics (reference: tests/util/test_logger.py)."""

import csv
import json
import os.path as osp
from collections import defaultdict

import pytest

from imitation_amd.util import logger


def _csv(path):
    out = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            for k, v in row.items():
                out[k].append(float(v) if v != "" else "")
    return dict(out)


def _json(path):
    lines = [json.loads(l) for l in open(path)]
    keys = set().union(*lines)
    return {k: [l.get(k, "") for l in lines] for k in keys}


def test_no_accum(tmp_path):
    h = logger.configure(str(tmp_path), ["csv", "json"])
    h.record("A", -1)
    h.record("A", 1)  # overwrites, not averaged
    h.record("B", 1)
    h.dump()
    h.record("A", 2)
    h.dump()
    h.record("B", 3)
    h.dump()
    expect = {"A": [1, 2, ""], "B": [1, "", 3]}
    assert _csv(tmp_path / "progress.csv") == expect
    assert _json(tmp_path / "progress.json") == expect


def test_unknown_format():
    with pytest.raises(ValueError, match="Unknown format specified"):
        logger.make_output_format("txt", "log_dir")


def test_reentry_fails(tmp_path):
    h = logger.configure(str(tmp_path))
    with h.accumulate_means("foo"):
        with pytest.raises(RuntimeError, match="Nested"):
            with h.accumulate_means("bar"):
                pass


def test_name_to_value_means(tmp_path):
    h = logger.configure(str(tmp_path))
    with h.accumulate_means("foo"):
        h.record("A", 1)
        assert h.name_to_value["raw/foo/A"] == 1
        h.record("B", 10)
        h.dump()
        h.record("B", 20)
    assert h.name_to_value["mean/foo/A"] == 1
    assert h.name_to_value["mean/foo/B"] == 15 and h.name_to_count["mean/foo/B"] == 2
    h.dump()
    assert len(h.name_to_value) == 0


def test_hard(tmp_path):
    h = logger.configure(str(tmp_path))
    h.record("no_context", 1)
    with h.accumulate_means("disc"):
        h.record("C", 2)
        h.record("D", 2)
        h.dump()
        h.record("C", 4)
        h.dump()
    with h.accumulate_means("gen"):
        h.record("E", 2)
        h.dump()
        h.record("E", 0)
        h.dump()
    with h.accumulate_means("disc"):
        h.record("C", 3)
        h.dump()
    h.dump()
    assert _csv(tmp_path / "progress.csv") == {"mean/gen/E": [1], "mean/disc/C": [3], "mean/disc/D": [2], "no_context": [1]}
    assert _csv(tmp_path / "raw" / "gen" / "progress.csv") == {"raw/gen/E": [2, 0]}
    assert _csv(tmp_path / "raw" / "disc" / "progress.csv") == {"raw/disc/C": [2, 4, 3], "raw/disc/D": [2, "", ""]}


def test_prefixes(tmp_path):
    h = logger.configure(str(tmp_path))
    with h.add_accumulate_prefix("foo"), h.accumulate_means("bar"):
        h.record("A", 1)
        h.dump()
    with h.accumulate_means("blat"), h.add_key_prefix("k"):
        h.record("C", 3)
        h.dump()
    h.dump()
    assert _csv(tmp_path / "progress.csv") == {"mean/foo/bar/A": [1], "mean/blat/k/C": [3]}
    assert _csv(tmp_path / "raw" / "foo" / "bar" / "progress.csv") == {"raw/foo/bar/A": [1]}
    with pytest.raises(RuntimeError):
        with h.accumulate_means("x"), h.add_accumulate_prefix("y"):
            pass
    with pytest.raises(RuntimeError):
        with h.add_key_prefix("z"):
            pass


def test_tensorboard_event_file(tmp_path):
    h = logger.configure(str(tmp_path), ["tensorboard"])
    h.record("x", 1.5)
    h.dump(step=3)
    h.close()
    files = list(tmp_path.glob("events.out.tfevents.*"))
    assert files and files[0].stat().st_size > 0


def _read_tfrecords(path):
    """(tag, step, value) of every scalar Event in a TF event file, checking each record's
    masked CRC32C with the pure-Python implementation."""
    import struct

    from imitation_amd.rl import logger as sb_logger

    out = []
    data = path.read_bytes()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        hdr = data[i:i + 8]
        assert struct.unpack_from("<I", data, i + 8)[0] == sb_logger._masked_crc(hdr)
        ev = data[i + 12:i + 12 + n]
        assert struct.unpack_from("<I", data, i + 12 + n)[0] == sb_logger._masked_crc(ev)
        i += 16 + n
        if b"brain.Event" in ev:
            continue
        # Event: 0x09 <f64 wall> 0x10 <varint step> 0x2a <len> summary
        j = 9
        step, shift = 0, 0
        j += 1
        while True:
            b = ev[j]
            step |= (b & 0x7F) << shift
            j += 1
            shift += 7
            if b < 0x80:
                break
        summ = ev[j + 2:]
        val = summ[2:]
        tlen = val[1]
        tag = val[2:2 + tlen].decode()
        (v,) = struct.unpack_from("<f", val, 2 + tlen + 1)
        out.append((tag, step, v))
    return out


def test_tensorboard_native_encoder_matches_python():
    """``_C.tb_scalar_records`` (csrc/runtime/tb_events.cpp) is byte-identical to the Python
    protobuf + CRC32C encoder, incl. multi-byte varints (long tags, large steps)."""
    from imitation_amd import _native
    from imitation_amd.rl import logger as sb_logger

    C = _native.load(build_if_missing=False)
    for b in (b"", b"a", b"123456789", bytes(range(256)) * 3):
        assert C.crc32c(b) == sb_logger._crc32c(b)
        assert C.masked_crc32c(b) == sb_logger._masked_crc(b)
    assert C.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    tags = ["x", "mean/gen/train/value_loss", "t" * 200]
    vals = [1.5, -3.25e-7, 12345.0]
    for step in (0, 3, 300, 2**40 + 7):
        assert C.tb_scalar_records(1.25e9, step, tags, vals) == sb_logger.encode_scalar_records(1.25e9, step, tags, vals)


@pytest.mark.parametrize("background", [True, False])
def test_tensorboard_writer_thread_round_trip(tmp_path, background, monkeypatch):
    """Dumps queued to the writer thread are all on disk, in order, after flush / close."""
    monkeypatch.setenv("IMITATION_AMD_TB_THREAD", "1" if background else "0")
    h = logger.configure(str(tmp_path), ["tensorboard"])
    for s in range(50):
        h.record("a", float(s))
        h.record("b", 2.0 * s)
        h.dump(step=s)
    h.close()
    files = list(tmp_path.glob("events.out.tfevents.*"))
    recs = _read_tfrecords(files[0])
    assert recs == [(k, s, v) for s in range(50) for k, v in (("a", float(s)), ("b", 2.0 * s))]


def test_free_form_text_levels(tmp_path):
    """Reference test_free_form: free-form messages reach log.txt at or above the level; inside
    accumulate_means they still go to the default output."""
    from imitation_amd.rl import logger as sb_logger

    h = logger.configure(str(tmp_path), ["log"])
    h.log("info 1")
    h.info("info 2")
    h.warn("warn 1")
    h.error("error 1")
    h.debug("hidden")
    h.set_level(level=sb_logger.DEBUG)
    h.debug("debug 1")
    with h.accumulate_means("foo"):
        h.info("info inner")
    h.debug("debug outer")
    h.close()
    with open(osp.join(str(tmp_path), "log.txt")) as f:
        assert f.readlines() == ["info 1\n", "info 2\n", "warn 1\n", "error 1\n", "debug 1\n", "info inner\n",
                                 "debug outer\n"]


def test_dump_after_close_raises(tmp_path):
    h = logger.configure(str(tmp_path))
    h.record("A", 1)
    with h.accumulate_means("foo"):
        h.record("B", 2)
    h.dump()
    h.close()
    h.record("foo", 42)
    with pytest.raises(ValueError, match="closed file"):
        h.dump()


def test_prefix_context_errors(tmp_path):
    h = logger.configure(str(tmp_path))
    with pytest.raises(RuntimeError):
        with h.accumulate_means("foo"), h.add_accumulate_prefix("bar"):
            pass
    h2 = logger.configure(str(tmp_path / "b"))
    with pytest.raises(RuntimeError):
        with h2.add_key_prefix("bar"):
            pass
