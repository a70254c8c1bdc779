"""W&B output format with a stand-in ``wandb`` module (``wandb`` is not installed here; the
upstream suite mocks it the same way): logged keys / steps, excluded keys, finish on close."""

import sys
import types

from imitation_amd.util import logger


class _FakeWandb(types.ModuleType):
    def __init__(self):
        super().__init__("wandb")
        self.logged, self.finished = [], 0

    def log(self, data, step=None, commit=None):
        self.logged.append((dict(data), step, commit))

    def finish(self):
        self.finished += 1


def test_wandb_format_logs_and_finishes(tmp_path, monkeypatch):
    fake = _FakeWandb()
    monkeypatch.setitem(sys.modules, "wandb", fake)
    log = logger.configure(tmp_path, format_strs=["wandb", "csv"])
    log.record("a", 1.0)
    log.record("hidden", 2.0, exclude="wandb")
    with log.accumulate_means("gen"):
        log.record("b", 3.0)
        log.dump(step=7)
    log.dump(step=11)
    keys = {k for d, _, _ in fake.logged for k in d}
    assert "a" in keys and "hidden" not in keys
    assert any(step == 11 and "a" in d for d, step, _ in fake.logged)
    assert any(commit for _, _, commit in fake.logged)
    log.close()
    assert fake.finished >= 1  # the root logger and each accumulate_means sub-logger own a writer
