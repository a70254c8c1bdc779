"""The native env runtime under AddressSanitizer + UBSan (host code only)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("bash") is None, reason="needs hipcc")
def test_native_envs_clean_under_asan_ubsan(tmp_path):
    out = subprocess.run(["bash", os.path.join(ROOT, "tools/sanitize/run.sh"), str(tmp_path / "fuzz"), "300"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "env_fuzz ok" in out.stdout
