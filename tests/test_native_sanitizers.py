"""Host sanitizer runs of the C++ runtime (csrc/native): ASan + UBSan, then TSan.

Builds csrc/native/test/selftest.cpp against the runtime sources (CRC32C, TFRecord/tfevents,
TF-V2 bundle, idx, threaded BatchPrefetcher) with g++ and runs it. GPU-side sanitizers are not
available on the MI355X pool, so this covers the host code only (the reference
relies on TF's own sanitizer builds of the equivalent C++).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_native_runtime_under_sanitizers(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "native_sanitize.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("native selftest ok") == 2 and "sanitizers clean" in out, out[-4000:]
