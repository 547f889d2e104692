"""Host engine self-test (csrc/tests/engine_selftest.cc), plain + ASAN/UBSAN + TSAN.

The reference guarded its task table and completion paths with irqsave
spinlocks and refcounts (kmod/nvme_strom.c:648-731, 1148-1187) and relied on
kernel lockdep for race detection; here the same concurrency surface is
exercised from many threads under the host sanitizers.  TSAN exits non-zero
(66) on any report, so a race fails this test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("make") is None, reason="make not available")
@pytest.mark.parametrize("variant", ["selftest", "selftest-asan", "selftest-tsan"])
def test_engine_selftest(variant, tmp_path):
    r = subprocess.run(["make", "-s", f"build/{variant}"], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, STROM_STAT_SHM="0", TMPDIR=str(tmp_path),
               TSAN_OPTIONS="report_signal_unsafe=0")
    r = subprocess.run([os.path.join(ROOT, "build", variant)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "engine_selftest: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr
