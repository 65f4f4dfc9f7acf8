"""Host-side sanitizer run of the native runtime.

The KServe wire codec (csrc/runtime/kserve_wire.cpp) is compiled together with
a fuzz / round-trip driver under AddressSanitizer + UndefinedBehaviorSanitizer
and run: malformed, truncated and length-inflated responses must be rejected
without any out-of-bounds access.  GPU ASan / XNACK are not available on the
GPU pool, so device code is covered by numerics tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_wire_codec_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "wire_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", os.path.join(ROOT, "csrc/runtime/kserve_wire.cpp"),
           os.path.join(ROOT, "csrc/tests/wire_fuzz.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "wire fuzz ok" in r.stdout
