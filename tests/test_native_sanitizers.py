"""Host-side sanitizer run of the native runtime.

The KServe wire codec (csrc/runtime/kserve_wire.cpp), the JPEG entropy decoder
(jpeg_entropy.cpp) and the host preprocess (cpu_image.cpp) are compiled
together with fuzz / round-trip drivers under AddressSanitizer +
UndefinedBehaviorSanitizer (the decoder's thread pool also under
ThreadSanitizer) and run: malformed, truncated and length-inflated inputs
must be rejected without any out-of-bounds access or data race.  The RCCL
communicator wrappers (rccl_comm.cpp: grouped p2p plan building and every
argument check) are built against host-only stand-ins of the RCCL / HIP
headers (csrc/tests/rccl_stub/) whose entry points record each call and touch
exactly the bytes a real transfer would, so a wrong element count or dtype is
a heap overflow under ASan.  GPU ASan / XNACK are not available on the
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


def _jpeg_files(tmp_path):
    import io

    from PIL import Image

    from triton_client_amd.utils.synthetic import camera_frame

    files = []
    for i, kw in enumerate([dict(subsampling=2), dict(subsampling=1, restart_marker_blocks=3), dict(subsampling=0)]):
        buf = io.BytesIO()
        Image.fromarray(camera_frame(72, 104, seed=i)).save(buf, format="JPEG", quality=85, **kw)
        p = tmp_path / f"f{i}.jpg"
        p.write_bytes(buf.getvalue())
        files.append(str(p))
    buf = io.BytesIO()
    Image.fromarray(camera_frame(72, 104, seed=9)).convert("L").save(buf, format="JPEG")
    (tmp_path / "g.jpg").write_bytes(buf.getvalue())
    return files + [str(tmp_path / "g.jpg")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_jpeg_decoder_and_preprocess_under_sanitizers(tmp_path, san):
    exe = str(tmp_path / "jpeg_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           os.path.join(ROOT, "csrc/runtime/jpeg_entropy.cpp"), os.path.join(ROOT, "csrc/runtime/cpu_image.cpp"),
           os.path.join(ROOT, "csrc/tests/jpeg_fuzz.cpp"), "-o", exe]
    if san != "thread":
        cmd.insert(5, "-fno-sanitize-recover=undefined")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "300" if san == "thread" else "2000", *_jpeg_files(tmp_path)], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "jpeg fuzz ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_rccl_plan_building_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "rccl_plan_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "csrc/tests/rccl_stub"),
           os.path.join(ROOT, "csrc/runtime/rccl_comm.cpp"), os.path.join(ROOT, "csrc/tests/rccl_plan_fuzz.cpp"),
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "rccl plan fuzz ok" in r.stdout
