"""GraphRunner capture hygiene (pipelines/graph.py): the round-3 crash in
``torch.cuda.graphs.capture_end`` came from a step that forked work onto a
third stream without joining it back.  The runner must turn that — and a native
launch onto a stream outside the capture — into a clean GraphCaptureError.
Each case runs in a child process, so a crash fails the test instead of the
test runner."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = textwrap.dedent("""
    import sys, torch
    sys.path.insert(0, %r)
    from triton_client_amd import _native
    from triton_client_amd.pipelines.graph import GraphRunner, GraphCaptureError
    _native.kernels()
    x = torch.zeros(1 << 16, device="cuda")
    y = torch.zeros(1 << 16, device="cuda")
    side = torch.cuda.Stream()
""" % ROOT)


def _child(body: str):
    r = subprocess.run([sys.executable, "-c", PRELUDE + textwrap.dedent(body)], cwd=ROOT, capture_output=True,
                       text=True, timeout=240)
    return r.returncode, r.stdout + r.stderr


def test_unjoined_fork_raises_instead_of_crashing(cuda):
    rc, out = _child("""
        def step():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y.add_(1.0)          # forked, never joined back
            x.add_(1.0)
            return x
        g = GraphRunner(step)
        try:
            g.capture()
        except GraphCaptureError as e:
            print("CLEAN", e)
        torch.cuda.synchronize()
        # the runner is still usable afterwards: a correct step captures and replays
        def good():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y.add_(1.0)
            x.add_(2.0)
            main.wait_stream(side)
            return x
        x.zero_(); y.zero_()
        r = GraphRunner(good, warmup=1)
        r.capture()
        x.zero_(); y.zero_()
        for _ in range(3):
            r()
        torch.cuda.synchronize()
        print("GOOD", float(x[0]), float(y[0]))
    """)
    assert rc == 0, out[-3000:]
    assert "CLEAN" in out and "unjoined" in out, out[-3000:]
    assert "GOOD 6.0 3.0" in out, out[-3000:]


def test_native_launch_outside_the_capture_raises(cuda):
    rc, out = _child("""
        from triton_client_amd.ops.image import draw_boxes_
        f = torch.zeros((1, 16, 16, 3), dtype=torch.uint8, device="cuda")
        box = torch.tensor([[[1.0, 1.0, 8.0, 8.0]]], device="cuda")
        cls = torch.zeros((1, 1), dtype=torch.int32, device="cuda")
        cnt = torch.ones((1,), dtype=torch.int32, device="cuda")
        other = torch.cuda.Stream()
        def step():
            draw_boxes_(f, box, cls, cnt, 1, stream=other)   # explicit stream outside the capture
            return f
        try:
            GraphRunner(step, warmup=1).capture()
        except GraphCaptureError as e:
            print("CLEAN", e)
        torch.cuda.synchronize()
    """)
    assert rc == 0, out[-3000:]
    assert "CLEAN" in out and "not part of the graph" in out, out[-3000:]


def test_raw_unjoined_capture_outcome_is_recorded(cuda):
    """Root cause, as observed: plain torch.cuda.graph over an unjoined fork (no
    runner).  Whatever HIP does with it (error or crash), it must not succeed
    silently; the outcome is printed for the record (profiles/r4/)."""
    rc, out = _child("""
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                main = torch.cuda.current_stream()
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    y.add_(1.0)
                x.add_(1.0)
            print("ENDED_WITHOUT_ERROR")
        except Exception as e:
            print("RAISED", type(e).__name__, str(e)[:300])
    """)
    print(f"raw unjoined capture: rc={rc} tail={out[-600:]!r}")
    assert "ENDED_WITHOUT_ERROR" not in out or rc != 0
