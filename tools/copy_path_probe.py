"""Which copy path does the HIP runtime take for each kind of source the served models copy from?

The served-path trace (profiles/r5/served/trace_summary_final.txt) shows 1,801 blit-kernel copies
(``__amd_rocclr_copyBuffer``, 111 us each) in the server beside its SDMA copies.  This issues each
kind of copy the server's plans issue, with a distinct size per kind so a kernel / copy trace names
them:

  A  torch pinned (hipHostMalloc) -> device            (the plans' own pinned staging)
  B  hipHostRegister'd /dev/shm mapping -> device      (a system shared-memory request input, _direct)
  C  plain pageable numpy -> device
  D  device -> device (torch copy_)
  E  device -> hipHostRegister'd /dev/shm mapping       (a system shared-memory output slice)
  F  device -> torch pinned

    python tools/copy_path_probe.py   (device events per kind via torch.profiler; a rocprofv3 run crashed at exit)
"""
import mmap
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SIZES = {"A": 3 << 20, "B": (3 << 20) + 4096, "C": (3 << 20) + 8192, "D": (3 << 20) + 12288,
         "E": (3 << 20) + 16384, "F": (3 << 20) + 20480}


def _device_events(fn) -> dict:
    """Names of the device-side events one call of ``fn`` produces (blit kernel vs DMA copy), via torch.profiler:
    in-process, so nothing depends on the tracer's exit path."""
    from torch.profiler import ProfilerActivity, profile

    try:
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            fn()
            torch.cuda.synchronize()
    except Exception as e:  # profiler unavailable: the timings still stand
        return {"error": repr(e)}
    names = {}
    for ev in prof.events():
        if getattr(ev, "device_type", None) is not None and "CUDA" in str(ev.device_type):
            names[ev.name] = names.get(ev.name, 0) + 1
    return names


def main() -> int:
    from triton_client_amd.server.shm import _host_register

    reps = int(os.environ.get("REPS", "20"))
    dev = torch.device("cuda:0")
    path = f"/dev/shm/tca_copyprobe_{os.getpid()}"
    total = 1 << 26
    fd = os.open(path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
    os.ftruncate(fd, total)
    mm = mmap.mmap(fd, total, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    reg = _host_register(mm, total)
    shm = np.frombuffer(mm, np.uint8)
    out = {"registered": bool(reg)}
    src_b = dst_e = None
    try:
        d = {k: torch.empty(v, dtype=torch.uint8, device=dev) for k, v in SIZES.items()}
        pin = {k: torch.empty(SIZES[k], dtype=torch.uint8).pin_memory() for k in "AF"}
        page = np.zeros(SIZES["C"], np.uint8)
        src_b = torch.from_numpy(shm[:SIZES["B"]])
        dst_e = torch.from_numpy(shm[1 << 25:(1 << 25) + SIZES["E"]])
        d2 = torch.empty(SIZES["D"], dtype=torch.uint8, device=dev)
        kinds = {
            "A": lambda: d["A"].copy_(pin["A"], non_blocking=True),
            "B": lambda: d["B"].copy_(src_b, non_blocking=True),
            "C": lambda: d["C"].copy_(torch.from_numpy(page), non_blocking=True),
            "D": lambda: d2.copy_(d["D"], non_blocking=True),
            "E": lambda: dst_e.copy_(d["E"], non_blocking=True),
            "F": lambda: pin["F"].copy_(d["F"], non_blocking=True),
        }
        for k, fn in kinds.items():
            fn()
            torch.cuda.synchronize()
            out.setdefault("device_events", {})[k] = _device_events(fn)
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            out[k] = {"bytes": SIZES[k], "us": round(dt * 1e6, 1), "GBps": round(SIZES[k] / dt / 1e9, 1)}
            print(k, out[k], flush=True)
    finally:
        torch.cuda.synchronize()
        if reg:  # unregister before the mapping goes: the runtime's exit path walks registered ranges
            torch.cuda.cudart().cudaHostUnregister(int(shm.ctypes.data))
        del src_b, dst_e, shm
        try:
            mm.close()
        except BufferError:
            pass
        os.unlink(path)
    import json
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
