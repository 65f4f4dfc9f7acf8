"""Device-to-device copy rates from another process's memory mapped with hipIpcOpenMemHandle (the devshm
wire's server side) against the same copy from this process's own memory, plus a kernel that reads each.

    python tools/ipc_copy_probe.py [--mib 8] [--reps 50]

The parent starts the reader process before it touches the GPU (no fork of a GPU-initialised process),
then allocates the buffer, fills it and sends the 64-byte handle over the child's stdin."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def reader(nbytes: int, reps: int) -> int:
    import torch

    from triton_client_amd.utils.hip_ipc import OpenedHandle

    h = bytes.fromhex(sys.stdin.readline().strip())
    dev = torch.device("cuda", 0)
    opened = OpenedHandle(h, nbytes, 0)
    ipc = opened.tensor
    own = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    own.copy_(ipc)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    res = {"mib": nbytes / 2**20, "reps": reps, "checksum_match": bool(torch.equal(own, ipc))}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        return {"ms": round(ms, 4), "GB_s": round(nbytes / ms / 1e6, 1)}

    res["copy_from_ipc"] = timed(lambda: dst.copy_(ipc))
    res["copy_from_own"] = timed(lambda: dst.copy_(own))
    res["copy_into_ipc"] = timed(lambda: ipc.copy_(own))
    f_ipc, f_own = ipc.view(torch.float32), own.view(torch.float32)
    res["kernel_read_ipc"] = timed(lambda: f_ipc.sum())
    res["kernel_read_own"] = timed(lambda: f_own.sum())
    opened.close()
    print(json.dumps(res), flush=True)
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--reader", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    nbytes = a.mib << 20
    if a.reader:
        return reader(nbytes, a.reps)
    child = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--reader", "--mib", str(a.mib),
                              "--reps", str(a.reps)], stdin=subprocess.PIPE, text=True)
    import torch

    from triton_client_amd.utils.hip_ipc import DeviceAllocation

    alloc = DeviceAllocation(nbytes, "cuda:0")
    alloc.tensor.copy_(torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda:0"))
    torch.cuda.synchronize()
    child.stdin.write(alloc.handle.hex() + "\n")
    child.stdin.flush()
    rc = child.wait(120)
    alloc.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
