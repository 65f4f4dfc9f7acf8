"""CPU / NUMA affinity of a rank process: bind it to its GPU's host-side socket.

On an 8-GPU MI355X node every GPU hangs off one socket's PCIe root complex.  A
data-parallel rank moves ~20 GB/s of sensor payload per GPU (150 MB per 7.5 ms
step) through page-locked host memory and decodes its JPEGs on
host threads; both should run on the cores and memory of the GPU's own NUMA
node, not cross the socket interconnect.  :func:`bind_to_gpu` is called by
:func:`~triton_client_amd.parallel.dp.init_distributed` *before* the process's
first GPU call, so every thread it later starts (decoder pools, copy threads)
and every pinned buffer it first touches inherit the binding.

The GPU's PCI function is found through sysfs without touching the HIP
runtime: AMD display / accelerator functions (vendor 0x1002, PCI class 0x03)
in bus order — the order the runtime enumerates them — filtered by
``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` when those list indices.
The binding is the intersection of the device's ``local_cpulist`` with the
CPUs this process may already use (a container's cpuset is respected); if that
is empty, or anything is unreadable, nothing changes.  ``TCA_NUMA_BIND=0``
disables it.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional, Set

PCI = "/sys/bus/pci/devices"


def parse_cpulist(text: str) -> Set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    out: Set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def amd_gpus(root: str = PCI) -> List[str]:
    """PCI device directories of AMD GPUs (vendor 0x1002, class 0x03xxxx), bus order."""
    out = []
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if _read(os.path.join(d, "vendor")) != "0x1002":
            continue
        cls = _read(os.path.join(d, "class")) or ""
        if cls.startswith("0x03"):
            out.append(d)
    return out


def _visible(n: int) -> List[int]:
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                idx = [int(x) for x in v.split(",") if x.strip()]
            except ValueError:  # UUIDs: no index mapping from sysfs alone
                return list(range(n))
            return [i for i in idx if 0 <= i < n]
    return list(range(n))


def gpu_cpus(local_rank: int, root: str = PCI) -> Optional[Set[int]]:
    """CPUs local to the ``local_rank``-th visible GPU, or None."""
    devs = amd_gpus(root)
    vis = _visible(len(devs))
    if not vis:
        return None
    d = devs[vis[local_rank % len(vis)]]
    text = _read(os.path.join(d, "local_cpulist"))
    return parse_cpulist(text) if text else None


def bind_to_gpu(local_rank: int, root: str = PCI) -> Optional[Set[int]]:
    """Restrict this process to its GPU's local CPUs (see the module doc);
    returns the CPU set applied, or None when nothing changed."""
    if os.environ.get("TCA_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    try:
        cpus = gpu_cpus(local_rank, root)
        if not cpus:
            return None
        allowed = os.sched_getaffinity(0)
        want = cpus & allowed
        if not want or want == allowed:
            return None
        os.sched_setaffinity(0, want)
        return want
    except (OSError, ValueError):
        return None
