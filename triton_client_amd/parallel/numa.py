"""CPU / NUMA affinity of a rank process: bind it to its GPU's host-side socket.

On an 8-GPU MI355X node every GPU hangs off one socket's PCIe root complex.  A
data-parallel rank moves ~20 GB/s of sensor payload per GPU (150 MB per 7.5 ms
step) through page-locked host memory and decodes its JPEGs on
host threads; both should run on the cores and memory of the GPU's own NUMA
node, not cross the socket interconnect.  :func:`bind_to_gpu` is called by
:func:`~triton_client_amd.parallel.dp.init_distributed` *before* the process's
first GPU call; it binds every thread the process already has
(``/proc/self/task``) and so every thread started later (decoder pools, copy
threads) and every pinned buffer first touched later inherits the binding.

The GPU's PCI function is found without touching the HIP runtime, in the order
the runtime enumerates agents:

1. the KFD topology (``/sys/class/kfd/kfd/topology/nodes/N``): GPU nodes are the
   ones with ``simd_count > 0``, in node order; ``domain`` + ``location_id``
   (bus << 8 | devfn) name the PCI function;
2. otherwise PCI sysfs: vendor 0x1002 functions of class 0x03xxxx (display) or
   0x12xxxx (processing accelerator — how Instinct parts enumerate), bus order.

``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` index lists filter that order.
The binding is the intersection of the device's ``local_cpulist`` with the CPUs
this process may already use (a container's cpuset is respected).  When that
changes nothing — a ``numa_node`` of -1 (firmware did not report locality, so
``local_cpulist`` is every CPU), or an empty intersection — nothing changes, and
:func:`describe` says why.  ``TCA_NUMA_BIND=0`` disables it.
"""
from __future__ import annotations

import glob
import logging
import os
from typing import Dict, List, Optional, Set

PCI = "/sys/bus/pci/devices"
KFD = "/sys/class/kfd/kfd/topology/nodes"

log = logging.getLogger("triton_client_amd.numa")


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


def _props(path: str) -> Dict[str, int]:
    out = {}
    for line in (_read(path) or "").splitlines():
        k, _, v = line.partition(" ")
        try:
            out[k] = int(v)
        except ValueError:
            pass
    return out


def kfd_gpus(kfd: str = KFD, pci: str = PCI) -> List[str]:
    """PCI device directories of the KFD GPU nodes, in node (= HSA agent) order."""
    nodes = []
    for d in glob.glob(os.path.join(kfd, "*")):
        name = os.path.basename(d)
        if not name.isdigit():
            continue
        p = _props(os.path.join(d, "properties"))
        if p.get("simd_count", 0) <= 0 or "location_id" not in p:
            continue
        loc, dom = p["location_id"], p.get("domain", 0)
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}"
        nodes.append((int(name), os.path.join(pci, bdf)))
    return [path for _, path in sorted(nodes)]


def amd_gpus(root: str = PCI) -> List[str]:
    """PCI device directories of AMD GPUs (vendor 0x1002, class 0x03xxxx display or
    0x12xxxx processing accelerator), bus order."""
    out = []
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if _read(os.path.join(d, "vendor")) != "0x1002":
            continue
        cls = _read(os.path.join(d, "class")) or ""
        if cls.startswith("0x03") or cls.startswith("0x12"):
            out.append(d)
    return out


def gpu_devices(root: str = PCI, kfd: str = KFD) -> List[str]:
    devs = kfd_gpus(kfd, root)
    return devs if devs else amd_gpus(root)


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


def gpu_pci(local_rank: int, root: str = PCI, kfd: str = KFD) -> Optional[str]:
    devs = gpu_devices(root, kfd)
    vis = _visible(len(devs))
    if not vis:
        return None
    return devs[vis[local_rank % len(vis)]]


def gpu_cpus(local_rank: int, root: str = PCI, kfd: str = KFD) -> Optional[Set[int]]:
    """CPUs local to the ``local_rank``-th visible GPU, or None."""
    d = gpu_pci(local_rank, root, kfd)
    text = _read(os.path.join(d, "local_cpulist")) if d else None
    return parse_cpulist(text) if text else None


def describe(local_rank: int, root: str = PCI, kfd: str = KFD) -> dict:
    """What :func:`bind_to_gpu` would do for ``local_rank`` and why (read-only)."""
    info = {"kfd_gpus": len(kfd_gpus(kfd, root)), "pci_gpus": len(amd_gpus(root)), "gpu_pci": None,
            "numa_node": None, "local_cpus": None, "allowed_cpus": None, "would_bind": None, "reason": ""}
    d = gpu_pci(local_rank, root, kfd)
    if d is None:
        info["reason"] = "no AMD GPU found in the KFD topology or PCI sysfs"
        return info
    info["gpu_pci"] = os.path.basename(d)
    nn = _read(os.path.join(d, "numa_node"))
    info["numa_node"] = int(nn) if nn not in (None, "") else None
    cpus = gpu_cpus(local_rank, root, kfd)
    allowed = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else set()
    info["allowed_cpus"] = len(allowed)
    if not cpus:
        info["reason"] = "the GPU's local_cpulist is unreadable"
        return info
    info["local_cpus"] = len(cpus)
    want = cpus & allowed
    if not want:
        info["reason"] = "the GPU's local CPUs are outside this process's cpuset"
    elif want == allowed:
        info["reason"] = ("numa_node -1: the firmware reports no locality (local_cpulist is every CPU)"
                          if info["numa_node"] == -1 else "this process already runs on the GPU's local CPUs only")
    else:
        info["would_bind"] = len(want)
        info["reason"] = f"bind to the {len(want)} CPUs of NUMA node {info['numa_node']}"
    return info


def _set_all_threads(cpus: Set[int]) -> int:
    """sched_setaffinity on every thread of this process; -> threads bound."""
    n = 0
    tids = [int(t) for t in os.listdir("/proc/self/task")] if os.path.isdir("/proc/self/task") else [0]
    for tid in tids:
        try:
            os.sched_setaffinity(tid, cpus)
            n += 1
        except OSError:  # the thread exited meanwhile
            pass
    return n


def bind_to_gpu(local_rank: int, root: str = PCI, kfd: str = KFD) -> Optional[Set[int]]:
    """Restrict this process (every thread it has, and so every thread it starts
    later) to its GPU's local CPUs (see the module doc); returns the CPU set applied,
    or None when nothing changed (logged with the reason)."""
    if os.environ.get("TCA_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    try:
        info = describe(local_rank, root, kfd)
        if not info["would_bind"]:
            log.info("rank %d: no CPU binding (%s)", local_rank, info["reason"])
            return None
        want = gpu_cpus(local_rank, root, kfd) & os.sched_getaffinity(0)
        threads = _set_all_threads(want)
        log.info("rank %d: GPU %s, NUMA node %s: bound %d threads to %d CPUs", local_rank, info["gpu_pci"],
                 info["numa_node"], threads, len(want))
        return want
    except (OSError, ValueError):
        return None
