"""NUMA binding on the real MI355X box: the GPU is found in the KFD topology (or
PCI sysfs, Instinct class 0x12), and either the binding shrinks the CPU set to the
GPU's socket or the reason it cannot is reported (e.g. numa_node -1).  Reading
sysfs is a CPU read; the binding itself runs in a child process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, os
from triton_client_amd.parallel import numa
allowed = set(os.sched_getaffinity(0))
local = numa.gpu_cpus(0)
before = len(allowed)
info = numa.describe(0)
got = numa.bind_to_gpu(0)
after = set(os.sched_getaffinity(0))
print(json.dumps({"info": info, "before": before, "after": len(after),
                  "applied": None if got is None else len(got),
                  "already_local": local is not None and allowed <= local,
                  "after_local": local is not None and after <= local}))
"""


def test_numa_binding_on_the_box(cuda):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("TCA_NUMA_BIND", None)
    out = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(r))
    keep = os.environ.get("GRAFT_REPO_ROOT")
    if keep:  # the box's answer, kept with the run's outputs
        os.makedirs(os.path.join(keep, "gpurun_out"), exist_ok=True)
        with open(os.path.join(keep, "gpurun_out", "numa_describe.json"), "w") as f:
            json.dump(r, f, indent=1)
    info = r["info"]
    assert info["kfd_gpus"] + info["pci_gpus"] > 0 and info["gpu_pci"], r
    if info["would_bind"]:
        assert r["applied"] == r["after"] == info["would_bind"] < r["before"], r
    else:
        assert r["after"] == r["before"] and info["reason"], r
    if info["numa_node"] is not None and info["numa_node"] >= 0:
        # a GPU with a NUMA node: afterwards the process runs on that node's CPUs only -- by a
        # shrink, or because its cpuset was already inside them (checked on the sets, not a string)
        assert r["after_local"], r
        assert r["after"] < r["before"] or r["already_local"], r
