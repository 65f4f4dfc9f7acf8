"""In-tree native build: hipcc (gfx950) → shared libraries under
``triton_client_amd/_lib`` (git-ignored, but they travel to the GPU box with
the repo snapshot).

* ``libtca_kernels.so`` — every ``csrc/kernels/*.hip`` (the HIP kernels and
  their C-ABI launchers).
* ``libtca_runtime.so`` — ``csrc/runtime/*.cpp`` host runtime (KServe wire
  codec, pinned staging pool, RCCL communicator, bag I/O) built with hipcc
  so it can call the HIP runtime and RCCL directly.

No torch headers are involved, so a full rebuild is a few seconds per file
and the libraries are loaded with ``ctypes`` (``triton_client_amd._native``).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import json
import os
import shutil
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "triton_client_amd", "_lib")
BUILDDIR = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("TCA_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"-I{os.path.join(CSRC, 'include')}", "-Wno-unused-result"]
KERNEL_FLAGS = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]


def _headers() -> List[str]:
    return glob.glob(os.path.join(CSRC, "include", "*.h"))


def _stale(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed: {' '.join(cmd)}\n{r.stdout}")


def _compile(src: str, obj: str, flags: List[str]) -> str:
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    _run([HIPCC, *COMMON_FLAGS, *flags, "-c", src, "-o", obj])
    return obj


def _stamp_changed(name: str, flags: List[str], link: List[str]) -> bool:
    """mtimes alone would reuse objects built for another arch / flag set (e.g.
    host objects copied into an image): the compiler, arch and flags of the
    last build are kept in a stamp next to the objects; any change rebuilds."""
    want = json.dumps({"hipcc": HIPCC, "arch": ARCH, "common": COMMON_FLAGS, "flags": flags, "link": link},
                      sort_keys=True)
    stamp = os.path.join(BUILDDIR, name + ".stamp")
    try:
        with open(stamp) as f:
            same = f.read() == want
    except OSError:
        same = False
    if not same:
        os.makedirs(BUILDDIR, exist_ok=True)
        with open(stamp, "w") as f:
            f.write(want)
    return not same


LAST = {}  # what the last build() did: compiled objects and relinked libraries (build provenance)


def _build_lib(name: str, sources: List[str], flags: List[str], link: List[str], jobs: int, force: bool) -> str:
    out = os.path.join(LIBDIR, name)
    force = _stamp_changed(name, flags, link) or force
    hdrs = _headers()
    objs = []
    todo = []
    for s in sources:
        o = os.path.join(BUILDDIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s, *hdrs]):
            todo.append((s, o))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda so: _compile(so[0], so[1], flags), todo))
    relinked = bool(force or todo or _stale(out, objs))
    if relinked:
        os.makedirs(LIBDIR, exist_ok=True)
        tmp = out + ".tmp"
        _run([HIPCC, "-shared", *flags, "-o", tmp, *objs, *link])
        os.replace(tmp, out)
    LAST[name] = {"compiled": [os.path.relpath(s_, ROOT) for s_, _ in todo], "sources": len(sources),
                  "relinked": relinked, "forced": bool(force)}
    return out


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> List[str]:
    jobs = jobs or min(8, os.cpu_count() or 4)
    kern = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    rt = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    outs = [_build_lib("libtca_kernels.so", kern, KERNEL_FLAGS, [], jobs, force)]
    if rt:
        rccl_link = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        outs.append(_build_lib("libtca_runtime.so", rt, ["-D__HIP_PLATFORM_AMD__"], rccl_link, jobs, force))
    if verbose:
        for o in outs:
            print(f"[tca-build] {os.path.relpath(o, ROOT)} ({os.path.getsize(o) // 1024} KiB)", file=sys.stderr)
    _write_provenance(outs)
    return outs


def _write_provenance(outs: List[str]) -> dict:
    """build/native/last_build.json: arch, compiler, which sources this build compiled,
    whether each library was relinked, and each library's sha256 (what the tests load)."""
    import hashlib
    import time

    rec = {"time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "arch": ARCH, "hipcc": HIPCC,
           "libs": {}}
    for o in outs:
        name = os.path.basename(o)
        with open(o, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        rec["libs"][name] = dict(LAST.get(name, {}), sha256=digest, bytes=os.path.getsize(o))
    rec["build_mode"] = ("full" if all(v.get("forced") for v in rec["libs"].values()) else
                         "incremental" if any(v.get("compiled") for v in rec["libs"].values()) else "up-to-date")
    os.makedirs(BUILDDIR, exist_ok=True)
    with open(os.path.join(BUILDDIR, "last_build.json"), "w") as f:
        json.dump(rec, f, indent=1)
    return rec


if __name__ == "__main__":
    build(force="--force" in sys.argv)
