"""Summarise a served-path trace (tools/gpu_served_trace.sh: rocprofv3 kernel + memory-copy
traces of the server and every client process): per process, kernel / copy time and the
union of its GPU activity over the busiest window, plus the server's top kernels and copy
durations by direction.

    python tools/served_trace_summary.py gpurun_out/r5/srvtrace [--server PID]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("dir")
    ap.add_argument("--server", default=None, help="server PID (default: the process with the most kernels)")
    a = ap.parse_args(argv)
    procs = {}
    for kp in glob.glob(os.path.join(a.dir, "*_kernel_trace.csv")):
        pid = os.path.basename(kp).split("_")[0]
        cp = kp.replace("_kernel_trace.csv", "_memory_copy_trace.csv")
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in _rows(kp)]
        cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]) for r in _rows(cp)] \
            if os.path.exists(cp) else []
        procs[pid] = (ks, cs)
    server = a.server or max(procs, key=lambda p: len(procs[p][0]))
    sk, sc = procs[server]
    # the window: from the clients' first to last GPU activity (their device preprocess / post and
    # copies: the timed run, without the server's model build and calibration)
    cl = [x for p, (ks, cs) in procs.items() if p != server for x in ks + cs]
    t0, t1 = min(x[0] for x in cl), max(x[1] for x in cl)
    win = t1 - t0

    def clip(iv):
        return [(max(s, t0), min(e, t1)) for s, e, *_ in iv if e > t0 and s < t1]
    print(f"window: {win / 1e6:.1f} ms (the clients' first to last GPU activity; server {server})")
    allact = []
    print(f"{'pid':>8} {'role':>7} {'kernels':>8} {'k_busy%':>8} {'copies':>7} {'c_busy%':>8} {'union%':>7}")
    for pid, (ks, cs) in sorted(procs.items()):
        kc, cc = clip(ks), clip(cs)
        allact += kc + cc
        role = "server" if pid == server else "client"
        print(f"{pid:>8} {role:>7} {len(kc):8d} {100 * _union(kc) / win:8.1f} {len(cc):7d} {100 * _union(cc) / win:8.1f} "
              f"{100 * _union(kc + cc) / win:7.1f}")
    print(f"GPU busy (every process's kernels and copies): {100 * _union(allact) / win:.1f}% of the window")
    per = defaultdict(lambda: [0, 0])
    for s, e, n in sk:
        if e > t0 and s < t1:
            per[n][0] += 1
            per[n][1] += e - s
    print("server top kernels (us total, calls):")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {t / 1e3:9.1f} {c:6d}  {n[:90]}")
    byd = defaultdict(list)
    for s, e, d in sc:
        if e > t0 and s < t1:
            byd[d].append(e - s)
    print("server copies by direction (count, total ms, median us):")
    for d, v in sorted(byd.items()):
        v.sort()
        print(f"  {d:40s} {len(v):6d} {sum(v) / 1e6:9.2f} {v[len(v) // 2] / 1e3:9.1f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
