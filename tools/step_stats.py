#!/usr/bin/env python3
"""Per-step, setup-excluded kernel summary of a rocprofv3 kernel-trace CSV.

A *step* starts at a launch of the marker kernel (default ``pc2_count`` for a
LiDAR run, use ``prep_`` for a camera-only run).  The first ``--skip`` marked
steps (setup, calibration, warm-up) are dropped and the last ``--steps``
complete steps are aggregated: per kernel, calls and µs per step, share of the
kernels' summed time, plus each step's wall span (first start → next marker).

    python tools/step_stats.py trace.csv --marker pc2_count --steps 5 [--top 40]
"""
import argparse
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kernel_stats import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="pc2_count")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sequence", action="store_true",
                    help="also list the last step's dispatches in launch order (duration, grid, kernel)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit(f"marker {a.marker!r} launched {len(idx)} times")
    n = min(a.steps, len(idx) - 1)
    starts = idx[-(n + 1):]
    tot, cnt = defaultdict(float), defaultdict(int)
    spans = []
    for s, e in zip(starts[:-1], starts[1:]):
        spans.append((int(rows[e]["Start_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e3)
        for r in rows[s:e]:
            k = short(r["Kernel_Name"])
            tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
    ksum = sum(tot.values()) / n
    # GPU-busy time: the union of the step's kernel intervals (any kernel running), and the
    # idle gaps (no kernel on the device at all) inside the step
    busy = []
    for s, e in zip(starts[:-1], starts[1:]):
        t_end = int(rows[e]["Start_Timestamp"])
        iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t_end)) for r in rows[s:e])
        u, cs, ce = 0, None, None
        for b_, e_ in iv:
            if cs is None or b_ > ce:
                if cs is not None:
                    u += ce - cs
                cs, ce = b_, e_
            else:
                ce = max(ce, e_)
        if cs is not None:
            u += ce - cs
        busy.append(u / 1e3)
    print(f"# {n} steps (marker {a.marker!r}); step span mean {sum(spans) / n:.1f} us "
          f"(min {min(spans):.1f}, max {max(spans):.1f}); kernel time sum {ksum:.1f} us/step; "
          f"GPU busy (union of kernels) {sum(busy) / n:.1f} us/step = {100 * sum(busy) / sum(spans):.1f}% of the span")
    print(f"{'us/step':>9} {'share':>6} {'calls':>6}  kernel")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
        print(f"{v / n:9.1f} {100 * v / n / ksum:5.1f}% {cnt[k] / n:6.1f}  {k}")
    if a.sequence:
        s, e = starts[-2], starts[-1]
        t0 = int(rows[s]["Start_Timestamp"])
        print(f"\n# last step in launch order (start / end: us from the marker's start; q: queue)\n"
              f"{'#':>4} {'us':>8} {'start':>8} {'end':>8} {'q':>3} {'grid':>10}  kernel")
        for i, r in enumerate(rows[s:e]):
            b_, e_ = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
            q = r.get("Queue_Id", "")
            print(f"{i:4d} {(e_ - b_) / 1e3:8.1f} {b_ / 1e3:8.1f} {e_ / 1e3:8.1f} {q:>3} {grid:>10}  "
                  f"{short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
