#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 ``--kernel-trace`` database (the default
rocpd SQLite output, ``<dir>/<name>_results.db``): calls, total / mean µs,
share of GPU time, plus VGPR / AGPR / LDS of each kernel.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 40] [--per-step N]
"""
import argparse
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kernel_stats import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--per-step", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tot, cnt, res = defaultdict(float), defaultdict(int), {}
    for name, dur, vg, ag, lds in c.execute(
            "select name, duration, vgpr_count, accum_vgpr_count, lds_size from kernels"):
        k = short(name)
        tot[k] += dur / 1e3
        cnt[k] += 1
        res[k] = (vg, ag, lds)
    all_us = sum(tot.values())
    div = a.per_step or 1
    print(f"total GPU kernel time {all_us / 1e3:.3f} ms" + (f" ({all_us / div / 1e3:.3f} ms/step over {div} steps)"
                                                           if a.per_step else ""))
    print(f"{'kernel':112s} {'calls':>7s} {'total_us':>11s} {'mean_us':>9s} {'share':>6s} {'vgpr':>5s} {'agpr':>5s} "
          f"{'lds':>7s}")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
        vg, ag, lds = res[k]
        print(f"{k:112s} {cnt[k]:7d} {v / div:11.1f} {v / cnt[k]:9.2f} {100 * v / all_us:5.1f}% {vg:5d} {ag:5d} "
              f"{lds:7d}")


if __name__ == "__main__":
    main()
