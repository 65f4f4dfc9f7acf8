#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV from ``--kernel-trace`` or
``rocpd2csv``): per-kernel call count, total / mean µs, share of GPU time.

    python tools/kernel_stats.py trace.csv [--top 30] [--per-step N]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)  # drop argument lists
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"<.*>", lambda m: "<" + m.group(0)[1:60] + ("…>" if len(m.group(0)) > 62 else ""), n)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--per-step", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    tot, cnt = defaultdict(float), defaultdict(int)
    with open(a.csv) as f:
        r = csv.DictReader(f)
        for row in r:
            name = row.get("Kernel_Name") or row.get("KernelName") or row.get("kernel_name") or row.get("Name")
            s = row.get("Start_Timestamp") or row.get("BeginNs") or row.get("start")
            e = row.get("End_Timestamp") or row.get("EndNs") or row.get("end")
            if name is None or s is None or e is None:
                continue
            k = short(name)
            tot[k] += (int(e) - int(s)) / 1e3
            cnt[k] += 1
    all_us = sum(tot.values())
    div = a.per_step or 1
    print(f"total GPU kernel time {all_us / 1e3:.3f} ms" + (f" ({all_us / div / 1e3:.3f} ms/step over {div} steps)"
                                                           if a.per_step else ""))
    print(f"{'kernel':112s} {'calls':>7s} {'total_us':>11s} {'mean_us':>9s} {'share':>6s}")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
        print(f"{k:112s} {cnt[k]:7d} {v / div:11.1f} {v / cnt[k]:9.2f} {100 * v / all_us:5.1f}%")


if __name__ == "__main__":
    main()
