#!/usr/bin/env python3
"""Scalar vs vector instruction mix per kernel from one rocprofv3 --pmc pass (SQ_WAVES SQ_INSTS_VALU
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES):
a CU has one scalar unit for its 32 waves, so a kernel issuing more SALU than VALU instructions can
be bound by it (the PillarVFE was: profiles/r6/vfe_pmc/).

    python tools/salu_table.py <counter_collection.csv> [--min-waves 64]
"""
import csv
import sys
from collections import defaultdict


def _short(name: str) -> str:
    """'void (anonymous namespace)::conv_wino_kernel<4, 4, 2, true, false, false>(float const*, ...)' ->
    'conv_wino_kernel<4, 4, 2, true, false, false>' (splitting at the first '(' kept only 'void ')."""
    for p in ("void ", "(anonymous namespace)::"):
        name = name.replace(p, "")
    depth = 0
    for i, c in enumerate(name):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0:
            return name[:i][:80]
    return name[:80]


def main():
    args = sys.argv[1:]
    min_waves = 64
    if "--min-waves" in args:
        i = args.index("--min-waves")
        min_waves = int(args[i + 1])
        del args[i:i + 2]
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in args:
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = _short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    rows = []
    for k, v in vals.items():
        n = max(1, len(disp[k]))
        if v.get("SQ_WAVES", 0) / n < min_waves:
            continue
        valu, salu = v.get("SQ_INSTS_VALU", 0), v.get("SQ_INSTS_SALU", 0)
        rows.append((salu / max(valu, 1), k, n, valu / n, salu / n, v.get("SQ_INSTS_SMEM", 0) / n,
                     v.get("SQ_ACTIVE_INST_SCA", 0) / max(v.get("SQ_ACTIVE_INST_VALU", 1), 1)))
    print("| kernel | dispatches | VALU / dispatch | SALU / dispatch | SMEM / dispatch | SALU / VALU | active SCA / VALU |")
    print("|---|---|---|---|---|---|---|")
    for ratio, k, n, valu, salu, smem, act in sorted(rows, reverse=True):
        print(f"| {k} | {n} | {valu:,.0f} | {salu:,.0f} | {smem:,.0f} | {ratio:.2f} | {act:.2f} |")


if __name__ == "__main__":
    main()
