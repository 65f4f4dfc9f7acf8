#!/usr/bin/env python3
"""One row per kernel from rocprofv3 --pmc counter CSVs (tools/gpu_pmc_cmd.sh passes): dispatches, time,
MFMA busy, approximate HBM bandwidth and LDS bank conflicts -- the per-kernel roofline check.

    python tools/pmc_table.py <csv> [<csv> ...] [--min-us 5] [--only substr,substr]

Time = GRBM_GUI_ACTIVE / 8 XCDs / 2.4 GHz.  MFMA busy as tools/pmc_summary.py.  HBM bytes =
(TCC_EA0_RDREQ_sum + TCC_EA0_WRREQ_sum) x 64 B (the request size is not counted separately, so
this is an estimate).  The check column: >= 30% MFMA busy or >= 60% of 8 TB/s.
"""
import csv
import sys
from collections import defaultdict

CLK = 2.4e9


def main():
    args = sys.argv[1:]
    min_us = 5.0
    only = None
    if "--only" in args:
        i = args.index("--only")
        only = args[i + 1].split(",")
        del args[i:i + 2]
    if "--min-us" in args:
        i = args.index("--min-us")
        min_us = float(args[i + 1])
        del args[i:i + 2]
    vals = defaultdict(lambda: defaultdict(list))
    for fn in args:
        with open(fn) as f:
            for row in csv.DictReader(f):
                vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    rows = []
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "GRBM_GUI_ACTIVE" not in m:
            continue
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        us = cyc / CLK * 1e6
        if us < min_us:
            continue
        n = max(len(v) for v in cs.values())
        mfma = 100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc) if "SQ_VALU_MFMA_BUSY_CYCLES" in m else None
        hbm = None
        if "TCC_EA0_RDREQ_sum" in m and "TCC_EA0_WRREQ_sum" in m:
            hbm = (m["TCC_EA0_RDREQ_sum"] + m["TCC_EA0_WRREQ_sum"]) * 64 / (us * 1e-6) / 1e12
        ok = (mfma is not None and mfma >= 30) or (hbm is not None and hbm >= 4.8)
        name = k.replace("(anonymous namespace)::", "").removeprefix("void ")
        name = name.split("(")[0][:70]
        if only and not any(o in name for o in only):
            continue
        rows.append((us, name, n, mfma, hbm, m.get("SQ_LDS_BANK_CONFLICT"), ok))
    rows.sort(reverse=True)
    print("| kernel | dispatches (pass 1) | µs / dispatch | MFMA busy | HBM TB/s (est.) | LDS conflicts | >= 30% MFMA or >= 60% HBM |")
    print("|---|---|---|---|---|---|---|")
    for us, name, n, mfma, hbm, cf, ok in rows:
        f = lambda v, fmt: "-" if v is None else fmt.format(v)  # noqa: E731
        print(f"| `{name}` | {n} | {us:.1f} | {f(mfma, '{:.1f}%')} | {f(hbm, '{:.2f}')} | {f(cf, '{:,.0f}')} | "
              f"{'yes' if ok else 'no'} |")


if __name__ == "__main__":
    main()
