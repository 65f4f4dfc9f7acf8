#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs of one kernel (tools/gpu_conv_pmc.sh
passes) into per-dispatch means and derived metrics.

    python tools/pmc_summary.py <kernel-substring> <csv> [<csv> ...]

Derived (MI355X: 256 CUs x 4 SIMDs in 8 XCDs; GRBM_GUI_ACTIVE is summed over
the 8 XCDs, so the kernel's cycles are GRBM_GUI_ACTIVE / 8):
  MFMA busy   SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)
  VALU / MFMA non-MFMA VALU instructions per MFMA instruction
  wave time   waiting (SQ_WAIT_ANY) / issue-stalled (SQ_WAIT_INST_ANY) / issuing
              (SQ_ACTIVE_INST_ANY), shares of SQ_WAVE_CYCLES
  L2 hit      TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import csv
import sys
from collections import defaultdict


def main():
    kern, files = sys.argv[1], sys.argv[2:]
    vals = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if kern in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        sys.exit(f"no dispatch of a kernel matching {kern!r}")
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    print(f"| counter | mean per dispatch |\n|---|---|")
    for k in sorted(m):
        print(f"| {k} | {m[k]:,.0f} |")
    d = []
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        d.append(f"MFMA busy: {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.1f}%")
    if "SQ_INSTS_VALU" in m and m.get("SQ_INSTS_MFMA"):
        d.append(f"non-MFMA VALU per MFMA: {(m['SQ_INSTS_VALU'] - m['SQ_INSTS_MFMA']) / m['SQ_INSTS_MFMA']:.2f}")
    if all(k in m for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES")):
        w = m["SQ_WAVE_CYCLES"]
        d.append(f"wave time: waiting {100 * m['SQ_WAIT_ANY'] / w:.0f}%, issue-stalled "
                 f"{100 * m['SQ_WAIT_INST_ANY'] / w:.0f}%, issuing {100 * m['SQ_ACTIVE_INST_ANY'] / w:.0f}%")
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        d.append(f"L2 hit: {100 * m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.1f}%")
    if "SQ_LDS_BANK_CONFLICT" in m:
        d.append(f"LDS bank conflicts: {m['SQ_LDS_BANK_CONFLICT']:,.0f}")
    print("\nDerived:\n" + "\n".join(f"- {x}" for x in d))


if __name__ == "__main__":
    main()
