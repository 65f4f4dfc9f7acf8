"""Where do a served run's blit-kernel copies (``__amd_rocclr_copyBuffer``) come from?  Joins each
copyBuffer dispatch of a rocprofv3 kernel trace to the HIP API call that issued it (same
Correlation_Id in the hip-runtime trace) and groups them by (process, API function, grid size):
the grid size is proportional to the bytes the blit moves, so it tells the camera frame, the
voxel tensor and the YOLO output apart.

    python tools/copybuffer_origin.py <trace dir from tools/gpu_served_trace.sh with HIP=1>
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _grid(r) -> int:
    for k in ("Grid_Size", "Grid_Size_X"):
        if k in r and r[k]:
            return int(r[k])
    return -1


def main(argv=None) -> int:
    d = (argv or sys.argv[1:])[0]
    groups = defaultdict(lambda: [0, 0])
    for kp in sorted(glob.glob(os.path.join(d, "*_kernel_trace.csv"))):
        pid = os.path.basename(kp).split("_")[0]
        hp = kp.replace("_kernel_trace.csv", "_hip_api_trace.csv")
        api = {r["Correlation_Id"]: r["Function"] for r in _rows(hp)} if os.path.exists(hp) else {}
        for r in _rows(kp):
            if "copyBuffer" not in r["Kernel_Name"]:
                continue
            key = (pid, api.get(r["Correlation_Id"], "?"), r["Kernel_Name"], _grid(r))
            groups[key][0] += 1
            groups[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"{'pid':>8} {'calls':>6} {'mean us':>8} {'grid':>10}  api / kernel")
    for (pid, fn, kn, g), (n, t) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        print(f"{pid:>8} {n:6d} {t / n / 1e3:8.1f} {g:10d}  {fn} / {kn[:40]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
