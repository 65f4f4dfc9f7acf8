"""Print the last N kernels of a rocprofv3 kernel-trace CSV with start/end
offsets (µs) and queue: shows how a replayed step's branches overlap."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']:>3} {r['Kernel_Name'][:80]}")
