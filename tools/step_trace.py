"""Print the kernels of one bench step from a rocprofv3 kernel-trace CSV.

usage: python tools/step_trace.py <run_kernel_trace.csv> [marker-kernel-substring]
The step is the span between the last two launches of the marker kernel."""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "vox_cell"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    s, e = idx[-2], idx[-1]
    tot = 0.0
    for r in rows[s:e]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        tot += d
        print(f"{d:8.1f} {r['Grid_Size_X']:>9} {r['Workgroup_Size_X']:>5} {r['Kernel_Name'][:90]}")
    span = (int(rows[e]["Start_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1000
    print(f"kernel sum {tot:.1f} us, step span {span:.1f} us")


if __name__ == "__main__":
    main()
