#!/usr/bin/env python3
"""Per-config medians of a tools/gpu_knob_sweep.sh run: reads its "<config> <round> <value>" lines (the gpurun
output or a saved copy) and prints one row per config, best median first.

    python tools/knob_table.py profiles/r6/knobs/sweep1.txt
"""
import collections
import statistics
import sys


def main(argv=None) -> int:
    runs = collections.defaultdict(list)
    for line in open((argv or sys.argv[1:])[0]):
        p = line.split()
        if len(p) == 3 and p[1].isdigit():
            try:
                runs[p[0]].append(float(p[2]))
            except ValueError:
                pass
    base = statistics.median(runs["default"]) if runs.get("default") else None
    print(f"{'config':10s} {'median':>9s} {'vs default':>10s}  runs")
    for k, v in sorted(runs.items(), key=lambda kv: -statistics.median(kv[1])):
        m = statistics.median(v)
        rel = f"{(m / base - 1) * 100:+.1f}%" if base else "-"
        print(f"{k:10s} {m:9.1f} {rel:>10s}  {', '.join(f'{x:.1f}' for x in v)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
