#!/usr/bin/env python3
"""Per-step kernel times from a rocprofv3 --kernel-trace CSV of bench.py:
the last STEP's launches in order, and per-kernel totals per step.
Usage: trace_step.py run_kernel_trace.csv [steps_total]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    tot = defaultdict(float)
    for r in rows:
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        tot[name] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:16]:
        print('%-45s %9.1f us/step' % (k[:45], v / steps))


if __name__ == '__main__':
    main()
