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
    # the last step's library dispatches in order (from its last k_classify
    # group: the 4th-last k_classify launch of the trace onwards)
    lib = [r for r in sorted(rows, key=lambda r: int(r['Start_Timestamp']))
           if r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').startswith('k_')]
    cls = [i for i, r in enumerate(lib) if 'k_classify' in r['Kernel_Name']]
    first = cls[-4] if len(cls) >= 4 else 0
    print('--- last step, in order')
    for r in lib[first:]:
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        print('%-45s %9.1f us  grid %s' % (name[:45], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                                           r.get('Grid_Size', r.get('Grid_Size_X', '?'))))


if __name__ == '__main__':
    main()
