#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 --kernel-trace CSV: name, calls, total ms,
mean ms (optionally only launches after the first N ms of the trace)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = defaultdict(float)
n = defaultdict(int)
for r in rows[skip:]:
    name = r['Kernel_Name']
    name = name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:60]
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    tot[name] += d
    n[name] += 1
for k in sorted(tot, key=lambda k: -tot[k]):
    print('%-60s %5d %10.3f %8.4f' % (k, n[k], tot[k], tot[k] / n[k]))
