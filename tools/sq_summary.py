#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counter CSVs (one pass, e.g. the SQ
VALU/issue counters + GRBM_GUI_ACTIVE of tools/profile_round.sh) ->
profiles/<config>_sq.json, the file bench.py reads for `roofline.valu`.
Usage: sq_summary.py COUNTER_CSV OUT_JSON"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(path)):
        name = row['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        acc[name][row['Counter_Name']] += float(row['Counter_Value'])
    res = {k: dict(v) for k, v in acc.items()}
    json.dump(res, open(out, 'w'), indent=1, sort_keys=True)
    for k, v in res.items():
        if v.get('GRBM_GUI_ACTIVE'):
            busy = 2.0 * v.get('SQ_INSTS_VALU', 0) / (1024 * v['GRBM_GUI_ACTIVE'] / 8.0)
            print('%-40s VALU busy %.3f' % (k[:40], busy))


if __name__ == '__main__':
    main()
