#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs of a bench run into
profiles/<config>_pass1_pmc.json: HBM bytes per step of the pass-1 kernels.

FETCH_SIZE is in KiB and tallies 64 B per memory request.  Calibrated on the
box with tools/fetch_calib.hip against known byte counts
(profiles/r03l_fetch_calibration.json): 16-B-per-lane streaming reads and
consecutive 32-B records per lane report 0.50 of their bytes (x2, as
MI355X_MICROARCH.md §HBM says for wide streaming reads), random 32-B reads
2.0x and random 64-B reads 1.04x (one 64-B tally per read).  Each kernel is
converted with the factor of its dominant read pattern: the streaming
kernels (k_classify, k_count, k_part_hist, k_part_scatter, the scans) x2,
k_reduce (segment reads plus random 64-B slot read-modify-writes) x1.  The
cap kernels read streaming since round 4: k_cap_scatter(_lds) walks the used
list and k_reduce's used-ordered key copy in order (16 B per entry, no slot
gathers; the per-rule bound and segment tables are L2-resident) and
k_cap_select reads its segments in order, so both take x2; before round 4
k_cap_scatter gathered 64-B slots (random 64-B reads, x1.04) and x2
overstated it.
WRITE_SIZE * 1024 is taken as is.  Usage: pmc_summary.py FETCH_CSV WRITE_CSV
OUT_JSON LINES STEPS_TOTAL (STEPS_TOTAL = warmup + timed steps of the profiled
bench run, + 1 untimed stats step when the run had one)."""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, counter):
    vals = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(path)):
        if row.get('Counter_Name') != counter:
            continue
        d = int(row['Dispatch_Id'])
        vals[d] += float(row['Counter_Value'])
        names[d] = row['Kernel_Name']
    return vals, names


def main():
    fetch_csv, write_csv, out, lines, steps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), \
        int(sys.argv[5])
    f, fn = per_dispatch(fetch_csv, 'FETCH_SIZE')
    w, wn = per_dispatch(write_csv, 'WRITE_SIZE')
    # every pass-1 launch of every slice: classification, deferred tails,
    # aggregation (record append, region histogram, region scatter, per-region
    # reduction) -- the kernels bracketed by the pass-1 HIP events
    # ('k_reduce<1' covers the <1, 3072, 16> and <1, 4096, 15> instantiations)
    kinds = ('k_classify', 'k_tail', 'k_count<', 'k_count16<', 'k_count_flush', 'k_cnt_', 'k_aggregate', 'k_part_hist',
             'k_scan_blocks', 'k_scan_sums', 'k_scan_add', 'k_part_scatter', 'k_seg_starts', 'k_hot_plan',
             'k_hot_combine<1>', 'k_reduce<1', 'k_cap_mark', 'k_cap_scatter', 'k_cap_select')
    # pass-1 launches only: the classifier instantiated with emission (the
    # classify-only launches of bench's untimed checks are excluded)
    # (k_classify<kImg, kEmit, kMode, kNarrow>: kEmit is the second argument)
    import re
    no_emit = lambda name: re.search(r'k_classify<[^,>]+, false', name) is not None or \
        ('k_tail' in name and 'false>' in name) or 'k_classify_pair<false>' in name
    pick = lambda name: any(k in name for k in kinds) and not no_emit(name)
    factor = lambda name: 1.0 if 'k_reduce' in name else 2.0
    read = 1024 * sum(v * factor(fn[d]) for d, v in f.items() if pick(fn[d])) / steps
    write = 1024 * sum(v for d, v in w.items() if pick(wn[d])) / steps
    split = {}
    for k in kinds:
        split[k] = {'read_bytes_per_step': 1024 * sum(v * factor(fn[d]) for d, v in f.items()
                                                      if k in fn[d] and pick(fn[d])) / steps,
                    'write_bytes_per_step': 1024 * sum(v for d, v in w.items() if k in wn[d] and pick(wn[d])) / steps}
    res = {'hbm_bytes_per_step': read + write, 'read_bytes_per_step': read, 'write_bytes_per_step': write,
           'lines_per_step': lines, 'steps_seen': steps, 'bytes_per_line': (read + write) / lines,
           'kernels': split,
           'method': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes), pass-1 launches, '
                     'FETCH_SIZE x2 for the streaming kernels and x1 for k_reduce (calibrated: '
                     'profiles/r03l_fetch_calibration.json)'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
