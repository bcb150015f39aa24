#!/bin/bash
# BASELINE config 3 at its full stated size on ONE MI355X: 1B lines (28 GB of
# tuples, timestamps and order keys resident in HBM), checks on.
set -o pipefail
OUT=gpurun_out/${1:-r06_1b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1100 python -u bench.py --lines 1000000000 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/bench_1b.json" 2> "$OUT/bench_1b.err" || { tail -30 "$OUT/bench_1b.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('1B', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['roofline']['frac'], d['roofline']['pass1'], d['checks'])" "$OUT/bench_1b.json"
echo done
