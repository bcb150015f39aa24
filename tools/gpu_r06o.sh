#!/bin/bash
# The text job at 100M lines (BASELINE config 3 rules) with the final build.
set -o pipefail
OUT=gpurun_out/${1:-r06o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --text --lines 100000000 --steps 3 --warmup 1 > "$OUT/text100.json" 2> "$OUT/text100.err" || { tail -20 "$OUT/text100.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text100', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['phases_ms'], d['checks'])" "$OUT/text100.json"
echo done
