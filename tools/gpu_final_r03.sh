#!/bin/bash
# Round-3 closing measurements: cfg3 profiles (trace, FETCH_SIZE, WRITE_SIZE,
# SQ) of HEAD, the text path at 16M and 100M lines, and the text kernels'
# trace.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${1:-r03ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/profile_round.sh "$OUT/cfg3" || { echo "profile cfg3 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --text --no-cpu-baseline > "$OUT/text.json" 2> "$OUT/text.err" \
  || { tail -20 "$OUT/text.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text16m', d['value']/1e6, d['phases_ms'], d['checks']['ok'])" "$OUT/text.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --no-cpu-baseline --no-check --steps 3 --warmup 1 > "$OUT/trace_text.json" \
  2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
timeout -k 10 900 python -u bench.py --text --lines 100000000 --no-cpu-baseline --steps 3 --warmup 1 \
  > "$OUT/text_100m.json" 2> "$OUT/text_100m.err" || { tail -20 "$OUT/text_100m.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text100m', d['value']/1e6, d['phases_ms'], d['checks']['ok'])" "$OUT/text_100m.json"
echo done
