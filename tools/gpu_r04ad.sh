#!/bin/bash
# Kernel traces of the text job (no checks) at 16M and 100M lines.
set -o pipefail
OUT=gpurun_out/${1:-r04ad}
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in 16000000 100000000; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text$L" -o run --output-format csv -- \
    python3 bench.py --text --lines $L --no-cpu-baseline --no-check --steps 3 --warmup 1 \
    > "$OUT/text$L.json" 2> "$OUT/text$L.err" || { tail -20 "$OUT/text$L.err"; exit 1; }
  f=$(find "$OUT/trace_text$L" -name '*kernel_trace.csv' | head -1)
  cp "$f" "$OUT/kernel_trace_text$L.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/text${L}_summary.txt" 2>&1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'])" "$OUT/text$L.json"
  head -25 "$OUT/text${L}_summary.txt"
done
echo done
