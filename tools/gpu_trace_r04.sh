#!/bin/bash
# Round-4 kernel traces (rocprofv3 --kernel-trace --stats): cfg3 and the text
# path at 16M lines; per-dispatch CSVs are kept for the per-slice analysis.
set -o pipefail
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg3" -o run --output-format csv -- \
  python3 bench.py --config cfg3 --no-cpu-baseline --no-check --steps 3 --warmup 1 \
  > "$OUT/trace_cfg3.json" 2> "$OUT/trace_cfg3.err" || { tail -20 "$OUT/trace_cfg3.err"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --lines 16000000 --no-cpu-baseline --no-check --steps 3 --warmup 1 \
  > "$OUT/trace_text.json" 2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
for t in cfg3 text; do
  f=$(find "$OUT/trace_$t" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_trace_$t.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_${t}_summary.txt" 2>&1
done
echo done
