#!/bin/bash
# Diagnosis call: kernel trace of the default bench (per-dispatch durations of
# the last step, tools/trace_step.py) and the LDS / wait counters
# (tools/profile_lds.sh).  Usage: tools/gpu_diag.sh TAG [bench args]
set -o pipefail
TAG=${1:-diag}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-config1 --no-check --steps 3 --warmup 1 "$@" > "$OUT/trace.json" 2> "$OUT/trace.err" \
  || { tail -20 "$OUT/trace.err"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" 5 > "$OUT/trace_step.txt" 2>&1
cp "$f" "$OUT/kernel_trace.csv"
head -60 "$OUT/trace_step.txt"
timeout -k 10 900 tools/profile_lds.sh "$OUT/lds" "$@" || exit 1
for p in lds wait; do
  c=$(find "$OUT/lds/$p" -name '*counter_collection.csv' | head -1)
  [ -n "$c" ] && python3 tools/sq_summary.py "$c" "$OUT/${p}_counters.json" > /dev/null
done
echo done
