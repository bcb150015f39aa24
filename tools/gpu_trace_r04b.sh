#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of cfg3, cfg2 and the text
# path (16M lines, register-window parse), and the world-1 merge trace.
set -o pipefail
OUT=gpurun_out/${1:-r04j}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in cfg3 cfg2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$cfg" -o run --output-format csv -- \
    python3 bench.py --config $cfg --no-cpu-baseline --no-check --steps 3 --warmup 1 \
    > "$OUT/trace_$cfg.json" 2> "$OUT/trace_$cfg.err" || { tail -20 "$OUT/trace_$cfg.err"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --lines 16000000 --no-cpu-baseline --no-check --steps 3 --warmup 1 --opt PARSE_MODE=2 \
  > "$OUT/trace_text.json" 2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
for t in cfg3 cfg2 text; do
  f=$(find "$OUT/trace_$t" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_trace_$t.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_${t}_summary.txt" 2>&1
done
RSA_MERGE_TRACE=1 timeout -k 10 400 python -u bench.py --gpus 1 --force-dist --no-cpu-baseline --steps 5 --warmup 2 \
  > "$OUT/force_dist.json" 2> "$OUT/force_dist.err" || { tail -20 "$OUT/force_dist.err"; exit 1; }
grep "merge rank" "$OUT/force_dist.err" | tail -2
echo done
