#!/bin/bash
# PMC/SQ profiles of the given configs (tools/profile_round.sh passes) and their summaries.
# Usage: tools/gpu_prof.sh TAG CFG [CFG...]; lines per GPU from bench.py's CONFIGS.
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
for cfg in "$@"; do
  OUT=gpurun_out/$TAG/$cfg
  mkdir -p "$OUT"
  timeout -k 10 1100 bash tools/profile_round.sh "$OUT" --config $cfg > "$OUT.log" 2>&1 || { tail -20 "$OUT.log"; exit 1; }
  lines=$(python3 -c "import sys; sys.argv=['x']; import bench; print(bench.CONFIGS['$cfg']['lines'])")
  f=$(find "$OUT/fetch" -name '*counter_collection.csv' | head -1)
  w=$(find "$OUT/write" -name '*counter_collection.csv' | head -1)
  q=$(find "$OUT/sq" -name '*counter_collection.csv' | head -1)
  t=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
  python3 tools/pmc_summary.py "$f" "$w" "$OUT/${cfg}_pass1_pmc.json" "$lines" 3 > /dev/null && \
  python3 tools/sq_summary.py "$q" "$OUT/${cfg}_sq.json" > "$OUT/sq_busy.txt" && \
  python3 tools/ktrace_summary.py "$t" > "$OUT/kernel_totals.txt" 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('$OUT/${cfg}_pass1_pmc.json'));print('$cfg', round(d['bytes_per_line'],1), 'B/line')"
  head -3 "$OUT/sq_busy.txt"
done
echo done
