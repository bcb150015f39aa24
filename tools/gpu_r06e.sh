#!/bin/bash
# Kernel traces of the default library and a profiling variant on the same box
# (per-kernel totals per step), cfg3 default bench.
set -o pipefail
OUT=gpurun_out/${1:-r06e}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in ruleset-analysis_amd/_build/libruleset_hip.so "$@"; do
  n=$(basename "$L" .so)
  RSA_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-config1 --no-check --steps 5 --warmup 2 > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
  t=$(find "$OUT/$n" -name '*kernel_trace.csv' | head -1)
  python3 tools/ktrace_summary.py "$t" > "$OUT/$n.totals.txt" 2>&1
  echo "== $n"; head -12 "$OUT/$n.totals.txt"
done
echo done
