#!/bin/bash
# GPU suite (per-launch hot-plan and cap counters zeroed in k_seg_starts instead of
# four memsets), cfg3/cfg5/cfg2 benches, cfg3 trace.
set -o pipefail
OUT=gpurun_out/${1:-r04ah}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for cfg in cfg3 cfg5 cfg2; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 \
    > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/bench_$cfg.json"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg3" -o run --output-format csv -- \
  python3 bench.py --config cfg3 --no-cpu-baseline --no-check --steps 5 --warmup 2 \
  > "$OUT/trace_cfg3.json" 2> "$OUT/trace_cfg3.err" || { tail -20 "$OUT/trace_cfg3.err"; exit 1; }
f=$(find "$OUT/trace_cfg3" -name '*kernel_trace.csv' | head -1)
cp "$f" "$OUT/kernel_trace_cfg3.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_cfg3_summary.txt" 2>&1
head -12 "$OUT/trace_cfg3_summary.txt"
echo done
