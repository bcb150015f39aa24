#!/bin/bash
# One GPU call: the -m gpu suite, then bench lines of the configs named on the
# command line (default: cfg3).  Every GPU step has its own time limit and the
# first failure ends the call.
#   tools/gpu_check.sh TAG [cfg ...]      (TAG names gpurun_out/TAG/)
set -o pipefail
TAG=${1:-check}; shift || true
CFGS=${*:-cfg3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
for c in $CFGS; do
  extra=""
  [ "$c" = cfg4 ] && extra="--steps 5 --warmup 2"
  timeout -k 10 600 python -u bench.py --config "$c" --no-cpu-baseline $extra $BENCH_ARGS \
    > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -30 "$OUT/bench_$c.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];p=r['pass1'];print(sys.argv[2],'%.3f G lines/s  %.3f ms/step  classify %.3f  aggregate %.3f  checks %s'%(d['value']/1e9,d['ms_per_step'],p['classify_ms'],p['aggregate_ms'],(d.get('checks') or {}).get('ok')))" "$OUT/bench_$c.json" "$c"
done
# extra GPU steps (each a command line, run under a time limit)
if [ -n "$EXTRA" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > "$OUT/extra.log" 2>&1 || { tail -30 "$OUT/extra.log"; exit 1; }
  tail -5 "$OUT/extra.log"
fi
# kernel traces (rocprofv3 --kernel-trace --stats) of the configs in $TRACE
for c in $TRACE; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$c" -o run --output-format csv -- \
    python3 bench.py --config "$c" --no-cpu-baseline --no-check --steps 3 --warmup 1 \
    > "$OUT/trace_$c.json" 2> "$OUT/trace_$c.err" || { tail -20 "$OUT/trace_$c.err"; exit 1; }
  f=$(find "$OUT/trace_$c" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_${c}_summary.txt" 2>&1
  true
done
