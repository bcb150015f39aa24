#!/bin/bash
# Filter-slice schedule A/B: FILTER_STEPS 3 (default) against 4 (one more
# bound refinement after 64M lines) on cfg3, cfg5, cfg2.
set -o pipefail
OUT=gpurun_out/${1:-r04af}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in cfg3 cfg5 cfg2; do
  for s in 3 4; do
    timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 --opt FILTER_STEPS=$s \
      > "$OUT/bench_${cfg}_s$s.json" 2> "$OUT/bench_${cfg}_s$s.err" || { tail -20 "$OUT/bench_${cfg}_s$s.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/bench_${cfg}_s$s.json"
  done
done
echo done
