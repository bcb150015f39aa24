#!/bin/bash
# Table-region count sweep (RSA_OPT_MIN_REGIONS_LOG2 10 / 11 / 12) on cfg3, cfg4, cfg5.
set -o pipefail
OUT=gpurun_out/${1:-r04ak}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in cfg4 cfg5 cfg3; do
  for r in 10 11 12; do
    timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-check --steps 6 --warmup 2 \
      --opt MIN_REGIONS_LOG2=$r > "$OUT/${cfg}_r$r.json" 2> "$OUT/${cfg}_r$r.err" || { tail -20 "$OUT/${cfg}_r$r.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3))" "$OUT/${cfg}_r$r.json"
  done
done
echo done
