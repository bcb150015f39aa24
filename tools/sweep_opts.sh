#!/bin/bash
# Bench sweep over the auto-filter options on the GPU box (one bench process per
# setting, each under its own time limit; stops at the first failure).
set -eo pipefail
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
for s in "FILTER_STEPS=3 FILTER_SLICE=256" "FILTER_STEPS=2 FILTER_SLICE=256" "FILTER_STEPS=4 FILTER_SLICE=256" \
         "FILTER_STEPS=3 FILTER_SLICE=128" "FILTER_STEPS=3 FILTER_SLICE=512" "FILTER_STEPS=4 FILTER_SLICE=1024" \
         "FILTER_STEPS=1 FILTER_SLICE=64" "FILTER_STEPS=2 FILTER_SLICE=64"; do
  args=""
  for kv in $s; do args="$args --opt $kv"; done
  tag=$(echo "$s" | tr ' =' '__')
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 $args > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  echo "$s $(python3 -c "import json,sys; d=json.load(open('$OUT/$tag.json')); print(round(d['value']/1e9,3), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))")"
done
