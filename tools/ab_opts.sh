#!/bin/bash
# A/B of runtime options on the default bench workload (GPU box):
#   tools/ab_opts.sh OUTDIR "OPT=V OPT=V" "OPT=V" ... [-- extra bench args]
#   (one quoted set per variant, "" = defaults)
# Each variant runs twice, interleaved; prints ms/step and the pass-1 split.
set -eo pipefail
OUT=$1; shift
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p "$OUT"
k=0
for rep in 1 2; do
  k=0
  for set in "${SETS[@]}"; do
    k=$((k + 1))
    args=()
    for kv in $set; do args+=(--opt "$kv"); done
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-config1 --no-check --steps 10 "${args[@]}" "$@" > "$OUT/v$k.$rep.json" 2>/dev/null
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print('%-34s %8.3f ms  classify %.3f  aggregate %.3f' % (sys.argv[2] or 'defaults', d['ms_per_step'], k['classify_ms'], k['aggregate_ms']))" "$OUT/v$k.$rep.json" "$set"
  done
done
