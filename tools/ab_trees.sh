#!/bin/bash
# A/B of whole trees (image builder + library) on the same box: each DIR holds
# a checkout with its built library; runs bench.py from each, interleaved.
#   tools/ab_trees.sh OUTDIR DIR1 DIR2 ... [-- extra bench args]
set -eo pipefail
OUT=$1; shift
DIRS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do DIRS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p "$OUT"
for rep in 1 2; do
  for D in "${DIRS[@]}"; do
    n=$(basename "$D"); [ "$n" = "." ] && n=tree
    (cd "$D" && timeout -k 10 240 python bench.py --no-cpu-baseline --no-config1 --no-check --steps 10 "$@") > "$OUT/$n.$rep.json" 2>/dev/null
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print('%-10s %8.3f ms  classify %.3f  aggregate %.3f  classify/launch %.4f' % (sys.argv[2], d['ms_per_step'], k['classify_ms'], k['aggregate_ms'], d['roofline']['ms_per_launch']))" "$OUT/$n.$rep.json" "$n"
  done
done
