#!/bin/bash
# A/B of library variants on the default bench workload (GPU box):
#   tools/ab_bench.sh OUTDIR lib1.so lib2.so ... [-- extra bench args]
# Each variant runs twice, interleaved; prints ms/step and the pass-1 split.
set -eo pipefail
OUT=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p "$OUT"
for rep in 1 2; do
  for L in "${LIBS[@]}"; do
    n=$(basename "$L" .so)
    RSA_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-config1 --no-check --steps 10 "$@" > "$OUT/$n.$rep.json" 2>/dev/null
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print('%-12s %8.3f ms  classify %.3f  aggregate %.3f  classify/launch %.4f' % (sys.argv[2], d['ms_per_step'], k['classify_ms'], k['aggregate_ms'], d['roofline']['ms_per_launch']))" "$OUT/$n.$rep.json" "$n"
  done
done
