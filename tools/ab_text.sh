#!/bin/bash
# A/B of library variants on the text job (GPU box):
#   tools/ab_text.sh OUTDIR LINES lib1.so lib2.so ...
# Each variant runs twice, interleaved; prints ms/step and the phase split.
set -eo pipefail
OUT=$1; LINES=$2; shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    RSA_HIP_LIB=$L timeout -k 10 400 python bench.py --text --lines "$LINES" --steps 3 --warmup 1 --no-check > "$OUT/$n.$rep.json" 2>/dev/null
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('%-24s %8.3f ms  %s' % (sys.argv[2], d['ms_per_step'], json.dumps({k: round(v, 2) for k, v in d['phases_ms'].items()})))" "$OUT/$n.$rep.json" "$n"
  done
done
