#!/bin/bash
# Filter schedule on BASELINE config 4 (few capped rules among 3.45M): the
# default three bound refinements vs one / two, and no auto filter.
set -o pipefail
OUT=gpurun_out/${1:-r06v}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/ab_opts.sh "$OUT/cfg4" "" "FILTER_STEPS=1" "FILTER_STEPS=2" "AUTO_FILTER=0" -- --config cfg4 || exit 1
echo done
