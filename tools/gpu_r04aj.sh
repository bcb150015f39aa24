#!/bin/bash
# cfg4 (global bucket image, 53 VGPRs: room at 8 waves/SIMD) A/B of the
# k_classify prefetch switch: none / next tuple / next tuple + order + timestamp
# / auto (2 for the global-image variant only); cfg3 base vs auto.
set -o pipefail
OUT=gpurun_out/${1:-r04aj}
mkdir -p "$OUT"
export TMPDIR=/tmp
L=ruleset-analysis_amd/_build/ab
timeout -k 10 700 bash tools/ab_bench.sh "$OUT/cfg4" $L/base.so $L/pf1.so $L/pf2.so $L/auto.so -- --config cfg4 --steps 6 && \
timeout -k 10 300 bash tools/ab_bench.sh "$OUT/cfg3" $L/base.so $L/auto.so
echo done
