#!/bin/bash
# cfg5 (bucket index in LDS, 52 VGPRs) A/B: prefetch off (auto) vs tuple + order + timestamp (auto2).
set -o pipefail
OUT=gpurun_out/${1:-r04al}
mkdir -p "$OUT"
export TMPDIR=/tmp
L=ruleset-analysis_amd/_build/ab
timeout -k 10 700 bash tools/ab_bench.sh "$OUT/cfg5" $L/auto.so $L/auto2.so -- --config cfg5 --steps 6
echo done
