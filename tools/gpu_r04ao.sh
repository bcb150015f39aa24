#!/bin/bash
# k_reduce<1> with 4096 LDS entries (regions <= 2^15 slots so the bitmaps fit: 156 KiB, 5 VGPRs spilled) vs 3072.
set -o pipefail
OUT=gpurun_out/${1:-r04ao}
mkdir -p "$OUT"
export TMPDIR=/tmp
L=ruleset-analysis_amd/_build/ab
timeout -k 10 400 bash tools/ab_bench.sh "$OUT/cfg5" $L/cur.so $L/r4096.so -- --config cfg5 --steps 6 && \
timeout -k 10 300 bash tools/ab_bench.sh "$OUT/cfg3" $L/cur.so $L/r4096.so
echo done
