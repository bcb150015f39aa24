#!/bin/bash
# k_reduce<1> LDS table size / occupancy A/B: 3072 entries at one workgroup per
# CU (current), 2048 entries (90 KiB), 1024 entries at two workgroups per CU.
set -o pipefail
OUT=gpurun_out/${1:-r04an}
mkdir -p "$OUT"
export TMPDIR=/tmp
L=ruleset-analysis_amd/_build/ab
timeout -k 10 500 bash tools/ab_bench.sh "$OUT/cfg5" $L/cur.so $L/r2048w4.so $L/r1024w8.so -- --config cfg5 --steps 6 && \
timeout -k 10 400 bash tools/ab_bench.sh "$OUT/cfg3" $L/cur.so $L/r2048w4.so $L/r1024w8.so
echo done
