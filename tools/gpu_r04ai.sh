#!/bin/bash
# k_classify A/B: next-tuple prefetch (1) and next order/timestamp prefetch (2),
# each at two workgroups per CU (64 VGPRs) and one (FORCE_LARGE, 128 VGPRs).
set -o pipefail
OUT=gpurun_out/${1:-r04ai}
mkdir -p "$OUT"
export TMPDIR=/tmp
L=ruleset-analysis_amd/_build/ab
timeout -k 10 900 bash tools/ab_bench.sh "$OUT" $L/base.so $L/pf1.so $L/pf2.so $L/lg.so $L/lgpf1.so $L/lgpf2.so
echo done
