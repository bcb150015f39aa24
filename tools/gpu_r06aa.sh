#!/bin/bash
# k_reduce<1> LDS table size: 3072 entries, one workgroup per CU (default) vs
# 1024 entries, two per CU (more waves to hide the latency, 3x the flushes) vs
# 2048 entries, one per CU.  Parity tests of the 1024 variant first.
set -o pipefail
OUT=gpurun_out/${1:-r06aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=ruleset-analysis_amd/_build
RSA_HIP_LIB=$V/var/libruleset_hip_red1k.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampled.py -x -q --timeout 600 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -40 "$OUT/parity.log"; exit 1; }
tail -2 "$OUT/parity.log"
bash tools/ab_bench.sh "$OUT/cfg3" $V/libruleset_hip.so $V/var/libruleset_hip_red1k.so $V/var/libruleset_hip_red2k.so || exit 1
bash tools/ab_bench.sh "$OUT/cfg2" $V/libruleset_hip.so $V/var/libruleset_hip_red1k.so -- --config cfg2 || exit 1
echo done
