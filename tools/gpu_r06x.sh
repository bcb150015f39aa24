#!/bin/bash
# Region sort tiles two per CU (RSA_PART_TILES_CU) vs power-of-two tiles for
# >= 384 workgroups: GPU parity tests, then a same-box A/B (cfg3, cfg5, cfg2).
set -o pipefail
OUT=gpurun_out/${1:-r06x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampled.py tests/test_gpu_dist.py -x -q --timeout 600 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -40 "$OUT/parity.log"; exit 1; }
tail -2 "$OUT/parity.log"
V=ruleset-analysis_amd/_build
bash tools/ab_bench.sh "$OUT/cfg3" $V/libruleset_hip.so $V/var/libruleset_hip_tilespow2.so || exit 1
bash tools/ab_bench.sh "$OUT/cfg5" $V/libruleset_hip.so $V/var/libruleset_hip_tilespow2.so -- --config cfg5 || exit 1
bash tools/ab_bench.sh "$OUT/cfg2" $V/libruleset_hip.so $V/var/libruleset_hip_tilespow2.so -- --config cfg2 || exit 1
echo done
