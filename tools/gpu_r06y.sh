#!/bin/bash
# Tiles per CU for the tiled counting sorts: 2 (default) vs 1 / 3 / 4 on cfg3
# and cfg5; the rule-block counting sort (cfg4) with per-CU tiles vs the
# power-of-two tiles.  GPU parity tests first.
set -o pipefail
OUT=gpurun_out/${1:-r06y}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4.py -x -q --timeout 600 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -40 "$OUT/parity.log"; exit 1; }
tail -2 "$OUT/parity.log"
V=ruleset-analysis_amd/_build
bash tools/ab_bench.sh "$OUT/cfg3" $V/libruleset_hip.so $V/var/libruleset_hip_tpc1.so $V/var/libruleset_hip_tpc3.so $V/var/libruleset_hip_tpc4.so || exit 1
bash tools/ab_bench.sh "$OUT/cfg5" $V/libruleset_hip.so $V/var/libruleset_hip_tpc1.so $V/var/libruleset_hip_tpc4.so -- --config cfg5 || exit 1
bash tools/ab_bench.sh "$OUT/cfg4" $V/libruleset_hip.so $V/var/libruleset_hip_cntpow2.so -- --config cfg4 || exit 1
echo done
