#!/bin/bash
# Equal contiguous parts of the used list per workgroup for the cap scatter and
# the emission (persistent grids) vs fixed chunks dealt round-robin (HEAD).
set -o pipefail
OUT=gpurun_out/${1:-r06z}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampled.py tests/test_gpu_dist.py -x -q --timeout 600 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -40 "$OUT/parity.log"; exit 1; }
tail -2 "$OUT/parity.log"
V=ruleset-analysis_amd/_build
bash tools/ab_bench.sh "$OUT/cfg3" $V/libruleset_hip.so $V/var/libruleset_hip_fixedchunks.so || exit 1
bash tools/ab_bench.sh "$OUT/cfg5" $V/libruleset_hip.so $V/var/libruleset_hip_fixedchunks.so -- --config cfg5 || exit 1
bash tools/ab_bench.sh "$OUT/cfg4" $V/libruleset_hip.so $V/var/libruleset_hip_fixedchunks.so -- --config cfg4 || exit 1
echo done
