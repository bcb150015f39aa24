#!/bin/bash
# Same-box A/B of the group records: ab_A = 80-B groups (four 4-word table
# descriptors), tree = 48-B groups (2-word descriptors, displacements right
# before the slots); cfg3 and cfg2.  Then the GPU parity tests of the index.
set -o pipefail
OUT=gpurun_out/${1:-r06i}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/ab_trees.sh "$OUT/cfg3" ab_A . || exit 1
bash tools/ab_trees.sh "$OUT/cfg2" ab_A . -- --config cfg2 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/parity.log" 2>&1 || { tail -30 "$OUT/parity.log"; exit 1; }
tail -2 "$OUT/parity.log"
echo done
