#!/bin/bash
# Three ranks on one GPU through rsa_merge, and the merge ABI's error paths.
set -o pipefail
OUT=gpurun_out/${1:-r06t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_gpu_dist.py::test_three_ranks_one_gpu_uneven_owners" "tests/test_gpu_dist.py::test_merge_abi_errors" -x -v --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -4 "$OUT/tests.log"
echo done
