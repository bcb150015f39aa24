#!/bin/bash
# The loopback (world 1, no process group) rsa_merge test and smoke().
set -o pipefail
OUT=gpurun_out/${1:-r06p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_gpu_dist.py::test_loopback_forced_exchange_in_process" -x -v --timeout 300 --timeout-method thread > "$OUT/loopback.log" 2>&1 || { tail -40 "$OUT/loopback.log"; exit 1; }
tail -3 "$OUT/loopback.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
echo done
