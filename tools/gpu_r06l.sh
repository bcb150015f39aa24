#!/bin/bash
# The sampled full-slice parity tests (cfg3 rules at 16M lines, cfg4 at 4M lines) against the C oracle.
set -o pipefail
OUT=gpurun_out/${1:-r06l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sampled.py "tests/test_gpu_cfg4.py::test_cfg4_sampled_lines_at_4m" -x -v --timeout 600 --timeout-method thread --durations=5 > "$OUT/sampled_tests.log" 2>&1 || { tail -40 "$OUT/sampled_tests.log"; exit 1; }
tail -12 "$OUT/sampled_tests.log"
echo done
