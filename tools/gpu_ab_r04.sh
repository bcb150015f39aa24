#!/bin/bash
# Round-4 A/B call: parity tests of the pass-1 kernels, then the cfg3 bench
# with the default library and the classify variants (one workgroup per CU,
# next-tuple prefetch).  Every GPU step has its own time limit.
set -o pipefail
OUT=gpurun_out/${1:-r04f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/ab_bench.sh "$OUT/ab" ruleset-analysis_amd/_build/libruleset_hip.so \
  ruleset-analysis_amd/_build/var/libruleset_hip_large.so ruleset-analysis_amd/_build/var/libruleset_hip_largepf.so
