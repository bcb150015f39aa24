#!/bin/bash
# Text-path A/B: the general (slow) parse from LDS rows vs from global memory.
set -o pipefail
OUT=gpurun_out/${1:-r06f}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/ab_text.sh "$OUT/text30" 30000000 ruleset-analysis_amd/_build/libruleset_hip.so ruleset-analysis_amd/_build/var/libruleset_hip_slowlds.so ruleset-analysis_amd/_build/var/libruleset_hip_slowlds_w6.so || exit 1
RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_slowlds.so timeout -k 10 600 python -u -m pytest tests/test_textparse.py -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/textparse_tests.log" 2>&1 || { tail -30 "$OUT/textparse_tests.log"; exit 1; }
tail -2 "$OUT/textparse_tests.log"
echo done
