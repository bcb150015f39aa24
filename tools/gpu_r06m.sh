#!/bin/bash
# Coalesced 16-KiB rounds in the line split (k_nl_offsets): the GPU text
# tests, then a same-box A/B of the text job against the per-thread-64-B build.
set -o pipefail
OUT=gpurun_out/${1:-r06m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py tests/test_multifile.py tests/test_reducer_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/text_tests.log" 2>&1 || { tail -30 "$OUT/text_tests.log"; exit 1; }
tail -2 "$OUT/text_tests.log"
bash tools/ab_text.sh "$OUT/ab" 30000000 ruleset-analysis_amd/_build/libruleset_hip.so ruleset-analysis_amd/_build/var/libruleset_hip_nocoal.so || exit 1
echo done
