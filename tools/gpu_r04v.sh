#!/bin/bash
# Text 16M A/B: scan descriptors prefetched (default) vs read per byte.
set -o pipefail
OUT=gpurun_out/${1:-r04v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in base nopf base nopf; do
  lib=""; [ $v = nopf ] && lib=ruleset-analysis_amd/_build/var/libruleset_hip_nopf.so
  RSA_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --text --lines 16000000 --no-cpu-baseline --no-check --steps 5 --warmup 1 \
    > "$OUT/text16_$v.json" 2> "$OUT/text16_$v.err" || { tail -20 "$OUT/text16_$v.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'])" "$OUT/text16_$v.json"
done
echo done
