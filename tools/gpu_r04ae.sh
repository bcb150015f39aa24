#!/bin/bash
# Text-path GPU tests and benches after the line split's coalesced slab loads
# (512-thread workgroups, 32-KiB blocks).
set -o pipefail
OUT=gpurun_out/${1:-r04ae}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "text or split or parse or offsets or reducer" \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for L in 16000000 100000000; do
  timeout -k 10 400 python -u bench.py --text --lines $L --no-cpu-baseline --steps 3 --warmup 1 \
    > "$OUT/text$L.json" 2> "$OUT/text$L.err" || { tail -20 "$OUT/text$L.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks'])" "$OUT/text$L.json"
done
echo done
