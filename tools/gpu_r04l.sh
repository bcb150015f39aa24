#!/bin/bash
# Text path after the reduction fixes: tests, 16M trace, 100M-line bench.
set -o pipefail
OUT=gpurun_out/${1:-r04l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py tests/test_multifile.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --lines 16000000 --no-cpu-baseline --steps 3 --warmup 1 \
  > "$OUT/trace_text.json" 2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks']['ok'])" "$OUT/trace_text.json"
f=$(find "$OUT/trace_text" -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_trace_text.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_text_summary.txt" 2>&1
head -24 "$OUT/trace_text_summary.txt"
timeout -k 10 900 python -u bench.py --text --lines 100000000 --no-cpu-baseline --steps 3 --warmup 1 \
  > "$OUT/text100.json" 2> "$OUT/text100.err" || { tail -20 "$OUT/text100.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks']['ok'])" "$OUT/text100.json"
echo done
