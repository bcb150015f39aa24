#!/bin/bash
# Text path: 100M-line kernel trace; register-capped window parse A/B at 16M.
set -o pipefail
OUT=gpurun_out/${1:-r04p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py tests/test_multifile.py tests/test_reducer_stream.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in base pw5; do
  lib=""; [ $v = pw5 ] && lib=ruleset-analysis_amd/_build/var/libruleset_hip_pw5.so
  RSA_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --text --lines 16000000 --no-cpu-baseline --steps 3 --warmup 1 \
    > "$OUT/text16_$v.json" 2> "$OUT/text16_$v.err" || { tail -20 "$OUT/text16_$v.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks']['ok'])" "$OUT/text16_$v.json"
done
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text100" -o run --output-format csv -- \
  python3 bench.py --text --lines 100000000 --no-cpu-baseline --no-check --steps 1 --warmup 1 \
  > "$OUT/trace_text100.json" 2> "$OUT/trace_text100.err" || { tail -20 "$OUT/trace_text100.err"; exit 1; }
f=$(find "$OUT/trace_text100" -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_trace_text100.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_text100_summary.txt" 2>&1
head -40 "$OUT/trace_text100_summary.txt"
echo done
