#!/bin/bash
# Round-3 text-path call: GPU tests of the parse / reducer / fused text job,
# the --text bench, a kernel trace of it, the reducer drop-in throughput and
# the merge at world 1.  Every GPU step has its own time limit; the first
# failure ends the call.
set -o pipefail
OUT=gpurun_out/${1:-r03q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py tests/test_reducer_stream.py tests/test_keytext.py \
  tests/test_multifile.py tests/test_cli_dropin.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --text --no-cpu-baseline > "$OUT/text.json" 2> "$OUT/text.err" \
  || { tail -20 "$OUT/text.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text', d['value']/1e6, 'M lines/s', d['phases_ms'])" "$OUT/text.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --no-cpu-baseline --no-check --steps 3 --warmup 1 > "$OUT/trace_text.json" \
  2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
timeout -k 10 300 python -u tools/bench_reducer.py > "$OUT/reducer.json" 2> "$OUT/reducer.err" \
  || { tail -20 "$OUT/reducer.err"; exit 1; }
cat "$OUT/reducer.json"
RSA_MERGE_TRACE=1 timeout -k 10 400 python -u bench.py --gpus 1 --force-dist --no-cpu-baseline --steps 5 --warmup 2 \
  > "$OUT/force_dist.json" 2> "$OUT/force_dist.err" || { tail -20 "$OUT/force_dist.err"; exit 1; }
grep "merge rank" "$OUT/force_dist.err" | tail -1
grep '^{' "$OUT/force_dist.json" | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('force-dist', d['ms_per_step'])"
