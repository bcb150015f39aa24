#!/bin/bash
# Round-3 record call: the whole -m gpu suite, smoke(), the bench lines of
# every config, the text path at 100M lines, and kernel traces of cfg3 and
# cfg4.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${1:-r03z}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
  || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('default', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'])" "$OUT/bench_default.json"
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" \
    || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value']/1e9, d['ms_per_step'], (d.get('checks') or {}).get('ok'))" "$OUT/bench_$c.json" $c
done
timeout -k 10 900 python -u bench.py --text --lines 100000000 --no-cpu-baseline --steps 3 --warmup 1 \
  > "$OUT/text_100m.json" 2> "$OUT/text_100m.err" || { tail -20 "$OUT/text_100m.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text100m', d['value']/1e6, d['phases_ms'], (d.get('checks') or {}).get('ok'))" "$OUT/text_100m.json"
for c in cfg3 cfg4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$c" -o run --output-format csv -- \
    python3 bench.py --config $c --no-cpu-baseline --no-check --steps 3 --warmup 1 > "$OUT/trace_$c.json" \
    2> "$OUT/trace_$c.err" || { tail -20 "$OUT/trace_$c.err"; exit 1; }
done
echo done
