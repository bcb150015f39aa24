#!/bin/bash
# Record call: full -m gpu suite, smoke(), the default bench line
# (cfg3 with cpu_baseline), the rocprofv3 kernel trace/stats of that same
# command, and the cfg2/cfg4/cfg5 bench lines.
set -o pipefail
OUT=gpurun_out/${1:-record}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('default', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['roofline']['frac'], d['cpu_baseline'])" "$OUT/bench_default.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv -- \
  python3 bench.py > "$OUT/trace_default.json" 2> "$OUT/trace_default.err" || { tail -20 "$OUT/trace_default.err"; exit 1; }
f=$(find "$OUT/trace_default" -name '*kernel_trace.csv' | head -1)
s=$(find "$OUT/trace_default" -name '*kernel_stats.csv' | head -1)
cp "$s" "$OUT/kernel_stats_default.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_default_summary.txt" 2>&1
head -8 "$OUT/trace_default_summary.txt"
for cfg in cfg2 cfg4 cfg5; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 \
    > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/bench_$cfg.json"
done
echo done
