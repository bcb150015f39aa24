#!/bin/bash
# Round-4 traces (cfg3, cfg2, text 16M) + text-parse ablation variants + world-1 merge trace.
set -o pipefail
OUT=gpurun_out/${1:-r04j}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in cfg3 cfg2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$cfg" -o run --output-format csv -- \
    python3 bench.py --config $cfg --no-cpu-baseline --no-check --steps 3 --warmup 1 \
    > "$OUT/trace_$cfg.json" 2> "$OUT/trace_$cfg.err" || { tail -20 "$OUT/trace_$cfg.err"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_text" -o run --output-format csv -- \
  python3 bench.py --text --lines 16000000 --no-cpu-baseline --no-check --steps 3 --warmup 1 \
  > "$OUT/trace_text.json" 2> "$OUT/trace_text.err" || { tail -20 "$OUT/trace_text.err"; exit 1; }
for t in cfg3 cfg2 text; do
  f=$(find "$OUT/trace_$t" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_trace_$t.csv" && python3 tools/ktrace_summary.py "$f" > "$OUT/trace_${t}_summary.txt" 2>&1
done
for v in tp1 tp2; do
  for mode in 0 2; do
    RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_$v.so timeout -k 10 300 python -u bench.py --text \
      --lines 16000000 --no-cpu-baseline --no-check --steps 3 --warmup 1 --opt PARSE_MODE=$mode \
      > "$OUT/text_${v}_m$mode.json" 2> "$OUT/text_${v}_m$mode.err" || { tail -20 "$OUT/text_${v}_m$mode.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['phases_ms'])" "$OUT/text_${v}_m$mode.json"
  done
done
RSA_MERGE_TRACE=1 timeout -k 10 400 python -u bench.py --gpus 1 --force-dist --no-cpu-baseline --steps 5 --warmup 2 \
  > "$OUT/force_dist.json" 2> "$OUT/force_dist.err" || { tail -20 "$OUT/force_dist.err"; exit 1; }
grep "merge rank" "$OUT/force_dist.err" | tail -2
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('force-dist', d['ms_per_step'])" "$OUT/force_dist.json"
echo done
