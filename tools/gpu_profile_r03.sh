#!/bin/bash
# Round-3 profiling call: FETCH_SIZE calibration of the pass-1 access shapes,
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of cfg4 and cfg5, and a kernel trace
# of the merge at world 1.  Every GPU step has its own time limit; the first
# failure ends the call.
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib" -o pmc --output-format csv -- \
  tools/_build/fetch_calib > "$OUT/calib.json" 2> "$OUT/calib.err" || { tail -5 "$OUT/calib.err"; exit 1; }
for c in cfg4 cfg5; do
  tools/profile_round.sh "$OUT/$c" --config "$c" || { echo "profile $c failed"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_dist" -o run --output-format csv -- \
  python3 bench.py --gpus 1 --force-dist --no-cpu-baseline --no-check --steps 3 --warmup 1 \
  > "$OUT/trace_dist.json" 2> "$OUT/trace_dist.err" || { tail -20 "$OUT/trace_dist.err"; exit 1; }
# text parse A/B: the word-cached LDS accessor vs one LDS read per byte
for v in base nocache; do
  lib=ruleset-analysis_amd/_build/libruleset_hip.so
  [ "$v" = nocache ] && lib=ruleset-analysis_amd/_build/var/libruleset_hip_nocache.so
  RSA_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --text --lines 8000000 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-check > "$OUT/text_$v.json" 2> "$OUT/text_$v.err" || { tail -5 "$OUT/text_$v.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['phases_ms'])" "$OUT/text_$v.json" $v
done
echo done
