#!/bin/bash
# The distributed job over RCCL at world 1 (--force-dist, nccl): full-size
# checks of the merged result, gather timing and exchange summary.
set -o pipefail
OUT=gpurun_out/${1:-r06g}
mkdir -p "$OUT"
export TMPDIR=/tmp
RSA_MERGE_TRACE=1 timeout -k 10 600 python -u bench.py --gpus 1 --force-dist --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/force_dist.json" 2> "$OUT/force_dist.err" || { tail -30 "$OUT/force_dist.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('force-dist', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['checks'], d['gather'], d['merge_exchange'])" "$OUT/force_dist.json"
grep "merge rank" "$OUT/force_dist.err" | tail -3
echo done
