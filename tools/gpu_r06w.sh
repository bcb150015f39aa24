#!/bin/bash
# Four ranks sharing the GPU at full cfg3 size through the library merge
# (gloo host-buffer transport): checks and the measured exchange volumes.
set -o pipefail
OUT=gpurun_out/${1:-r06w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 4 --share-gpu --backend gloo --steps 2 --warmup 1 > "$OUT/bench_share4.json" 2> "$OUT/bench_share4.err" || { tail -30 "$OUT/bench_share4.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('share4', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['config']['merge'], d['checks']['ok'], d['gather'], d['merge_exchange'])" "$OUT/bench_share4.json"
echo done
