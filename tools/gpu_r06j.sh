#!/bin/bash
# The library-side merge (rsa_merge / rsa_merge_rccl): the GPU dist tests, the
# world-1 RCCL job with every collective forced (full cfg3 size, checks vs the
# single-GPU records), and the 2-rank shared-GPU job through the host-buffer
# transport at full size.
set -o pipefail
OUT=gpurun_out/${1:-r06j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 420 --timeout-method thread > "$OUT/dist_tests.log" 2>&1 || { tail -40 "$OUT/dist_tests.log"; exit 1; }
tail -3 "$OUT/dist_tests.log"
RSA_MERGE_TRACE=1 timeout -k 10 600 python -u bench.py --gpus 1 --force-dist --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/force_dist.json" 2> "$OUT/force_dist.err" || { tail -30 "$OUT/force_dist.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('force-dist', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['config']['merge'], d['checks'], d['gather'], d['merge_exchange'])" "$OUT/force_dist.json"
grep "merge rank" "$OUT/force_dist.err" | tail -2
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --backend gloo --steps 3 --warmup 1 > "$OUT/bench_share2.json" 2> "$OUT/bench_share2.err" || { tail -30 "$OUT/bench_share2.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('share2', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['config']['merge'], d['checks'], d['gather'], d['merge_exchange'])" "$OUT/bench_share2.json"
echo done
