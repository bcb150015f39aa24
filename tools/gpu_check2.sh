#!/bin/bash
# GPU suite + smoke + default bench + the 2-rank (shared-GPU) distributed job
# at full cfg3 size: merged-result checks, timed gather and exchange volume.
set -o pipefail
OUT=gpurun_out/${1:-check2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --no-config1 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('default', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['roofline']['frac'], d['roofline']['pass1'], d['checks']['ok'])" "$OUT/bench_default.json"
timeout -k 10 900 python -u bench.py --gpus 2 --share-gpu --backend gloo --steps 3 --warmup 1 > "$OUT/bench_share2.json" 2> "$OUT/bench_share2.err" || { tail -20 "$OUT/bench_share2.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('share2', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['checks'], d['gather'], d['merge_exchange'])" "$OUT/bench_share2.json"
echo done
