#!/bin/bash
# Default bench line (with the CPU baselines) + the full-size GPU test.
set -o pipefail
OUT=gpurun_out/${1:-r06h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['cpu_baseline'];print('default', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['checks']['ok'], {k: c[k] for k in ('value','cores','sample')}, c['single_core']['value'], c['config1']['hadoop_like']['value'])" "$OUT/bench_default.json"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > "$OUT/fullsize.log" 2>&1 || { tail -30 "$OUT/fullsize.log"; exit 1; }
tail -1 "$OUT/fullsize.log"
echo done
