#!/bin/bash
# Region count from the previous job's records (RSA_OPT_REGION_RECORDS): the new
# parity test first, the whole suite, then the cfg benches.
set -o pipefail
OUT=gpurun_out/${1:-r04am}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "region_count or cap_count_on_device" \
  --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -3 "$OUT/pytest_new.log"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for cfg in cfg3 cfg4 cfg5 cfg2; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 6 --warmup 2 \
    > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/bench_$cfg.json"
done
echo done
