#!/bin/bash
# Full GPU suite (recount fast path), cfg benches, text scan-descriptor A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for cfg in cfg3 cfg5 cfg2; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 \
    > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/bench_$cfg.json"
done
for v in base nopf; do
  lib=""; [ $v = nopf ] && lib=ruleset-analysis_amd/_build/var/libruleset_hip_nopf.so
  RSA_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --text --lines 16000000 --no-cpu-baseline --no-check --steps 5 --warmup 1 \
    > "$OUT/text16_$v.json" 2> "$OUT/text16_$v.err" || { tail -20 "$OUT/text16_$v.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'])" "$OUT/text16_$v.json"
done
echo done
