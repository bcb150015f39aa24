#!/bin/bash
# Text path (prefix staging, LDS finisher) + region-count A/B on cfg2/cfg3.
set -o pipefail
OUT=gpurun_out/${1:-r04n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_textparse.py tests/test_multifile.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for L in 16000000 100000000; do
  timeout -k 10 900 python -u bench.py --text --lines $L --no-cpu-baseline --steps 3 --warmup 1 \
    > "$OUT/text_$L.json" 2> "$OUT/text_$L.err" || { tail -20 "$OUT/text_$L.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks']['ok'])" "$OUT/text_$L.json"
done
RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_okfull.so timeout -k 10 600 python -u bench.py --text --lines 16000000 \
  --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/text_okfull.json" 2> "$OUT/text_okfull.err" || { tail -20 "$OUT/text_okfull.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], round(d['value']/1e6,1), d['phases_ms'], d['checks']['ok'])" "$OUT/text_okfull.json"
for cfg in cfg2 cfg3; do
  for r in 8 10; do
    timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 --warmup 2 --opt MIN_REGIONS_LOG2=$r \
      > "$OUT/${cfg}_r$r.json" 2> "$OUT/${cfg}_r$r.err" || { tail -20 "$OUT/${cfg}_r$r.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print(sys.argv[1], round(d['value']/1e9,3), round(d['ms_per_step'],3), 'cls', round(k['classify_ms'],3), 'agg', round(k['aggregate_ms'],3), d['checks']['ok'])" "$OUT/${cfg}_r$r.json"
  done
done
echo done
