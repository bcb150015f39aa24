#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r04i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { tail -20 "$OUT/bench_cfg3.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['roofline']['pass1'];print('cfg3 %.3f G lines/s %.3f ms classify %.3f aggregate %.3f checks %s'%(d['value']/1e9,d['ms_per_step'],k['classify_ms'],k['aggregate_ms'],d['checks']['ok']))" "$OUT/bench_cfg3.json"
timeout -k 10 600 python -u bench.py --text --lines 16000000 --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/bench_text16.json" 2> "$OUT/bench_text16.err" || { tail -20 "$OUT/bench_text16.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text16 %.1f M lines/s'%(d['value']/1e6), d['phases_ms'], d.get('checks'))" "$OUT/bench_text16.json"
timeout -k 10 600 python -u bench.py --text --lines 16000000 --no-cpu-baseline --steps 3 --warmup 1 --opt PARSE_MODE=2 > "$OUT/bench_text16_win.json" 2> "$OUT/bench_text16_win.err" || { tail -20 "$OUT/bench_text16_win.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('text16 win %.1f M lines/s'%(d['value']/1e6), d['phases_ms'], d.get('checks'))" "$OUT/bench_text16_win.json"
