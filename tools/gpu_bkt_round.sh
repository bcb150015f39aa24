# One GPU round for the index comparison: parity tests of every index kind,
# then cfg3 and cfg4 benches per kind (tools/gpu_bkt_round.sh).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4.py -x -q --timeout 300 --timeout-method thread -k "index_and_scan or deferred or bucket or uncapped or 10k_rules_spread or capped_zipf or cfg4_parity" > gpurun_out/bkt_tests.log 2>&1 || { tail -30 gpurun_out/bkt_tests.log; exit 1; }
tail -2 gpurun_out/bkt_tests.log
for k in pht bucket bucket-filtered; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-check --steps 5 --index $k > gpurun_out/idx_cfg3_$k.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('cfg3', sys.argv[2], 'ms/step %.3f classify/launch %.4f' % (d['ms_per_step'], r['ms_per_launch']))" gpurun_out/idx_cfg3_$k.json $k
done
for k in pht bucket bucket-filtered; do
  timeout -k 10 400 python bench.py --config cfg4 --no-cpu-baseline --no-check --steps 3 --warmup 1 --index $k > gpurun_out/idx_cfg4_$k.json 2>gpurun_out/idx_cfg4_$k.err || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('cfg4', sys.argv[2], 'ms/step %.3f classify/launch %.4f' % (d['ms_per_step'], r['ms_per_launch']))" gpurun_out/idx_cfg4_$k.json $k
done
