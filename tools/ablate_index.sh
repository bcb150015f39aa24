# Classification ablations (PROFILING ONLY, results invalid) of both indexes on
# the default bench workload: tools/ablate_index.sh [PROFILE_CLASSIFY values...]
set -e
for v in ${@:-0 1 2 4}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 5 --opt PROFILE_CLASSIFY=$v > gpurun_out/abl_b$v.json 2>/dev/null
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('bucket prof', sys.argv[2], 'classify/launch %.4f' % d['roofline']['ms_per_launch'])" gpurun_out/abl_b$v.json $v
done
