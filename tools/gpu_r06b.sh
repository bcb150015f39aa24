#!/bin/bash
# The 2-rank shared-GPU distributed job at full cfg3 size, an A/B of k_reduce
# variants and the phase-profiling build's k_reduce<1> breakdown.
set -o pipefail
OUT=gpurun_out/${1:-r06b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --backend gloo --steps 3 --warmup 1 > "$OUT/bench_share2.json" 2> "$OUT/bench_share2.err" || { tail -30 "$OUT/bench_share2.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('share2', round(d['value']/1e9,3), round(d['ms_per_step'],3), d['checks'], d['gather'], d['merge_exchange'])" "$OUT/bench_share2.json"
RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_phaseprof.so RSA_PHASE_PROF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config1 --no-check --steps 5 > "$OUT/phaseprof.json" 2> "$OUT/phaseprof.err" || { tail -20 "$OUT/phaseprof.err"; exit 1; }
grep phase_prof "$OUT/phaseprof.err"
bash tools/ab_bench.sh "$OUT/ab" ruleset-analysis_amd/_build/libruleset_hip.so ruleset-analysis_amd/_build/var/libruleset_hip_nopair.so ruleset-analysis_amd/_build/var/libruleset_hip_fill5.so ruleset-analysis_amd/_build/var/libruleset_hip_fill7.so
echo done
