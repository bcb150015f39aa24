#!/bin/bash
# Phase profile of the recount (k_reduce<2>) beside k_reduce<1> (profiling build).
set -o pipefail
OUT=gpurun_out/${1:-r06n}
mkdir -p "$OUT"
export TMPDIR=/tmp
RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_phaseprof.so RSA_PHASE_PROF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config1 --no-check --steps 5 > "$OUT/phaseprof.json" 2> "$OUT/phaseprof.err" || { tail -20 "$OUT/phaseprof.err"; exit 1; }
grep phase_prof "$OUT/phaseprof.err"
echo done
