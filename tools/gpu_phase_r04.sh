set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
for cfg in cfg3 cfg5 cfg2; do
  RSA_PHASE_PROF=1 RSA_HIP_LIB=ruleset-analysis_amd/_build/var/libruleset_hip_phase.so timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-check --steps 5 --warmup 2 > gpurun_out/r04c/phase_$cfg.json 2> gpurun_out/r04c/phase_$cfg.err || exit 1
  grep phase_prof gpurun_out/r04c/phase_$cfg.err
done
