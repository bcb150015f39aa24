#!/bin/bash
# LDS / stall counters of the default bench workload (one rocprofv3 --pmc pass
# each, MI355X_MICROARCH.md §rocprofv3 PMC slots): LDS instructions and bank
# conflicts, wait/issue/active cycles.  Usage: tools/profile_lds.sh OUTDIR [bench args]
set -eo pipefail
OUT=${1:-gpurun_out/prof_lds}
shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d "$OUT/lds" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > "$OUT/bench_lds.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE \
  -d "$OUT/wait" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > "$OUT/bench_wait.log" 2>&1
echo done
