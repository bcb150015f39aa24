#!/bin/bash
# Profiles of the default bench workload, run on the GPU box:
#   kernel trace + stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE;
#   SQ VALU/issue counters + GRBM_GUI_ACTIVE), each in its own run as
#   MI355X_MICROARCH.md §rocprofv3 PMC slots requires.
# Usage: tools/profile_round.sh OUTDIR [extra bench args]
set -eo pipefail
OUT=${1:-gpurun_out/prof}
shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 5 --warmup 2 "$@" > "$OUT/bench_trace.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > "$OUT/bench_fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > "$OUT/bench_write.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/sq" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > "$OUT/bench_sq.log" 2>&1
echo done
