#!/bin/bash
# Cap-selection volume per filter slice (RSA_DEBUG=1: capped rules, their
# entries, keys scattered) for cfg3 and cfg5.
set -o pipefail
OUT=gpurun_out/${1:-r04z}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in cfg3 cfg5; do
  RSA_DEBUG=1 timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-check --steps 1 --warmup 1 \
    > "$OUT/dbg_$cfg.json" 2> "$OUT/dbg_$cfg.err" || { tail -20 "$OUT/dbg_$cfg.err"; exit 1; }
  grep -E "cap select|pass-1 launch" "$OUT/dbg_$cfg.err" | tail -24
done
echo done
