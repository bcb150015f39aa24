#!/bin/bash
# Cap scatter chunk size: 16384 (HEAD, capold), 8192 and 4096 entries per
# chunk (new form, span 1): more workgroups of the persistent grid busy.
set -o pipefail
OUT=gpurun_out/${1:-r06r}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=ruleset-analysis_amd/_build
bash tools/ab_bench.sh "$OUT/cfg3" $V/var/libruleset_hip_capold.so $V/var/libruleset_hip_capper8.so $V/var/libruleset_hip_capper4.so || exit 1
bash tools/ab_bench.sh "$OUT/cfg5" $V/var/libruleset_hip_capold.so $V/var/libruleset_hip_capper8.so $V/var/libruleset_hip_capper4.so -- --config cfg5 || exit 1
echo done
