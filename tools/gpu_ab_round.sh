#!/bin/bash
# One GPU call of the round-2 classify/partition work: A/B of library variants
# on cfg3, GPU parity of the default library, classify ablation probe.
set -eo pipefail
export TMPDIR=/tmp
B=ruleset-analysis_amd/_build
tools/ab_bench.sh gpurun_out/ab1 "$@" $B/libruleset_hip.so > gpurun_out/ab1.txt 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest2.log 2>&1
timeout -k 10 300 python tools/classify_probe.py --variants "base;GROUP_TASKS=0;PROFILE_CLASSIFY=1;PROFILE_CLASSIFY=2;PROFILE_CLASSIFY=4;PROFILE_SKIP=2" > gpurun_out/probe.log 2>&1
