set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4.py -x -q --timeout 300 --timeout-method thread -k "index_and_scan or deferred or pht or uncapped or 10k_rules_spread or capped_zipf or cfg4_parity" > gpurun_out/bkt_tests.log 2>&1 || { tail -30 gpurun_out/bkt_tests.log; exit 1; }
tail -2 gpurun_out/bkt_tests.log
bash tools/ab_bench.sh gpurun_out/ab_bkt3 ruleset-analysis_amd/_build/libruleset_hip.so ruleset-analysis_amd/_build/var/libruleset_hip_serial.so > gpurun_out/ab_bkt3.txt 2>&1
cat gpurun_out/ab_bkt3.txt
timeout -k 10 300 bash tools/ablate_index.sh 1 2 4 > gpurun_out/ablate3.txt 2>&1; cat gpurun_out/ablate3.txt
