#!/bin/bash
# round-3 closing run 2 (HEAD: dispatch-recorded events): GPU suite, smoke,
# driver's command, default bench; SQ counters of config 4's kernel
set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py > gpurun_out/bench_final.log 2>&1 || exit 1
bash tools/pmc_sq_workload.sh rtt_r03 rtt > gpurun_out/sq_rtt_r03.txt 2>&1
