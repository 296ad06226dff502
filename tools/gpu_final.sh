#!/bin/bash
# closing run on the GPU box with the tree's build: the whole GPU suite,
# smoke, the driver's bench command and the default bench
set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py > gpurun_out/bench_final.log 2>&1
