#!/bin/bash
# round-3 session j: dispatch-recorded launch events in the timed region --
# the driver's command three times (fresh processes), Pacman, parity subset
set -o pipefail
: > gpurun_out/bench_s20_j.jsonl
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/j_s20.log 2>&1 || { tail -20 gpurun_out/j_s20.log; exit 1; }
  grep '^{' gpurun_out/j_s20.log >> gpurun_out/bench_s20_j.jsonl
done
timeout -k 10 200 python3 bench.py --workload pacman --steps 200 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/j_pac.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_j.log 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rollout.py tests/test_pacman_engine.py \
    > gpurun_out/tests_j.log 2>&1
