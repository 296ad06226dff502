#!/bin/bash
# Round 6, step A: config 4 in one dispatch round (wg_step_kernel<7> at 123
# VGPRs), the GPU suite, the rtt and headline bench lines, and bench.py's
# multi-rank path executed once on the one-GPU box (2 ranks sharing cuda:0,
# gloo): gpurun_out/r06a/
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1
rc=$?; tail -n1 $O/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 $O/gpu.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --workload rtt --steps 100 --warmup 5 --no-cpu-baseline > $O/bench_rtt.log 2>&1 || { echo RTT FAIL; tail -20 $O/bench_rtt.log; exit 1; }
tail -n1 $O/bench_rtt.log | cut -c1-400
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo BENCH FAIL; tail -20 $O/bench_driver.log; exit 1; }
tail -n1 $O/bench_driver.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --share-gpu --steps 20 --warmup 5 > $O/bench_2ranks.log 2>&1 || { echo 2RANK FAIL; tail -30 $O/bench_2ranks.log; exit 1; }
tail -n1 $O/bench_2ranks.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --share-gpu --steps 20 --warmup 5 --global-envs 4096 > $O/bench_2ranks_g4096.log 2>&1 || { echo 2RANK4096 FAIL; tail -30 $O/bench_2ranks_g4096.log; exit 1; }
tail -n1 $O/bench_2ranks_g4096.log | cut -c1-300
