#!/bin/bash
# Round 6, step H: the config-4 barrier diet adopted (one-barrier counts, the
# observer's kept ballot on an existing barrier, the step-start rebuild
# skipped when the tables are current) -- the GPU suite, the checks build's
# parity tests, smoke, the driver's command, per-phase stamps of config 4,
# config 4 at 8192 envs, then the rtt rocprofv3 evidence (tools/prof_headline.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1
rc=$?; tail -n1 $O/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 $O/gpu.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_host_components.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/checks.log 2>&1
rc=$?; tail -n1 $O/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 $O/checks.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 $O/smoke.log; exit 1; }
tail -n1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo BENCH FAIL; tail -20 $O/bench_driver.log; exit 1; }
tail -n1 $O/bench_driver.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 1 --workload rtt --envs 8192 --steps 100 --warmup 5 --no-other --no-cpu-baseline > $O/bench_rtt8192.log 2>&1 || { echo RTT8192 FAIL; tail -20 $O/bench_rtt8192.log; exit 1; }
tail -n1 $O/bench_rtt8192.log | cut -c1-300
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python3 tools/stamps.py rtt 1024 > $O/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; tail -20 $O/stamps_rtt.log; exit 1; }
tail -n 25 $O/stamps_rtt.log
timeout -k 10 900 bash tools/prof_headline.sh r06rtt2 rtt > $O/prof.log 2>&1 || { echo PROF FAIL; tail -20 $O/prof.log; exit 1; }
tail -n 5 $O/prof.log
