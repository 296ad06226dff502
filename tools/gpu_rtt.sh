set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K="workgroup or config4 or wide or reach_the_target_configs or rtt_64"
GW_ENGINE_VARIANT=checks timeout -k 10 400 python -u -m pytest tests/test_engine_golden.py tests/test_engine_oracle.py -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/rtt_checks.log 2>&1
rc=$?; tail -5 gpurun_out/rtt_checks.log; [ $rc -eq 0 ] || { echo "CHECKS FAILED rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/rtt_checks.log | head -30; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_engine_golden.py tests/test_engine_oracle.py -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/rtt.log 2>&1
rc=$?; tail -5 gpurun_out/rtt.log; [ $rc -eq 0 ] || { echo "FAILED rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/rtt.log | head -30; exit 1; }
