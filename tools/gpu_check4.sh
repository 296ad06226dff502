timeout -k 10 300 python -u -m pytest tests/test_engine_golden.py -x -q --timeout 120 --timeout-method thread -k "shuffled or workgroup" > gpurun_out/wg_shuffle.log 2>&1 && \
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
