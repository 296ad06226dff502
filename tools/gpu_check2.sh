# shuffled-action fixtures, full GPU suite, bench variants (20-step single launch vs 5x20)
timeout -k 10 300 python -u -m pytest tests/test_dict_api.py -x -q --timeout 120 --timeout-method thread -k "shuffle" > gpurun_out/shuffle.log 2>&1 && \
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --fragment 20 > gpurun_out/bench_s100_f20.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 5 > gpurun_out/bench_s200.log 2>&1
