timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/bench_final.log 2>&1
