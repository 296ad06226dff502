timeout -k 10 300 python -u -m pytest tests/test_maze_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/maze.log 2>&1 && \
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
