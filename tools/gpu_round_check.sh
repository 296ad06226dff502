timeout -k 10 300 python -u -m pytest tests/test_maze_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/maze.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1
