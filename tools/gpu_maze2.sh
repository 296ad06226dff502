timeout -k 10 300 python -u -m pytest tests/test_maze_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/maze.log 2>&1 && \
timeout -k 10 120 python tools/maze_bench.py > gpurun_out/maze_bench.log 2>&1 && \
timeout -k 10 120 python tools/maze_bench.py --rows 32 --cols 32 --envs 2048 >> gpurun_out/maze_bench.log 2>&1 && \
bash tools/gpu_prof_r02c.sh
