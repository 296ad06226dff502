# maze tests, maze timing, rocprof of the maze kernel, RCCL path at world size 1
mkdir -p gpurun_out/prof_maze
timeout -k 10 300 python -u -m pytest tests/test_maze_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/maze.log 2>&1 && \
timeout -k 10 120 python tools/maze_bench.py > gpurun_out/maze_bench.log 2>&1 && \
timeout -k 10 120 python tools/maze_bench.py --rows 32 --cols 32 --envs 2048 >> gpurun_out/maze_bench.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_maze -o maze -- python3 tools/maze_bench.py > gpurun_out/maze_prof.log 2>&1 && \
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_rccl1.log 2>&1
