timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-other --preroll 20000 > gpurun_out/b20a.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-other > gpurun_out/b20b.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-other --preroll 20000 > gpurun_out/b20c.log 2>&1
