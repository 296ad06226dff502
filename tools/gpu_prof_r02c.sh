bash tools/profile.sh r02c team_battle rollout 100 > gpurun_out/prof_r02c_f100.out 2>&1 && \
bash tools/profile.sh r02c_f20 team_battle rollout 20 > gpurun_out/prof_r02c_f20.out 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_final.log 2>&1
