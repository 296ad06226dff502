# round-4 closing runs on the GPU box: bash tools/gpu_r04_final.sh <a|b>
#  a: the whole GPU suite, smoke(), the driver's bench command (with the CPU baseline)
#  b: rocprofv3 evidence of the kernels HEAD ships (headline, config 4)
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
if [ "${1:?a|b}" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04z_gputest.log 2>&1 || { echo TESTS FAIL; tail -40 gpurun_out/r04z_gputest.log; exit 1; }
  tail -1 gpurun_out/r04z_gputest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r04z_smoke.log; exit 1; }
  tail -1 gpurun_out/r04z_smoke.log
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04z_bench20.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r04z_bench20.log; exit 1; }
  tail -1 gpurun_out/r04z_bench20.log | cut -c1-400
else
  timeout -k 10 560 bash tools/prof_headline.sh r04z > gpurun_out/ph_r04z.log 2>&1 || { echo PROF FAIL; tail -20 gpurun_out/ph_r04z.log; exit 1; }
  timeout -k 10 560 bash tools/prof_headline.sh r04zrtt rtt > gpurun_out/ph_r04zrtt.log 2>&1 || { echo PROF RTT FAIL; tail -20 gpurun_out/ph_r04zrtt.log; exit 1; }
  grep -h "timed launch\|HBM traffic\|waiting" gpurun_out/ph_r04z/profiles/*summary.md gpurun_out/ph_r04zrtt/profiles/*summary.md
  if [ -f abmarl_amd/_build/libgw_engine_wunroll.so ]; then
    bash tools/ab_rtt.sh abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_wunroll.so || exit 1
  fi
fi
