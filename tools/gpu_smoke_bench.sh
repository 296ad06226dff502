set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench1.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench1.log; exit 1; }
tail -3 gpurun_out/bench1.log
