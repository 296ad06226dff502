# Pacman checks + A/B of HEAD against a previous build: bash tools/gpu_r04h.sh <lib.so>
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pacman or turn or f3" > gpurun_out/r04h_checks.log 2>&1 || { echo CHECKS FAIL; tail -30 gpurun_out/r04h_checks.log; exit 1; }
tail -1 gpurun_out/r04h_checks.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pacman or turn or f3" > gpurun_out/r04h_prod.log 2>&1 || { echo PROD FAIL; tail -30 gpurun_out/r04h_prod.log; exit 1; }
tail -1 gpurun_out/r04h_prod.log
bash tools/ab_pac.sh abmarl_amd/_build/libgw_engine.so ${1:?lib} abmarl_amd/_build/libgw_engine.so ${1}
