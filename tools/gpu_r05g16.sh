#!/bin/bash
# Round 5: Pacman's full-grid observation as aligned 16-byte group stores
# (build grp16) -- parity, A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out/r05g16
export TMPDIR=/tmp
L=abmarl_amd/_build/ab/grp16/libgw_engine.so
GW_ENGINE_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g16/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05g16/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05g16/tests.log; exit 1; }
timeout -k 10 600 bash tools/ab_libs.sh r05g16/ab_pac_roll "head=- grp16=$L" --workload pacman --steps 200 --warmup 5 --fragment 50 --preroll 200 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh r05g16/ab_pac_step "head=- grp16=$L" --workload pacman --mode step --steps 200 --warmup 5 --preroll 200 || exit 1
