#!/bin/bash
set -o pipefail
bash tools/gpu_ab_r03g.sh || exit 1
bash tools/gpu_ab_r03h.sh
