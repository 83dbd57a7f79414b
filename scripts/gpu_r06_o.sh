#!/bin/bash
# k_upd hand-off stores issued from inside the next GEMM (PPO_UPD_DEFER) vs the default: A/B on the
# metric bench, then the update parity tests on the defer library.   bash scripts/gpu_r06_o.sh <tag>
set -o pipefail
TAG=${1:-r06o}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ARMS="base:-:- defer:ppo.cpp_amd/lib/libppo_hip_defer.so:-" BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh $TAG 3 || exit 1
export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_defer.so
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py tests/test_gpu_e2e_teacher.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
