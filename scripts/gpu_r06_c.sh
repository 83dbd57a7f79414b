#!/bin/bash
# k_vbx critic pass (deferred per-step critic) tests, then the single-change k_upd A/B.
set -o pipefail
TAG=${1:-r06c}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
[ -n "$SKIPTESTS" ] || timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rollout.py tests/test_gpu_golden_widths.py -k "not update" \
  tests/test_gpu_parity.py::test_full_iteration_vs_oracle tests/test_gpu_ddppo.py \
  tests/test_apps_gpu.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
ARMS="off:ppo.cpp_amd/lib/libppo_hip_off.so:- chan:ppo.cpp_amd/lib/libppo_hip_chan.so:- bar:ppo.cpp_amd/lib/libppo_hip_bar.so:- pre:ppo.cpp_amd/lib/libppo_hip_pre.so:- bf:ppo.cpp_amd/lib/libppo_hip_bf.so:- ch2:ppo.cpp_amd/lib/libppo_hip_ch2.so:- new:-:-" \
  BENCH_ARGS="--no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh $TAG 2
