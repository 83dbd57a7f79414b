#!/bin/bash
# Round 6: update parity tests + the k_vbx critic test on the default library, the k_upd combination
# A/B, the dW L2-hot diagnostic (bf16x6) and the k_upd phase stamps.   bash scripts/gpu_r06_f.sh <tag>
set -o pipefail
TAG=${1:-r06f}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py \
  tests/test_gpu_e2e_teacher.py tests/test_gpu_e2e.py tests/test_gpu_rollout.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
grep -E "critic vs oracle" $OUT/tests.txt
ARMS="off:ppo.cpp_amd/lib/libppo_hip_off.so:- notop:ppo.cpp_amd/lib/libppo_hip_notop.so:- new:-:-" \
  BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh $TAG 3 || exit 1
bash scripts/gpu_r06_e.sh $TAG
