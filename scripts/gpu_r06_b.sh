#!/bin/bash
# k_upd round-6 change: the update parity tests on the new default library, then an A/B of the bench
# line: base (round-5 k_upd) / noearly / new (default).   bash scripts/gpu_r06_b.sh <tag>
set -o pipefail
TAG=${1:-r06b}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py tests/test_gpu_parity.py \
  tests/test_gpu_e2e_teacher.py tests/test_gpu_e2e.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
ARMS="base:ppo.cpp_amd/lib/libppo_hip_base.so:- noearly:ppo.cpp_amd/lib/libppo_hip_noearly.so:- new:-:-" \
  BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh $TAG 3
