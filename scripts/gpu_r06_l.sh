#!/bin/bash
# H1 recompute in k_dwf_bx: bitwise test vs the stored H1, the update parity tests, then store vs recompute A/B.
set -o pipefail
TAG=${1:-r06l}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py -k "h1_recompute" > $OUT/tests_rc.txt 2>&1 || { echo "recompute tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_rc.txt | head; tail -30 $OUT/tests_rc.txt; exit 1; }
tail -2 $OUT/tests_rc.txt
ARMS="store:-:h1_handoff=store rc:-:h1_handoff=recompute" BENCH_ARGS="--no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh $TAG 3 || exit 1
for a in store rc; do tail -1 $OUT/bench_${a}_3.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms_per_step"])'; done
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py \
  tests/test_gpu_e2e_teacher.py tests/test_gpu_e2e.py tests/test_gpu_rollout.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
