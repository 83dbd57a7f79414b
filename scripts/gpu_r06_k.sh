#!/bin/bash
# upd_split (k_upd + k_dwf in launch pairs of M / n rows): parity vs the oracle, then the A/B.
set -o pipefail
TAG=${1:-r06k}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py -k "split or metric_halfcheetah-" > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
ARMS="s1:-:upd_split=1 s2:-:upd_split=2 s4:-:upd_split=4 s8:-:upd_split=8" \
  BENCH_ARGS="--no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh $TAG 2
for a in s1 s4; do tail -1 $OUT/bench_${a}_2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms_per_step"])'; done
