#!/bin/bash
# k_upd's split-bf16 form (upd_mfma=bx6): its GPU tests, then the default bench line A/B against
# the fp32-MFMA k_upd (upd_mfma=16), alternating.   bash scripts/gpu_bx6.sh [tag]
set -o pipefail
TAG=${1:-bx6}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_update_headline.py \
  -k "bx6" > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "bx6 vs|worst|PASS|FAIL|Error|assert" $OUT/tests.log | tail -30; exit 1; }
grep -E "bx6 vs|worst|PASSED|FAILED" $OUT/tests.log
for rep in 1 2; do
  for opt in upd_mfma=16 upd_mfma=bx6; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cli --options $opt ${BENCH_ARGS} > $OUT/bench_${opt#*=}_$rep.log 2>&1 || { echo "bench $opt failed"; tail -5 $OUT/bench_${opt#*=}_$rep.log; exit 1; }
    echo "$opt rep$rep $(tail -1 $OUT/bench_${opt#*=}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
  done
done
