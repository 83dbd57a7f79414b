#!/bin/bash
# Round 5: the split-bf16 dW (k_dwf_bx, create option dw_mfma) — parity / accuracy tests, then the
# A/B at the metric config and at the N = 8 shard.   bash scripts/gpu_r05_c.sh <tag>
set -o pipefail
TAG=${1:-r05c}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_gpu_update_headline.py -k "bf16 or dw_mfma or split_bf16" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -60 $OUT/tests.txt; exit 1; }
grep -E "passed|failed" $OUT/tests.txt | tail -2
for E in 4096 512; do
  for D in f32 bf16x9 bf16x8; do
    timeout -k 10 120 python bench.py --num-envs $E --steps 20 --warmup 3 --no-cpu-baseline --no-cli --options dw_mfma=$D > $OUT/bench_e${E}_$D.log 2>&1 || { echo "bench $E $D failed"; tail -20 $OUT/bench_e${E}_$D.log; exit 1; }
    echo "E=$E $D $(tail -1 $OUT/bench_e${E}_$D.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bx9 -o kt -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cli --options dw_mfma=bf16x9 > $OUT/trace_bx9.log 2>&1) || { echo "trace failed"; exit 1; }
head -6 $OUT/trace_bx9/*kernel_stats.csv
echo r05c-done
