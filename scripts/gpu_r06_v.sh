#!/bin/bash
# gradnorm=fold vs slices A/B (metric bench, E = 512 shard, cfg1 / cfg2 / cfg4 shard) + the trainer-iteration test.
set -o pipefail
TAG=${1:-r06v}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_trainer_iteration_vs_oracle_at_metric_size" > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "params max|FAILED|Error" $OUT/tests.txt | head; exit 1; }
grep -E "params max|passed" $OUT/tests.txt
ARMS="slices:-:gradnorm=slices fold:-:gradnorm=fold" BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh ${TAG}_e4096 3 || exit 1
ARMS="slices:-:gradnorm=slices fold:-:gradnorm=fold" BENCH_ARGS="--no-fp32-leg --num-envs 512 --steps 40" bash scripts/gpu_ab_multi.sh ${TAG}_e512 3 || exit 1
for o in slices fold slices fold; do
  timeout -k 10 300 python scripts/bench_configs.py --iters 3 --warmup 2 --options gradnorm=$o > $OUT/configs_$o.jsonl 2>&1 || { echo "configs $o failed"; tail -5 $OUT/configs_$o.jsonl; exit 1; }
  grep config $OUT/configs_$o.jsonl | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d["kernels_ms_per_iteration"]; print("'$o'", d["config"], d["ms_per_iteration"], "colsum", k.get("colsum"), "gradnorm", k.get("gradnorm"))'
done
