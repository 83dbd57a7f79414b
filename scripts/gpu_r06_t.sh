#!/bin/bash
# gradnorm=fold (clip_grad_norm_'s sums of squares inside k_colsum) vs slices (k_gradnorm): the tests that
# touch the norm path, then A/B on the metric bench, the E = 512 shard and cfg1 / cfg2.
set -o pipefail
TAG=${1:-r06t}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rollout.py tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py tests/test_gpu_e2e_teacher.py \
  tests/test_gpu_e2e.py tests/test_gpu_comm.py "tests/test_gpu_parity.py::test_trainer_iteration_vs_oracle_at_metric_size" -s > $OUT/tests.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.txt | head; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
ARMS="slices:-:gradnorm=slices fold:-:gradnorm=fold" BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh ${TAG}_e4096 3 || exit 1
ARMS="slices:-:gradnorm=slices fold:-:gradnorm=fold" BENCH_ARGS="--no-fp32-leg --num-envs 512 --steps 40" bash scripts/gpu_ab_multi.sh ${TAG}_e512 3 || exit 1
for o in slices fold; do
  timeout -k 10 300 python scripts/bench_configs.py --iters 3 --warmup 2 --options gradnorm=$o > $OUT/configs_$o.jsonl 2>&1 || { echo "configs $o failed"; tail -5 $OUT/configs_$o.jsonl; exit 1; }
  grep config $OUT/configs_$o.jsonl | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("'$o'", d["config"], d["ms_per_iteration"], d["kernels_ms_per_iteration"].get("colsum"), d["kernels_ms_per_iteration"].get("gradnorm"))'
done
