#!/bin/bash
# CaRL conv1 split-bf16 form (conv1_mfma=bx3): its GPU tests, then the CaRL benchmark A/B against
# conv1_mfma=f32, alternating.   bash scripts/gpu_carla_bx.sh [tag]
set -o pipefail
TAG=${1:-carla_bx}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_carla.py \
  tests/test_gpu_carla_update.py -k "conv1 or update_vs or larger" > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "bx3|PASS|FAIL|Error|assert" $OUT/tests.log | tail -30; exit 1; }
grep -E "bx3|PASSED|FAILED" $OUT/tests.log
for rep in 1 2; do
  for opt in conv1_mfma=f32 conv1_mfma=bx3; do
    timeout -k 10 200 python scripts/bench_carla.py --batch 256 --update-batch 2048 --options $opt > $OUT/carla_${opt#*=}_$rep.jsonl 2>&1 || { echo "bench $opt failed"; tail -5 $OUT/carla_${opt#*=}_$rep.jsonl; exit 1; }
    echo "$opt rep$rep"; grep workload $OUT/carla_${opt#*=}_$rep.jsonl | cut -c1-200
  done
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bx3 -o kt -- \
  python3 $R/scripts/bench_carla.py --batch --update-batch 2048 --iters 5 --options conv1_mfma=bx3 > $OUT/trace_bx3.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
