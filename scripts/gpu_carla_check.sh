#!/bin/bash
# CaRL agent check: its -m gpu tests, the forward / update benchmark, a kernel trace of the batch-32
# forward.   bash scripts/gpu_carla_check.sh <tag>
set -o pipefail
TAG=${1:-carla}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_carla.py tests/test_gpu_carla_update.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 300 python3 scripts/bench_carla.py > $OUT/carla.jsonl 2>&1 || { echo "bench failed"; tail -20 $OUT/carla.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/carla.jsonl
for o in tail=layers tail=staged tail=fused; do
  timeout -k 10 120 python3 scripts/bench_carla.py --batch 32 --update-batch --iters 50 --options $o 2>&1 | grep workload || { echo "bench $o failed"; exit 1; }
done
# per-kernel trace of the per-layer path (the cooperative launch is not traced here)
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 $R/scripts/bench_carla.py --batch 32 --update-batch --iters 50 --options tail=staged > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-4 {} | head -20
