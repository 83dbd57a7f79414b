#!/bin/bash
# CaRL batch-32 forward: tests, bench, and the per-launch durations of the last traced forward.
#   bash scripts/gpu_carla_fwd.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-carlafwd}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_carla.py tests/test_gpu_carla_update.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
  tail -2 $OUT/tests.txt
fi
timeout -k 10 300 python3 scripts/bench_carla.py --batch 32 256 --update-batch --iters 50 > $OUT/carla.jsonl 2>&1 || { echo "bench failed"; tail -20 $OUT/carla.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/carla.jsonl
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- \
  python3 $R/scripts/bench_carla.py --batch 32 --update-batch --iters 20 > $OUT/kt.log 2>&1) || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
python3 scripts/carla_trace.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) forward
