#!/bin/bash
# conv1=packed (k_conv_img3) vs staged: tests, then the CaRL benchmark and kernel trace for both.
#   bash scripts/gpu_carla_c1.sh <tag>
set -o pipefail
TAG=${1:-carlac1}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -s \
  "tests/test_gpu_carla.py::test_packed_conv1_matches_staged" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
grep -E "passed|failed" $OUT/tests.txt | tail -1
for O in conv1=staged conv1=packed; do
  timeout -k 10 300 python scripts/bench_carla.py --options $O > $OUT/bench_${O#conv1=}.jsonl 2>&1 || { echo "bench $O failed"; tail -5 $OUT/bench_${O#conv1=}.jsonl; exit 1; }
  echo "$O"; cut -c1-200 $OUT/bench_${O#conv1=}.jsonl
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_packed -o kt -- \
    python3 $R/scripts/bench_carla.py --batch 256 --update-batch 2048 --iters 3 --options conv1=packed > $OUT/trace_packed.log 2>&1) || { echo "trace failed"; exit 1; }
head -6 $OUT/trace_packed/kt_kernel_stats.csv
