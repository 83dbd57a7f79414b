#!/bin/bash
# CaRL update A/B: the GPU tests matching a -k filter, then the 2 048-row update benchmark for two
# option strings, alternating, then a kernel trace (per-launch durations) of the second.
#   bash scripts/gpu_carla_ab.sh <tag> "<pytest -k>" "<options A>" "<options B>"
set -o pipefail
TAG=${1:-carla_ab}
KSEL=$2
OA=$3
OB=$4
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ -n "$KSEL" ]; then
  timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_carla.py \
    tests/test_gpu_carla_update.py -k "$KSEL" > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|assert" $OUT/tests.log | tail -30; exit 1; }
  grep -E "PASSED|FAILED" $OUT/tests.log
fi
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then opt=$OA; else opt=$OB; fi
    timeout -k 10 200 python scripts/bench_carla.py --batch 256 --update-batch 2048 --options "$opt" > $OUT/carla_${v}_$rep.jsonl 2>&1 || { echo "bench $opt failed"; tail -5 $OUT/carla_${v}_$rep.jsonl; exit 1; }
    echo "$v=$opt rep$rep"; grep workload $OUT/carla_${v}_$rep.jsonl | cut -c1-200
  done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- \
  python3 $R/scripts/bench_carla.py --batch --update-batch 2048 --iters 3 --options "$OB" > $OUT/trace.log 2>&1) || { echo "trace failed"; exit 1; }
python3 scripts/carla_trace.py $(find $OUT/trace -name "*kernel_trace.csv" | head -1) > $OUT/update_launches.txt
tail -14 $OUT/update_launches.txt
echo done
