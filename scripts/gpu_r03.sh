#!/bin/bash
# Round-3 GPU check: the given test files first (verbose), then the whole -m gpu suite and smoke().
#   bash scripts/gpu_r03.sh <tag> <test files...>
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $OUT/new_tests.log; exit 1; }
  tail -3 $OUT/new_tests.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_all.log 2>&1 || { echo "gpu suite failed"; grep -E "FAILED|Error|error" $OUT/gpu_all.log | head -20; tail -40 $OUT/gpu_all.log; exit 1; }
tail -2 $OUT/gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli > $OUT/bench_all.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_all.log; exit 1; }
  tail -1 $OUT/bench_all.log | cut -c1-600
  timeout -k 10 300 python bench.py --num-envs 512 --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli > $OUT/bench_e512.log 2>&1 || { echo "bench e512 failed"; tail -30 $OUT/bench_e512.log; exit 1; }
  tail -1 $OUT/bench_e512.log | cut -c1-600
  timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; tail -20 $OUT/configs.jsonl; exit 1; }
  cut -c1-300 $OUT/configs.jsonl
fi
echo done
