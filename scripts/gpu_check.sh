#!/bin/bash
# GPU-box check: parity tests, smoke(), default bench line (with CPU baseline), per-kernel bench.
#   bash scripts/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --profile-all --no-cpu-baseline > $OUT/bench_all.log 2>&1 || { echo "bench profile-all failed"; tail -30 $OUT/bench_all.log; exit 1; }
tail -1 $OUT/bench_all.log
echo done
