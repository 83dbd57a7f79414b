#!/bin/bash
set -o pipefail
TAG=${1:-dw2full}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden_widths.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py --only cfg2 > $OUT/c.log 2>&1 || { echo "cfg2 failed"; tail -20 $OUT/c.log; exit 1; }
  grep config $OUT/c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_iteration"]; print(d["ms_per_iteration"], "upd2", k["fwdbwd"], "dw", k["dw"])'
done
