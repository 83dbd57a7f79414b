#!/bin/bash
# k_dwf_dma A/B: the bitwise test, then bench.py with and without dw_dma=1 at E = 4096 and 512.
#   bash scripts/gpu_dwdma.sh <tag>
set -o pipefail
TAG=${1:-dwdma}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k fused_dw -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for E in 4096 512; do
  for o in "" dw_dma=1; do
    timeout -k 10 200 python bench.py --num-envs $E --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli ${o:+--options $o} > $OUT/b.log 2>&1 || { echo "bench E=$E $o failed"; tail -20 $OUT/b.log; exit 1; }
    echo "E=$E ${o:-default}: $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "dw", k["dw"], "colsum", k["colsum"], "upd", k["fwdbwd"])')" | tee -a $OUT/summary.txt
  done
done
