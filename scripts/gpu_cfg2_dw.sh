#!/bin/bash
# cfg2 k_dw2 row-chunk A/B (create option dw_rows): split-K partial bytes (k_dw2 writes, k_colsum
# reads) against k_dw2's parallelism.   bash scripts/gpu_cfg2_dw.sh <tag>
set -o pipefail
TAG=${1:-cfg2dw}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for o in "" dw_rows=512 dw_rows=384 dw_rows=128; do
  timeout -k 10 300 python3 scripts/bench_configs.py --only cfg2 ${o:+--options $o} > $OUT/c.log 2>&1 || { echo "cfg2 $o failed"; tail -20 $OUT/c.log; exit 1; }
  grep config $OUT/c.log | tee -a $OUT/summary.jsonl | cut -c1-420
done
