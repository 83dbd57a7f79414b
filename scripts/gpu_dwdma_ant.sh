#!/bin/bash
# k_dw_dma A/B: the bitwise tests, then the cfg4 shard with dw_dma=0 (k_dw) and the default.
#   bash scripts/gpu_dwdma_ant.sh <tag>
set -o pipefail
TAG=${1:-dwant}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden_widths.py tests/test_gpu_update_headline.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for o in dw_dma=0 ""; do
  timeout -k 10 300 python3 scripts/bench_configs.py --only cfg4_shard ${o:+--options $o} > $OUT/c.log 2>&1 || { echo "cfg4 $o failed"; tail -20 $OUT/c.log; exit 1; }
  grep config $OUT/c.log | tee -a $OUT/summary.jsonl | cut -c1-420
done
