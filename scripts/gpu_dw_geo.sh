#!/bin/bash
# k_dwf chunk geometry A/B (create options dw_rows / dw_slices) at the N = 8 / 4 / 1 shards.
#   bash scripts/gpu_dw_geo.sh <tag>
set -o pipefail
TAG=${1:-dwgeo}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
run() {  # E options
  timeout -k 10 200 python bench.py --num-envs $1 --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli ${2:+--options $2} > $OUT/b.log 2>&1 || { echo "bench E=$1 $2 failed"; tail -20 $OUT/b.log; exit 1; }
  echo "E=$1 ${2:-default}: $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "dw", k["dw"], "colsum", k["colsum"], "upd", k["fwdbwd"])')" | tee -a $OUT/summary.txt
}
run 512 && run 512 dw_rows=128 && run 512 dw_rows=128,dw_slices=1 && run 512 dw_rows=64,dw_slices=1 && \
run 1024 && run 1024 dw_rows=256 && run 1024 dw_rows=128,dw_slices=1 && \
run 4096 && run 4096 dw_rows=512 && run 4096 dw_slices=2 || exit 1
echo dwgeo-done
