#!/bin/bash
# k_dwf_dma priority A/B at E = 4096 and 512.   bash scripts/gpu_dwprio.sh <tag>
set -o pipefail
TAG=${1:-dwprio}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for E in 4096 512; do
  for o in "" dw_sched=1 "" dw_sched=1; do
    timeout -k 10 200 python bench.py --num-envs $E --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli ${o:+--options $o} > $OUT/b.log 2>&1 || { echo "bench E=$E $o failed"; tail -20 $OUT/b.log; exit 1; }
    echo "E=$E ${o:-default}: $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "dw", k["dw"], "upd", k["fwdbwd"])')" | tee -a $OUT/summary.txt
  done
done
