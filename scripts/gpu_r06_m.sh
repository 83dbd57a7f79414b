#!/bin/bash
# update_graph=1 (the minibatch loop replayed as one hipGraph) vs eager on the other configs.
set -o pipefail
TAG=${1:-r06m}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in 1 2; do
  timeout -k 10 300 python scripts/bench_configs.py --iters 4 --warmup 2 > $OUT/eager_$rep.jsonl 2>&1 || { echo "eager failed"; tail -5 $OUT/eager_$rep.jsonl; exit 1; }
  timeout -k 10 300 python scripts/bench_configs.py --iters 4 --warmup 2 --options update_graph=1 > $OUT/graph_$rep.jsonl 2>&1 || { echo "graph failed"; tail -5 $OUT/graph_$rep.jsonl; exit 1; }
  for f in eager graph; do grep config $OUT/${f}_$rep.jsonl | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("'$f'", d["config"], d["ms_per_iteration"])'; done
done
for E in 512 4096; do
  for o in update_graph=0 update_graph=1; do
    timeout -k 10 120 python bench.py --num-envs $E --steps 20 --warmup 3 --no-cpu-baseline --no-cli --no-fp32-leg --options $o > $OUT/bench_e${E}_$o.log 2>&1 || { echo "bench failed"; exit 1; }
    echo "E=$E $o $(tail -1 $OUT/bench_e${E}_$o.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
