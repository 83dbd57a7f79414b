#!/bin/bash
# rocprofv3 kernel trace of scripts/bench_configs.py (cfg2 + cfg4 shard) -> per-kernel CSV summary.
# usage (on the GPU box): scripts/prof_cfg.sh <out-dir> [extra env assignments are inherited]
set -e
OUT=${1:-gpurun_out/prof_cfg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o kt -- \
  python3 scripts/bench_configs.py --iters 1 --warmup 1
