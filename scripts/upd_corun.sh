#!/bin/bash
# k_upd co-run analysis on the GPU box (stamps build): per-phase cycles and kernel time with both
# trunks, the critic alone and the actor alone (PPO_UPD_TRUNK, diagnostic builds only).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/corun_${1:-dev}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in both 0 1; do
  if [ $V = both ]; then unset PPO_UPD_TRUNK; else export PPO_UPD_TRUNK=$V; fi
  timeout -k 10 240 python3 -u $R/scripts/diag_stamps.py $OUT/raw_$V.npy > $OUT/stamps_$V.txt 2>&1 || { tail -5 $OUT/stamps_$V.txt; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$V -o run -- python3 $R/scripts/diag_stamps.py > $OUT/prof_$V.log 2>&1 || { tail -5 $OUT/prof_$V.log; exit 1; }
  echo "== $V"; cat $OUT/stamps_$V.txt | grep -v Warning
  f=$(find $OUT/prof_$V -name "*kernel_stats.csv" | head -1); grep -E "k_upd|k_dwf" $f | cut -c1-160
done
