#!/bin/bash
# Round-5 first box: SQ counter sets of k_upd / k_upd32 / mix at the metric config (verdict item 4),
# and the E = 512 shard with and without update_graph=1 (item 3).   bash scripts/gpu_r05_a.sh <tag>
set -o pipefail
TAG=${1:-r05a}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for V in 16 32 mix; do
  CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --options upd_mfma=$V" \
    timeout -k 10 400 bash scripts/gpu_counters.sh ${TAG}_upd$V "$P1" "$P2" > $OUT/sq_upd$V.txt 2>&1 || { echo "counters $V failed"; tail -20 $OUT/sq_upd$V.txt; exit 1; }
  grep -E "^(fwdbwd|dw) " $OUT/sq_upd$V.txt
done
for G in 0 1; do
  timeout -k 10 120 python bench.py --num-envs 512 --steps 30 --warmup 3 --no-cpu-baseline --no-cli --options update_graph=$G > $OUT/e512_graph$G.log 2>&1 || { echo "e512 graph=$G failed"; tail -20 $OUT/e512_graph$G.log; exit 1; }
  tail -1 $OUT/e512_graph$G.log | cut -c1-300
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_e512 -o kt -- \
    python3 $R/bench.py --num-envs 512 --steps 10 --warmup 2 --no-cpu-baseline --no-cli > $OUT/trace_e512.log 2>&1) || { echo "trace failed"; exit 1; }
echo r05a-done
