#!/bin/bash
# SQ counters of the CaRL 2048-row update kernels (verdict r04 item 7).   bash scripts/gpu_carla_ctr.sh <tag>
set -o pipefail
TAG=${1:-carlactr}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
CTR_CMD="scripts/bench_carla.py --batch --update-batch 2048 --iters 2" timeout -k 10 500 bash scripts/gpu_counters.sh ${TAG} "$P1" "$P2" > $OUT/sq.txt 2>&1 || { echo "counters failed"; tail -20 $OUT/sq.txt; exit 1; }
grep -E "^(conv|wgrad|dgrad|conv1_fwd|conv1_wgrad|conv2_[a-z]*) " $OUT/sq.txt
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- \
    python3 $R/scripts/bench_carla.py --batch --update-batch 2048 --iters 3 > $OUT/trace.log 2>&1) || { echo "trace failed"; exit 1; }
head -12 $OUT/trace/kt_kernel_stats.csv
