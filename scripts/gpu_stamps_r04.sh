#!/bin/bash
# Round-4 phase stamps: k_upd2 (cfg2), k_upd (metric), persistent rollout (E=512 / 4096).
#   bash scripts/gpu_stamps_r04.sh <tag>
set -o pipefail
TAG=${1:-stamps}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 240 python3 scripts/diag_stamps2.py $OUT/upd2_raw.npy > $OUT/kupd2_phases.txt 2>&1 || { echo "upd2 stamps failed"; tail -20 $OUT/kupd2_phases.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd2_phases.txt
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "hc stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_hc.txt
timeout -k 10 120 python3 scripts/roll_stamps.py > $OUT/roll_stamps.txt 2>&1 || { echo "roll stamps failed"; tail -20 $OUT/roll_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/roll_stamps.txt
