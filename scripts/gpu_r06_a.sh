#!/bin/bash
# Round-6 first check: the tests this round touched, then one default bench line (fp32 leg, dW frac).
#   bash scripts/gpu_r06_a.sh <tag>
set -o pipefail
TAG=${1:-r06a}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_golden_widths.py -k gae tests/test_gpu_parity.py::test_gae_scan_matches_serial \
  tests/test_gpu_parity.py::test_cfg1_shape_iteration_vs_oracle \
  tests/test_gpu_carla_update.py::test_generic_wgrad_sample_groups_match_one_pass \
  tests/test_gpu_carla.py::test_packed_conv1_odd_block_counts_match_generic \
  tests/test_bench_gpu.py::test_bench_single_rank_line > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
grep -E "max \|adv" $OUT/tests.txt | head
timeout -k 10 400 python bench.py --no-cli --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-2500
