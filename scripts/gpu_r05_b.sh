#!/bin/bash
# Round 5: the new parity tests (teacher-forced AC e2e, cfg5 2048-row CaRL update, DD-PPO partial
# collections, CLI host/device at E = 4096, refused-create leak) and the cfg3 async-collection
# measurements (host cost 0 / 5 / 20 us per env step) with a kernel + marker trace.
#   bash scripts/gpu_r05_b.sh <tag>
set -o pipefail
TAG=${1:-r05b}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_e2e_teacher.py tests/test_gpu_ddppo.py tests/test_apps_gpu.py \
  "tests/test_gpu_update_headline.py::test_refused_options_free_the_context" \
  "tests/test_gpu_carla_update.py::test_update_cfg5_minibatch_2048_vs_torch" -s > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -60 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
bash scripts/async_sps.sh $TAG || exit 1
echo r05b-done
