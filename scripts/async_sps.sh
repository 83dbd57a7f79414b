#!/bin/bash
# cfg3 (AC-PPO HalfCheetah shapes, E = 4096, host envs in async collection groups): SPS of the drop-in
# CLI at host costs of 0 / 5 / 20 us per env step, then a rocprofv3 kernel + marker (roctx) trace of
# the 5 us run for the overlap analysis (scripts/async_overlap.py).   bash scripts/async_sps.sh <tag>
set -o pipefail
TAG=${1:-async}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG/async
mkdir -p $OUT
EXE=$R/ppo.cpp_amd/bin/ac_ppo_continuous_action
for US in 0 5 20; do
  for G in 0 16; do
    timeout -k 10 200 $EXE --env_id SyntheticCheetah-v0 --env_backend host --num_envs 4096 --num_steps 128 \
      --total_timesteps $((4096*128*4)) --num_eval_runs 1 --host_step_us $US --num_collect_groups $G \
      --exp_name_stem async_${US}_$G > $OUT/cli_us${US}_g$G.log 2>&1 || { echo "cli us=$US g=$G failed"; tail -20 $OUT/cli_us${US}_g$G.log; exit 1; }
    echo "us=$US groups=$G $(grep -m1 'collection groups' $OUT/cli_us${US}_g$G.log) $(grep SPS: $OUT/cli_us${US}_g$G.log | tr '\n' ' ')"
  done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/trace_us5 -o tr -- \
   $EXE --env_id SyntheticCheetah-v0 --env_backend host --num_envs 4096 --num_steps 128 \
   --total_timesteps $((4096*128*2)) --num_eval_runs 1 --host_step_us 5 --exp_name_stem async_trace > $OUT/trace_us5.log 2>&1) || { echo "trace failed"; tail -20 $OUT/trace_us5.log; exit 1; }
find $OUT/trace_us5 -name "*.csv" | head
echo async-done
