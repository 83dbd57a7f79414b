set -o pipefail
X=ppo.cpp_amd/bin/ac_ppo_continuous_action
ls ppo.cpp_amd/bin >/dev/null || X=$(find ppo.cpp_amd -name ac_ppo_continuous_action -type f | head -1)
C="--env_id SyntheticCheetah-v0 --num_envs 4096 --num_steps 128 --total_timesteps ${TOTAL:-5242880} --seed 1 --num_eval_runs 0"
mkdir -p gpurun_out/cli
timeout -k 10 180 $X $C --env_backend device --exp_name_stem cli_dev > gpurun_out/cli/dev.log 2>&1 || { tail -5 gpurun_out/cli/dev.log; exit 1; }
grep SPS gpurun_out/cli/dev.log | tail -2
for g in ${GROUPS_LIST:-2 4 8 16}; do
timeout -k 10 300 $X $C --env_backend host --num_collect_groups $g --exp_name_stem cli_host$g > gpurun_out/cli/host$g.log 2>&1 || { tail -5 gpurun_out/cli/host$g.log; exit 1; }
grep SPS gpurun_out/cli/host$g.log | tail -2
done
nproc; grep -m1 "model name" /proc/cpuinfo
