export PPO_HIP_LIB=$GRAFT_REPO_ROOT/ppo.cpp_amd/lib/libppo_hip_stamps.so ACT_MICRO_CASES="1,17,6,256"
for d in 0 1 2 3 4 7; do PPO_ACT_DIAG=$d timeout -k 10 100 python scripts/act_micro.py || exit 1; done
