#!/usr/bin/env python3
"""Per-iteration time of the BASELINE configs other than the metric one, on one MI355X with the
device-resident synthetic env of each config's shape (random-init agent):
  cfg2  ppo_continuous_action Humanoid-v4 (O=376, A=17), 2x64 tanh MLP, E=1024, T=2048, 32 x 10 updates
  cfg4  ac_ppo_continuous_action Ant-v5 (O=105, A=8), E=8192 over 8 GPUs -> the E=1024 shard of one GPU
        (no collectives here), T=128, 4 x 4 updates of 32 768 rows
  cfg1  ppo_continuous_action HalfCheetah-v5 defaults (E=1, T=2048, 32 x 10 updates of 64 rows) on the GPU
        path (the reference runs it on the CPU; its arithmetic is timed as bench.py's cpu_baseline cfg1)
Prints one JSON line per config: ms per iteration, env steps/s on this GPU and the HIP-event time
of every kernel class per iteration (the events themselves add a few us per launch)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import ppo_amd  # noqa: E402


def run(name, cfg, iters, warmup, options=None):
    tr = ppo_amd.Trainer(cfg, options=options)
    for _ in range(warmup):
        tr.iterate()
    tr.agent.sync()
    # untimed pass with per-kernel events, then a timed pass without them
    tr.agent.profile_reset()
    tr.agent.profile(0xFFFF)
    tr.iterate()
    tr.agent.sync()
    tr.agent.profile(0)
    prof = tr.agent.profile_read()
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.iterate()
    tr.agent.sync()
    dt = (time.perf_counter() - t0) / iters
    steps = cfg.num_envs * cfg.num_steps
    out = {"config": name, **({"options": options} if options else {}), "num_envs": cfg.num_envs, "num_steps": cfg.num_steps, "env_id": cfg.env_id,
           "ms_per_iteration": round(dt * 1e3, 3), "env_steps_per_s": round(steps / dt, 1),
           "kernels_ms_per_iteration": {k: round(v[0], 3) for k, v in prof.items()},
           "kernels_ms_note": "one separate iteration with a HIP-event pair around every kernel class: each pair "
                              "adds its own overhead, so the sum can exceed ms_per_iteration (timed without events)"}
    print(json.dumps(out), flush=True)
    tr.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--only", default="", help="cfg2, cfg4_shard or cfg1")
    ap.add_argument("--options", default=None, help="ppo_create_ex options (A/B runs)")
    args = ap.parse_args()
    ppo_amd.set_device(0)
    n = args.iters + args.warmup + 2
    if args.only in ("", "cfg2"):
        run("cfg2", ppo_amd.PPOConfig(env_id="Humanoid-v4", num_envs=1024, num_steps=2048,
                                      total_timesteps=1024 * 2048 * n), args.iters, args.warmup, args.options)
    if args.only in ("", "cfg4_shard"):
        run("cfg4_shard", ppo_amd.ACPPOConfig(env_id="Ant-v5", num_envs=1024, num_steps=128,
                                              total_timesteps=1024 * 128 * n), args.iters, args.warmup, args.options)
    if args.only in ("", "cfg1"):
        run("cfg1", ppo_amd.PPOConfig(env_id="HalfCheetah-v5", num_envs=1, num_steps=2048,
                                      total_timesteps=2048 * n), args.iters, args.warmup, args.options)


if __name__ == "__main__":
    main()
