#!/usr/bin/env python3
"""Forward throughput of the CaRL CNN agent (BASELINE config 5 shapes: bev uint8
[n, 15, 192, 192], 8 measurements, 3 value measurements, 2 actions) on one GPU: samples/s of
ppo_carla_forward with inputs resident in HBM, and the algorithmic MFMA rate (87.9 MFLOP per sample,
SURVEY §8d), and of the PPO minibatch update (ppo_carla_update, counted as 3x the forward:
forward + two backward GEMMs per layer)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402
import carla_inputs as CI  # noqa: E402

FLOP_PER_SAMPLE = 87_907_008  # SURVEY §8d (conv + MLP forward, 2 K N per layer)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="*", default=[32, 256])
    ap.add_argument("--update-batch", type=int, nargs="*", default=[256, 2048])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--options", default="", help="ppo_carla_create_ex options, e.g. tail=layers")
    args = ap.parse_args()
    ppo_amd.set_device(0)
    L = CI.layout()
    p = CI.params(L)
    for n in args.batch:
        ag = ppo_amd.CarlaAgent(max_batch=n, options=args.options or None)
        ag.load_params(p)
        bev, meas, vmeas, _ = CI.inputs(n)
        d = [ppo_amd.DeviceArray.from_numpy(bev, np.uint8), ppo_amd.DeviceArray.from_numpy(meas),
             ppo_amd.DeviceArray.from_numpy(vmeas)]
        A = ag.layout.A
        out = [ppo_amd.DeviceArray(sh) for sh in ((n, A), (n,), (n,), (n,), (n, A), (n, A))]
        for _ in range(3):
            ag.forward(*d, sample_type="sample", out=out)
        # rollout pattern: one forward, then wait for its actions (output buffers preallocated)
        t0 = time.perf_counter()
        for i in range(args.iters):
            ag.forward(*d, sample_type="sample", step_id=i, out=out)
        dt = (time.perf_counter() - t0) / args.iters
        # device time: forwards back to back, one wait at the end
        t0 = time.perf_counter()
        for i in range(args.iters):
            ag.forward(*d, sample_type="sample", step_id=i, out=out, sync=False)
        ppo_amd.lib().ppo_device_sync()
        dd = (time.perf_counter() - t0) / args.iters
        print(json.dumps({"workload": "carla_forward", "batch": n, "options": args.options, "ms_per_forward": round(dt * 1e3, 3),
                          "ms_per_forward_back_to_back": round(dd * 1e3, 3), "samples_per_s": round(n / dt, 1),
                          "tflops": round(n * FLOP_PER_SAMPLE / dt / 1e12, 2)}), flush=True)
        ag.close()
    for n in args.update_batch:
        ag = ppo_amd.CarlaAgent(max_batch=n, options=args.options or None)
        ag.load_params(p)
        rng = np.random.default_rng(1)
        bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
        f32 = lambda *shape: ppo_amd.DeviceArray.from_numpy(rng.uniform(-1, 1, shape).astype(np.float32))  # noqa: E731
        d = [ppo_amd.DeviceArray.from_numpy(bev, np.uint8), f32(n, 8), f32(n, 3), f32(n, 2), f32(n), f32(n), f32(n),
             f32(n)]
        for _ in range(2):
            ag.update(*d, want_stats=False)
        ppo_amd.lib().ppo_device_sync()
        t0 = time.perf_counter()
        its = max(3, args.iters // 4)
        for _ in range(its):
            ag.update(*d, want_stats=False)
        ppo_amd.lib().ppo_device_sync()
        dt = (time.perf_counter() - t0) / its
        print(json.dumps({"workload": "carla_update", "batch": n, "options": args.options, "ms_per_update": round(dt * 1e3, 3),
                          "samples_per_s": round(n / dt, 1),
                          "tflops": round(3 * n * FLOP_PER_SAMPLE / dt / 1e12, 2)}), flush=True)
        ag.close()


if __name__ == "__main__":
    main()
