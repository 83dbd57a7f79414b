#!/usr/bin/env python3
"""bench.py — env steps/s of the MI355X-native AC-PPO hot path (BASELINE.json metric).

One "step" = one full PPO iteration of ac_ppo_continuous_action on HalfCheetah-v5 shapes
(src/ac_ppo_continuous_action.cpp defaults: num_envs=4096, num_steps=128, num_minibatches=4,
update_epochs=4): rollout of T steps (agent act + env step for every env), GAE, and 16 optimizer
steps (gather, forward, loss, backward, grad all-reduce, clip_grad_norm_, Adam). The env is the
device-resident synthetic HalfCheetah-shaped env (MuJoCo is not available), so inputs are resident
in HBM when the timed region starts. value = env steps of all ranks / max-over-ranks wall time.

Multi-GPU: one process per GPU (torch.distributed.run); the reference shards num_envs over ranks
(num_envs_per_device = num_envs / world_size, ac:399), gradients are averaged with RCCL every
minibatch — strong scaling by default, --scaling weak keeps num_envs per GPU.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

ppo_amd = None  # imported in main(), after the launcher decision (ppo_amd loads libppo_hip.so)

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix = vector peak (spec)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "env steps/sec (SPS), HalfCheetah-v5 num_envs=4096 at 1/2/4/8 MI355X"


def algorithmic_work(O, A, H, E, T, MB, nh):
    """Algorithmic FLOPs / bytes per launch of each kernel (DESIGN.md 'Roofline accounting')."""
    M = E * T // MB
    fwd_row = (2 * O * H + 2 * H * H + 2 * H) + (2 * O * H + 2 * H * H + 2 * nh * H)
    bwd_row = (2 * H + 2 * H * H + 2 * H) + (2 * nh * H + 2 * H * H + 2 * nh * H)  # dh, dW3, dh1 (dW1/dW2: k_dw)
    return {
        "fwdbwd": ("flop", M * (fwd_row + bwd_row)),
        "dw": ("flop", 2 * (2 * H * H * M + 2 * H * O * M)),
        "act": ("flop", E * fwd_row),
        "gae": ("byte", E * T * 4 * 5),  # reads r, v, d; writes adv, ret
    }


PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense (no sparsity)


def bx6_mix_peak(O, A, H):
    """k_upd with upd_mfma=bx6: the share of its algorithmic FLOPs that run as split-bf16 piece
    products (layer 2 forward and dh1 = W2^T dz2 of both trunks: 4 x 2 H^2 per row) and the peak of
    that instruction mix: fp32 products on 16x16x4 f32 MFMAs at 157.3 TF/s, the rest at six bf16 piece
    products each on the 2.5 PF/s bf16 MFMA (417 TF/s of fp32 products)."""
    nh = 2 * A
    fwd_row = (2 * O * H + 2 * H * H + 2 * H) + (2 * O * H + 2 * H * H + 2 * nh * H)
    bwd_row = (2 * H + 2 * H * H + 2 * H) + (2 * nh * H + 2 * H * H + 2 * nh * H)
    share = 4 * 2 * H * H / (fwd_row + bwd_row)
    return share, 1.0 / (share / (PEAK_BF16_MFMA_TFLOPS / 6) + (1 - share) / PEAK_F32_MFMA_TFLOPS)


def host_cores():
    """CPU threads this job may use: the launcher's thread budget (OMP_NUM_THREADS, set to the box's
    CPU share), else the cgroup quota, else the affinity mask."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
        if n > 0:
            return n
    except ValueError:
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(E, T, MB, EP):
    """The reference's CPU arithmetic on this host, bounded sample: rollout inference on `cores`
    host threads (the reference's per-env collection threads, ac:575-618 / :641-698), update with
    one intra-op thread (ac:288-289)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    cores = host_cores()
    if os.path.exists(harness):
        try:
            out = subprocess.run([harness, "--bench", str(E), str(T), str(MB), str(EP), "300", str(cores)],
                                 capture_output=True, text=True, timeout=300, check=True).stdout.strip().splitlines()[-1]
            r = json.loads(out)
            res = {"value": round(r["sps"], 2), "unit": "env_steps/s", "cores": cores, "kind": "reference",
                   "cpu_model": cpu_model(), "value_1thread": round(r["sps_1thread"], 2),
                   "sample": (f"LibTorch CPU replay of the reference AC-PPO arithmetic (rl_utils.h Beta): "
                              f"{cores} host threads x {r['n_act']} batch-1 get_action_and_value calls "
                              f"({r['t_act_batch1_s']*1e3:.3f} ms per call aggregate, "
                              f"{r['t_act_batch1_1thread_s']*1e3:.3f} ms on 1 thread) + 1 optimizer step on "
                              f"M={r['M']} rows, 1 intra-op thread as ac:288 sets ({r['t_opt_step_s']:.2f} s) + GAE "
                              f"({r['t_gae_s']*1e3:.1f} ms), extrapolated to one iteration ({E*T} acts, {EP*MB} "
                              f"optimizer steps); env physics excluded")}
            try:  # BASELINE cfg1 (ppo_continuous_action defaults, CPU-only by design) beside the published SPS
                o1 = subprocess.run([harness, "--bench-ppo", "1", "2048", "32", "10", "2048"], capture_output=True,
                                    text=True, timeout=120, check=True).stdout.strip().splitlines()[-1]
                r1 = json.loads(o1)
                res["cfg1"] = {"value": round(r1["sps"], 1), "unit": "env_steps/s", "published": 1900,
                               "sample": "ppo_continuous_action HalfCheetah-v5 num_envs=1: 2048 batch-1 acts + 64 "
                                         "optimizer steps of 64 rows + GAE over T=2048 on 1 thread, extrapolated to "
                                         "one iteration (2048 acts, 320 steps); physics, checkpoint and logging "
                                         "excluded (the published ~1900 SPS includes MuJoCo)"}
            except Exception as e:  # noqa: BLE001
                print(f"[bench] cfg1 reference timing failed: {e}", file=sys.stderr)
            return res
        except Exception as e:  # noqa: BLE001
            print(f"[bench] reference harness failed: {e}", file=sys.stderr)
    # C restatement (oracle) — port baseline
    import oracle_lib as O
    L = O.layout_init(1, 17, 6, 256)
    rng = np.random.default_rng(0)
    p = (rng.standard_normal(L.P) * 0.05).astype(np.float32)
    p[L.hi], p[L.lo] = 1.0, -1.0
    p[L.ostd:L.ostd + 17] = 1.0
    Ms = 2048
    x = rng.standard_normal((Ms, 17)).astype(np.float32)
    a = rng.uniform(-0.9, 0.9, (Ms, 6)).astype(np.float32)
    cfg = O.LossCfg(0.1, 0.01, 0.5, 1, 1)
    t0 = time.perf_counter()
    O.minibatch_grad(L, p, x, a, np.zeros(Ms), rng.standard_normal(Ms), rng.standard_normal(Ms), np.zeros(Ms), cfg)
    t_row = (time.perf_counter() - t0) / Ms
    t0 = time.perf_counter()
    O.get_action_and_value(L, p, x[:512], 0)
    t_act = (time.perf_counter() - t0) / 512
    B = E * T
    t_iter = t_act * B + t_row * B * EP
    return {"value": round(B / t_iter, 2), "unit": "env_steps/s", "cores": 1, "kind": "port",
            "sample": f"C oracle: {Ms}-row minibatch gradient + 512 sampled acts, extrapolated to one iteration"}


def cli_sps(E, T, iterations):
    """SPS as the reference defines and prints it (ac:928-935: global_step / seconds since before
    iteration 0, so the rollout, GAE, update, per-iteration checkpoint and logging are all inside):
    the drop-in ac_ppo_continuous_action executable on the device env, last printed value."""
    exe = os.path.join(ROOT, "ppo.cpp_amd", "bin", "ac_ppo_continuous_action")
    if not os.path.exists(exe):
        return None
    cmd = [exe, "--env_id", "HalfCheetah-v5", "--env_backend", "device", "--num_envs", str(E), "--num_steps", str(T),
           "--total_timesteps", str(E * T * iterations), "--exp_name_stem", "bench_cli", "--num_eval_runs", "1"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True)
        sps = [float(l.split(":")[1]) for l in r.stdout.splitlines() if l.startswith("SPS:")]
        return {"value": sps[-1], "unit": "env_steps/s", "iterations": iterations,
                "cmd": " ".join(os.path.relpath(c, ROOT) if c == exe else c for c in cmd)} if sps else None
    except Exception as e:  # noqa: BLE001
        print(f"[bench] CLI run failed: {e}", file=sys.stderr)
        return None


FP32_OPTIONS = "upd_mfma=16,dw_mfma=f32"


def fp32_leg(cfg, E, args, work):
    """The bench workload again with every update GEMM on fp32 MFMAs (v_mfma_f32_16x16x4_f32: the
    LibTorch kFloat32 arithmetic of ac:816-888 without split-bf16 piece products), same warmup and
    timing as the headline; reported beside it, never as `value`."""
    opts = FP32_OPTIONS if not args.options else args.options + "," + FP32_OPTIONS
    tr = ppo_amd.Trainer(cfg, num_envs_per_device=E, rank=0, world_size=1, device=0, options=opts)
    try:
        for _ in range(args.warmup):
            tr.iterate()
        tr.agent.sync()
        tr.agent.profile_reset()
        tr.agent.profile(1 << 1)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.iterate()
        tr.agent.sync()
        el = time.perf_counter() - t0
        tr.agent.profile(0)
        prof = tr.agent.profile_read()
        res = {"options": opts, "kernels": tr.agent.kernel_info(), "steps": args.steps,
               "value": round(E * cfg.num_steps * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3)}
        if prof and "fwdbwd" in prof:
            ms, cnt = prof["fwdbwd"]
            tf = work["fwdbwd"][1] / (ms / 1e3 / cnt) / 1e12
            res["fwdbwd"] = {"avg_launch_ms": round(ms / cnt, 4), "achieved": round(tf, 3),
                             "frac": round(tf / PEAK_F32_MFMA_TFLOPS, 4)}
        return res
    finally:
        tr.close()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The one-process-per-GPU launch of this script for `--gpus n` (the reference's
    `mpirun -n G`, README.md:56-59): torch.distributed.run on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def relaunch(n):
    """`bench.py --gpus n` without an external launcher: start the n ranks as a child process (never
    an exec, and before anything in this process touches the GPU). Rank 0 prints the JSON line to
    the inherited stdout; this process exits with the launcher's status."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run(launcher_cmd(sys.argv[1:], n, free_port()), env=env)
    return r.returncode


def main():
    global ppo_amd
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--num-steps", type=int, default=128)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-all", action="store_true", help="HIP-event time every kernel class")
    ap.add_argument("--no-cli", action="store_true", help="skip the ac_ppo_continuous_action CLI SPS run")
    ap.add_argument("--no-fp32-leg", action="store_true",
                    help="skip the second timed run with every GEMM on fp32 MFMAs (upd_mfma=16,dw_mfma=f32)")
    ap.add_argument("--cli-iterations", type=int, default=30)
    ap.add_argument("--comm", choices=["rccl", "host"], default="rccl",
                    help="N > 1 data path: RCCL (one GPU per rank), or the host transport over gloo with every "
                         "rank on GPU 0 (rehearses this script's multi-rank path on a one-GPU box)")
    ap.add_argument("--comm-1rank", action="store_true",
                    help="N = 1 only: attach a one-rank RCCL communicator, so the distributed update path "
                         "(advantage-statistics and in-stream gradient all-reduces) runs and its cost can be timed")
    ap.add_argument("--options", default=None, help="ppo_create_ex options (kernel / geometry A/B runs)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(or drop the external launcher and let --gpus start the ranks)")
    import ppo_amd as _ppo_amd  # imports torch before loading libppo_hip.so: one HIP runtime serves both
    ppo_amd = _ppo_amd
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo (CPU) only for rendezvous, barriers and timing max
        dist.init_process_group("gloo")
    # one GPU per rank (the reference's cudaSetDevice(gpu_ids.at(local_rank)), ac:447-448 / :459-460);
    # only the host-transport rehearsal puts every rank on GPU 0 on purpose
    device = 0 if args.comm == "host" else local_rank
    ppo_amd.set_device(device)

    E_total = args.num_envs if args.scaling == "strong" else args.num_envs * world
    E = E_total // world
    T = args.num_steps
    cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=E_total, num_steps=T,
                              total_timesteps=E_total * T * (args.steps + args.warmup + 1))
    tr = ppo_amd.Trainer(cfg, num_envs_per_device=E, rank=rank, world_size=world, device=device,
                         options=args.options)
    dev_ord, dev_bus = tr.agent.device()
    if dev_ord != device:
        raise SystemExit(f"bench.py: rank {rank} asked for device {device} but its context is on {dev_ord}")
    devices = [(dev_ord, dev_bus)]
    if world > 1:
        import socket
        hosts = [None] * world
        dist.all_gather_object(hosts, (socket.gethostname(), dev_ord, dev_bus))
        devices = [(d, b) for _, d, b in hosts]
        # bus ids repeat across hosts (local rank 0 of every node is usually the same bus): a shared GPU
        # is the same (host, bus) pair
        shared = [hb for hb in set((h, b) for h, _, b in hosts) if sum((h, b) == hb for h, _, b in hosts) > 1]
        if args.comm == "rccl" and shared:
            raise SystemExit(f"bench.py: ranks share a GPU under RCCL ((host, PCI bus id) {sorted(shared)}); one GPU "
                             f"per rank is required")
    if world > 1:
        if args.comm == "host":
            import torch

            def allreduce(buf, average):
                t = torch.from_numpy(buf)  # the library's host staging buffer, reduced in place
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                if average:
                    t /= world
            tr.agent.comm_init_host(rank, world, allreduce)
        else:
            uid = [ppo_amd.Agent.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            tr.agent.comm_init(uid[0], rank, world)
        tr.agent.comm_broadcast_params(0)
    if world == 1 and args.comm_1rank:
        tr.agent.comm_init(ppo_amd.Agent.comm_unique_id(), 0, 1)
    comm_kind, _, comm_world = tr.agent.comm_info()
    if world > 1 and comm_world != world:
        raise SystemExit(f"bench.py: the {comm_kind} communicator reports {comm_world} ranks, expected {world}")

    for _ in range(args.warmup):
        tr.iterate()
    tr.agent.sync()
    # per-kernel HIP events on the context stream over the timed region (dominant kernel always)
    mask = 0xFFFF if args.profile_all else (1 << 1)
    tr.agent.profile_reset()
    tr.agent.profile(mask)
    if dist:
        dist.barrier()
    tr.agent.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.iterate()
    tr.agent.sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tr.agent.profile(0)
    prof = tr.agent.profile_read()
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    units = E_total * T * args.steps
    value = units / elapsed
    dw_prof = None
    if world == 1 and not args.profile_all:
        # dW's own fraction beside k_upd's: a few iterations after the timed region with HIP events
        # around the dW launches too (kept out of the timed region so it carries one event class only)
        tr.agent.profile_reset()
        tr.agent.profile((1 << 1) | (1 << 2))
        for _ in range(min(args.steps, 4)):
            tr.iterate()
        tr.agent.sync()
        tr.agent.profile(0)
        dw_prof = tr.agent.profile_read()
    if rank == 0:
        H, O_, A = 256, 17, 6
        work = algorithmic_work(O_, A, H, E, T, cfg.num_minibatches, 2 * A)
        kinfo = tr.agent.kernel_info()
        roof = None
        if prof:
            name = max(prof, key=lambda k: prof[k][0])
            ms, cnt = prof[name]
            avg_s = ms / 1e3 / cnt
            kind, amount = work.get(name, ("flop", 0))
            if kind == "flop":
                achieved = amount / avg_s / 1e12
                roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_F32_MFMA_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_MFMA_TFLOPS, 4), "traffic": None,
                        "kernel": name, "avg_launch_ms": round(ms / cnt, 4), "launches": cnt,
                        "algorithmic_per_launch": amount, "kernels": kinfo}
                if name == "fwdbwd" and "update=k_upd/bx6" in kinfo:
                    # the fp32 products of layer 2 and dh1 run as six bf16 piece products on the bf16
                    # MFMA (2.5 PF/s dense): the peak of the kernel's actual instruction mix
                    frac_bx, peak_mix = bx6_mix_peak(O_, A, H)
                    roof["bx6_flop_share"] = round(frac_bx, 4)
                    roof["peak_instruction_mix"] = round(peak_mix, 1)
                    roof["frac_instruction_mix"] = round(achieved / peak_mix, 4)
            else:
                achieved = amount / avg_s / 1e9
                roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None, "kernel": name,
                        "avg_launch_ms": round(ms / cnt, 4), "launches": cnt, "algorithmic_per_launch": amount}
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    tj = json.load(open(pmc))
                    if name in tj and tj[name].get("config") == f"E={E},T={T}":
                        # PMC counters cannot run inside the timed region: the bytes come from the two
                        # rocprofv3 passes (FETCH_SIZE, WRITE_SIZE) of this bench command named here
                        roof["traffic"] = tj[name]["hbm_bytes_per_launch"]
                        roof["traffic_source"] = tj.get("_source", "profiles/pmc_traffic.json")
                        if "dw" in tj and tj["dw"].get("config") == f"E={E},T={T}":
                            roof["traffic_dw"] = tj["dw"]["hbm_bytes_per_launch"]
                except Exception:  # noqa: BLE001
                    pass
        src = dw_prof or prof
        if roof is not None and src and "dw" in src:
            ms, cnt = src["dw"]
            dw_tf = work["dw"][1] / (ms / 1e3 / cnt) / 1e12
            roof["dw"] = {"kernel": kinfo.split("dw=")[-1].split()[0] if "dw=" in kinfo else "dw",
                          "avg_launch_ms": round(ms / cnt, 4),
                          "launches": cnt, "achieved": round(dw_tf, 3), "frac": round(dw_tf / PEAK_F32_MFMA_TFLOPS, 4),
                          "algorithmic_per_launch": work["dw"][1],
                          "timing": "HIP events on the context stream, iterations after the timed region"}
            if "bf16x6" in kinfo:  # every dW product is six bf16 piece products: 2.5 PF/s / 6
                roof["dw"]["peak_instruction_mix"] = round(PEAK_BF16_MFMA_TFLOPS / 6, 1)
                roof["dw"]["frac_instruction_mix"] = round(dw_tf / (PEAK_BF16_MFMA_TFLOPS / 6), 4)
                roof["dw"]["frac_note"] = ("frac = fp32-product FLOP/s over the fp32 MFMA spec (can pass 1: the products run "
                                           "as bf16 piece products); frac_instruction_mix = over the peak of the "
                                           "instructions issued (2.5 PF/s bf16 / 6 products)")
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "dtype_note": ("fp32 operands and fp32 accumulation; the update's 256-wide GEMMs and dW run each fp32 "
                           "product as six of its nine split-bf16 piece products on bf16 MFMAs (the dropped "
                           "mid*lo + lo*mid + lo*lo are < ~2^-21 of the product; DESIGN.md 3c), tested within 1.5x "
                           "of the fp32 MFMA form's distance from the fp64 oracle; results differ bitwise from the "
                           "fp32 MFMA form. fp32 MFMAs throughout: options upd_mfma=16,dw_mfma=f32 (the fp32_mfma "
                           "leg below)"),
            "data": "synthetic: device-resident HalfCheetah-shaped env (O=17, A=6), random-init AC agent",
            "config": {"workload": f"ac_ppo_continuous_action HalfCheetah-v5 num_envs={E_total} num_steps={T} "
                                   f"num_minibatches={cfg.num_minibatches} update_epochs={cfg.update_epochs}",
                       "num_envs": E_total, "num_envs_per_device": E, "num_steps": T,
                       "minibatch_per_device": E * T // cfg.num_minibatches, "parallelism": f"dp{world}",
                       "comm_ranks": comm_world, "comm_kind": comm_kind,
                       "devices": [d for d, _ in devices], "device_pci_bus_ids": [b for _, b in devices],
                       **({"comm": "host transport (gloo), all ranks on GPU 0: rehearsal, not a scaling number"}
                          if world > 1 and args.comm == "host" else {})},
            "roofline": roof,
        }
        if args.profile_all:
            out["kernels_ms_per_step"] = {k: round(v[0] / args.steps, 3) for k, v in prof.items()}
            out["kernels_ms_note"] = ("HIP-event pairs around every kernel class: the sum can exceed ms_per_step "
                                      "(each pair adds its own overhead to the class it brackets)")
    if world == 1 and not args.no_fp32_leg:
        # the same workload with every GEMM on fp32 MFMAs (no split-bf16 piece products)
        tr.close()
        tr = None
        out["fp32_mfma"] = fp32_leg(cfg, E, args, algorithmic_work(17, 6, 256, E, T, cfg.num_minibatches, 12))
    if rank == 0:
        if world == 1 and not args.no_cli:
            out["cli_value"] = cli_sps(E_total, T, args.cli_iterations)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(E, T, cfg.num_minibatches, cfg.update_epochs)
        print(json.dumps(out), flush=True)
    if tr is not None:
        tr.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
