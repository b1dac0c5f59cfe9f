#!/usr/bin/env python3
"""bench.py — descriptor decisions/s of the HIP rate-limit decision path (BASELINE.json).

Workload (N=1 line): BASELINE config 3 — 1e8 keys, Zipf s=1.1 over ranks mapped through a
fixed permutation, rule by rank % 3 (SECOND 10 / MINUTE 600 / HOUR 36000), 1e6 descriptors
per batch (one descriptor per request, hits_addend 1), `now` advancing 1 s per batch.
A step = one batch through the whole device path (fingerprint, radix sort, segmented scan,
table apply, decide). Inputs are resident in HBM before timing; outputs stay in HBM.

Multi-GPU (torchrun, one rank per GPU): the key space is hash-sharded one
shard per GPU. Every rank ingests its own 1e6-descriptor batch per step, routes each
descriptor to the GPU owning its key with an RCCL all-to-all (32-B records), the owners
decide, and the 24-B replies return with the reverse all-to-all (api-ratelimit_amd/router.py)
— weak scaling. value = descriptors decided for all ranks / max-over-ranks time.
--independent runs N unrouted replicas instead (each rank its own key space).

Also reported (rank 0): per-kernel HIP-event times over an extra K steps, the roofline
of the batch pipeline against §8(d)'s algorithmic bytes, and the CPU oracle timed on a
bounded sample of the same stream (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))

import hiprl  # noqa: E402
import router  # noqa: E402
import workload  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3])
    ap.add_argument("--desc", type=int, default=1_000_000, help="descriptors per batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--no-roofline-probe", action="store_true")
    ap.add_argument("--pipeline", choices=["v4", "lsd"], default="v4",
                    help="decision pipeline (v4 default; lsd = radix-sort only)")
    ap.add_argument("--independent", action="store_true",
                    help="N>1: unrouted replicas (each rank its own key space) instead of RCCL routing")
    ap.add_argument("--json-out", type=str, default="")
    ap.add_argument("--depth", type=int, default=2,
                    help="batches in flight through rl_submit_pipelined (2..3; --serial = 1). 2 is fastest "
                         "at config 3: a third batch's k4_hist starts at the end of batch k-2 and takes the "
                         "CUs the next k4_scan needs (DESIGN.md §3a)")
    ap.add_argument("--serial", action="store_true",
                    help="one batch in flight (rl_submit_device + rl_wait per step) instead of two (rl_submit_pipelined)")
    return ap.parse_args()


def random_access_roofline(eng, alg_bytes, U, pipe_ms, step_ms):
    import ctypes as C

    lp = ROOT / "tools" / "microbench" / "libroofline_probe.so"
    if not lp.exists() or U <= 0:
        return None
    lib = C.CDLL(str(lp))
    lib.rl_probe_roofline.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]
    lib.rl_probe_roofline.restype = C.c_int
    slots = sum(2 << int(x) for x in eng.cfg.log2_slots)  # 8 regions: unit x window parity
    gbs, rate, rus = C.c_double(), C.c_double(), C.c_double()
    if lib.rl_probe_roofline(slots, U, C.byref(gbs), C.byref(rate), C.byref(rus)):
        return None
    stream_bytes = alg_bytes - 64 * U
    t_roof_us = stream_bytes / (gbs.value * 1e9) * 1e6 + U / rate.value * 1e6
    return {"t_roof_us": round(t_roof_us, 2), "frac_of_step": round(t_roof_us / (step_ms * 1e3), 4),
            "frac_of_kernel_time": round(t_roof_us / (pipe_ms * 1e3), 4),
            "streaming_bytes": int(stream_bytes), "copy_GBps": round(gbs.value, 1),
            "table_slots": int(1 << (slots.bit_length() - 1)), "U": U,
            "slot_rmw_per_s": round(rate.value, 1), "slot_rmw_us": round(rus.value, 2),
            "atomics_per_s": round(U / (step_ms * 1e-3), 1),
            "definition": "SURVEY.md 8(d): t_roof = streaming_B / copy_BW + U / RMW_rate (U random 32-B slot "
                          "load + 64-bit atomicAdd on a table of the engine's size, power-of-two rounded); "
                          "frac = t_roof / t"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    d = args.desc
    if args.config == 3:
        gen, rules, log2 = workload.config3_batch, workload.CONFIG3_RULES, (22, 24, 25, 12)
        wl = "config3: 1e8 keys Zipf s=1.1, SECOND/MINUTE/HOUR by rank%3, 1 descriptor/request"
    elif args.config == 2:
        gen, rules, log2 = workload.config2_batch, workload.CONFIG2_RULES, (22, 12, 12, 12)
        wl = "config2: 1e6 uniform keys, SECOND L=5, 1 descriptor/request"
    else:
        gen, rules, log2 = workload.config1_batch, workload.CONFIG1_RULES, (16, 12, 12, 12)
        wl = "config1: examples/ratelimit rules, 1e4 keys"
    n_batches = args.warmup + args.steps * (1 if args.no_kernel_times else 2)
    # Each rank is its own key shard: seed the stream by rank.
    host_batches = []
    t_gen = time.time()
    for b in range(n_batches):
        if args.config == 1:
            hb = gen(b, d=d, seed=1 + 7919 * rank)
        else:
            hb = gen(b, d=d, seed=(3 if args.config == 3 else 2) + 7919 * rank)
        host_batches.append(hb)
    t_gen = time.time() - t_gen

    routed = world > 1 and not args.independent
    # an owner may receive up to every origin's batch (hot keys concentrate on their owner)
    cap = d * world if routed else d
    eng = hiprl.Engine(device=local, log2_slots=log2, max_batch_desc=cap, max_batch_req=cap,
                       max_blob_bytes=max(int(hb.blob.shape[0]) for hb in host_batches) + 64, sort_bits=48,
                       pipeline=args.pipeline)
    eng.load_rules(rules)

    dev_batches = [router.DeviceBatch.from_host(hb, dev) for hb in host_batches]
    # two output buffers: with two batches in flight each needs its own
    outs = [torch.empty(d * 20, dtype=torch.uint8, device=dev) for _ in range(hiprl.MAX_IN_FLIGHT)]
    thrs = [torch.empty(d, dtype=torch.int32, device=dev) for _ in range(hiprl.MAX_IN_FLIGHT)]
    rtr = None
    if routed:
        rtr = router.ShardRouter(router.EngineShard(eng, rank, world, dev, d))
    torch.cuda.synchronize()

    pipelined = rtr is None and not args.serial
    # The rl_batch of every batch and the output pointers are marshalled once, outside the timed
    # loop: a service's submitter builds them while the previous batch runs (Python ctypes
    # marshalling would otherwise sit between rl_wait and the next submit).
    DEPTH = min(args.depth, hiprl.MAX_IN_FLIGHT) if pipelined else 1
    sub_args = [(hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs()),
                 outs[b % DEPTH].data_ptr(), thrs[b % DEPTH].data_ptr()) for b, db in enumerate(dev_batches)]

    def run(b0, b1):
        """Batches [b0, b1): one step per batch. Pipelined: batch k+1 is submitted before batch k
        is waited for (the micro-batcher's double buffering); every batch is complete on return."""
        for j, b in enumerate(range(b0, b1)):
            db = dev_batches[b]
            if rtr is not None:
                rtr.step(db)
                continue
            if pipelined:
                eng.submit_pipelined_batch(*sub_args[b])  # output buffers rotate by batch
                if j >= DEPTH - 1:
                    eng.wait()
            else:
                args_ = (db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), outs[j & 1].data_ptr(), thrs[j & 1].data_ptr())
                eng.submit_device_async(*args_)
                eng.wait()
        if pipelined:
            for _ in range(min(DEPTH - 1, b1 - b0)):
                eng.wait()

    run(0, args.warmup)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.warmup, args.warmup + args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_desc = world * args.steps * d
    value = total_desc / elapsed

    # Per-kernel HIP-event timing over another K steps of the same stream.
    kernel = None
    uniq = []
    if not args.no_kernel_times:
        eng.set_timing(True)
        for b in range(args.warmup + args.steps, args.warmup + 2 * args.steps):
            run(b, b + 1)
            uniq.append(eng.last_batch_info()["unique_keys"])
        kt = eng.kernel_times()
        eng.set_timing(False)
        kernel = {k: dict(total_ms=v[0], launches=v[1]) for k, v in kt.items() if v[1]}
    info = eng.last_batch_info()
    if not uniq:
        uniq = [info["unique_keys"]]
    stats = eng.stats()

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    # Roofline of the batch pipeline against §8(d) algorithmic bytes.
    U = float(np.mean(uniq))
    hb_last = host_batches[-1]
    alg_bytes = workload.algorithmic_bytes(hb_last, int(U))
    roofline = None
    if kernel:
        per_batch_ms = {k: v["total_ms"] / args.steps for k, v in kernel.items()}
        pipe_ms = sum(v for k, v in per_batch_ms.items())
        dom = max((k for k in per_batch_ms if k != "memset"), key=lambda k: per_batch_ms[k])
        achieved = alg_bytes / (pipe_ms * 1e-3) / 1e9
        prof_dir = ROOT / "profiles"
        traffic = None
        # PMC traffic of this pipeline from the committed rocprofv3 --pmc passes (tools/profile_round.sh)
        tf = prof_dir / {"v4": "r01_v7_pmc_traffic.json", "v3": "r01_v3_pmc_traffic.json", "v2": "r01_v2_pmc_traffic.json",
                         "lsd": "r01_pmc_traffic.json"}[args.pipeline]
        if tf.exists():
            try:
                traffic = json.loads(tf.read_text()).get("hbm_bytes_per_batch")
            except Exception:
                traffic = None
        roofline = {
            "bound": "hbm", "kernel": "batch pipeline (all kernels of one batch, HIP events on the engine stream)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_batch": alg_bytes, "unique_keys_per_batch": int(U),
            "pipeline_us_per_batch": round(pipe_ms * 1e3, 2),
            "dominant_kernel": {"name": dom, "us_per_batch": round(per_batch_ms[dom] * 1e3, 2),
                                "launches_per_batch": kernel[dom]["launches"] / args.steps,
                                "avg_us_per_launch": round(kernel[dom]["total_ms"] * 1e3 / kernel[dom]["launches"], 2)},
            "kernels_us_per_batch": {k: round(v * 1e3, 2) for k, v in per_batch_ms.items()},
        }

    # SURVEY.md §8d random-access roofline: t_roof = streaming bytes / copy bandwidth + U /
    # random slot-RMW rate, both measured here on a table of the engine's size.
    if roofline is not None and not args.no_roofline_probe:
        ra = random_access_roofline(eng, alg_bytes, int(U), pipe_ms, elapsed / args.steps * 1e3)
        if ra:
            roofline["random_access"] = ra

    cpu = None
    if world == 1 and args.cpu_seconds > 0:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle as orc

        o = orc.Oracle()
        o.load_rules(rules)
        n_done, t_cpu, nb = 0, 0.0, 0
        for hb in host_batches:
            t1 = time.perf_counter()
            o.submit(hb)
            t_cpu += time.perf_counter() - t1
            n_done += hb.n_desc
            nb += 1
            if t_cpu >= args.cpu_seconds:
                break
        cpu = {"value": round(n_done / t_cpu, 1), "unit": "descriptor decisions/s", "cores": 1, "kind": "port",
               "sample": f"first {nb} batches ({n_done} descriptors) of the same stream through the C++ oracle "
                         f"(serial DoLimit over an in-memory Redis stand-in), {t_cpu:.1f} s"}

    line = {
        "metric": "descriptor decisions/sec, 100M keys Zipf, 1-8 GPUs; % of HBM peak" if args.config == 3
        else f"descriptor decisions/sec (config {args.config})",
        "value": round(value, 1),
        "unit": "descriptor decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded splitmix64 / bounded Zipf stream, generated on host, resident in HBM)",
        "config": {"workload": wl, "descriptors_per_batch": d, "requests_per_batch": d,
                   "parallelism": (f"key-sharded x{world}, RCCL all-to-all routing (32-B records out, 24-B replies back)"
                                   if routed else "single shard" if world == 1
                                   else f"x{world} independent replicas (no collective)"),
                   "pipeline": args.pipeline, "batches_in_flight": DEPTH,
                   "unique_keys_per_batch": int(U)},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "engine": {"resorts": stats["resorts"], "lsd_fallbacks": stats["lsd_fallbacks"], "hot_keys": stats["hot_keys"],
                   "batches": stats["batches"], "gen_s": round(t_gen, 1)},
    }
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        Path(args.json_out).write_text(s + "\n")
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
