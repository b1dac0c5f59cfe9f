#!/usr/bin/env python3
"""bench.py — descriptor decisions/s of the HIP rate-limit decision path (BASELINE.json).

Workload (N=1 line): BASELINE config 3 — 1e8 keys, Zipf s=1.1 over ranks mapped through a
fixed permutation, rule by rank % 3 (SECOND 10 / MINUTE 600 / HOUR 36000), 1e6 descriptors
per batch (one descriptor per request, hits_addend 1). `now` advances once every
--batches-per-second batches (default 8000, i.e. the rate this path runs at), so one SECOND
window holds thousands of batches and the table holds the live set a real deployment has:
before timing, --prefill batches (default 1.5 s of traffic) fill it — every MINUTE/HOUR key
drawn so far, the previous second's SECOND keys and half of the current second's — in
regions sized for it (2^27 slots per home unit and parity, 25.8 GB). A step = one batch
through the whole device path (fingerprint, bucket sort, segmented scan, table apply,
decide); inputs are resident in HBM before timing, outputs stay in HBM. Batches are made on
the device (tools/gen/workload_gen.hip, the workload.py construction) because one second of
traffic is 8000 distinct 1e6-descriptor batches.

Multi-GPU (torchrun, one rank per GPU): the key space is hash-sharded one
shard per GPU. Every rank ingests its own 1e6-descriptor batch per step, routes each
descriptor to the GPU owning its key with an RCCL all-to-all (32-B records; one combined
record per hot key per origin), the owners decide, and 8-B raw replies return with the reverse
all-to-all; the origins decide from them — weak scaling, three steps in flight (--router-depth). The step runs
through the C-ABI router (rl_router_submit / rl_router_wait, csrc/rl_router.cpp: the Go
host's entry point, its own RCCL communicator); --torch-router runs the round-2 step through
api-ratelimit_amd/router.py (torch.distributed) instead. value = descriptors decided for all ranks / max-over-ranks time.
--independent runs N unrouted replicas instead (each rank its own key space).

Also reported (rank 0): per-kernel HIP-event times over an extra K steps, the roofline of the
dominant kernel and the SURVEY §8(d) random-access roofline, table occupancy, the host
(PCIe) path end to end, and the CPU oracle timed on a bounded sample of the same stream on
1 and on N host threads (cpu_baseline).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))

import hiprl  # noqa: E402
import workload  # noqa: E402

# router.py imports torch, which maps the HIP runtime: imported where used, so the launcher
# process of `--gpus N` (launch_ranks) starts its ranks without it


def _router():
    import router

    return router

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
T0 = 1_700_000_020      # not minute-aligned: SECOND / MINUTE / HOUR keys in their own home regions
PMC_SUMMARIES = {3: ROOT / "profiles" / "r06_pmc_traffic.json", 4: ROOT / "profiles" / "r06_pmc_traffic_config4.json",
                 5: ROOT / "profiles" / "r06_pmc_traffic_config5.json"}
SOURCES = sorted((ROOT / "api-ratelimit_amd" / "csrc").glob("*.h*")) + sorted(
    (ROOT / "api-ratelimit_amd" / "csrc").glob("*.cpp")) + [ROOT / "include" / "rl_hip.h"]


def source_sha() -> str:
    h = hashlib.sha256()
    for p in SOURCES:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5],
                    help="BASELINE config: 3 (headline), 2, 1 (examples/ratelimit rules, 10k keys: the CPU row), 4 "
                         "(1e9 keys, 4-entry descriptors resolved on the device each step, local cache, shadow rules) "
                         "or 5 (60 simulated seconds, hits_addend U{1..8})")
    ap.add_argument("--desc", type=int, default=1_000_000, help="descriptors per batch")
    ap.add_argument("--batches-per-second", type=int, default=0,
                    help="batches per SECOND window (now advances once every K batches; 0: 8000, config 5: 16); "
                         "1 = round-1 mode")
    ap.add_argument("--prefill", type=int, default=-1,
                    help="untimed batches that fill the table before warmup (-1: 1.5 windows of K batches)")
    ap.add_argument("--log2-slots", type=int, default=27,
                    help="table slots per region (home unit x parity); 2^27 x 32 B x 6 regions = 25.8 GB, ~23 %% load "
                         "at config 3's live set (shorter probe chains than 2^26 at ~46 %%)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline sample budget per leg (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="N-thread CPU baseline (0 = min(16, cpus))")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--no-roofline-probe", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--host-formats", default="compact,full", help=argparse.SUPPRESS)  # traces: one format only
    ap.add_argument("--host-no-probe", action="store_true", help=argparse.SUPPRESS)  # traces: no link probes
    ap.add_argument("--pipeline", choices=["v4", "lsd"], default="v4",
                    help="decision pipeline (v4 default; lsd = radix-sort only)")
    ap.add_argument("--independent", action="store_true",
                    help="N>1: unrouted replicas (each rank its own key space) instead of RCCL routing")
    ap.add_argument("--json-out", type=str, default="")
    ap.add_argument("--depth", type=int, default=2, help="batches in flight through rl_submit_pipelined (2..3)")
    ap.add_argument("--serial", action="store_true", help="one batch in flight (rl_submit_device + rl_wait)")
    ap.add_argument("--logical-shards", type=int, default=0,
                    help="G > 0: one GPU, G engines as G logical shards behind the C-ABI router (rl_router, local "
                         "transport): G origin batches per step, records per owner and the step breakdown")
    ap.add_argument("--lib", type=str, default="", help=argparse.SUPPRESS)  # diagnostics: a variant library
    # tests: the routed (RCCL all-to-all) step on one rank, so the multi-GPU path runs on a 1-GPU box
    ap.add_argument("--force-routed", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--router-depth", type=int, default=3, help="routed steps in flight (rl_router_submit / _wait)")
    ap.add_argument("--no-combine", action="store_true", help="routed steps without hot-prefix combining")
    ap.add_argument("--xgmi-gbps", type=float, default=400.0,
                    help="--logical-shards estimate: all-to-all bandwidth per GPU and direction over xGMI (GB/s); "
                         "7 links x ~153 GB/s = 1.07 TB/s raw, RCCL all-to-all assumed to reach ~37%% of it")
    ap.add_argument("--torch-router", action="store_true",
                    help="routed steps through router.ShardRouter (torch.distributed over RCCL) instead of the "
                         "C-ABI router rl_router_step (the Go host's path, the default)")
    ap.add_argument("--dump-stamps", type=str, default="", help=argparse.SUPPRESS)  # -DRL_STAMPS variant: raw stamps
    ap.add_argument("--dump-host-times", type=str, default="", help=argparse.SUPPRESS)  # per-call submit / wait seconds
    ap.add_argument("--host-delay-us", type=float, default=0.0, help=argparse.SUPPRESS)  # diagnostic: spin before submit
    ap.add_argument("--master-port", type=int, default=0,
                    help="--gpus N > 1 without a launcher: rendezvous port of the ranks bench.py starts (0: pick one)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launch check: every rank joins a gloo group, prints the world it sees and exits (no GPU)")
    return ap.parse_args()


def launch_ranks(args) -> int | None:
    """`--gpus N` is the number of ranks, one per GPU. Under a launcher
    (torch.distributed.run sets WORLD_SIZE) every rank checks WORLD_SIZE == N and goes on.
    Without one and N > 1, bench.py starts the N ranks itself — a fresh
    `torch.distributed.run --nproc-per-node N` child, started BEFORE anything in this process
    touches the GPU (only the device count is read, which does not initialise it) — and
    returns the child's exit code. A box with fewer than N GPUs fails here, loudly, instead
    of measuring one GPU and calling it N. Returns None when this process is a rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if args.logical_shards:
        return None
    if env_world is not None:
        if int(env_world) != args.gpus and not (args.gpus == 1 and args.force_routed):
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
        return None
    if args.gpus <= 1:
        return None
    if not args.dry_launch:
        have = gpu_count_sysfs()
        if have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this box has {have}")
    port = args.master_port
    if not port:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"bench.py launcher: {launcher_device_report()}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def gpu_count_sysfs() -> int:
    """GPUs in the KFD topology (nodes whose gfx_target_version is non-zero; CPU nodes have 0),
    narrowed by a non-empty ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.
    Read from sysfs: the launcher neither opens /dev/kfd nor loads the HIP runtime
    (torch.cuda.device_count() falls back to hipGetDeviceCount when amdsmi fails)."""
    n = 0
    try:
        nodes = list(Path("/sys/class/kfd/kfd/topology/nodes").iterdir())
    except OSError:
        return 0
    for node in nodes:
        try:
            for line in (node / "properties").read_text().splitlines():
                key, _, val = line.partition(" ")
                if key == "gfx_target_version" and int(val) != 0:
                    n += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var, "").strip()
        if v:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launcher_device_report() -> str:
    """What this (launcher) process holds of the GPU: an open /dev/kfd, the HIP runtime mapped."""
    kfd = False
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                kfd |= os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd"
            except OSError:
                pass
    except OSError:
        pass
    try:
        with open("/proc/self/maps") as f:
            hip = "libamdhip64" in f.read()
    except OSError:
        hip = False
    return f"/dev/kfd open: {'yes' if kfd else 'no'}; HIP runtime loaded: {'yes' if hip else 'no'}"


def dry_launch_main(args):
    """Every rank joins the gloo group the routed bench uses for its barrier and time max,
    all-gathers (rank, world) and rank 0 prints what every rank saw. No GPU is touched."""
    import torch
    import torch.distributed as dist

    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if world > 1:
        dist.init_process_group("gloo")
        seen = [None] * world
        dist.all_gather_object(seen, {"rank": rank, "world": world, "local_rank": int(os.environ["LOCAL_RANK"])})
        t = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.destroy_process_group()
    else:
        seen, t = [{"rank": 0, "world": 1, "local_rank": 0}], torch.tensor([0.0])
    if rank == 0:
        print(json.dumps({"dry_launch": True, "n_gpus": args.gpus, "world": world, "ranks": seen,
                          "max_over_ranks": float(t.item())}), flush=True)


class DeviceGen:
    """Config-2/3/4/5 batches made on the device (tools/gen/libworkload_gen.so) into DeviceBatch
    buffers (config 4: with the batch's rl_resolve_batch arrays, the strings being the batch's own
    prefix bytes; its rule ids are resolved by the engine inside the step)."""

    PREFIX = {2: b"bench_k_", 3: b"bench_k_", 5: b"c5_k_"}

    def __init__(self, config: int, d: int, seed: int, K: int, dev):
        import torch

        self.torch, self.d, self.seed, self.K, self.dev, self.config = torch, d, seed, K, dev, config
        lib = C.CDLL(str(ROOT / "tools" / "gen" / "libworkload_gen.so"))
        vp, u32, u64, dbl = C.c_void_p, C.c_uint32, C.c_uint64, C.c_double
        lib.rlw_keys2.argtypes = [C.c_int, u64, dbl, dbl, dbl, dbl, u64, u64, u64, u32, vp, vp, vp, vp, u32, vp]
        lib.rlw_bytes2.argtypes = [u32, vp, vp, vp, vp, C.c_char_p, u32, vp]
        lib.rlw_bytes4.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp]
        self.lib = lib
        if config in (3, 4, 5):
            self.N = workload.CONFIG4_N if config == 4 else 100_000_000
            s = 1.1
            self.mode = {3: 0, 4: 3, 5: 2}[config]
            z = workload.Zipf(self.N, s)
            self.z = (s, float(z.hx1), float(z.hN), float(z.sq))
        else:
            self.N, self.mode, self.z = 1_000_000, 1, (0.0, 0.0, 0.0, 0.0)
        self.plen = len(self.PREFIX.get(config, b""))
        self.max_len = 28 if config == 4 else self.plen + 10  # bytes per prefix at most
        a = 2654435761
        while math.gcd(a, self.N) != 1:
            a += 2
        self.mult = a  # workload.permute
        self.key = torch.empty(d, dtype=torch.int64, device=dev)
        self.len = torch.empty(d, dtype=torch.int32, device=dev)

    def alloc(self):
        t, d, dev = self.torch, self.d, self.dev
        db = _router().DeviceBatch(t.empty(d * self.max_len + 64, dtype=t.uint8, device=dev),
                                t.zeros(d + 1, dtype=t.int32, device=dev), t.empty(d, dtype=t.int32, device=dev),
                                t.empty(d, dtype=t.int32, device=dev), t.empty(d, dtype=t.int64, device=dev),
                                t.ones(d, dtype=t.int32, device=dev), d * self.max_len)
        if self.config == 4:  # the rl_resolve_batch arrays (device)
            db.res = (t.empty(2 * d, dtype=t.int32, device=dev), t.empty(d + 1, dtype=t.int32, device=dev),
                      t.empty(16 * d, dtype=t.int32, device=dev))
        return db

    def make(self, b: int):
        db = self.alloc()
        self.fill(b, db)
        return db

    def fill(self, b: int, db):
        """Batch b (counter stream b): now = T0 + b // K."""
        t = self.torch
        st = t.cuda.current_stream(self.dev).cuda_stream
        hits = db.hits.data_ptr() if self.config == 5 else None
        rc = self.lib.rlw_keys2(self.mode, self.N, *self.z, self.seed, b, self.mult, self.d, self.key.data_ptr(),
                                db.rule.data_ptr(), self.len.data_ptr(), hits, self.plen, st)
        t.cumsum(self.len, 0, dtype=t.int32, out=db.off[1:])
        if self.config == 4:
            dom, first, ent = db.res
            rc |= self.lib.rlw_bytes4(self.d, self.key.data_ptr(), db.off.data_ptr(), db.blob.data_ptr(),
                                      db.req_of.data_ptr(), dom.data_ptr(), first.data_ptr(), ent.data_ptr(), st)
        else:
            rc |= self.lib.rlw_bytes2(self.d, self.key.data_ptr(), db.off.data_ptr(), db.blob.data_ptr(),
                                      db.req_of.data_ptr(), self.PREFIX[self.config], self.plen, st)
        db.now.fill_(T0 + b // self.K)
        if rc:
            raise RuntimeError("workload generator launch failed")

    def resolve_struct(self, db):
        """Config 4: the batch's rl_resolve_batch (device pointers; strings = its prefix bytes)."""
        dom, first, ent = db.res
        s = hiprl.RlResolveBatch()
        s.n_desc, s.n_entries, s.bytes_len, s.reserved = self.d, 4 * self.d, db.blob_bytes(), 0
        s.bytes, s.domain, s.entry_first, s.entry = db.blob.data_ptr(), dom.data_ptr(), first.data_ptr(), ent.data_ptr()
        s.override_rule = None
        return s


class HostGen:
    """Config-1 batches (examples/ratelimit rules, 10k keys, workload.config1_batch) made on the
    host and copied to the device once, before timing."""

    def __init__(self, d: int, seed: int, dev):
        self.d, self.seed, self.dev = d, seed, dev

    def make(self, b: int):
        return _router().DeviceBatch.from_host(workload.config1_batch(b, d=self.d, seed=self.seed, t0=T0), self.dev)


def random_access_roofline(eng, alg_bytes, U, pipe_ms, step_ms):
    lp = ROOT / "tools" / "microbench" / "libroofline_probe.so"
    if not lp.exists() or U <= 0:
        return None
    lib = C.CDLL(str(lp))
    lib.rl_probe_roofline.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]
    lib.rl_probe_roofline.restype = C.c_int
    slots = sum(2 << int(x) for x in eng.cfg.log2_slots)  # 8 regions: home unit x window parity
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


def pmc_traffic(dom: str, config: int):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc summary of
    this workload (tools/pmc_round.sh <tag> <steps> "" <config>), only if it was measured on these
    exact kernel sources."""
    PMC_SUMMARY = PMC_SUMMARIES.get(config)
    if PMC_SUMMARY is None or not PMC_SUMMARY.exists():
        return None, "no PMC summary committed", None
    try:
        pm = json.loads(PMC_SUMMARY.read_text())
    except Exception as ex:  # noqa: BLE001
        return None, f"unreadable PMC summary: {ex}", None
    if pm.get("source_sha") != source_sha():
        return None, f"PMC summary {PMC_SUMMARY.name} is for other kernel sources ({pm.get('source_sha')})", None
    if config != pm.get("config", 3):
        return None, f"PMC summary {PMC_SUMMARY.name} is of config {pm.get('config', 3)}", None
    k = pm.get("kernels", {}).get(dom)
    return ((k or {}).get("hbm_bytes_per_launch"), f"{PMC_SUMMARY.name} (source {pm['source_sha']})",
            pm.get("hbm_bytes_per_batch"))


def cpu_baseline(args, rules, d, seed, K, b0, eng=None):
    """The C++ oracle (serial DoLimit restatement) on host batches of the same stream (numpy
    generator, batch indices from b0): 1 thread, then N key-sharded threads on the same batches.
    Config 4: the sample's rule ids are resolved beforehand (untimed, the engine's host
    rl_resolve): the CPU leg times DoLimit only."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as orc

    n_thr = args.cpu_threads or min(16, os.cpu_count() or 1)
    if args.config == 1:
        def gen(b, d, seed, batches_per_s, t0):
            return workload.config1_batch(b, d=d, seed=seed, t0=t0)
    elif args.config == 4:
        def gen(b, d, seed, batches_per_s, t0):
            hb, r4 = workload.config4_batch(b, d=d, seed=seed, t0=t0, batches_per_s=batches_per_s)
            hb.rule = eng.resolve(r4)[:d].astype(np.uint32)
            return hb
    elif args.config == 5:
        def gen(b, d, seed, batches_per_s, t0):
            return workload.config5_batch(b, d=d, N=100_000_000, seed=seed, t0=t0, batches_per_s=batches_per_s)
    else:
        gen = workload.config3_batch if args.config == 3 else workload.config2_batch
    hbs, legs = [], {}
    for threads in (1, n_thr):
        o = orc.Oracle(local_cache=args.config == 4)
        o.load_rules(rules)
        n_done, t_cpu, nb = 0, 0.0, 0
        while t_cpu < args.cpu_seconds and nb < 64:
            if nb == len(hbs):
                hbs.append(gen(b0 + nb, d=d, seed=seed, batches_per_s=K, t0=T0))
            if threads > 1 and nb == 0:  # one warm-up submit: the thread pool and the map start cold
                o.submit(hbs[nb], threads=threads)
            t1 = time.perf_counter()
            o.submit(hbs[nb], threads=threads)
            t_cpu += time.perf_counter() - t1
            n_done += d
            nb += 1
        legs[threads] = (n_done / t_cpu, nb, t_cpu)
    v1, nb1, t1 = legs[1]
    vn, nbn, tn = legs[n_thr]
    return {"value": round(vn, 1), "unit": "descriptor decisions/s", "cores": n_thr, "kind": "port",
            "sample": f"{nbn} batches ({nbn * d} descriptors) of the same stream (host-generated, cold table) through "
                      f"the C++ oracle, key-sharded over {n_thr} threads, {tn:.1f} s",
            "single_core": {"value": round(v1, 1), "cores": 1,
                            "sample": f"{nb1} batches, serial DoLimit over an in-memory Redis stand-in, {t1:.1f} s"}}


def logical_shards_main(args):
    """G logical shards on one GPU (SURVEY.md §8e readiness without a multi-GPU box): every
    origin draws its batch from the same Zipf key distribution, so each hot key lands on one
    owner from every origin. Reports records per owner (max / mean), the router's step
    breakdown (each origin's pack and unpack and each owner's decide timed alone), the bytes
    each GPU would move over xGMI, and the G-GPU step estimate from them."""
    import torch

    G, d, K = args.logical_shards, args.desc, max(1, args.batches_per_second)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lg = args.log2_slots - int(math.ceil(math.log2(G)))  # each shard holds 1/G of the live set
    rules = workload.CONFIG3_RULES if args.config == 3 else workload.CONFIG2_RULES
    engines = []
    for _ in range(G):
        e = hiprl.Engine(device=0, log2_slots=(lg, lg, lg, 12), max_batch_desc=G * d, max_batch_req=G * d,
                         max_blob_bytes=G * d * 17 + 64, sort_bits=48, pipeline=args.pipeline,
                         lib_path=(ROOT / args.lib) if args.lib else None)
        e.load_rules(rules)
        engines.append(e)
    r = hiprl.Router(engines, max_desc=d, combine=not args.no_combine)
    gens = [DeviceGen(args.config, d, (3 if args.config == 3 else 2) + 7919 * g, K, dev) for g in range(G)]
    bufs = [[gen.alloc() for gen in gens] for _ in range(2)]
    outs = [torch.empty(d * 20, dtype=torch.uint8, device=dev) for _ in range(G)]
    thrs = [torch.empty(d, dtype=torch.int32, device=dev) for _ in range(G)]
    prefill = args.prefill if args.prefill >= 0 else 64

    def step(b):
        dbs = bufs[b % 2]
        for gen, db in zip(gens, dbs):
            gen.fill(b, db)
        torch.cuda.synchronize()
        r.step([hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs()) for db in dbs],
               [o.data_ptr() for o in outs], [t.data_ptr() for t in thrs])
        return r.stats()

    for b in range(prefill + args.warmup):
        step(b)
    rows = [step(prefill + args.warmup + j) for j in range(args.steps)]
    rec = np.array([x["recv"] for x in rows], np.float64)  # steps x owners
    mean_owner = rec.mean(axis=1)
    keys = ["pack_us", "exchange_us", "decide_us", "decide_max_us", "reply_us", "unpack_us", "step_us"]
    br = {k: round(float(np.mean([x[k] for x in rows])), 1) for k in keys}
    # G real GPUs, one origin and one owner each: an origin packs and unpacks its own batch
    # (pack_us / G, unpack_us / G: the origins were timed one at a time), the hottest owner
    # decides its records (decide_max_us), and each GPU sends and receives over xGMI about
    # (G-1)/G of its records (32 B) and replies (8 B): max over owners of what it receives.
    xg = args.xgmi_gbps * 1e3  # bytes per us
    rmax = float(rec.max(axis=1).mean())
    xch_rec_us = (G - 1) / G * max(float(mean_owner.mean()), rmax) * hiprl.ROUTE_RECORD_BYTES / xg
    xch_rep_us = (G - 1) / G * max(float(mean_owner.mean()), rmax) * 8 / xg
    compute_us = br["pack_us"] / G + br["decide_max_us"] + br["unpack_us"] / G
    serial_us = compute_us + xch_rec_us + xch_rep_us
    # two steps in flight (rl_router_submit / _wait): exchanges overlap the other step's compute
    piped_us = max(compute_us, xch_rec_us + xch_rep_us)
    line = {"mode": "logical_shards", "n_shards": G, "descriptors_per_origin_batch": d, "steps": args.steps,
            "prefill_steps": prefill, "config": args.config, "log2_slots_per_shard": lg,
            "combining": not args.no_combine, "combined_steps": int(rows[-1]["combined_steps"]),
            "repacks": int(rows[-1]["repacks"]), "hot_groups_origin0": int(rows[-1]["hot_groups"]),
            "records_per_owner_mean": round(float(mean_owner.mean()), 1),
            "records_per_owner_max": int(rec.max()),
            "records_per_origin_batch": d,
            "owner_imbalance_max_over_mean": round(float((rec.max(axis=1) / mean_owner).mean()), 3),
            "records_per_owner_last_step": [int(x) for x in rows[-1]["recv"]],
            "step_breakdown_us": br,
            "xgmi_assumed_GBps_per_direction": args.xgmi_gbps,
            "estimate_us": {"pack_per_origin": round(br["pack_us"] / G, 1), "decide_hottest_owner": br["decide_max_us"],
                            "unpack_per_origin": round(br["unpack_us"] / G, 1),
                            "records_xgmi": round(xch_rec_us, 1), "replies_xgmi": round(xch_rep_us, 1),
                            "serial_step": round(serial_us, 1), "pipelined_step": round(piped_us, 1)},
            "estimated_step_us_on_G_gpus": round(piped_us, 1),
            "estimated_desc_per_s_on_G_gpus": round(G * d / (piped_us * 1e-6), 1),
            "estimated_desc_per_s_on_G_gpus_serial": round(G * d / (serial_us * 1e-6), 1),
            "note": "one GPU, G engines (local transport: exchanges are device copies, each origin's pack / unpack and "
                    "each owner's decide timed alone); estimate on G GPUs = max(pack/G + hottest decide + unpack/G, "
                    "xGMI time of the hottest owner's records + replies at the assumed bandwidth), two steps in "
                    "flight; serial = their sum"}
    print(json.dumps(line), flush=True)
    if args.json_out:
        Path(args.json_out).write_text(json.dumps(line) + "\n")
    r.close()


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        return rc
    if args.dry_launch:
        return dry_launch_main(args)
    if args.logical_shards:
        return logical_shards_main(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == args.gpus or (args.gpus == 1 and args.force_routed), (world, args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    args.native_router = not args.torch_router
    if world > 1 or args.force_routed:
        import torch.distributed as dist
        # the C-ABI router's own communicator bootstraps over loopback (one node); torch.distributed
        # (gloo) only shares its id and carries the barrier and the max over ranks of the time
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        if world == 1:  # --force-routed without a launcher (e.g. under rocprofv3): a group of one
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29561"), ("RANK", "0"), ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        if args.native_router:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    d, K = args.desc, max(1, args.batches_per_second or (16 if args.config == 5 else 8000))
    lg = args.log2_slots
    tree = None
    if args.config == 3:
        rules, log2 = workload.CONFIG3_RULES, (lg, lg, lg, 12)
        wl = "config3: 1e8 keys Zipf s=1.1, SECOND/MINUTE/HOUR by rank%3, 1 descriptor/request"
    elif args.config == 4:
        import rl_config
        # 1e9 keys: a larger live set than config 3's; 2^28 slots per region (51.5 GB)
        lg = 28 if args.log2_slots == 27 else lg
        log2 = (lg, lg, lg, 12)
        tree = rl_config.RateLimitConfig([("config4.yaml", workload.config4_yaml(4))])
        rules = [(r[0], r[1], k % 2 == 0) for k, r in enumerate(tree.rule_table())]  # every other rule shadow
        wl = ("config4: 1e9 keys Zipf s=1.1, 4-entry descriptors (a, b, c, d) resolved on the device in every step "
              "(rl_resolve_device; batch k+1's right after batch k's submit) by a 4-level descriptor tree "
              "(workload.config4_yaml(4)), local over-limit cache on, every other rule in shadow mode, "
              "1 descriptor/request")
    elif args.config == 5:
        rules, log2 = workload.CONFIG5_RULES, (lg, lg, lg, 12)
        wl = (f"config5: 60 simulated seconds ({K} batches per second, 59 s of prefill), 1e8 keys Zipf s=1.1, "
              "SECOND 20 / MINUTE 400 / HOUR 9000 by rank%3, hits_addend U{1..8}, near-limit ratio 0.8, "
              "1 descriptor/request")
    elif args.config == 2:
        rules, log2 = workload.CONFIG2_RULES, (lg, 12, 12, 12)
        wl = "config2: 1e6 uniform keys, SECOND L=5, 1 descriptor/request"
    else:
        if d == 1_000_000:  # (the default): config 1 is 10k keys, one batch of 10k requests per second
            d = 10_000
        K = 1
        # (a window start that is a multiple of 60 / 3600 / 86400 s makes the key string's home
        # unit MINUTE / HOUR / DAY, DESIGN.md §4: those regions take a whole batch too)
        rules, log2 = workload.CONFIG1_RULES, (20, 16, 16, 16)
        wl = ("config1: examples/ratelimit rules (rl.foo.baz SECOND 1, mongo_cps SECOND 500), 10k keys, "
              "1 descriptor/request, now +1 s per batch")
    prefill = args.prefill if args.prefill >= 0 else (59 * K if args.config == 5 else K + K // 2 if K > 1 else 0)
    seed = {1: 1, 2: 2, 3: 3, 4: 4, 5: 5}[args.config] + 7919 * rank  # each rank its own stream
    routed = (world > 1 or args.force_routed) and not args.independent
    # an owner may receive up to every origin's batch (hot keys concentrate on their owner)
    cap = d * world if routed else d
    eng = hiprl.Engine(device=local, log2_slots=log2, max_batch_desc=cap, max_batch_req=cap,
                       max_blob_bytes=cap * 32 + 64, sort_bits=48, pipeline=args.pipeline,
                       lib_path=(ROOT / args.lib) if args.lib else None, local_cache=args.config == 4)
    if tree is not None:
        tree.install(eng)  # the descriptor tree and its rule table (rl_load_tree, rl_load_rules)
    eng.load_rules(rules)
    # config 4: rule ids resolved on the device in every step (before the batch's submit; routed:
    # before timing, since the router's pack runs on the router's own stream)
    gen = HostGen(d, seed, dev) if args.config == 1 else DeviceGen(args.config, d, seed, K, dev)
    rtr = nrt = None
    if routed and args.native_router:
        ids = [hiprl.Router.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        nrt = hiprl.Router([eng], max_desc=d, n_shards=world, rank=rank, rccl_id=ids[0], combine=not args.no_combine)
    elif routed:
        router = _router()
        rtr = router.ShardRouter(router.EngineShard(eng, rank, world, dev, d))
    pipelined = not routed and not args.serial
    DEPTH = min(args.depth, hiprl.MAX_IN_FLIGHT) if pipelined else 1
    RDEPTH = max(1, min(3, args.router_depth)) if nrt is not None else 1
    outs = [torch.empty(d * 20, dtype=torch.uint8, device=dev) for _ in range(hiprl.MAX_IN_FLIGHT)]
    thrs = [torch.empty(d, dtype=torch.int32, device=dev) for _ in range(hiprl.MAX_IN_FLIGHT)]

    host_t = {"submit": [], "wait": [], "step": []}  # host seconds per engine call / per loop step (pipelined)

    def run(dbs, first=0, depth=None):
        """One step per batch. Pipelined: batch k+1 is submitted before batch k is waited for (the
        micro-batcher's double buffering; routed: rl_router_submit / rl_router_wait, two steps in
        flight); every batch is complete on return."""
        pend = 0
        hprev = 0.0
        rdepth = RDEPTH if depth is None else depth
        # config 4: every batch's rule ids resolved on the device inside the step, one batch ahead
        # (batch k+1's right after batch k's submit, so it can run beside k's kernels; each batch
        # has its own rule array, and the engine orders a submit after the resolves before it)
        # (RL_BENCH_RESOLVE_LATE=1, diagnostics: each batch resolved just before its own submit)
        late = os.environ.get("RL_BENCH_RESOLVE_LATE") == "1"
        resolve4 = args.config == 4 and nrt is None and rtr is None and not late
        if resolve4 and dbs:
            eng.resolve_device(gen.resolve_struct(dbs[0]), dbs[0].rule.data_ptr())
        for j, db in enumerate(dbs):
            if rtr is not None:
                rtr.step(db)
                continue
            if late and args.config == 4 and nrt is None:
                eng.resolve_device(gen.resolve_struct(db), db.rule.data_ptr())
            sb = hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs())
            o, t = outs[(first + j) % len(outs)].data_ptr(), thrs[(first + j) % len(thrs)].data_ptr()
            if nrt is not None:
                nrt.submit([sb], [o], [t])
                pend += 1
                if pend == rdepth:
                    nrt.wait()
                    pend -= 1
                continue
            if pipelined:
                if args.host_delay_us:  # (diagnostic: how the next batch's k4_hist start moves the step)
                    tq = time.perf_counter() + args.host_delay_us * 1e-6
                    while time.perf_counter() < tq:
                        pass
                h0 = time.perf_counter()
                if j:
                    host_t["step"].append(h0 - hprev)
                hprev = h0
                eng.submit_pipelined_batch(sb, o, t)
                if resolve4 and j + 1 < len(dbs):
                    eng.resolve_device(gen.resolve_struct(dbs[j + 1]), dbs[j + 1].rule.data_ptr())
                h1 = time.perf_counter()
                host_t["submit"].append(h1 - h0)
                pend += 1
                if pend == DEPTH:
                    eng.wait()
                    host_t["wait"].append(time.perf_counter() - h1)
                    pend -= 1
            else:
                eng.submit_device_async(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), o, t)
                if resolve4 and j + 1 < len(dbs):
                    eng.resolve_device(gen.resolve_struct(dbs[j + 1]), dbs[j + 1].rule.data_ptr())
                eng.wait()
        for _ in range(pend):
            if nrt is not None:
                nrt.wait()
            else:
                eng.wait()

    # Prefill (untimed): one batch generated at a time into a ring of buffers, the engine two
    # batches behind (a buffer is refilled only after the batch that used it completed).
    t_fill = time.time()
    ring = [gen.alloc() for _ in range(4)] if prefill else []
    pend = 0
    for b in range(prefill):
        db = ring[b % len(ring)]
        gen.fill(b, db)
        torch.cuda.current_stream(dev).synchronize()
        if args.config == 4:
            eng.resolve_device(gen.resolve_struct(db), db.rule.data_ptr())
            if nrt is not None or rtr is not None:
                torch.cuda.synchronize()  # (the router's pack runs on its own stream)
        if rtr is not None:
            rtr.step(db)
            continue
        sb = hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs())
        o, t = outs[b % len(outs)].data_ptr(), thrs[b % len(thrs)].data_ptr()
        if nrt is not None:
            nrt.submit([sb], [o], [t])
        else:
            eng.submit_pipelined_batch(sb, o, t)
        pend += 1
        if pend == 2:
            nrt.wait() if nrt is not None else eng.wait()
            pend -= 1
    for _ in range(pend):
        nrt.wait() if nrt is not None else eng.wait()
    t_fill = time.time() - t_fill
    fallbacks_prefill = eng.stats()["lsd_fallbacks"]
    # Timed batches (and warmup and kernel-timing batches) resident before timing.
    n_kt = 0 if args.no_kernel_times else args.steps
    b0 = prefill
    dbs = [gen.make(b0 + j) for j in range(args.warmup + args.steps + n_kt)]
    torch.cuda.synchronize()
    if args.config == 4 and (nrt is not None or rtr is not None):
        for db in dbs:  # routed: rule ids resolved before timing (the N = 1 line resolves inside the step)
            eng.resolve_device(gen.resolve_struct(db), db.rule.data_ptr())
        torch.cuda.synchronize()
    run(dbs[:args.warmup])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    fb0 = eng.stats()["lsd_fallbacks"]
    for v in host_t.values():
        v.clear()
    t0 = time.perf_counter()
    run(dbs[args.warmup:args.warmup + args.steps], args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # (outside the timed region)
    host_us = {k: {"mean": round(sum(v) / max(1, len(v)) * 1e6, 1),
                   "p50": round(float(np.median(v)) * 1e6, 1) if v else None,
                   "max": round(max(v) * 1e6, 1) if v else None} for k, v in host_t.items()}
    if args.dump_host_times:
        Path(args.dump_host_times).write_text(json.dumps({k: [round(x * 1e6, 2) for x in v] for k, v in host_t.items()}))
    fb_timed = eng.stats()["lsd_fallbacks"] - fb0
    rstats = nrt.stats() if nrt is not None else None
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.native_router else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_desc = world * args.steps * d
    value = total_desc / elapsed
    step_ms = elapsed / args.steps * 1e3

    # Per-kernel HIP-event timing over another K steps of the same stream (one stream, unoverlapped).
    kernel, uniq = None, []
    if n_kt:
        eng.set_timing(True)
        for j in range(args.warmup + args.steps, len(dbs)):
            run([dbs[j]], j)
            uniq.append(eng.last_batch_info()["unique_keys"])
        kt = eng.kernel_times()
        eng.set_timing(False)
        kernel = {k: dict(total_ms=v[0], launches=v[1]) for k, v in kt.items() if v[1]}
    if not uniq:
        uniq = [eng.last_batch_info()["unique_keys"]]
    if args.dump_stamps:  # diagnostic build: per-block phase stamps of the last batch
        st4 = np.zeros((4096, 8), np.uint64)
        eng.lib.rl_debug_st4.argtypes = [C.c_void_p]
        eng.lib.rl_debug_st4(st4.ctypes.data)
        np.save(args.dump_stamps, st4)
    stats = eng.stats()
    occ = eng.occupancy()

    # Host (PCIe) path (what a Go service sees: host batches, three in flight), in the compact
    # wire format (rl_batch_c: prefix bytes + one word per descriptor + one per request in, 8-B
    # raw replies out) and, for comparison, in the full rl_batch format (20-B statuses out):
    #  - the link bound: one batch's exact copies moved by the link alone, H2D and D2H on two
    #    streams (tools/pcie_probe.py's shapes);
    #  - staged: batches built in place in the engine's pinned slots (rl_host_acquire_c /
    #    rl_host_acquire), as a Go batcher writes its requests straight into C memory: only H2D,
    #    kernels (+ the compact form's expansion) and D2H are timed (each slot holds its batch
    #    from an untimed first pass; the batches repeat, which changes counters, not the cost);
    #    results read in the slot (rl_wait_raw_view / rl_wait_view);
    #  - host_decide: rl_decide_raw (GetResponseDescriptorStatus on the host, the work the
    #    reference's Go BaseRateLimiter does per descriptor) over those replies, ns per
    #    descriptor on 1 thread and desc/s on `threads` threads splitting each batch;
    #  - frac_of_pcie_bound = that bound / the measured per-batch time.
    host = None
    if not args.no_host_path and not routed:
        hbatches = []
        for db in dbs[args.warmup:args.warmup + args.steps]:
            n = int(db.off[-1].item())
            hbatches.append(hiprl.Batch(db.blob[:n].cpu().numpy(), db.off.cpu().numpy().view(np.uint32),
                                        db.rule.cpu().numpy().view(np.uint32), db.req_of.cpu().numpy().view(np.uint32),
                                        db.now.cpu().numpy(), db.hits.cpu().numpy().view(np.uint32)))
        cbatches = [hiprl.compact_batch(b) for b in hbatches]

        def link_probe(sz_in, sz_out, n=20):
            """ms per batch for the link to move one batch's exact copies (H2D arrays on one
            stream, D2H arrays on another; pinned host buffers): H2D alone, D2H alone, and both
            directions concurrently."""
            hin = [torch.empty(x, dtype=torch.uint8).pin_memory() for x in sz_in]
            din = [torch.empty(x, dtype=torch.uint8, device=dev) for x in sz_in]
            hout = [torch.empty(x, dtype=torch.uint8).pin_memory() for x in sz_out]
            dout = [torch.empty(x, dtype=torch.uint8, device=dev) for x in sz_out]
            s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

            def run(k, do_in, do_out):
                for _ in range(k):
                    if do_in:
                        with torch.cuda.stream(s1):
                            for h, dd in zip(hin, din):
                                dd.copy_(h, non_blocking=True)
                    if do_out:
                        with torch.cuda.stream(s2):
                            for h, dd in zip(hout, dout):
                                h.copy_(dd, non_blocking=True)

            res = []
            for do_in, do_out in ((True, False), (False, True), (True, True)):
                run(2, do_in, do_out)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                run(n, do_in, do_out)
                torch.cuda.synchronize()
                res.append((time.perf_counter() - t1) / n)
            return res

        def fill(sl, b):
            n = int(b.blob.shape[0])
            sl["blob"][:n] = b.blob
            sl["off"][:b.n_desc + 1] = b.off
            sl["rule"][:b.n_desc] = b.rule
            sl["req_of"][:b.n_desc] = b.req_of
            sl["now"][:b.n_req] = b.now
            sl["hits"][:b.n_req] = b.hits

        def fill_c(sl, cb):
            n = int(cb.blob.shape[0])
            sl["blob"][:n] = cb.blob
            sl["desc_word"][:cb.n_desc] = cb.desc_word
            sl["req_word"][:cb.n_req] = cb.req_word

        held = {}  # pinned slot (blob address) -> the batch built in it
        pv, pt = C.c_void_p(), C.c_void_p()

        def host_round(bs, build, compact):
            pend = 0
            for b in bs:
                sl = eng.host_acquire_c() if compact else eng.host_acquire()
                key = (compact, sl["blob"].ctypes.data)
                if build:
                    (fill_c if compact else fill)(sl, b)
                    held[key] = b
                else:  # the batch this slot already holds (built in place once)
                    b = held[key]
                if compact:
                    eng.submit_c_staged(b.n_desc, b.n_req, int(b.blob.shape[0]), b.now_base, sl)
                else:
                    eng.submit_staged(b.n_desc, b.n_req, int(b.blob.shape[0]), sl)
                pend += 1
                if pend == hiprl.MAX_IN_FLIGHT:
                    if compact:
                        eng._check(eng.lib.rl_wait_raw_view(eng.h, C.byref(pv)), "rl_wait_raw_view")
                    else:
                        eng._check(eng.lib.rl_wait_view(eng.h, C.byref(pv), C.byref(pt)), "rl_wait_view")
                    pend -= 1
            for _ in range(pend):
                if compact:
                    eng._check(eng.lib.rl_wait_raw_view(eng.h, C.byref(pv)), "rl_wait_raw_view")
                else:
                    eng._check(eng.lib.rl_wait_view(eng.h, C.byref(pv), C.byref(pt)), "rl_wait_view")

        nb3 = hiprl.MAX_IN_FLIGHT
        reps = max(3 * len(hbatches), 30)
        res = {}
        fmts = args.host_formats.split(",")
        for compact, src in ((True, cbatches), (False, hbatches)):
            if ("compact" if compact else "full") not in fmts:
                res[compact] = (float("nan"), src[:1])
                continue
            # the untimed first pass builds a batch in every slot; the timed rounds reuse them
            host_round(src[:nb3], True, compact)
            rep = [src[k % nb3] for k in range(reps)]
            host_round(rep[:2], False, compact)
            th = time.perf_counter()
            host_round(rep, False, compact)
            res[compact] = ((time.perf_counter() - th) / len(rep), rep)
        t_c, rep_c = res[True]
        t_f, rep_f = res[False]
        h2d_c = sum(cb.wire_bytes() + 32 for cb in rep_c) / len(rep_c)
        d2h_c = 8 * d
        h2d_f = sum(int(b.blob.shape[0]) + 32 + 4 * (b.n_desc + 1) + 8 * b.n_desc + 12 * b.n_req for b in rep_f) / len(rep_f)
        d2h_f = sum(20 * b.n_desc + 4 * b.n_req for b in rep_f) / len(rep_f)
        cb0, ab = cbatches[0], hbatches[0]
        nan3 = (float("nan"),) * 3
        lc = nan3 if args.host_no_probe else link_probe([int(cb0.blob.shape[0]) + 32, 8 * cb0.n_desc], [8 * cb0.n_desc])
        lf = nan3 if args.host_no_probe else link_probe(
            [int(ab.blob.shape[0]) + 32, 4 * (ab.n_desc + 1), 4 * ab.n_desc, 4 * ab.n_desc, 8 * ab.n_req, 4 * ab.n_req],
            [20 * ab.n_desc, 4 * ab.n_req])
        # host decisions from raw replies (rl_decide_raw), 1 and `threads` threads
        import concurrent.futures as cf
        eng.submit_c(cb0)
        raw0 = eng.wait_raw_into(cb0.n_desc)
        st0 = np.empty(cb0.n_desc, hiprl.STATUS_DTYPE)
        th0 = np.empty(cb0.n_req, np.uint32)
        tq = time.perf_counter()
        for _ in range(3):
            eng.decide_raw(cb0, raw0, 0, cb0.n_desc, st0, th0)
        t_dec1 = (time.perf_counter() - tq) / 3
        nthr = 8
        cuts = [cb0.n_desc * k // nthr for k in range(nthr + 1)]  # one descriptor per request: any cut
        with cf.ThreadPoolExecutor(nthr) as ex:
            def dec_all():
                list(ex.map(lambda k: eng.decide_raw(cb0, raw0, cuts[k], cuts[k + 1], st0, th0), range(nthr)))
            dec_all()
            tq = time.perf_counter()
            for _ in range(5):
                dec_all()
            t_decn = (time.perf_counter() - tq) / 5
        host = {"value": round(d / t_c, 1), "unit": "descriptor decisions/s",
                "format": "compact (rl_submit_c / rl_wait_raw_view)",
                "ms_per_batch": round(t_c * 1e3, 4),
                "bytes_per_desc": {"h2d": round(h2d_c / d, 2), "d2h": round(d2h_c / d, 2)},
                "bytes_per_batch": {"h2d": int(h2d_c), "d2h": int(d2h_c)},
                "link_ms_per_batch": {"h2d": round(lc[0] * 1e3, 4), "d2h": round(lc[1] * 1e3, 4),
                                      "both": round(lc[2] * 1e3, 4)},
                "pcie_bound_ms_per_batch": round(max(lc[0], lc[1]) * 1e3, 4),
                "frac_of_pcie_bound": round(max(lc[0], lc[1]) / t_c, 3),
                "achieved_GBps": {"h2d": round(h2d_c / t_c / 1e9, 1), "d2h": round(d2h_c / t_c / 1e9, 1)},
                "device_kernels_ms_per_batch": round(step_ms, 4),
                "host_decide": {"ns_per_desc_1_thread": round(t_dec1 / cb0.n_desc * 1e9, 2), "threads": nthr,
                                "value": round(cb0.n_desc / t_decn, 1), "unit": "descriptor statuses/s"},
                # the compact form's statuses are made on the host (rl_decide_raw): a caller gets
                # decisions at the slower of the two rates (the copy-in/out pipeline and the decide,
                # running on separate host threads), which the full format avoids
                "end_to_end": {"value": round(min(d / t_c, cb0.n_desc / t_decn), 1),
                               "bound_by": "host decide (rl_decide_raw)" if cb0.n_desc / t_decn < d / t_c
                               else "PCIe copies + kernels",
                               "unit": "descriptor decisions/s"},
                "full_format": {"value": round(d / t_f, 1), "ms_per_batch": round(t_f * 1e3, 4),
                                "bytes_per_desc": {"h2d": round(h2d_f / d, 2), "d2h": round(d2h_f / d, 2)},
                                "link_ms_per_batch": {"h2d": round(lf[0] * 1e3, 4), "d2h": round(lf[1] * 1e3, 4),
                                                      "both": round(lf[2] * 1e3, 4)},
                                "frac_of_pcie_bound": round(max(lf[0], lf[1]) / t_f, 3)},
                "note": "compact: prefix bytes + a 4-B word per descriptor (length | rule) + a 4-B word per request "
                        "(hits | time delta) H2D, expanded on the device; 8-B raw replies (INCRBY post-value or "
                        "local-cache hit) D2H; statuses made on the host by rl_decide_raw (host_decide, run by the "
                        "caller's threads as the reference's Go BaseRateLimiter would). full_format: rl_batch in, "
                        "20-B statuses + ThrottleMillis out. staged in the engine's pinned slots, 3 in flight, "
                        "H2D + kernels + D2H timed; bound = the link moving one batch's exact copies, the slower "
                        "direction alone"}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    U = float(np.mean(uniq))
    nbytes = int(dbs[-1].off[-1].item())
    alg_bytes = nbytes + 12 * d + 12 * d + 20 * d + 4 * d + 64 * int(U)  # workload.algorithmic_bytes, r = d
    alg_def = ("achieved = algorithmic bytes of one batch (SURVEY §8d: prefixes + 12 B/desc + 16 B/req + 20 B/desc out "
               "+ 64 B per unique key) / the dominant kernel's average launch time (HIP events on the engine stream, "
               "kernels unoverlapped)")
    kernel_alg = {}  # a kernel whose work is not the whole §8d batch: its own algorithmic bytes
    if args.config == 4 and not routed:
        # + the resolve step's inputs and output (the reference's descriptor entries): domain (off, len)
        # 8 B, entry_first 4 B, 4 entries x 16 B, the rule id written 4 B per descriptor
        alg_bytes += 80 * d
        alg_def += "; config 4: + 80 B/desc of rl_resolve_batch inputs and rule-id output (resolved in the step)"
        # k_resolve reads the strings (the descriptors' prefix bytes) and the 80 B/desc above, nothing
        # of the decision's bytes (priced at its own work, config_impl.go:274-323)
        for kname in ("k_resolve", "k_resolve_exact"):
            kernel_alg[kname] = nbytes + 80 * d
        alg_def += ("; a dominant k_resolve is priced at its own bytes: the prefix bytes it walks + 80 B/desc, "
                    "the k4_* kernels at the batch's §8d bytes without the resolve's 80 B/desc")
    if routed and rstats is not None:
        # an owner's launch decides the records it received, not a whole batch: price it at those
        # (32-B record in, 8-B raw reply out per record, 64 B per unique key of the owner batch)
        n_rec = int(rstats["recv"][rank]) or d
        alg_bytes = 40 * n_rec + 64 * int(U)
        alg_def = ("routed: achieved = the owner batch's algorithmic bytes (its received records: 32-B record in + 8-B "
                   "raw reply out each, + 64 B per unique key of the owner batch) / the dominant kernel's average "
                   "launch time on that batch (HIP events, unoverlapped); not a whole-batch figure")
    roofline = None
    if kernel:
        per_batch_ms = {k: v["total_ms"] / args.steps for k, v in kernel.items()}
        pipe_ms = sum(per_batch_ms.values())
        dom = max((k for k in per_batch_ms if k != "memset"), key=lambda k: per_batch_ms[k])
        dom_us = kernel[dom]["total_ms"] * 1e3 / kernel[dom]["launches"]
        # The dominant kernel priced at the batch's algorithmic bytes (SURVEY §8d's per-descriptor
        # figure x the descriptors one launch processes): every decision kernel of a batch handles
        # all of its descriptors, so each launch is held to the whole batch's bytes (config 4:
        # without the resolve's; k_resolve at its own, kernel_alg).
        dom_bytes = kernel_alg.get(dom, alg_bytes - (80 * d if kernel_alg else 0))
        achieved = dom_bytes / (dom_us * 1e-6) / 1e9
        # (the PMC summary profiles the unrouted step: no counter figure for an owner batch)
        traffic, tsrc, traffic_batch = pmc_traffic(dom, args.config) if not routed else (None, None, None)
        roofline = {
            "bound": "hbm", "kernel": dom,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "traffic_per_batch": traffic_batch,
            "traffic_over_algorithmic": round(traffic_batch / alg_bytes, 3) if traffic_batch else None,
            "algorithmic_bytes_per_batch": alg_bytes, "unique_keys_per_batch": int(U),
            "dominant_kernel_algorithmic_bytes": dom_bytes,
            "dominant_kernel_avg_us": round(dom_us, 2),
            "pipeline_us_per_batch": round(pipe_ms * 1e3, 2),
            "pipeline_achieved_GBps": round(alg_bytes / (pipe_ms * 1e-3) / 1e9, 1),
            "kernels_us_per_batch": {k: round(v * 1e3, 2) for k, v in per_batch_ms.items()},
            "definition": alg_def,
        }
        if not args.no_roofline_probe:
            ra = random_access_roofline(eng, alg_bytes, int(U), pipe_ms, step_ms)
            if ra:
                roofline["random_access"] = ra

    cpu = None
    if world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, rules, d, seed, K, b0, eng)

    live_frac = [round(occ["live"][r] / occ["slots"][r], 4) for r in range(8)]
    if routed and nrt is not None:
        parallelism = (f"key-sharded x{world}, RCCL all-to-all routing through the C-ABI router (32-B records out, one "
                       f"per hot key per origin with combining; 8-B raw replies back; {RDEPTH} steps in flight)")
    elif routed:
        parallelism = (f"key-sharded x{world}, RCCL all-to-all routing through router.ShardRouter (32-B records out, "
                       f"24-B replies back)")
    else:
        parallelism = "single shard" if world == 1 else f"x{world} independent replicas (no collective)"
    line = {
        "metric": "descriptor decisions/sec, 100M keys Zipf, 1-8 GPUs; % of HBM peak" if args.config == 3
        else f"descriptor decisions/sec (config {args.config})",
        "value": round(value, 1),
        "unit": "descriptor decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded splitmix64 / bounded Zipf stream, generated on the device, resident in HBM)",
        "config": {"workload": wl, "descriptors_per_batch": d, "requests_per_batch": d,
                   "batches_per_second_window": K, "prefill_batches": prefill,
                   "parallelism": parallelism,
                   "pipeline": args.pipeline, "batches_in_flight": RDEPTH if nrt is not None else DEPTH,
                   "combining": (not args.no_combine) if nrt is not None else None,
                   "unique_keys_per_batch": int(U)},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "host_path": host,
        "router": ({k: rstats[k] for k in ("recv", "sent", "combined", "combined_steps", "repacks", "hot_groups",
                                           "pack_us", "exchange_us", "decide_us", "reply_us", "unpack_us", "step_us")}
                   if rstats else None),
        "table": {"live_keys": stats["live_keys"], "region_live_fraction": live_frac, "region_slots": occ["slots"],
                  "bytes": int(sum(occ["slots"])) * 32},
        "engine": {"resorts": stats["resorts"], "lsd_fallbacks_prefill": fallbacks_prefill,
                   "lsd_fallbacks_timed": fb_timed, "hot_keys": stats["hot_keys"], "batches": stats["batches"],
                   "prefill_s": round(t_fill, 1), "source_sha": source_sha(),
                   # host time per step inside rl_submit_pipelined / rl_wait (pipelined single-GPU path only):
                   # submit is launch overhead the device may idle behind; wait is time the host blocks
                   "host_us_per_step": host_us if pipelined else None},
    }
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        Path(args.json_out).write_text(s + "\n")
    if nrt is not None:
        nrt.close()
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
