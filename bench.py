#!/usr/bin/env python3
"""Benchmark: Mpps classified (device-resident), 64 B packets x 64 PMR rules.

One step = one pass of the receive-path classifier (parse + RX checksum
verdict + PMR -> CoS walk, odpg_classify) over one batch of 2^20 synthetic
frames already resident in HBM, writing the 4-byte verdict per packet (CoS
index + RX checksum status, the per-packet outputs the north star names). A
second timed loop repeats the launches with the loopback_recv pktio counters
(and the per-CoS / per-queue delivery counts) added in every launch, into the
sharded device counters odp_pktio_stats reads; it is reported as
`with_pktio_counters`.

Launch:  python bench.py [--gpus N --steps K --warmup W --config c2]
         torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
`python bench.py --gpus N` with N > 1 and no launcher environment starts the
N rank processes itself (a torch.distributed.run child process, before any
GPU call) and exits with its status; under a launcher WORLD_SIZE must equal
--gpus. n_gpus in the line is the process group's size.
Packets are independent: each rank classifies its own shard (weak scaling,
no data-path collective). Rank 0 compiles the rule table once and broadcasts
the image (odpg_rules_compile / odpg_table_import); the only other collective
is the end-of-run all-reduce of the CoS / pktio counters (odp_cls_cos_stats
semantics). --backend picks RCCL ("nccl", default) or gloo; ranks beyond the
visible GPUs share them (LOCAL_RANK modulo the device count), so a 2-rank
gloo run on one GPU exercises the whole multi-rank path. --source gpu0 adds
a second workload: each step's batch originates on rank 0's GPU, is
scattered over the ranks and the verdicts gathered back.

Rank 0 prints one JSON line (contract in the task description) with a
`roofline` object (kernel time from HIP events on the classify stream) and a
`cpu_baseline` object (the CPU restatement timed on this host's cores). The
default 1-GPU run also measures the other BASELINE configs (C1, C2x, C3, C4,
C5) in the same process and summarises them in `other_configs` (--others).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def log(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    print(msg, file=sys.stderr, flush=True)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "Mpps classified (device-resident), 64B pkts × 64 PMR rules"


# BASELINE.json's other configs (C1, C3, C4 on one GPU, C5) and SURVEY §8(d)'s
# second C2 rule mix, measured beside the headline by the default run
OTHER_CONFIGS = ("c1", "c2x", "c3", "c4", "c5")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--runs", type=int, default=5,
                    help="timed loops of exactly --steps launches each (after one warmup); "
                         "the line reports the median run (SURVEY.md 8(d))")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c2x", "c3", "c4", "c5", "tx"])
    ap.add_argument("--fwd-mode", default="hash", choices=["hash", "lpm"],
                    help="c5 only: l3fwd lookup mode")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--buffers", type=int, default=0,
                    help="rotating input batches (default: enough to exceed the 256 MiB "
                         "Infinity Cache so every launch streams from HBM)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stats", action="store_true",
                    help="skip the second timed loop (launches with pktio counters)")
    ap.add_argument("--kernel-mode", type=int, default=0,
                    help="0 auto, 1 wave-cooperative walk, 2 evaluate-all, 3 hash walk")
    ap.add_argument("--diag", default="full",
                    choices=["full", "parse", "parse-nochk", "l3", "none"],
                    help="diagnostic floors (not the metric): 'parse' = parse + checksum "
                         "verdicts without CoS matching, 'none' = frame loads + result "
                         "stores only")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the host-buffer path (pinned H2D + kernel + D2H)")
    ap.add_argument("--backend", default=os.environ.get("ODPG_DIST_BACKEND", "nccl"),
                    choices=["nccl", "gloo"], help="torch.distributed backend for N > 1")
    ap.add_argument("--source", default="sharded", choices=["sharded", "gpu0"],
                    help="gpu0: also time scatter-from-rank-0 + classify + gather-to-root "
                         "(initialises the process group even for one rank)")
    ap.add_argument("--spawn-check", action="store_true",
                    help="ranks print their rank / world size and exit before any GPU "
                         "call (tests the launcher path on CPU)")
    ap.add_argument("--others", default=None,
                    help="comma list of further configs measured in the same process and "
                         "summarised in the line's `other_configs` (default on a 1-GPU "
                         "headline run: " + ",".join(OTHER_CONFIGS) + "; 'none' to skip)")
    ap.add_argument("--others-cpu-seconds", type=float, default=6.0,
                    help="CPU-baseline seconds per further config")
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: one rank process per GPU through a
    torch.distributed.run child (never an exec of this process), rendezvous
    on 127.0.0.1; returns the child's exit status."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if args.spawn_check:
        print(json.dumps({"rank": rank, "world": world}), flush=True)
        return
    dist = None
    if world > 1 or args.source == "gpu0":
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        ndev = torch.cuda.device_count()
        local = local % ndev if ndev else local     # ranks may share a GPU
        torch.cuda.set_device(local)
        tdist.init_process_group(args.backend, rank=rank, world_size=world)
        dist = tdist
        world = tdist.get_world_size()

    out = run_config(args, world, rank, local, dist)
    others = args.others
    if others is None:
        others = ",".join(OTHER_CONFIGS) if world == 1 and args.config == "c2" and \
            args.diag == "full" else "none"
    if out is not None and others != "none":
        out["other_configs"] = measure_others(args, others.split(","), world, rank, local, dist)
    if out is not None:
        # compact separators: the line (with other_configs) stays near 2 KB,
        # inside the tail the driver keeps
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_config(args, world, rank, local, dist):
    """One config's measurement; rank 0 gets the line's dict, others None."""
    if args.config == "c5":
        return bench_l3fwd(args, world, rank, local, dist)
    if args.config == "tx":
        return bench_tx(args, world, rank, local, dist)
    return bench_classify(args, world, rank, local, dist)


def measure_others(args, cfgs, world, rank, local, dist):
    """The other configs in this process, each with fewer timed launches and
    a shorter CPU-baseline leg; a compact summary per config (progress on
    stderr): value (Mpps, this run's clock), kernel_ms (HIP events on the
    launch stream), frac of HBM peak, traffic_x (committed PMC bytes per
    launch / algorithmic), counted_kernel_ms (pktio counters on), and the
    CPU baseline (cpu: the per-GPU core share, as the headline's
    cpu_baseline.cores; cpu_1thread: one thread)."""
    import copy
    res = {}
    for c in cfgs:
        a = copy.copy(args)
        a.config, a.others, a.e2e, a.source = c, "none", False, "sharded"
        # 100 warmup launches: the first ~10 ms of heavy traffic run with
        # the memory side still clocking up (DESIGN §3 "C3 under the trace")
        a.steps, a.warmup, a.runs = min(args.steps, 100), 100, 3
        a.cpu_seconds = args.others_cpu_seconds
        a.batch = 1 << 20
        t0 = time.perf_counter()
        log(f"other config {c} ...")
        r = run_config(a, world, rank, local, dist)
        if r is None:
            continue
        rf = r["roofline"]
        alg = rf["bytes_per_pkt"] * rf["pkts_per_launch"]
        cpu = r.get("cpu_baseline") or {}
        e = {"value": round(r["value"]), "kernel_ms": rf["kernel_ms"], "frac": round(rf["frac"], 3),
             "traffic_x": round(rf["traffic"] / alg, 3) if rf.get("traffic") else None}
        if "with_pktio_counters" in r:
            e["counted_kernel_ms"] = r["with_pktio_counters"]["kernel_ms"]
        if cpu:
            e["cpu"] = round(cpu.get("value"), 1)
            e["cpu_1thread"] = round(cpu.get("value_1thread"), 1)
        res[c] = e
        log(f"other config {c}: {e} ({time.perf_counter() - t0:.1f} s)")
    return res


def bench_classify(args, world, rank, local, dist):
    """C1 / C2 / C2x / C3 / C4: odpg_classify launches (bench.py docstring)."""
    import ctypes as C

    import numpy as np

    from odp_amd import _lib as L
    from odp_amd import cls, gen, gpu, shard

    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    if args.config == "c4":
        assert cls.set_limits(2048, 2048, 32) == 0
    pktio = cls.loop_pktio(pktin=opt)
    if args.config == "c1":
        gen.build_c1_rules(cls, pktio)
        nrules = 1
        frames_fn = gen.c1_frames
        workload = ("C1: 64B IPv4/UDP x 1 PMR (SIP 10.10.10.0/24 -> queue1, "
                    "example/classifier rule)")
    elif args.config == "c4":
        gen.build_c4_rules(cls, pktio)
        nrules = 1024
        frames_fn = gen.c2_frames
        workload = "C4: 64B IPv4/UDP x 1024 PMR (32x SIP/21 -> 32x31 UDP_DPORT), raised limits"
    elif args.config == "c2x":
        gen.build_c2x_rules(cls, pktio)
        nrules = 60
        frames_fn = gen.c2x_frames
        workload = ("C2x: 64B Eth/VLAN/QinQ IPv4 UDP|TCP + IPv6/UDP + multicast x 60 PMR over "
                    "the other term kinds (ETHTYPE_0, DMAC, IPPROTO, IP_DSCP, VLAN_ID_0/X, "
                    "VLAN_PCP, DIP6, CUSTOM_L3/FRAME, TCP_DPORT, UDP_S/DPORT), pktin "
                    "ipv4+udp+tcp checksum verify (SURVEY 8(d) C2 second rule mix)")
    elif args.config == "c3":
        gen.build_c3_rules(cls, pktio)
        nrules = 256
        frames_fn = gen.c3_frames
        workload = ("C3: IMIX 7:4:1 64/570/1518B, 80/20 IPv4/IPv6, 50/50 UDP/TCP, ~2% "
                    "checksum errors/zero/fragments x 256 PMR DAG over 63 CoS + error CoS, "
                    "pktin ipv4+udp+tcp checksum verify, (offset,len) descriptors")
    else:
        gen.build_c2_rules(cls, pktio)
        nrules = 64
        frames_fn = gen.c2_frames
        workload = ("C2: 64B IPv4/UDP x 64 PMR (default -> 8x SIP_ADDR/19 -> 8x7 UDP_DPORT "
                    "-> 55 leaf CoS), pktin ipv4+udp+tcp checksum verify")
    assert cls.pktio_start(pktio) == 0
    rules = cls.pktio_rules(pktio)
    # the table is compiled once, on rank 0, and its image broadcast
    dev = f"cuda:{local}" if dist is not None and args.backend == "nccl" else None
    image = gpu.compile_rules(rules) if rank == 0 else None
    image = shard.broadcast_bytes(image, dist, dev)

    n = args.batch
    # each rank owns a distinct shard of the synthetic capture
    frames = frames_fn(n, seed=gen.C_SEED + rank)
    desc = None
    if isinstance(frames, tuple):            # descriptor layout (C3)
        frames, desc = frames
        stride = 0
        frame_bytes = float(desc["len"].mean())
        bytes_per_pkt = frame_bytes + 8 + 4  # frame + descriptor + verdict
    else:
        stride = 64
        frame_bytes = stride
        bytes_per_pkt = stride + 4           # frame + verdict
    ctx = gpu.Context(local)
    ctx.set_kernel_mode(args.kernel_mode)
    tbl = ctx.table(image=image)
    nbuf = args.buffers or max(2, -(-300 * (1 << 20) // frames.nbytes))
    fbufs, obufs, dbufs = [], [], []
    for _ in range(nbuf):
        fb = ctx.buffer(frames.nbytes)
        fb.upload(frames)
        fbufs.append(fb)
        if desc is not None:
            db = ctx.buffer(desc.nbytes)
            db.upload(desc)
            dbufs.append(db)
        obufs.append(ctx.buffer(4 * n))
    cnt = ctx.counters(tbl)
    layer, do_cls = {"full": (L.LAYER_ALL, 1), "parse": (L.LAYER_ALL, 0),
                     "parse-nochk": (L.LAYER_ALL, 0), "l3": (L.LAYER_L3, 0),
                     "none": (L.LAYER_NONE, 0)}[args.diag]
    if args.diag in ("parse-nochk", "l3"):
        opt = 0
    batches = [L.odpg_batch_t(fb.ptr, dbufs[k].ptr if dbufs else None, stride, n, opt, layer,
                              do_cls) for k, fb in enumerate(fbufs)]
    # the timed launches produce what the north star names per packet: the
    # verdict word (CoS index, L3/L4 checksum status, error / drop bits). A
    # second timed loop adds the loopback_recv pktio counters (in_packets /
    # in_octets / in_errors / in_discards, loop.c:304-374) and the per-queue
    # delivery counts (_odp_cos_queue_stats_add) to every launch: sharded
    # device counters (odpg.h), folded once when read.
    results = [L.odpg_result_t(ob.ptr, None, None, None, None) for ob in obufs]
    results_st = [L.odpg_result_t(ob.ptr, None, None, None, cnt.h) for ob in obufs]
    lib = L.lib

    def launch(i, res):
        rc = lib.odpg_classify(ctx.h, tbl.h, C.byref(batches[i % nbuf]), C.byref(res[i % nbuf]))
        if rc:
            raise RuntimeError(f"odpg_classify rc={rc}")

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()

    def timed(res):
        return timed_runs(args, ctx, lambda i: launch(i, res), barrier, dist, dev)

    wall, kernel_ms, enq_ms, run_ms = timed(results)
    counted = None
    if not args.no_stats:
        wall_st, kernel_ms_st, _, run_ms_st = timed(results_st)
        # the read-time fold, then CoS / pktio counters summed over GPUs (RCCL)
        folded = cnt.fold()
        tf0 = time.perf_counter()          # a steady-state fold (code loaded)
        cnt.fold()
        fold_ms = (time.perf_counter() - tf0) * 1e3
        stats = shard.reduce_counters(np.concatenate([folded["pktio"], folded["cos"]]),
                                      dist, dev)
        # (experiment builds, ODPG_LIB, may skip the counter commit)
        if args.diag == "full" and not os.environ.get("ODPG_LIB"):
            # loopback_recv accounting: every packet is either delivered
            # error-free (in_packets) or counted in in_errors (error CoS /
            # parse error)
            launches = args.warmup + args.steps * max(1, args.runs)
            assert int(stats[0]) + int(stats[2]) == n * world * launches, ("packets lost",
                                                                             stats[:4])
            if args.config != "c3":
                assert int(stats[0]) == n * world * launches, ("not every packet was delivered",
                                                               stats[:4])
        counted = {"value": round(n * world * args.steps / wall_st / 1e6, 1),
                   "ms_per_step": round(wall_st * 1e3 / max(args.steps, 1), 5),
                   "kernel_ms": round(kernel_ms_st, 5),
                   "runs_ms_per_step": run_ms_st,
                   "fold_ms": round(fold_ms, 3),
                   "what": "same launches + pktio/queue counters; fold_ms: read-time fold"}

    ms_per_step = wall * 1e3 / max(args.steps, 1)
    total_pkts = n * world * args.steps
    value = total_pkts / wall / 1e6
    achieved = bytes_per_pkt * n / (kernel_ms * 1e-3) / 1e9

    out = None
    if rank == 0:
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None, "kernel_ms": round(kernel_ms, 5),
                    "bytes_per_pkt": round(bytes_per_pkt, 2), "pkts_per_launch": n}
        roofline["traffic"], roofline["traffic_source"] = pmc_traffic(args.config)
        cpu = None
        if not args.no_cpu and world == 1:
            cpu = cpu_baseline(rules, frames, desc, n, stride, opt, args)
        out = {
            "metric": METRIC if args.config == "c2" else (
                METRIC.replace("64B pkts", "IMIX pkts").replace("64 PMR", f"{nrules} PMR")
                + " + RX checksum verify" if args.config == "c3"
                else METRIC.replace("64 PMR", f"{nrules} mixed-term PMR")
                if args.config == "c2x" else METRIC.replace("64 PMR", f"{nrules} PMR")),
            "value": round(value, 1), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "runs": max(1, args.runs), "runs_ms_per_step": run_ms,
            "host_enqueue_ms_per_step": round(enq_ms / max(args.steps, 1), 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": workload, "batch_per_gpu": n,
                       "frame_bytes": round(frame_bytes, 2),
                       "pmr_rules": nrules, "rotating_buffers": nbuf,
                       "kernel_mode": ["auto", "walk", "evaluate-all", "hash-walk"][args.kernel_mode],
                       "parallelism": f"dp{world} (packet shards, no collective)"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if counted:
            out["with_pktio_counters"] = counted
        if args.diag != "full":
            out["diag"] = args.diag
        if args.e2e:
            out["e2e_host_path"] = e2e(ctx, tbl, frames, desc, n, stride, opt)
        if dist is not None:
            out["distributed"] = {
                "backend": args.backend, "world": world,
                "collectives": ["broadcast (table image)", "all_reduce max (wall clock)",
                                "all_reduce sum (counters)"]
                + (["scatter (frames)", "gather (verdicts)"] if args.source == "gpu0" else [])}
    if args.source == "gpu0" and dist is not None and stride:
        sg = bench_scatter_gather(args, ctx, tbl, frames, n, stride, opt, world, rank, local,
                                  dist)
        if out is not None:
            out["scatter_gather"] = sg
    cnt.close()
    del tbl
    for b in fbufs + obufs + dbufs:
        b.free()
    ctx.close()
    return out


def timed_runs(args, ctx, launch, barrier, dist, dev):
    """warmup, then args.runs loops of exactly args.steps launches, each
    between barriers (device sync + process-group barrier); returns the
    median run's (wall seconds, mean HIP-event ms per launch on the launch
    stream, host ms spent enqueueing the launches) and every run's wall ms
    per step. The wall clock is the max over ranks per run."""
    import ctypes as C

    from odp_amd import _lib as L
    from odp_amd import shard
    lib = L.lib
    for i in range(args.warmup):
        launch(i)
    runs = []
    for _ in range(max(1, args.runs)):
        barrier()
        t0 = time.perf_counter()
        lib.odpg_event_record(ctx.h, 0)
        for i in range(args.steps):
            launch(i)
        lib.odpg_event_record(ctx.h, 1)
        te = time.perf_counter()
        ctx.sync()
        t1 = time.perf_counter()
        barrier()
        ev_ms = C.c_float(0)
        L.check(lib.odpg_event_elapsed_ms(ctx.h, 0, 1, C.byref(ev_ms)), "event")
        runs.append((shard.max_over_ranks(t1 - t0, dist, dev),
                     ev_ms.value / max(args.steps, 1), (te - t0) * 1e3))
    order = sorted(range(len(runs)), key=lambda k: runs[k][0])
    med = runs[order[len(runs) // 2]]
    return med[0], med[1], med[2], [round(r[0] * 1e3 / max(args.steps, 1), 5) for r in runs]


def bench_scatter_gather(args, ctx, tbl, frames, n, stride, opt, world, rank, local, dist):
    """SURVEY §8(e) optional path: the whole batch (world x n frames) sits in
    rank 0's HBM; per step it is scattered over the ranks (RCCL over xGMI, or
    gloo through host memory), each rank classifies its shard, and the verdict
    shards are gathered on rank 0. Timed like the headline loop (barriers,
    max over ranks); value = world * n packets per step / time."""
    import ctypes as C

    import numpy as np
    import torch

    from odp_amd import _lib as L
    from odp_amd import shard
    on_gpu = args.backend == "nccl"
    cdev = torch.device(f"cuda:{local}") if on_gpu else torch.device("cpu")
    per = torch.from_numpy(np.ascontiguousarray(frames).reshape(n, stride))
    whole = per.repeat(world, 1).to(cdev) if rank == 0 else None
    mine = torch.empty((n, stride), dtype=torch.uint8, device=cdev)
    verd = torch.empty(n, dtype=torch.int32, device=cdev)
    fb = ob = None
    if not on_gpu:                  # gloo moves host tensors: stage them
        fb, ob = ctx.buffer(n * stride), ctx.buffer(4 * n)
    src = mine.data_ptr() if on_gpu else fb.ptr
    dst = verd.data_ptr() if on_gpu else ob.ptr
    b = L.odpg_batch_t(src, None, stride, n, opt, L.LAYER_ALL, 1)
    r = L.odpg_result_t(dst, None, None, None, None)

    def step():
        shard.scatter_shards(whole, mine, dist)
        if on_gpu:                  # the shard in HBM, classified in place
            torch.cuda.current_stream().synchronize()
        else:
            fb.upload(mine.numpy())
        L.check(L.lib.odpg_classify(ctx.h, tbl.h, C.byref(b), C.byref(r)), "odpg_classify")
        ctx.sync()
        if not on_gpu:
            verd.copy_(torch.from_numpy(ob.download(np.int32, n)))
        return shard.gather_to_root(verd, dist)

    for _ in range(max(1, args.warmup // 4)):
        step()
    ctx.sync()
    dist.barrier()
    steps = max(1, args.steps // 4)
    t0 = time.perf_counter()
    for _ in range(steps):
        got = step()
    if on_gpu:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    wall = shard.max_over_ranks(t1 - t0, dist, cdev if on_gpu else None)
    if rank == 0:
        # every shard is the same capture: the gathered verdicts repeat
        g = got.cpu().numpy().reshape(world, n)
        assert all(np.array_equal(g[0], g[k]) for k in range(world)), "gathered shards differ"
    for x in (fb, ob):
        if x is not None:
            x.free()
    return {"value": round(world * n * steps / wall / 1e6, 1),
            "ms_per_step": round(wall * 1e3 / steps, 4), "steps": steps,
            "backend": args.backend,
            "what": "batch on rank 0's GPU: scatter (64 B/pkt) + classify + gather 4 B "
                    "verdicts to rank 0, per step"}


def pmc_traffic(config):
    """HBM bytes per launch of the timed kernel from the committed rocprofv3
    PMC summary (profiles/pmc_traffic_<config>.json, tools/pmc.sh +
    tools/pmc_summary.py: FETCH_SIZE x 2 on gfx950 + WRITE_SIZE), or None;
    and where the figure comes from: the summary records a fingerprint of the
    kernel sources it was collected on (tools/kernel_fingerprint.py), so a
    figure from other kernels is reported as stale, not as this run's."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_fingerprint import fingerprint
    tf = os.path.join(ROOT, "profiles", f"pmc_traffic_{config}.json")
    try:
        rec = json.load(open(tf))
    except (OSError, ValueError):
        return None, "no PMC summary for this config"
    src = f"profiles/pmc_traffic_{config}.json (rocprofv3 --pmc, separate run"
    if rec.get("kernel_sources_sha256") == fingerprint():
        src += ", these kernel sources)"
    else:
        src += "; STALE: other kernel sources)"
    return rec.get("bytes_per_launch"), src


def bench_tx(args, world, rank, local, dist):
    """Loop pktio TX side (include/odpg_tx.h): loopback_fix_checksums +
    get_dest_queue over 2^20 64 B IPv4/UDP frames per launch, IPv4 + UDP
    checksums inserted in place, crc32c queue pick over 8 loop queues."""
    import ctypes as C

    import numpy as np

    from odp_amd import _lib as L
    from odp_amd import gen, gpu, shard

    n = args.batch
    frames = gen.c2_frames(n, seed=gen.C_SEED + rank).reshape(n, 64).copy()
    frames[:, 24:26] = 0                 # IPv4 header checksum
    frames[:, 40:42] = 0                 # UDP checksum
    frames = frames.reshape(-1)
    ctx = gpu.Context(local)
    nbuf = args.buffers or max(2, -(-300 * (1 << 20) // frames.nbytes))
    fbufs, obufs = [], []
    for _ in range(nbuf):
        fb = ctx.buffer(frames.nbytes)
        fb.upload(frames)
        fbufs.append(fb)
        obufs.append(ctx.buffer(4 * n))
    hp = L.HASH_IPV4_UDP | L.HASH_IPV4
    cfg = L.odpg_tx_cfg_t(L.PKTOUT_IPV4_CHKSUM | L.PKTOUT_UDP_CHKSUM | L.PKTOUT_TCP_CHKSUM,
                          L.PKTOUT_LOOP_CAPA, hp, 8, 0, 0)
    batches = [L.odpg_tx_batch_t(fb.ptr, None, 64, n, None) for fb in fbufs]
    lib = L.lib

    def launch(i):
        rc = lib.odpg_tx_prepare(ctx.h, C.byref(batches[i % nbuf]), C.byref(cfg),
                                 obufs[i % nbuf].ptr)
        if rc:
            raise RuntimeError(f"odpg_tx_prepare rc={rc}")

    dev = f"cuda:{local}" if dist is not None and args.backend == "nccl" else None

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()
    wall, kernel_ms, enq_ms, run_ms = timed_runs(args, ctx, launch, barrier, dist, dev)
    out = obufs[(args.steps - 1) % nbuf].download(np.uint32, n)
    assert np.all(out & L.TX_OUT_IPV4) and np.all(out & L.TX_OUT_UDP)
    value = n * world * args.steps / wall / 1e6
    bytes_per_pkt = 64 + 4 + 4           # frame read + two checksum fields + out word
    achieved = bytes_per_pkt * n / (kernel_ms * 1e-3) / 1e9
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle

            def tx_slice(lo, hi):
                oracle.tx_prepare(frames[lo * 64:hi * 64], hi - lo, stride=64,
                                  pktout_cfg=cfg.pktout_cfg, hash_proto=hp, num_qs=8)
            cpu = cpu_baseline_mt(tx_slice, n, args, "TX")
        res = {
            "metric": "Mpps TX-prepared (device-resident), 64B pkts, IPv4+UDP checksum insert "
                      "+ crc32c loop queue pick",
            "value": round(value, 1), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / max(args.steps, 1), 5),
            "runs": max(1, args.runs), "runs_ms_per_step": run_ms,
            "host_enqueue_ms_per_step": round(enq_ms / max(args.steps, 1), 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "loop pktio TX: 64B IPv4/UDP with zeroed checksums, pktout "
                                   "ipv4+udp+tcp insert, hash ipv4_udp+ipv4 over 8 queues",
                       "batch_per_gpu": n, "frame_bytes": 64, "rotating_buffers": nbuf,
                       "parallelism": f"dp{world} (packet shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(args.config)[0],
                         "traffic_source": pmc_traffic(args.config)[1],
                         "kernel_ms": round(kernel_ms, 5),
                         "bytes_per_pkt": bytes_per_pkt, "pkts_per_launch": n},
            "cpu_baseline": cpu,
        }
    for b in fbufs + obufs:
        b.free()
    ctx.close()
    return res if rank == 0 else None


def bench_l3fwd(args, world, rank, local, dist):
    """C5: example/l3fwd forwarding decision (include/odpg_fwd.h) over 10 M
    distinct flows of 64 B frames, routes over <= 32 subnets; frames are
    rewritten in place (TTL, checksum, MACs) every step, as l3fwd does."""
    import ctypes as C

    import numpy as np

    from odp_amd import _lib as L
    from odp_amd import gen, gpu, shard

    n = args.batch if args.batch != (1 << 20) else gen.C5_FLOWS
    mode = L.FWD_LPM if args.fwd_mode == "lpm" else L.FWD_HASH
    routes = gen.c5_routes()
    frames = gen.c5_frames(n, routes, seed=gen.C_SEED + rank)
    ctx = gpu.Context(local)
    fw = gpu.Forwarder(ctx, routes, mode=mode)
    nbuf = args.buffers or max(2, -(-300 * (1 << 20) // frames.nbytes))
    fbufs, obufs = [], []
    for _ in range(nbuf):
        fb = ctx.buffer(frames.nbytes)
        fb.upload(frames)
        fbufs.append(fb)
        obufs.append(ctx.buffer(4 * n))
    batches = [L.odpg_fwd_batch_t(fb.ptr, 64, n, 0, 0) for fb in fbufs]
    lib = L.lib

    def launch(i):
        rc = lib.odpg_l3fwd(ctx.h, fw.h, C.byref(batches[i % nbuf]), obufs[i % nbuf].ptr)
        if rc:
            raise RuntimeError(f"odpg_l3fwd rc={rc}")

    dev = f"cuda:{local}" if dist is not None and args.backend == "nccl" else None

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()
    wall, kernel_ms, enq_ms, run_ms = timed_runs(args, ctx, launch, barrier, dist, dev)
    out = obufs[(args.steps - 1) % nbuf].download(np.int32, n)
    assert (out >= 0).all(), "every C5 packet is IPv4 and forwarded"
    value = n * world * args.steps / wall / 1e6
    bytes_per_pkt = 64 + 32 + 4          # frame read + header rewrite + port
    achieved = bytes_per_pkt * n / (kernel_ms * 1e-3) / 1e9
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle

            def fwd_passes(lo, hi, reps):
                return oracle.l3fwd_passes(fw.routes, fw.param, frames[lo * 64:hi * 64], 64,
                                           hi - lo, reps)
            cpu = cpu_baseline_mt(None, n, args, "C5", passes=fwd_passes)
        res = {
            "metric": f"Mpps forwarded (device-resident), 64B pkts, l3fwd {args.fwd_mode}, "
                      "10M flows",
            "value": round(value, 1), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / max(args.steps, 1), 5),
            "runs": max(1, args.runs), "runs_ms_per_step": run_ms,
            "host_enqueue_ms_per_step": round(enq_ms / max(args.steps, 1), 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"C5: example/l3fwd {args.fwd_mode} mode, {len(routes)} "
                                   "routes (nested /8../28), 10M distinct 5-tuple flows, "
                                   "64B IPv4 UDP/TCP, in-place TTL/checksum/MAC rewrite",
                       "batch_per_gpu": n, "frame_bytes": 64, "routes": len(routes),
                       "rotating_buffers": nbuf,
                       "parallelism": f"dp{world} (packet shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(args.config)[0],
                         "traffic_source": pmc_traffic(args.config)[1],
                         "kernel_ms": round(kernel_ms, 5),
                         "bytes_per_pkt": bytes_per_pkt, "pkts_per_launch": n,
                         "bytes_note": ("SURVEY.md 8(d) prices C5 at 196 B/pkt (frame + a "
                                        "hash-table probe); the interval table replaces "
                                        "the probe with an LDS search, so 64 B read + "
                                        "32 B header rewrite + 4 B port = 100 B. The "
                                        "kernel writes each frame's whole 64 B back "
                                        "(coalesced): partial-sector writes of the "
                                        "32 B measured slower (263 vs 252 us), so its "
                                        "HBM traffic is 132 B/pkt")},
            "cpu_baseline": cpu,
        }
    del fw
    for b in fbufs + obufs:
        b.free()
    ctx.close()
    return res if rank == 0 else None


def cpu_baseline(rules, frames, desc, n, stride, opt, args):
    """The CPU restatement of linux-generic's classifier (oracle/, a literal
    port of the reference's per-packet path) timed on this host's cores over
    the same batch, ~cpu_seconds of work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import statistics

    import oracle
    cpus, share = cpu_share()
    threads = args.cpu_threads or len(cpus)
    cpus = (cpus * (threads // len(cpus) + 1))[:threads]
    sub = min(n, 1 << 18)
    # single-thread calibration pass (pinned)
    t = time.perf_counter()
    oracle.classify_mt(rules, frames, sub, stride=stride, desc=desc, opt=opt, nthreads=1, reps=1,
                       cpus=cpus[:1])
    one = sub / (time.perf_counter() - t) / 1e6
    # all cores of the share, pinned, median of 5 runs; each
    # run is ~cpu_seconds / 5 of work
    runs = 5
    reps = max(1, int(args.cpu_seconds / runs * one * threads * 1e6 / n * 0.8))
    rates = []
    used = threads
    for _ in range(runs):
        t = time.perf_counter()
        _, used = oracle.classify_mt(rules, frames, n, stride=stride, desc=desc, opt=opt,
                                     nthreads=threads, reps=reps, cpus=cpus)
        rates.append(n * reps / (time.perf_counter() - t) / 1e6)
        log(f"cpu baseline: {used} threads {rates[-1]:.1f} Mpps")
    # SURVEY.md §8(d) also asks for every core (nproc). Where the host
    # grants this job fewer cores than its affinity mask lists (the GPU box:
    # OMP_NUM_THREADS=16 of 256), a run over the whole mask measures that
    # quota, not the cores, and is not reported
    allc = None
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    if len(aff) > used:
        allc = {"value": None,
                "note": f"not measured: {len(aff)} CPUs in the mask, {used} granted"}
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(statistics.median(rates), 2), "unit": "Mpps", "cores": used,
            "kind": "port", "value_1thread": round(one, 2), "cpu_model": model,
            "runs_mpps": [round(r, 2) for r in rates], "all_cores": allc,
            "sample": f"median of {runs} runs x {reps} passes over the {n}-pkt "
                      f"{args.config.upper()} batch in host DRAM, {used} threads pinned ({share})"}


def cpu_baseline_mt(work, n, args, what, passes=None):
    """A CPU restatement whose C entry point works on a packet range
    (work(lo, hi), a ctypes call that releases the GIL) timed on the host's
    per-GPU core share: one pinned thread per core over its own slice of the
    batch, median of 5 runs of ~cpu_seconds / 5 each, plus a 1-thread
    calibration figure (1 thread and all cores). With
    `passes(lo, hi, reps)` instead (an entry point with per-call setup, such
    as l3fwd's warmed flow cache), each thread makes one call of `reps`
    passes and reports their time without the setup; the rate is all
    threads' packets over the slowest thread's pass time."""
    import statistics
    import threading

    cpus, share = cpu_share()
    threads = args.cpu_threads or len(cpus)
    cpus = (cpus * (threads // len(cpus) + 1))[:threads]

    def run_passes(nthr, seconds, rate_hint):
        per = max(1, n // nthr)
        reps = max(1, int(seconds * rate_hint * 1e6 / per))
        secs = [0.0] * nthr

        def body(t):
            try:
                os.sched_setaffinity(0, {cpus[t]})      # this thread only
            except (AttributeError, OSError):
                pass
            lo = t * per
            secs[t] = passes(lo, min(n, lo + per), reps)
        th = [threading.Thread(target=body, args=(t,)) for t in range(nthr)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        return per * reps * nthr / max(secs) / 1e6

    def run(nthr, seconds):
        per = max(1, n // nthr)
        done = [0] * nthr
        stop = time.perf_counter() + seconds

        def body(t):
            try:
                os.sched_setaffinity(0, {cpus[t]})      # this thread only
            except (AttributeError, OSError):
                pass
            lo = t * per
            hi = min(n, lo + per)
            while time.perf_counter() < stop:
                work(lo, hi)
                done[t] += hi - lo
        th = [threading.Thread(target=body, args=(t,)) for t in range(nthr)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        return sum(done) / (time.perf_counter() - t0) / 1e6
    rates = []
    if passes is not None:
        n1 = min(n, 1 << 20)
        one = n1 / passes(0, n1, 1) / 1e6             # calibration: one pass, 1 thread
        for _ in range(5):
            rates.append(run_passes(threads, args.cpu_seconds / 5, one))
            log(f"cpu baseline {what}: {threads} threads {rates[-1]:.1f} Mpps")
    else:
        one = run(1, min(args.cpu_seconds / 5, 4.0))
        for _ in range(5):
            rates.append(run(threads, args.cpu_seconds / 5))
            log(f"cpu baseline {what}: {threads} threads {rates[-1]:.1f} Mpps")
    return {"value": round(statistics.median(rates), 2), "unit": "Mpps", "cores": threads,
            "kind": "port", "value_1thread": round(one, 2),
            "runs_mpps": [round(r, 2) for r in rates],
            "sample": f"median of 5 runs of ~{args.cpu_seconds / 5:.0f} s, {threads} threads "
                      f"pinned one per core ({share}), each over its own {n // threads}-packet "
                      f"slice of the {what} batch in host DRAM, passes repeated"
                      + ("; per-call setup (l3fwd's route table / warmed flow cache) outside "
                         "the timed passes, as the reference builds it before its workers; "
                         "1-thread figure: one pass over 2^20 packets" if passes is not None
                         else "; 1-thread figure: one thread over the whole batch")}


def cpu_share():
    """CPUs the CPU baseline may use: the affinity mask, capped at the host's
    declared per-GPU share (the GPU box sets OMP_NUM_THREADS to the 16 cores
    it grants one GPU job; its affinity mask lists the whole machine).
    Returns (cpu list, description)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and 0 < int(cap) < len(aff):
        return aff[:int(cap)], f"{int(cap)} of {len(aff)} CPUs, OMP_NUM_THREADS={cap}"
    return aff, f"all {len(aff)} CPUs of the affinity mask"


def e2e(ctx, tbl, frames, desc, n, stride, opt):
    """Host (pinned) buffers -> H2D -> classify -> D2H verdicts (odpg_classify_host:
    three staging sets cycling over a copy stream and the compute stream)."""
    import ctypes as C

    import numpy as np

    from odp_amd import _lib as L
    lib = L.lib
    hp = C.c_void_p()
    L.check(lib.odpg_host_alloc_pinned(frames.nbytes, C.byref(hp)), "pinned")
    ho = C.c_void_p()
    L.check(lib.odpg_host_alloc_pinned(4 * n, C.byref(ho)), "pinned")
    C.memmove(hp.value, frames.ctypes.data, frames.nbytes)
    dptr = None
    if desc is not None:
        hd = C.c_void_p()
        L.check(lib.odpg_host_alloc_pinned(desc.nbytes, C.byref(hd)), "pinned")
        C.memmove(hd.value, desc.ctypes.data, desc.nbytes)
        dptr = hd.value
    b = L.odpg_batch_t(hp.value, dptr, stride, n, opt, L.LAYER_ALL, 1)
    r = L.odpg_result_t(ho.value, None, None, None)
    res = {}
    for chunk in (1 << 16, 1 << 17, 1 << 18, 1 << 19):
        lib.odpg_classify_host(ctx.h, tbl.h, C.byref(b), C.byref(r), chunk)
        reps = 10
        t = time.perf_counter()
        for _ in range(reps):
            L.check(lib.odpg_classify_host(ctx.h, tbl.h, C.byref(b), C.byref(r), chunk), "host")
        dt = (time.perf_counter() - t) / reps
        res[f"chunk_{chunk}"] = {"mpps": round(n / dt / 1e6, 1),
                                 "gbps_h2d": round(frames.nbytes / dt / 1e9, 2)}
    lib.odpg_host_free_pinned(hp.value)
    if dptr:
        lib.odpg_host_free_pinned(dptr)
    lib.odpg_host_free_pinned(ho.value)
    del np
    return res


if __name__ == "__main__":
    main()
