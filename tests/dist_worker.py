"""One rank of the multi-process shard test (tests/test_dist.py), launched
with torch.distributed.run like bench.py. Classifies this rank's packet
shard, sums the counter block over ranks and gathers the verdicts.

    --backend gloo --engine oracle   CPU (runs anywhere)
    --backend gloo --engine gpu      product path on cuda:LOCAL_RANK, gloo collectives
    --config c2 | c4 | c5            the C2 rules, the C4 1024-PMR rules (limits
                                     raised before any create, as bench.py does),
                                     or example/l3fwd over the C5 routes
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from odp_amd import _lib as L  # noqa: E402
from odp_amd import cls, gen, shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npkt", type=int, default=40000)
    ap.add_argument("--engine", default="oracle", choices=["oracle", "gpu"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"])
    a = ap.parse_args()
    dist.init_process_group("gloo")
    if a.config == "c5":
        return main_l3fwd(a)
    rank, world = dist.get_rank(), dist.get_world_size()
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    if a.config == "c4":
        assert cls.set_limits(2048, 2048, 32) == 0
    pktio = cls.loop_pktio(pktin=opt)
    if a.config == "c4":
        gen.build_c4_rules(cls, pktio)
    else:
        gen.build_c2_rules(cls, pktio, stats=True)
    assert cls.pktio_start(pktio) == 0
    rules = cls.pktio_rules(pktio)
    # the table image: compiled on rank 0 only and broadcast (bench.py's
    # path); every rank checks it against its own compile of the same rules
    from odp_amd import gpu
    image = shard.broadcast_bytes(gpu.compile_rules(rules) if rank == 0 else None, dist)
    image_bad = shard.reduce_counters([int(image != gpu.compile_rules(rules))], dist)[0]
    frames = gen.c2_frames(a.npkt).reshape(a.npkt, 64)
    start, count = shard.shard_range(a.npkt, rank, world)
    mine = np.ascontiguousarray(frames[start:start + count])
    ctx = tbl = None
    if a.engine == "gpu":
        ndev = max(1, L.lib.odpg_device_count())     # ranks may share one GPU
        ctx = gpu.Context(int(os.environ.get("LOCAL_RANK", "0")) % ndev)
        tbl = ctx.table(image=image)

    def run(fr, n):
        if a.engine == "gpu":
            res = ctx.classify(tbl, fr, n, stride=64, opt=opt)
        else:
            import oracle
            res = oracle.classify(rules, fr, n, stride=64, opt=opt)
        return res["out"], res["stats"]

    out, stats = run(mine, count)
    total = shard.reduce_counters(stats, dist)
    allout = shard.gather_verdicts(out, dist, a.npkt, world)
    slowest = shard.max_over_ranks(float(rank), dist)
    # scatter-from-root / gather-to-root (equal shards of a batch on rank 0)
    import torch
    per = a.npkt // world
    whole = torch.from_numpy(np.ascontiguousarray(frames[:per * world])) if rank == 0 else None
    recv = torch.empty((per, 64), dtype=torch.uint8)
    shard.scatter_shards(whole, recv, dist)
    sout, _ = run(recv.numpy(), per)
    gathered = shard.gather_to_root(torch.from_numpy(sout.astype(np.int32)), dist)
    if tbl is not None:
        del tbl
        ctx.close()
    if rank == 0:
        with open(a.out, "w") as f:
            json.dump({"world": world, "stats": [int(x) for x in total],
                       "out_sha": int(np.bitwise_xor.reduce(allout.astype(np.uint64) *
                                                            np.arange(1, a.npkt + 1, dtype=np.uint64))),
                       "n_out": int(len(allout)), "max_rank": slowest,
                       "image_bad_ranks": int(image_bad), "image_bytes": len(image),
                       "scatter_gather_equal": bool(np.array_equal(
                           gathered.numpy().astype(np.uint32), allout[:per * world]))}, f)
        np.save(a.out + ".npy", allout)
    dist.destroy_process_group()


def main_l3fwd(a):
    """example/l3fwd (C5 routes, hash mode) over packet shards: every rank
    builds the forwarder from the same route list (odpg_fwd_create is a
    deterministic host compile), forwards its shard, and the ports and
    rewritten frames are gathered on rank 0"""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    routes = gen.c5_routes()
    frames = gen.c5_frames(a.npkt, routes, flows=a.npkt).reshape(a.npkt, 64)
    start, count = shard.shard_range(a.npkt, rank, world)
    mine = np.ascontiguousarray(frames[start:start + count]).reshape(-1)
    from odp_amd import gpu
    if a.engine == "gpu":
        ndev = max(1, L.lib.odpg_device_count())
        ctx = gpu.Context(int(os.environ.get("LOCAL_RANK", "0")) % ndev)
        fw = gpu.Forwarder(ctx, routes, mode=L.FWD_HASH)
        port, fr = fw.run(mine, 64, count)
        fr = np.asarray(fr)[:mine.nbytes]
        del fw
        ctx.close()
    else:
        import oracle
        port, fr = oracle.l3fwd(gpu.make_routes(routes), gpu.make_fwd_param(L.FWD_HASH, 4),
                                mine, 64, count)
    ports = shard.gather_verdicts(np.asarray(port).astype(np.uint32), dist, a.npkt, world)
    # the rewritten frames: equal-size pieces gathered as int64 words
    counts = [shard.shard_range(a.npkt, r, world)[1] for r in range(world)]
    buf = np.zeros((max(counts), 64), np.uint8)
    buf[:count] = np.asarray(fr, np.uint8).reshape(count, 64)
    t = torch.from_numpy(buf.view(np.int64).copy())
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    allfr = np.concatenate([p.numpy().view(np.uint8).reshape(-1, 64)[:c]
                            for p, c in zip(parts, counts)])
    if rank == 0:
        with open(a.out, "w") as f:
            json.dump({"world": world, "n_out": int(len(ports))}, f)
        np.save(a.out + ".npy", ports.astype(np.int32))
        np.save(a.out + ".frames.npy", allfr)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
