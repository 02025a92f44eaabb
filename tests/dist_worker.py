"""One rank of the multi-process shard test (tests/test_dist.py), launched
with torch.distributed.run like bench.py. Classifies this rank's packet
shard, sums the counter block over ranks and gathers the verdicts.

    --backend gloo --engine oracle   CPU (runs anywhere)
    --backend gloo --engine gpu      product path on cuda:LOCAL_RANK, gloo collectives
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
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    pktio = cls.loop_pktio(pktin=opt)
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


if __name__ == "__main__":
    main()
