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
    frames = gen.c2_frames(a.npkt).reshape(a.npkt, 64)
    start, count = shard.shard_range(a.npkt, rank, world)
    mine = np.ascontiguousarray(frames[start:start + count])
    if a.engine == "gpu":
        from odp_amd import gpu
        ndev = max(1, L.lib.odpg_device_count())     # ranks may share one GPU
        ctx = gpu.Context(int(os.environ.get("LOCAL_RANK", "0")) % ndev)
        tbl = ctx.table(rules)
        res = ctx.classify(tbl, mine, count, stride=64, opt=opt)
        out, stats = res["out"], res["stats"]
        del tbl
        ctx.close()
    else:
        import oracle
        res = oracle.classify(rules, mine, count, stride=64, opt=opt)
        out, stats = res["out"], res["stats"]
    total = shard.reduce_counters(stats, dist)
    allout = shard.gather_verdicts(out, dist, a.npkt, world)
    slowest = shard.max_over_ranks(float(rank), dist)
    if rank == 0:
        with open(a.out, "w") as f:
            json.dump({"world": world, "stats": [int(x) for x in total],
                       "out_sha": int(np.bitwise_xor.reduce(allout.astype(np.uint64) *
                                                            np.arange(1, a.npkt + 1, dtype=np.uint64))),
                       "n_out": int(len(allout)), "max_rank": slowest}, f)
        np.save(a.out + ".npy", allout)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
