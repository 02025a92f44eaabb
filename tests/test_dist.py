"""Multi-process sharding: world_size-2 runs under
torch.distributed.run with gloo. The sharded job's gathered verdicts and
all-reduced counter block must equal one whole-batch run of the same input.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from odp_amd import shard

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 256, 1000003):
        for w in (1, 2, 3, 8):
            seen = 0
            for r in range(w):
                s, c = shard.shard_range(n, r, w)
                assert s == seen and c >= 0
                seen += c
            assert seen == n
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, engine, n=40000, world=2, config="c2"):
    out = str(tmp_path / f"dist_{engine}_{config}.json")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(HERE, "dist_worker.py"),
           "--npkt", str(n), "--engine", engine, "--out", out, "--config", config]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.load(open(out)), np.load(out + ".npy")


def _whole(n, config="c2"):
    import oracle
    from odp_amd import _lib as L
    from odp_amd import cls, gen
    opt = L.PKTIN_IPV4_CHKSUM | L.PKTIN_UDP_CHKSUM | L.PKTIN_TCP_CHKSUM
    cls.reset()
    if config == "c4":
        assert cls.set_limits(2048, 2048, 32) == 0
    pktio = cls.loop_pktio(pktin=opt)
    if config == "c4":
        gen.build_c4_rules(cls, pktio)
    else:
        gen.build_c2_rules(cls, pktio, stats=True)
    assert cls.pktio_start(pktio) == 0
    rules = cls.pktio_rules(pktio)
    frames = gen.c2_frames(n)
    ref = oracle.classify(rules, frames, n, stride=64, opt=opt)
    cls.reset()
    return ref


def test_two_rank_gloo_matches_whole_batch(tmp_path):
    n = 40000
    got, allout = _run(tmp_path, "oracle", n)
    ref = _whole(n)
    assert got["world"] == 2 and got["n_out"] == n and got["max_rank"] == 1.0
    np.testing.assert_array_equal(allout, ref["out"])
    assert got["stats"] == [int(x) for x in ref["stats"]]
    assert got["stats"][0] == n          # every packet delivered to a CoS queue
    # rank 0's compiled image reached rank 1 byte-exact; scatter/gather path
    assert got["image_bad_ranks"] == 0 and got["image_bytes"] > 0
    assert got["scatter_gather_equal"]


@pytest.mark.gpu
def test_two_rank_gpu_shards_match_whole_batch(tmp_path):
    """Both ranks classify on the GPU through the C-ABI; gloo carries the
    counter all-reduce and the verdict gather."""
    n = 40000
    got, allout = _run(tmp_path, "gpu", n)
    ref = _whole(n)
    np.testing.assert_array_equal(allout, ref["out"])
    assert got["stats"] == [int(x) for x in ref["stats"]]


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu(tmp_path):
    """bench.py itself with world size 2 over gloo, both ranks on one GPU:
    the table image broadcast, per-rank shards, max-over-ranks timing, the
    counter all-reduce and the scatter-from-rank-0 / gather-to-root loop."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "4", "--batch", str(1 << 16), "--no-cpu", "--backend", "gloo",
           "--source", "gpu0", "--others", "none"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["with_pktio_counters"]["value"] > 0
    assert d["scatter_gather"]["value"] > 0 and d["scatter_gather"]["backend"] == "gloo"


def test_bench_spawns_its_ranks_without_a_launcher():
    """`python bench.py --gpus N` (no WORLD_SIZE) starts N ranks itself through
    a torch.distributed.run child; each sees world N (checked before any GPU
    call, so this runs on CPU)."""
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "3",
           "--backend", "gloo", "--spawn-check"]
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="1"), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = []
    for x in r.stdout.splitlines():
        try:
            d = json.loads(x[x.index("{"):]) if "{" in x else None
        except ValueError:
            continue
        if isinstance(d, dict) and "rank" in d:
            recs.append(d)
    assert sorted(d["rank"] for d in recs) == [0, 1, 2], r.stdout[-2000:]
    assert all(d["world"] == 3 for d in recs)


def test_bench_refuses_a_world_size_mismatch():
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2",
           "--spawn-check"]
    r = subprocess.run(cmd, env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "launcher started 1 ranks" in r.stderr


@pytest.mark.gpu
def test_bench_rccl_path_on_one_gpu():
    """bench.py with the RCCL ("nccl") process group at world size 1: the
    table-image broadcast, the max / sum all-reduces and the scatter-from-
    rank-0 / gather-to-root loop run as RCCL collectives on the MI355X (the
    8-GPU run's code path, one rank)."""
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "1",
           "--steps", "20", "--warmup", "4", "--batch", str(1 << 16), "--no-cpu",
           "--backend", "nccl", "--source", "gpu0", "--others", "none"]
    env = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["distributed"]["backend"] == "nccl" and d["distributed"]["world"] == 1
    assert d["scatter_gather"]["value"] > 0 and d["scatter_gather"]["backend"] == "nccl"


@pytest.mark.gpu
def test_bench_other_configs():
    """The default 1-GPU run's `other_configs`: further configs measured in
    the same process, one compact entry each (value, kernel time, roofline
    fraction, traffic ratio, counted-launch time, CPU baseline)."""
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--steps", "20",
           "--warmup", "4", "--runs", "1", "--batch", str(1 << 16), "--cpu-seconds", "1",
           "--others", "c1,c3,c5", "--others-cpu-seconds", "1"]
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="2"), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    assert len(line[0]) < 2048    # three entries here; all five stay near 2 KB
    d = json.loads(line[0])
    oc = d["other_configs"]
    assert sorted(oc) == ["c1", "c3", "c5"]
    for c, e in oc.items():
        assert e["value"] > 0 and e["kernel_ms"] > 0 and 0 < e["frac"] < 1.2, (c, e)
        assert e["cpu"] > 0 and e["cpu_1thread"] > 0, (c, e)
    assert oc["c1"]["counted_kernel_ms"] > 0 and "counted_kernel_ms" not in oc["c5"]


def _whole_l3fwd(n):
    import oracle
    from odp_amd import _lib as L
    from odp_amd import gen, gpu
    routes = gen.c5_routes()
    frames = gen.c5_frames(n, routes, flows=n)
    return oracle.l3fwd(gpu.make_routes(routes), gpu.make_fwd_param(L.FWD_HASH, 4), frames,
                        64, n)


@pytest.mark.parametrize("engine", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_two_rank_c4_image_and_verdicts(tmp_path, engine):
    """C4 (1024 PMRs, limits raised with set_limits(2048, 2048, 32) before
    any create): rank 0's broadcast image equals each rank's own compile,
    and the gathered verdicts and reduced counters equal one whole-batch
    run."""
    n = 24000
    got, allout = _run(tmp_path, engine, n, config="c4")
    ref = _whole(n, "c4")
    assert got["world"] == 2 and got["n_out"] == n
    assert got["image_bad_ranks"] == 0 and got["image_bytes"] > 0
    np.testing.assert_array_equal(allout, ref["out"])
    # pktio counters; no C4 CoS has stats_enable, so every CoS word is zero
    # (the GPU block may stop after the pktio words)
    want = [int(x) for x in ref["stats"]]
    assert got["stats"][:4] == want[:4] and got["stats"][0] == n
    assert not any(got["stats"][4:]) and not any(want[4:])
    assert got["scatter_gather_equal"]
    assert len(np.unique(ref["out"] & 0xFFFF)) > 100


@pytest.mark.parametrize("engine", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_two_rank_c5_l3fwd(tmp_path, engine):
    """example/l3fwd over two packet shards: gathered ports and rewritten
    frames equal one whole-batch run of the oracle"""
    n = 30000
    got, ports = _run(tmp_path, engine, n, config="c5")
    out = str(tmp_path / f"dist_{engine}_c5.json")
    frames = np.load(out + ".frames.npy")
    o_port, o_fr = _whole_l3fwd(n)
    assert got["world"] == 2 and got["n_out"] == n
    np.testing.assert_array_equal(ports, np.asarray(o_port).astype(np.int32))
    np.testing.assert_array_equal(frames.reshape(-1), np.asarray(o_fr).reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c4", "c5"])
def test_bench_two_ranks_one_gpu_c4_c5(tmp_path, config):
    """bench.py --config c4 / c5 --gpus 2 --backend gloo, both ranks on one
    GPU (the configs BASELINE names at 8 GPUs): n_gpus is the process group's
    size and every rank ran its shard."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2",
           "--config", config, "--steps", "10", "--warmup", "2", "--runs", "2",
           "--batch", str(1 << 16), "--no-cpu", "--backend", "gloo"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["config"]["batch_per_gpu"] == 1 << 16
