"""example/l3fwd forwarding (include/odpg_fwd.h).

CPU tests pin the oracle's restatement: the reference example test
(udp64.pcap through route 10.0.0.0/24 -> IF1, platform/linux-generic/test/
example/l3fwd/pktio_env + example/l3fwd/odp_l3fwd_run.sh), the newest-first
route scan, the LPM trie's construction quirks read off odp_l3fwd_lpm.c, and
the TTL / checksum update. GPU tests compare odpg_l3fwd() with the oracle
bit for bit (output ports and every rewritten frame byte).
"""
import numpy as np
import pytest

import oracle
from helpers import GOLDEN
from odp_amd import _lib as L
from odp_amd import gen, gpu


def ip(s):
    return gen.ip4(s)


def R(addr, depth, port, k=0):
    return (ip(addr) if isinstance(addr, str) else addr, depth, port,
            [0x02, 0, 0, 0, 0x10, port], [0x02, 0, 0, 1, k, port])


def frames_to(dsts, proto=gen.PROTO_UDP, ttl=64):
    n = len(dsts)
    return gen.ipv4_frames(n, 64, np.full(n, ip("172.16.0.1"), np.uint64),
                           np.array(dsts, np.uint64), proto, 1000, 2000, ttl=ttl).reshape(-1)


def ip_hdr_ok(fr, l3=14):
    h = fr[l3:l3 + 20].astype(np.uint32)
    s = int((h[0::2] << 8).sum() + h[1::2].sum())
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s == 0xFFFF


def run_oracle(routes, frames, mode=L.FWD_HASH, stride=64, sif=0, error_check=False):
    num = len(frames) // stride
    return oracle.l3fwd(gpu.make_routes(routes), gpu.make_fwd_param(mode, 4), frames, stride,
                        num, sif, error_check)


# ---- reference fixture ----------------------------------------------------
def test_example_l3fwd_pcap():
    """odp_l3fwd_run.sh: -i IF0,IF1 -r "10.0.0.0/24,IF1"; the run passes when
    every packet of udp64.pcap (100 x 10.0.0.1 -> 10.0.0.2) leaves on IF1."""
    pk = [bytes.fromhex(h) for h in GOLDEN["pcap"]["perf_udp64"]]
    buf = np.zeros((len(pk), 64), np.uint8)
    for k, p in enumerate(pk):
        buf[k, :len(p)] = np.frombuffer(p, np.uint8)
    routes = [R("10.0.0.0", 24, 1)]
    out, fr = run_oracle(routes, buf.reshape(-1))
    assert (out == 1).all()
    fr = fr.reshape(-1, 64)
    assert (fr[:, 22] == buf[:, 22] - 1).all()                   # TTL - 1
    assert all(ip_hdr_ok(f) for f in fr)                         # checksum still valid
    assert (fr[:, 0:6] == routes[0][4]).all() and (fr[:, 6:12] == routes[0][3]).all()


# ---- find_fwd_db_entry: newest route first ---------------------------------
def test_hash_newest_route_wins():
    routes = [R("10.1.0.0", 16, 1, 0), R("10.1.2.0", 24, 2, 1), R("10.0.0.0", 8, 3, 2)]
    out, _ = run_oracle(routes, frames_to([ip("10.1.2.3"), ip("10.1.9.9"), ip("10.200.0.1"),
                                           ip("11.0.0.1")]), sif=0)
    # 10.0.0.0/8 was added last, so it is scanned first and wins everywhere it covers
    assert list(out) == [3, 3, 3, 0]
    # most specific added last: it is scanned first
    routes = [R("10.0.0.0", 8, 3, 2), R("10.1.0.0", 16, 1, 0), R("10.1.2.0", 24, 2, 1)]
    out, _ = run_oracle(routes, frames_to([ip("10.1.2.3"), ip("10.1.9.9"), ip("10.7.0.1")]))
    assert list(out) == [2, 1, 3]


def test_hash_no_route_swaps_mac():
    fr = frames_to([ip("192.0.2.1")])
    out, f2 = run_oracle([R("10.0.0.0", 8, 1)], fr, sif=2)
    assert out[0] == 2
    assert (f2[0:6] == fr[6:12]).all() and (f2[6:12] == fr[6:12]).all()


# ---- the hash-mode flow cache (odp_l3fwd_db.c:178-335, 474-508) ------------
# Expected ports below are read off the reference code: init_fwd_hash_cache
# caches addr + i for i < 2^(32 - depth), newest route first, and returns at
# the first address already cached or when the 2^22 flows are used up;
# find_fwd_db_entry answers from the cache, else from the masked first match
# (depth 32: "1u << 32" is a shift by 0 on x86-64, mask 0).
def test_hash_host_bits_route_is_served_by_the_warmed_cache():
    out, _ = run_oracle([R("10.0.0.5", 24, 1)],
                        frames_to([ip("10.0.0.5"), ip("10.0.1.4"), ip("10.0.0.4"),
                                   ip("10.0.1.5")]), sif=3)
    assert list(out) == [1, 1, 3, 3]      # 256 warmed hosts from .5; the scan never matches


def test_hash_depth32_routes():
    out, _ = run_oracle([R("10.0.0.7", 32, 2)], frames_to([ip("10.0.0.7"), ip("10.0.0.8")]),
                        sif=0)
    assert list(out) == [2, 0]
    # 0.0.0.0/32 (newest): mask 0 matches every address the cache does not
    # hold; the older /24's hosts were warmed after it and stay on the /24
    out, _ = run_oracle([R("10.0.0.0", 24, 1), R(0, 32, 3)],
                        frames_to([ip("10.0.0.9"), ip("192.0.2.1"), 0, ip("10.0.1.1")]), sif=0)
    assert list(out) == [1, 3, 3, 3]


def test_hash_warmup_stops_at_first_cached_address():
    """The newest route (host bits set) warms 9.255.255.0 .. 10.0.0.255; the
    older /24's first host is then already cached, so the warm-up returns:
    10.0.0.9 stays on the newer route although the scan would pick the /24."""
    routes = [R("10.0.0.0", 24, 1), R("9.255.255.0", 23, 2)]
    out, _ = run_oracle(routes, frames_to([ip("10.0.0.9"), ip("10.0.1.200"), ip("10.0.2.1"),
                                           ip("9.255.255.0"), ip("9.255.254.255")]), sif=0)
    assert list(out) == [2, 0, 0, 2, 0]


def test_hash_warmup_wraps_and_is_capped():
    # 255.255.255.0 with depth 16 warms 65536 hosts, wrapping into 0.0.x.x
    out, _ = run_oracle([R("255.255.255.0", 16, 1)],
                        frames_to([ip("255.255.255.9"), ip("0.0.1.1"), ip("0.0.254.255"),
                                   ip("0.0.255.0")]), sif=2)
    assert list(out) == [1, 1, 1, 2]
    # a /8 with host bits: only the first 2^22 hosts fit in the flow store
    out, _ = run_oracle([R("10.0.0.1", 8, 1)],
                        frames_to([ip("10.0.0.1"), ip("10.64.0.0"), ip("10.64.0.1")]), sif=2)
    assert list(out) == [1, 1, 2]


# ---- fib_tbl_insert / fib_tbl_lookup quirks (odp_l3fwd_lpm.c) ---------------
def test_lpm_short_prefix_sets_one_first_level_node():
    """depth <= 16 writes only fib_rt_tbl[ip >> 16] (:184-201)."""
    port, valid = oracle.fib_lookup(gpu.make_routes([R("10.0.0.0", 8, 3)]),
                                    [ip("10.0.5.5"), ip("10.1.0.1")])
    assert list(valid) == [True, False] and port[0] == 3


def test_lpm_split_children_stay_invalid():
    """A split copies next_hop / depth into the new children but not the
    valid bit (:107-122): after /16 then /24, the /16's other addresses miss."""
    routes = [R("10.0.1.0", 24, 2), R("10.0.0.0", 16, 1)]   # /16 inserted first (newest first)
    port, valid = oracle.fib_lookup(gpu.make_routes(routes),
                                    [ip("10.0.1.7"), ip("10.0.2.5"), ip("10.0.200.1")])
    assert list(valid) == [True, False, False] and port[0] == 2


def test_lpm_prefix_inside_stride_updates_single_child():
    """A route ending inside a 4-bit stride updates next[ip >> ip_width]
    only (:124-130): 10.0.64.0/18 lands on the child for bits 0001."""
    port, valid = oracle.fib_lookup(gpu.make_routes([R("10.0.64.0", 18, 5)]),
                                    [ip("10.0.64.1"), ip("10.0.16.1"), ip("10.0.31.255")])
    assert list(valid) == [False, True, True] and list(port[1:]) == [5, 5]


def test_lpm_deeper_update_keeps_longer_prefix():
    """fib_update_node replaces a valid leaf only if its depth <= the new one."""
    routes = [R("10.0.1.0", 24, 2), R("10.0.1.0", 20, 4)]   # /20 inserted first
    port, valid = oracle.fib_lookup(gpu.make_routes(routes), [ip("10.0.1.1")])
    assert valid[0] and port[0] == 2


# ---- drop_err_pkts ---------------------------------------------------------
def test_drops_non_ipv4_and_errors():
    v4 = frames_to([ip("10.0.0.9")]).reshape(1, 64)
    v6 = gen.ipv6_frames(1, 64, 1, 2, gen.PROTO_UDP, 1, 2)
    bad = v4.copy()
    bad[0, 14] = 0x44                                   # IHL 4 -> ip_err
    fr = np.concatenate([v4, v6, bad]).reshape(-1)
    routes = [R("10.0.0.0", 8, 1)]
    out, f2 = run_oracle(routes, fr)
    assert list(out) == [1, -1, 1]                      # errors pass without -e
    out, f3 = run_oracle(routes, fr, error_check=True)
    assert list(out) == [1, -1, -1]
    assert (f3.reshape(3, 64)[1:] == fr.reshape(3, 64)[1:]).all()   # dropped: untouched


def test_ttl_checksum_update_keeps_header_valid():
    routes = gen.c5_routes()
    fr = gen.c5_frames(5000, routes)
    for mode in (L.FWD_HASH, L.FWD_LPM):
        out, f2 = run_oracle(routes, fr, mode=mode)
        f2 = f2.reshape(-1, 64)
        assert (out >= 0).all()
        assert all(ip_hdr_ok(f) for f in f2[:500])
        assert (f2[:, 22] == 63).all()


# ---- GPU parity ------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode", [L.FWD_HASH, L.FWD_LPM])
@pytest.mark.parametrize("n", [1, 300, 1 << 16])
def test_gpu_c5_parity(gpu_ctx, mode, n):
    routes = gen.c5_routes()
    fr = gen.c5_frames(n, routes, seed=n)
    fw = gpu.Forwarder(gpu_ctx, routes, mode=mode)
    g_out, g_fr = fw.run(fr, 64, n, src_port=1)
    o_out, o_fr = run_oracle(routes, fr, mode=mode, sif=1)
    np.testing.assert_array_equal(g_out, o_out)
    np.testing.assert_array_equal(g_fr[:fr.nbytes], o_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("error_check", [False, True])
@pytest.mark.parametrize("stride", [64, 128, 256])
def test_gpu_generic_frames_parity(gpu_ctx, error_check, stride):
    """Non-plain frames (VLAN, IPv6, ARP, options, truncation, bad headers)
    through the generic parse path, several strides, both modes."""
    import rulesets
    frames = rulesets.mutate_corpus(3000, seed=stride, max_len=stride)
    buf = np.zeros((len(frames), stride), np.uint8)
    for k, f in enumerate(frames):
        buf[k, :min(len(f), stride)] = np.frombuffer(f[:stride], np.uint8)
    # route most of the address space the corpus uses
    routes = [R("10.0.0.0", 8, 1, 0), R("192.168.0.0", 16, 2, 1), R("10.10.10.0", 24, 3, 2)]
    for mode in (L.FWD_HASH, L.FWD_LPM):
        fw = gpu.Forwarder(gpu_ctx, routes, mode=mode)
        g_out, g_fr = fw.run(buf.reshape(-1), stride, len(frames), error_check=error_check)
        o_out, o_fr = run_oracle(routes, buf.reshape(-1), mode=mode, stride=stride,
                                 error_check=error_check)
        np.testing.assert_array_equal(g_out, o_out)
        np.testing.assert_array_equal(g_fr[:buf.nbytes], o_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [L.FWD_HASH, L.FWD_LPM])
def test_gpu_stride64_mixed_waves(gpu_ctx, mode):
    """The persistent stride-64 kernel with tiles of plain frames (register
    path, whole frames written back through the LDS transpose) next to
    tiles holding mutated frames (generic path per lane); ragged last tile."""
    import rulesets
    routes = gen.c5_routes()
    n = 64 * 91 + 17
    fr = gen.c5_frames(n, routes, seed=77).reshape(n, 64).copy()
    mut = rulesets.mutate_corpus(2000, seed=29, max_len=64)
    k = 0
    for t in range(1, (n + 63) // 64, 3):
        for j in range(t * 64, min(n, t * 64 + 64), 4):
            m = np.frombuffer(bytes(mut[k % len(mut)])[:64], np.uint8)
            fr[j, :] = 0
            fr[j, :len(m)] = m
            k += 1
    fr = fr.reshape(-1)
    for error_check in (False, True):
        fw = gpu.Forwarder(gpu_ctx, routes, mode=mode)
        g_out, g_fr = fw.run(fr, 64, n, src_port=2, error_check=error_check)
        o_out, o_fr = run_oracle(routes, fr, mode=mode, sif=2, error_check=error_check)
        np.testing.assert_array_equal(g_out, o_out)
        np.testing.assert_array_equal(g_fr[:fr.nbytes], o_fr)


@pytest.mark.gpu
def test_gpu_example_pcap(gpu_ctx):
    pk = [bytes.fromhex(h) for h in GOLDEN["pcap"]["perf_udp64"]]
    buf = np.zeros((len(pk), 64), np.uint8)
    for k, p in enumerate(pk):
        buf[k, :len(p)] = np.frombuffer(p, np.uint8)
    fw = gpu.Forwarder(gpu_ctx, [R("10.0.0.0", 24, 1)])
    out, fr = fw.run(buf.reshape(-1), 64, len(pk))
    assert (out == 1).all()
    o_out, o_fr = run_oracle([R("10.0.0.0", 24, 1)], buf.reshape(-1))
    np.testing.assert_array_equal(fr[:buf.nbytes], o_fr)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [L.FWD_HASH, L.FWD_LPM])
def test_gpu_c5_full_size(gpu_ctx, mode):
    """The C5 bench launch itself: 10 M distinct flows in one batch."""
    n = gen.C5_FLOWS
    routes = gen.c5_routes()
    fr = gen.c5_frames(n, routes)
    fw = gpu.Forwarder(gpu_ctx, routes, mode=mode)
    g_out, g_fr = fw.run(fr, 64, n)
    o_out, o_fr = run_oracle(routes, fr, mode=mode)
    np.testing.assert_array_equal(g_out, o_out)
    np.testing.assert_array_equal(g_fr[:fr.nbytes], o_fr)


def _random_routes(rng, nr):
    out = []
    for k in range(nr):
        d = int(rng.choice([8, 12, 16, 20, 23, 24, 28, 30, 31, 32, int(rng.integers(1, 33))]))
        a = int(rng.integers(0, 1 << 32))
        if rng.random() < 0.5:                      # half aligned, half with host bits
            a &= ((1 << d) - 1) << (32 - d)
        if rng.random() < 0.2:                      # overlap an earlier route
            a = (out[int(rng.integers(0, len(out)))][0] + int(rng.integers(0, 300))) % (1 << 32) \
                if out else a
        out.append(R(a, d, k % 4, k))
    return out


def _probe_dsts(rng, routes, n):
    d = []
    for a, dep, *_ in routes:
        n_h = 1 << (32 - dep)
        for off in (0, 1, n_h - 1, n_h, n_h + 1, -1, n_h // 2, 1 << 22, (1 << 22) - 1):
            d.append((a + off) % (1 << 32))
        m = ((1 << dep) - 1) << (32 - dep)
        d += [a & m, ((a & m) + n_h - 1) % (1 << 32)]
    d += [0, 0xFFFFFFFF] + list(rng.integers(0, 1 << 32, n))
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_gpu_hash_flow_cache_parity(gpu_ctx, seed):
    """Random route sets of every depth, half with host bits, overlapping and
    wrapping: the GPU's interval table vs the oracle's literal flow cache."""
    rng = np.random.default_rng(seed)
    routes = _random_routes(rng, int(rng.integers(1, 33)))
    dsts = _probe_dsts(rng, routes, 4000)
    fr = frames_to(dsts)
    fw = gpu.Forwarder(gpu_ctx, routes, mode=L.FWD_HASH)
    g_out, g_fr = fw.run(fr, 64, len(dsts), src_port=3)
    o_out, o_fr = run_oracle(routes, fr, sif=3)
    np.testing.assert_array_equal(g_out, o_out)
    np.testing.assert_array_equal(g_fr[:fr.nbytes], o_fr)


@pytest.mark.gpu
def test_gpu_hash_flow_cache_cases(gpu_ctx):
    cases = [([R("10.0.0.5", 24, 1)], ["10.0.0.5", "10.0.1.4", "10.0.0.4", "10.0.1.5"]),
             ([R("10.0.0.0", 24, 1), R(0, 32, 3)], ["10.0.0.9", "192.0.2.1", "0.0.0.0"]),
             ([R("10.0.0.0", 24, 1), R("9.255.255.0", 23, 2)],
              ["10.0.0.9", "10.0.1.200", "10.0.2.1", "9.255.255.0", "9.255.254.255"]),
             ([R("255.255.255.0", 16, 1)], ["255.255.255.9", "0.0.1.1", "0.0.254.255",
                                            "0.0.255.0"]),
             ([R("10.0.0.1", 8, 1)], ["10.0.0.1", "10.64.0.0", "10.64.0.1"])]
    for routes, qs in cases:
        fr = frames_to([ip(q) for q in qs])
        g_out, _ = gpu.Forwarder(gpu_ctx, routes, mode=L.FWD_HASH).run(fr, 64, len(qs),
                                                                       src_port=2)
        o_out, _ = run_oracle(routes, fr, sif=2)
        np.testing.assert_array_equal(g_out, o_out)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [64, 128])
def test_gpu_hash_more_than_128_intervals(gpu_ctx, stride):
    """32 disjoint /24 routes with host bits set: each adds its masked scan
    range and its unaligned warmed range, 4 points per route + 0 = 129
    interval starts, so the destinations of the last routes sit at interval
    index >= 128, past a 7-step binary search (fwd.hip search)."""
    routes = [R((ip("10.0.0.0") | (k << 8)) + 0x55, 24, k % 4, k) for k in range(32)]
    dsts = []
    for k in range(32):
        b = ip("10.0.0.0") | (k << 8)
        dsts += [b, b + 0x54, b + 0x55, b + 0xFF, b + 0x100 + 0x54, b + 0x100 + 0x55]
    dsts += [ip("10.0.32.0"), ip("10.0.31.255"), 0, 0xFFFFFFFF]
    fr = frames_to(dsts).reshape(-1, 64)
    if stride != 64:
        fr = np.concatenate([fr, np.zeros((len(dsts), stride - 64), np.uint8)], axis=1)
    fr = fr.reshape(-1)
    fw = gpu.Forwarder(gpu_ctx, routes, mode=L.FWD_HASH)
    g_out, g_fr = fw.run(fr, stride, len(dsts), src_port=3)
    o_out, o_fr = run_oracle(routes, fr, stride=stride, sif=3)
    np.testing.assert_array_equal(g_out, o_out)
    np.testing.assert_array_equal(g_fr[:fr.nbytes], o_fr)
    assert len(set(int(x) for x in o_out)) == 4
