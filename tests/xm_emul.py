"""Host emulation of the lean descriptor kernel's classification stage
(classify_gf.hip: the hit map over the compiled TBL_XMASK region and the
match_pmr_cos walk on it), reading the table image that odpg_rules_compile
emits (odpg_internal.h: dtable_hdr_t, XM_HDR_WORDS, XM_GROUP_WORDS,
xm_layout_t). Parse results come from the oracle's metadata, so a CPU test
can check the compiler's region (rule bits, AND-chain groups, collision-free
slot tables, per-bit destinations) against the oracle's classification
without a GPU. Test infrastructure only."""
import struct

import numpy as np

HDR_FIELDS = ("num_cos default_cos error_cos flags num_pmr num_terms cos_off pmr_off term_off "
              "slot_off simple_off run_off num_runs hgroup_off num_hgroups hent_off num_hent "
              "cinfo_off pinfo_off slot_mask wgroup_off num_wgroups went_off num_went "
              "mgroup_off num_mgroups ment_off num_ment pinfo2_off cgroup_off num_cgroups "
              "cent_off num_cent pinfo3_off pinfo4_off def_cgmask xcos_off xlist_off num_xlist "
              "num_xwords xm_off num_xment xm_slot_bytes num_xflat blob_bytes xm_nw xm_nbits "
              "xm_ngroups xm_kx").split()
TBL_XMASK = 0x1000
XM_HDR_WORDS = 16
XM_GROUP_WORDS = 16
SLOT_VLANX, SLOT_L3, SLOT_L4, SLOT_LEN = 5, 6, 16, 18
IFL_VLAN_QINQ = 12
FL_ERROR_MASK = 0xFE000000
COS_NONE, COS_LOOP = 0xFFFF, 0xFFFD


def xm_layout(nw, num_xment, slot_bytes, num_cos, nbits, num_xflat):
    """odpg_internal.h xm_layout_of (word offsets)"""
    nx = (num_xment + 4) & ~3     # at least one zero entry (a miss's bit map)
    L = {"masks": 0}
    if nw == 2:                   # entries interleaved {map0, map1, value, 0}
        L.update(estride=4, values=2, vstride=4, slots=4 * nx)
    else:
        L.update(estride=nw, values=nx * nw, vstride=1)
        L["slots"] = L["values"] + nx
    L["xci"] = L["slots"] + ((slot_bytes + 15) & ~15) // 4
    L["xpd"] = L["xci"] + 2 * ((num_cos + 1) & ~1)
    L["xflat"] = L["xpd"] + 4 * nbits
    L["lds_words"] = L["xflat"] + 8 * num_xflat
    return L


class XmTable:
    def __init__(self, img):
        hdr_bytes = struct.unpack_from("<4I", img, 0)[2]
        vals = struct.unpack_from("<%dI" % len(HDR_FIELDS), img, 16)
        self.h = h = dict(zip(HDR_FIELDS, vals))
        for k in ("default_cos", "error_cos"):
            h[k] = struct.unpack("<i", struct.pack("<I", h[k]))[0]
        assert 16 + 4 * len(HDR_FIELDS) <= 16 + hdr_bytes
        blob = img[16 + hdr_bytes:]
        self.flags = h["flags"]
        if not self.flags & TBL_XMASK:
            return
        w = np.frombuffer(blob, np.uint32, offset=h["xm_off"])
        self.nw, self.nbits, self.ngroups, nx, _, nxf = (int(x) for x in w[:6])
        sb = h["xm_slot_bytes"]
        assert (self.nw, self.nbits, self.ngroups) == (h["xm_nw"], h["xm_nbits"], h["xm_ngroups"])
        assert (nx, sb, nxf) == (h["num_xment"], 0, h["num_xflat"])
        self.chain = self._big(w[8:16])
        # group order: [0, n0) plain unguarded, [n0, n1) plain guarded,
        # [n1, n2) chain unguarded, [n2, ngroups) chain guarded
        self.gcut = (int(w[7]) & 0xFF, (int(w[7]) >> 8) & 0xFF, (int(w[7]) >> 16) & 0xFF)
        self.ngor = self.gcut[1]
        self.kpos = [(int(w[4]) >> (8 * k)) & 0xFF for k in range(3)]
        self.kx = (int(w[4]) >> 24) & 1
        assert self.kx == h["xm_kx"]
        self.groups = w[XM_HDR_WORDS:XM_HDR_WORDS + XM_GROUP_WORDS * self.ngroups] \
            .reshape(-1, XM_GROUP_WORDS).astype(np.uint64)
        base = XM_HDR_WORDS + XM_GROUP_WORDS * self.ngroups
        ncos = h["num_cos"]
        L = xm_layout(self.nw, nx, sb, ncos, self.nbits, nxf)
        lds = w[base:base + L["lds_words"]]
        ent = lds[:L["slots"]]
        es, vs = L["estride"], L["vstride"]
        self.masks = np.stack([ent[L["masks"] + w::es][:nx] for w in range(self.nw)], 1) \
            if nx else None
        self.values = ent[L["values"]::vs][:nx]
        self.xci = lds[L["xci"]:L["xci"] + 2 * ncos].reshape(-1, 2)
        self.xpd = lds[L["xpd"]:L["xpd"] + 4 * self.nbits].reshape(-1, 4)
        self.xflat = lds[L["xflat"]:L["xflat"] + 8 * nxf].reshape(-1, 8)
        self.xfc = w[base + L["lds_words"]:base + L["lds_words"] + ncos]
        cos = np.frombuffer(blob, np.uint8, 12 * ncos, h["cos_off"]).reshape(-1, 12)
        self.cos_valid = cos[:, 10].astype(bool)
        self.cos_nrule = cos[:, 4].astype(np.uint32) | (cos[:, 5].astype(np.uint32) << 8)

    def _big(self, words):
        x = 0
        for k in range(self.nw):
            x |= int(words[k]) << (32 * k)
        return x

    def hit_map(self, frame, meta):
        """the packet's hit map (kernel `keys`), as one integer"""
        l2, l3, l4 = int(meta["l2_offset"]), int(meta["l3_offset"]), int(meta["l4_offset"])
        inf = int(meta["input_flags"]) & 0xFFFFFFFF
        n = len(frame)
        buf = bytes(frame) + bytes(96)
        vlanx = 14 + (4 if (int(meta["input_flags"]) >> IFL_VLAN_QINQ) & 1 else 0)

        def rd32(pos):
            if pos >= n:
                return 0
            b = bytearray(buf[pos:pos + 4])
            for k in range(4):
                if pos + k >= n:
                    b[k] = 0
            return struct.unpack("<I", bytes(b))[0]

        def key(slot):
            if slot < SLOT_VLANX:
                return rd32(l2 + 4 * slot)
            if slot == SLOT_VLANX:
                return rd32(vlanx)
            if slot < SLOT_L4:
                return rd32(l3 + 4 * (slot - SLOT_L3))
            if slot < SLOT_LEN:
                return rd32(l4 + 4 * (slot - SLOT_L4))
            return n

        full = (1 << (32 * self.nw)) - 1
        hm = self.chain
        # the kernel's 16-word key vector (classify_gf.hip): slot s < 16 at
        # word s, slots 16..18 at the words xhdr[4] names (unless kx)
        kvec = {}
        if not self.kx:
            for s in range(16):
                kvec[s] = key(s)
            assert len(set(self.kpos)) == 3 and max(self.kpos) < 16, self.kpos
            for k in range(3):
                assert not any(int(g[2]) >> 8 == self.kpos[k] for g in self.groups)
                kvec[self.kpos[k]] = key(16 + k)
        for gi, g in enumerate(self.groups):
            mul, shf, kw, eb, gthr, req, gmask, l3mask = (int(x) for x in g[:8])
            slot = kw >> 8
            guarded = gthr != 0
            assert guarded == (self.gcut[0] <= gi < self.gcut[1] or gi >= self.gcut[2])
            kword = key(slot) if self.kx else kvec[kw & 15]
            # direct entries: slot (value * mul) >> shift; an empty slot's
            # map is zero, so a probe landing there acts as a miss
            h = 0
            if (inf & req) == req and n >= (l3 & l3mask) + gthr:
                kv = kword & gmask
                e = eb + (((kv * mul) & 0xFFFFFFFF) >> shf)
                if int(self.values[e]) == kv:
                    h = self._big(self.masks[e])
            if gi >= self.ngor:
                na = self._big(g[8:16])
                hm = ((hm & (h | na)) | (h & ~self.chain)) & full
            else:
                hm |= h
        return hm, key, l3, n, inf

    def walk(self, frame, meta):
        """(cos, mark, matched) of a packet the oracle parsed without error
        (cls_select_cos's default-CoS branch + match_pmr_cos)"""
        hm, key, l3, n, inf = self.hit_map(frame, meta)
        dc = self.h["default_cos"]
        if dc < 0 or not self.cos_valid[dc]:
            return (COS_NONE if dc < 0 else dc), 0, False
        cos, mark, any_match, steps = dc, 0, False, 0
        if self.cos_nrule[dc] == 0:
            return cos, 0, False
        crs = int(self.xci[cos][0])
        cxf = int(self.xfc[cos]) if len(self.xflat) else 0
        while True:
            lo, cnt = crs & 0xFFFF, crs >> 16
            x = (hm >> lo) & ((1 << cnt) - 1)
            best = (x & -x).bit_length() - 1 + lo if x else None
            j, jend, acc = cxf & 0xFFFF, (cxf & 0xFFFF) + (cxf >> 16), True
            while j < jend:
                r, q = self.xflat[j][:4], self.xflat[j][4:]
                if best is not None and int(q[0]) >= best:
                    break
                rx, ry, rz, rw = (int(v) for v in r)
                acc = acc and (inf & rx) == rx and \
                    (not (rw >> 31) or n > ((0 if (rw >> 30) & 1 else l3) + ((rw >> 8) & 0xFFFF))) \
                    and (key(rw & 0xFF) & ry) == rz
                if int(q[1]):
                    if acc:
                        best = int(q[0])
                        break
                    acc = True
                elif not acc:
                    j = int(q[2])
                    acc = True
                j += 1
            if best is None:
                return cos, mark, any_match
            pd = self.xpd[best]
            cos, mark, crs, cxf = int(pd[0]) & 0xFFFF, int(pd[0]) >> 16, int(pd[1]), int(pd[2])
            any_match = True
            steps += 1
            if steps >= self.h["num_cos"]:
                return COS_LOOP, mark, any_match
            if crs >> 16 == 0:
                return cos, mark, any_match
