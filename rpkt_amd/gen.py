"""Seeded synthetic batches for the BASELINE.json configs (host C++ generator).

Config ids follow BASELINE.json `configs` (1-based like SURVEY.md §8d):
  1 benches/rpkt: 1,000 x 64 B Ether/IPv4/UDP with the rpkt_build.rs header values
  2 1,048,576 x 64 B Ether/IPv4/UDP, stride 64, 1 % bad IPv4 checksum
  3 1,048,576 x 1500 B Ether/IPv4/TCP, stride 1500, random payload, 1 % bad IP / TCP
  4 8,388,608 IMIX 64/570/1500 at 7:4:1, 50/50 TCP/UDP, packed + u32 offsets
  5 4,194,304 x U[64,1518] B, 802.1Q or QinQ, IPv4 options, TCP options, packed
  6 fuzz: every parse status, frames of 0..300 B and 1000..1600 B, packed
  7 262,144 x 8000 B jumbo Ether/IPv4/{TCP,UDP} as mbuf chains: 2048-B data room,
    2176-B mempool slots (128-B headroom) in shuffled order (rpkt-dpdk
    examples/jumboframe_tx.rs:45; mempool_alloc(.., 2048 + 128, ..) in tests/pbuf.rs)
  8 chain fuzz: config-6 style frames up to 9000 B cut into 1..6 segments at random
    and header-boundary positions (empty segments included), odd slot alignments
  9 protocol mix for the layer walk: 1,048,576 frames drawn from the reference's
    captures, a third cut short and a third with random header bytes (make_mix)
 10 dual stack, 1,048,576 x 64 B, stride 64: IPv4/UDP or IPv6/UDP at 50/50, 1 % bad
    L4 (and IPv4 header) checksums; parsed with RPKT_F_IPV6
 11 dual stack, 1,048,576 x 1500 B, stride 1500: IPv4 or IPv6 with 0-3 extension
    headers (HopByHop, DestOptions, Routing types 0/2/4 with segments left or not,
    atomic Fragment, AH), TCP or UDP, a quarter 802.1Q-tagged, 1 % bad checksums
 12 dual-stack fuzz: every IPv4 and IPv6 status (truncation, bad payload_len, bad or
    short extension headers, non-atomic fragments, chains past RPKT_MAX_IP6_EXT,
    other upper-layer protocols, UDP checksum 0 over IPv6), packed
 13 tunnel mix, 1,048,576 x 1500 B, stride 1500: 40 % VXLAN (outer UDP checksum 0 or
    set), 36 % GTP-U G-PDUs with 0-3 extension headers of every type the reference
    parses, 24 % GRE v0 (checksum / key / sequence bits, IPv4 or transparent Ethernet
    inside); inner IPv4 or IPv6 (+ extension headers), TCP or UDP; 1 % bad sums at
    every level; parsed with rpkt_gpu_parse_tunnel_batch (RPKT_F_IPV6)
 14 tunnel fuzz: config 13's shapes at 40..1518 B with inner-frame faults, random
    tunnel-header bytes, GTP lengths / message types / extension bytes, GRE
    versions, truncations, packed
"""
import ctypes
import os

import numpy as np

from .build import GEN_LIB, build_gen

DEFAULT_N = {1: 1000, 2: 1 << 20, 3: 1 << 20, 4: 8 << 20, 5: 4 << 20, 6: 1 << 16,
             7: 1 << 18, 8: 1 << 15, 9: 1 << 20, 10: 1 << 20, 11: 1 << 20, 12: 1 << 16,
             13: 1 << 20, 14: 1 << 16}
DEFAULT_SEED = {1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 7, 8: 8, 9: 9, 10: 10, 11: 11, 12: 12,
                13: 13, 14: 14}
STRIDED = {1: 64, 2: 64, 3: 1500, 10: 64, 11: 1500, 13: 1500}
CHAINED = (7, 8)
DUAL_STACK = (10, 11, 12)                                 # generated with IPv6 frames
# config 2 = extract + IPv4 header sum; the dual-stack configs parse with RPKT_F_IPV6
FLAGS = {1: 3, 2: 1, 3: 3, 4: 3, 5: 3, 6: 3, 7: 3, 8: 3, 10: 11, 11: 11, 12: 11, 13: 11, 14: 11}
TUNNEL = (13, 14)                                         # tunnel mixes (VXLAN, GTP-U, GRE)
MBUF_ROOM, MBUF_HEADROOM = 2048, 128                      # RTE_MBUF_DEFAULT_DATAROOM, headroom
# header-boundary cut positions for the chain fuzz (Ether 14, tags 18/22, IPv4 +20..60, L4 +8/20)
FUZZ_CUTS = (0, 1, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 26, 30, 33, 34, 35, 38,
             42, 46, 54, 58, 62, 66, 74, 82, 94, 102, 118, 128, 142)
# ... and for dual-stack configs the IPv6 ones (header 54/58/62 + 40, extension headers
# of 8..24 B, the L4 header after them)
FUZZ_CUTS6 = FUZZ_CUTS + (20, 53, 55, 56, 60, 70, 78, 86, 94, 96, 98, 102, 110, 126, 134, 150)

_lib = None


def lib():
    global _lib
    if _lib is None:
        build_gen()   # no-op unless the source is newer than the library
        L = ctypes.CDLL(GEN_LIB)
        L.rpkt_gen_lengths.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_void_p]
        L.rpkt_gen_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.rpkt_gen_fill.restype = ctypes.c_int
        L.rpkt_gen_scatter.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p,
                                                               ctypes.c_int]
        L.rpkt_gen_scatter.restype = ctypes.c_int
        _lib = L
    return _lib


class HostBatch:
    """A generated batch in host memory: frames (uint8) + layout."""

    def __init__(self, config, n, seed, frames, offsets, stride, frame_len):
        self.config, self.n, self.seed = config, n, seed
        self.frames, self.offsets = frames, offsets
        self.stride, self.frame_len = stride, frame_len

    @property
    def frame_bytes(self):
        return int(self.offsets[-1]) if self.offsets is not None else self.n * self.stride

    def lens(self):
        if self.offsets is not None:
            return np.diff(self.offsets.astype(np.int64))
        return np.full(self.n, self.frame_len or self.stride, dtype=np.int64)


def make_batch(config, n=None, seed=None, threads=None, packed=None, first=0):
    """Generate frames [first, first + n) of config `config`.  packed=None uses the
    config's own layout (strided for 1-3); packed frames start at arbitrary byte
    offsets.  A shard generated with `first` equals that slice of the full batch."""
    n = DEFAULT_N[config] if n is None else n
    seed = DEFAULT_SEED[config] if seed is None else seed
    threads = threads or min(16, os.cpu_count() or 1)
    lens = np.zeros(max(n, 1), dtype=np.uint32)
    lib().rpkt_gen_lengths(config, seed, first, n, lens.ctypes.data)
    lens = lens[:n]
    use_packed = (config not in STRIDED) if packed is None else packed
    if not use_packed:
        stride = STRIDED[config]
        frames = np.zeros(n * stride, dtype=np.uint8)
        lib().rpkt_gen_fill(config, seed, first, n, lens.ctypes.data, None, stride,
                            frames.ctypes.data, threads)
        return HostBatch(config, n, seed, frames, None, stride, 0)
    slots = lens.astype(np.uint64)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(slots, out=offsets[1:])
    total = int(offsets[-1])
    if total >= (1 << 32) - 256:
        raise ValueError("batch of %d bytes exceeds the 4 GiB descriptor range" % total)
    offsets32 = offsets.astype(np.uint32)
    frames = np.zeros(total + 16, dtype=np.uint8)
    lib().rpkt_gen_fill(config, seed, first, n, lens.ctypes.data, offsets32.ctypes.data, 0,
                        frames.ctypes.data, threads)
    return HostBatch(config, n, seed, frames[:total], offsets32, 0, 0)


class HostChains:
    """Frames as mbuf chains in host memory: an arena `buf` holding every segment,
    `segs` = (offset, length) u32 pairs, chain p = segments chain_first[p] ..
    chain_first[p+1]-1 (the rpkt_chains_t layout of include/rpkt_gpu.h)."""

    def __init__(self, config, n, seed, buf, segs, chain_first, pkt_lens):
        self.config, self.n, self.seed = config, n, seed
        self.buf, self.segs, self.chain_first = buf, segs, chain_first
        self.pkt_lens = pkt_lens

    @property
    def n_segs(self):
        return int(self.segs.shape[0])

    def lens(self):
        return self.pkt_lens.astype(np.int64)

    def frame(self, p):
        """Chain p's bytes, concatenated (host-side view for tests)."""
        a, b = int(self.chain_first[p]), int(self.chain_first[p + 1])
        return b"".join(self.buf[o:o + l].tobytes() for o, l in self.segs[a:b])


def _mbuf_cuts(lens, room):
    nseg = np.maximum((lens + room - 1) // room, 1)
    seg_len = np.full(int(nseg.sum()), room, dtype=np.int64)
    last = np.cumsum(nseg) - 1
    seg_len[last] = lens - (nseg - 1) * room
    return nseg, seg_len


def _fuzz_cuts(lens, rng, cuts_at=FUZZ_CUTS):
    nsegs, seg_lens = [], []
    for L in lens.tolist():
        k = int(rng.integers(1, 7))
        cuts = rng.integers(0, L + 1, size=k - 1).tolist()
        if k > 1 and rng.integers(0, 2):
            cuts[0] = min(cuts_at[int(rng.integers(0, len(cuts_at)))], L)
        cuts = sorted(cuts)
        edges = [0] + cuts + [L]
        nsegs.append(k)
        seg_lens.extend(edges[i + 1] - edges[i] for i in range(k))
    return np.array(nsegs, dtype=np.int64), np.array(seg_lens, dtype=np.int64)


def make_chains(config, n=None, seed=None, threads=None, layout=None):
    """Generate frames of `config` and lay them out as mbuf chains.  layout "mbuf":
    2048-B segments in 2176-B slots (128-B headroom), slots in a seeded shuffled
    order; "fuzz": random cuts (see FUZZ_CUTS), odd slot offsets."""
    n = DEFAULT_N[config] if n is None else n
    seed = DEFAULT_SEED[config] if seed is None else seed
    threads = threads or min(16, os.cpu_count() or 1)
    layout = layout or ("mbuf" if config == 7 else "fuzz")
    hb = make_batch(config, n, seed, threads, packed=True)
    lens = hb.lens()
    rng = np.random.default_rng(seed * 7919 + 17)
    if layout == "mbuf":
        nseg, seg_len = _mbuf_cuts(lens, MBUF_ROOM)
        slot_bytes, pad = MBUF_ROOM + MBUF_HEADROOM, np.full(seg_len.size, MBUF_HEADROOM)
    else:
        nseg, seg_len = _fuzz_cuts(lens, rng, FUZZ_CUTS6 if config in DUAL_STACK else FUZZ_CUTS)
        slot_bytes, pad = 0, rng.integers(0, 64, size=seg_len.size)
    n_segs = seg_len.size
    chain_first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nseg, out=chain_first[1:])
    # source offset of each segment inside the packed frame buffer
    frame_base = np.repeat(hb.offsets[:-1].astype(np.int64), nseg)
    cum = np.cumsum(seg_len) - seg_len
    within = cum - cum[np.repeat(chain_first[:-1], nseg)]
    src_off = (frame_base + within).astype(np.uint64)
    slot = rng.permutation(n_segs).astype(np.int64)
    if slot_bytes:                                   # fixed mempool slots
        dst_off = (slot * slot_bytes + pad).astype(np.uint64)
        total = n_segs * slot_bytes
    else:                                            # packed in shuffled order, odd gaps
        room = seg_len + pad
        start = np.zeros(n_segs, dtype=np.int64)
        start[slot] = np.cumsum(room[slot]) - room[slot]
        dst_off = (start + pad).astype(np.uint64)
        total = int(room.sum()) + 64
    if total >= (1 << 32) - 256:
        raise ValueError("chain arena of %d bytes exceeds the 4 GiB descriptor range" % total)
    buf = np.zeros(total, dtype=np.uint8)
    sl32 = seg_len.astype(np.uint32)
    lib().rpkt_gen_scatter(hb.frames.ctypes.data, src_off.ctypes.data, dst_off.ctypes.data,
                           sl32.ctypes.data, n_segs, buf.ctypes.data, threads)
    segs = np.stack([dst_off.astype(np.uint32), sl32], axis=1)
    return HostChains(config, n, seed, buf, np.ascontiguousarray(segs),
                      chain_first.astype(np.uint32), lens.astype(np.uint32))


def fixture_frames(root=None):
    """The reference's captures (tests/golden/packets/*.dat), sorted by name."""
    d = root or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "tests", "golden", "packets")
    out = []
    for fn in sorted(os.listdir(d)):
        with open(os.path.join(d, fn)) as fh:
            s = fh.read().strip()
        out.append(bytes(int(s[i:i + 2], 16) for i in range(0, len(s), 2)))
    return out


def make_mix(n=1 << 20, seed=9, fuzz=True):
    """Config 9 (the protocol-walk workload): frames drawn from the reference's 53
    captures (ARP, 802.3/LLC/STP, QinQ, MPLS, PPPoE, GRE v0/v1, VXLAN, GTPv1/v2,
    IPv6 extension headers, IPv4 options, TCP, UDP), packed.  With `fuzz`, a third
    of them are cut at a random length and a third get 1-3 random header bytes."""
    base = fixture_frames()
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(base), n)
    lens = np.array([len(b) for b in base], dtype=np.int64)[pick]
    mode = rng.integers(0, 3, n) if fuzz else np.zeros(n, dtype=np.int64)
    cut = np.where(mode == 1, (rng.random(n) * (lens + 1)).astype(np.int64), lens)
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(cut, out=offsets[1:])
    frames = np.zeros(int(offsets[-1]) + 16, dtype=np.uint8)
    pool = [np.frombuffer(b, dtype=np.uint8) for b in base]
    order = np.argsort(pick, kind="stable")
    for k in range(len(base)):                        # vectorised copy per capture
        idx = order[np.searchsorted(pick[order], k):np.searchsorted(pick[order], k + 1)]
        if not idx.size:
            continue
        L = len(pool[k])
        rows = np.minimum(cut[idx], L)
        tgt = offsets[idx][:, None] + np.arange(L)[None, :]
        mask = np.arange(L)[None, :] < rows[:, None]
        frames[tgt[mask]] = np.broadcast_to(pool[k], (idx.size, L))[mask]
    flip = np.nonzero(mode == 2)[0]
    nb = rng.integers(1, 4, flip.size)
    for j in range(3):
        sel = flip[nb > j]
        pos = offsets[sel] + (rng.random(sel.size) * np.minimum(cut[sel], 80)).astype(np.int64)
        ok = cut[sel] > 0
        frames[pos[ok]] = rng.integers(0, 256, ok.sum(), dtype=np.uint8)
    return HostBatch(9, n, seed, frames[:int(offsets[-1])], offsets.astype(np.uint32), 0, 0)
