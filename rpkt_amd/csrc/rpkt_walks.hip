// rpkt_walks.hip — per-frame walks over a batch: the IPv4/TCP option iterators and the
// protocol-layer walk driven by the pktfmt-derived table.
#include "rpkt_common.h"
#include "rpkt_opts.h"
#include "rpkt_proto_table.h"

#include <map>
#include <mutex>

namespace {

// ---- option iterators: TcpOptionsIter / Ipv4OptionsIter over a parsed batch ----
// One wave per 64 frames.  The records give each frame's option slices; only the
// 16-B chunks that overlap a slice are loaded (frames without options cost their
// record read and the 64-B output only).  Lane-per-frame walk over LDS bytes with
// the per-type parse rules of the generated option views (rpkt_opts.h;
// oracle/rpkt_oracle_opts.c cites them); results staged through LDS and stored as
// 4 KiB of coalesced rows.  (rpkt_gpu_parse_options_batch runs the same walks inside
// the parse, on the header window it already holds.)
constexpr int kOptChunks = 8;                  // 128 B from the 16-B phase of the first
constexpr int kOptSlot = 132;                  // option byte: both slices span at most
                                               // ihl4 + 40 <= 100 B, + 15 of phase
struct OptScratch {
    uint8_t win[kWave * kOptSlot];             // 8448 B (stride 33 dwords: conflict-free),
};                                             // so four blocks (16 waves) fit a CU
static_assert(kWave * 21 * 4 <= kWave * kOptSlot, "record stage fits the option window");

// C16: the records are rpkt_rec16_t (16 B: one coalesced dwordx4 per lane) instead of
// rpkt_rec_t (80 B, staged through LDS); the walks need status, IP protocol, l3, l4 and
// the TCP data offset (payload_off - l4 for a TCP frame that parsed OK), which both hold.
template <bool C16>
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void options_kernel(const uint8_t* __restrict__ frames, uint32_t fb,
                    const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                    uint32_t n, const void* __restrict__ recs_any, rpkt_opts_t* __restrict__ opts) {
    __shared__ __attribute__((aligned(16))) OptScratch scratch[kWavesPerBlock];
    // the option-type rules of both iterators (a per-lane type: LDS, not a switch)
    __shared__ uint8_t rules[512];
    opt_rules_fill(rules);
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    OptScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    const Frame fr = spans.get(i);

    // records of the tile (coalesced): status, IP protocol, l3 / l4 offsets, TCP doff
    uint32_t status, proto, l3, l4, doff4;
    uint32_t nh0 = 256u;                                 // IPv6: the first next_header
    bool is6;                                            // an IPv6 record (RPKT_F_IPV6)
    if constexpr (C16) {
        const u32x4* in = reinterpret_cast<const u32x4*>(recs_any);
        const u32x4 r = i < n ? __builtin_nontemporal_load(&in[i]) : u32x4{0u, 0u, 0u, 0u};
        status = r.x & 0xffu;                            // rpkt_rec16_t, include/rpkt_gpu.h
        proto = (r.x >> 16) & 0xffu;
        l3 = r.y & 0xffffu;
        l4 = r.y >> 16;
        doff4 = (r.z & 0xffffu) - l4;                    // payload_off - l4: TCP, status OK
        is6 = ((r.x >> 24) & 4u) != 0u;                  // verdict bit 2
    } else {
        const rpkt_rec_t* recs = reinterpret_cast<const rpkt_rec_t*>(recs_any);
        const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
        const u32x4* in = reinterpret_cast<const u32x4*>(recs + p0);
        u32x4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t c = k * kWave + lane;
            // records and option bytes are read once: non-temporal loads (-2.6 %)
            v[k] = (c / 5 < nrec) ? __builtin_nontemporal_load(&in[c]) : u32x4{0u, 0u, 0u, 0u};
        }
        uint32_t* st = reinterpret_cast<uint32_t*>(W.win);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t c = k * kWave + lane, r = c / 5, pc = c % 5;
            uint32_t* d = st + r * 21 + pc * 4;
            d[0] = v[k].x;
            d[1] = v[k].y;
            d[2] = v[k].z;
            d[3] = v[k].w;
        }
        wave_sync();
        const uint32_t w0 = st[lane * 21 + 0], w8 = st[lane * 21 + 8];
        const uint32_t w14 = st[lane * 21 + 14], w16 = st[lane * 21 + 16];
        const uint32_t w5 = st[lane * 21 + 5], w7 = st[lane * 21 + 7];
        wave_sync();
        status = w0 & 0xffu;
        // the dispatch ethertype: the outer one, or the last VLAN tag's
        const uint32_t nv = (w0 >> 8) & 0xffu;
        const uint32_t et = nv == 0u ? w0 >> 16 : (nv == 1u ? w5 & 0xffffu : w5 >> 16);
        is6 = et == 0x86ddu && status != RPKT_S_ETH_SHORT && status != RPKT_S_VLAN_SHORT &&
              status != RPKT_S_NOT_IPV4;
        proto = (w8 >> 8) & 0xffu;
        l3 = w16 & 0xffffu;
        l4 = w16 >> 16;
        doff4 = ((w14 >> 12) & 0xfu) * 4u;
        nh0 = (w7 >> 16) & 0xffu;                        // ip6_next_header, record byte 30
    }
    OptSlices S = opt_slices(status, proto, l3, l4, doff4, is6);
    // the window: the option slices; for an IPv6 record, the extension chain [l3 + 40, l4)
    // (and the TCP slice after it) when they fit, so that Ipv6OptionsIter reads LDS
    // instead of memory (ip6_walk, OptDw).  The chain's first next_header (frame byte
    // l3 + 6) comes from the 80-B record, or, with compact records, from a dword load
    // issued with the window's.  (Round 5 started the window at l3 + 4 for that byte: 10 %
    // of config 11's chains then missed the window, and 92 % of its waves waited on
    // dependent global reads; from l3 + 40, 0.8 % and 18 %.)
    if constexpr (C16) {
        if (S.ip6 && S.l4 > S.l3 + 40u) nh0 = (gdword(rs, fb, fr.off + S.l3 + 4u) >> 16) & 0xffu;
    }
    S.nh0 = nh0;
    uint32_t need_lo = S.need_lo, need_hi = S.need_hi;
    bool need = S.need;
    if (S.ip6 && S.l4 > S.l3 + 40u) {
        const uint32_t lo6 = S.l3 + 40u, hi6 = S.need && S.need_hi > S.l4 ? S.need_hi : S.l4;
        if (hi6 - lo6 + ((fr.off + lo6) & 15u) + 16u <= (uint32_t)(kOptChunks * 16)) {
            need_lo = lo6;
            need_hi = hi6;
            need = true;
        }
    }

    // window chunks that overlap the option bytes -> LDS slots
    {
        u32x4 d[kOptChunks];
        uint32_t addr[kOptChunks];
        uint32_t fix = 0;
#pragma unroll
        for (int k = 0; k < kOptChunks; ++k) {
            const int c = k * kWave + lane;
            const int q = c / kOptChunks, j = c % kOptChunks;
            const uint32_t lo = (uint32_t)__shfl((int)(need ? fr.off + need_lo : 0u), q, kWave);
            const uint32_t hi = (uint32_t)__shfl((int)(need ? fr.off + need_hi : 0u), q, kWave);
            const uint32_t a = (lo & ~15u) + 16u * j;
            addr[k] = a < hi ? a : fb;
            fix |= (uint32_t)straddles(addr[k], fb) << k;
        }
#pragma unroll
        for (int k = 0; k < kOptChunks; ++k) d[k] = load16_fast<2>(rs, addr[k]);
#pragma unroll
        for (int k = 0; k < kOptChunks; ++k) {
            const int c = k * kWave + lane;
            u32x4 v = d[k];
            if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
            uint32_t* dst = reinterpret_cast<uint32_t*>(&W.win[(c / kOptChunks) * kOptSlot +
                                                              (c % kOptChunks) * 16]);
            dst[0] = v.x;
            dst[1] = v.y;
            dst[2] = v.z;
            dst[3] = v.w;
        }
    }
    wave_sync();

    // the frame bytes the slot holds: the loaded chunks from the 16-B phase of need_lo
    const uint32_t phw = (fr.off + need_lo) & 15u;
    const uint32_t wspan = (need_hi - need_lo + phw + 15u) & ~15u;
    const OptDw d6{&W.win[lane * kOptSlot], phw - need_lo, need ? need_lo - phw : 0u,
                   need ? need_lo - phw + (wspan < kOptChunks * 16u ? wspan : kOptChunks * 16u) : 0u,
                   fr.off, fb, rs};
#if RPKT_OPT_PAIRED
    walk_options_paired(W.win, lane, lane * kOptSlot + (phw - need_lo), S, rules, opts, p0, n, d6);
#else
    const OptWin s{&W.win[lane * kOptSlot], phw - need_lo};
    uint32_t o[16];
    walk_options(s, S, rules, o);
    store_opts(reinterpret_cast<uint32_t*>(W.win), lane, o, opts, p0, n, S, d6);
#endif
}

// ---- protocol layer walk: the pktfmt-derived table interpreted per frame ----
// kProtos / kGroups / kMembers (rpkt_proto_table.h, generated by tools/pktfmt_table.py
// from the reference's pktfmt specs) hold, per protocol, exactly what its generated
// parse / payload / group_parse are functions of; walk_group interprets them with the
// pktfmt codegen rules (pktfmt/src/codegen/parse.rs:138-244, payload.rs:23-87).
// One lane per frame over a 128-B LDS slot.  128 B keeps the block under 40 KB of LDS,
// so four blocks (16 waves) fit a CU.  A header that runs past the slot (deep tunnel
// stacks) refills that lane's slot from the header on, with eight 16-B loads in flight
// at once.
//
// Lanes walk different protocols, so a step is written as straight-line selects over
// table values rather than branches on them (a divergent switch costs the wave the
// union of its cases plus exec-mask bookkeeping for each), and the step's LDS reads
// form a chain of two round trips: the group record (64 B: the group word, its first
// two member tests and its first member's protocol, whose next-layer rule is folded
// in), then the next header's first 20 bytes.  Rarer needs (members past the second,
// the byte-keyed lookup groups, a member other than the first) are read under
// wave-uniform branches, taken only by waves that have a lane needing them.
#ifndef RPKT_LAY_CHUNKS
#define RPKT_LAY_CHUNKS 8
#endif
// Development switches (same-process A/B in DESIGN.md, layers_kernel; all off in the
// product build)
#ifndef RPKT_LAY_STAGE_REC
#define RPKT_LAY_STAGE_REC 0     // 1: records stored through the slots, 64 B per 4 lanes
#endif
#ifndef RPKT_LAY_COOP_FILL
#define RPKT_LAY_COOP_FILL 0     // 1: ... and the new frames' windows loaded cooperatively
#endif
#ifndef RPKT_LAY_HALF
#define RPKT_LAY_HALF 0          // 1: refills fetch the slot's first half, the rest on demand
#endif
// A wave takes new frames once RPKT_LAY_TAKE_MIN of its walks ended (or none is still
// walking); ended lanes wait until then.  Same process, byte-identical, vs taking at every
// ended walk (1): capture mix 58.1 -> 57.2 us, config 2 43.2 -> 43.1, config 5 313.3 ->
// 304.5 (16); 8 and 32 in between (profiles/r05_lay_take/).
#ifndef RPKT_LAY_TAKE_MIN
#define RPKT_LAY_TAKE_MIN 16
#endif
#ifndef RPKT_LAY_STAGE_MIN
#define RPKT_LAY_STAGE_MIN 16    // ... when at least this many walks of the wave end together
#endif

constexpr int kLayChunks = RPKT_LAY_CHUNKS;    // 128 B slot from a 16-B boundary
constexpr int kLayFill = RPKT_LAY_HALF ? kLayChunks / 2 : kLayChunks;   // chunks per refill
constexpr int kLaySlot = 16 * kLayChunks + 4;  // 33 dwords: conflict-free lanes
static_assert((kLaySlot / 4) % 2 == 1, "odd dword stride");
struct LayScratch {
    uint8_t win[kWave * kLaySlot];             // 8448 B
#if RPKT_LAY_STAGE_REC
    uint32_t emap[kWave];                      // lanes whose walk ended, by rank
#endif
};

struct LayerWin {
    uint8_t* base;                             // the lane's slot
    uint32_t bias;                             // frame byte x at base[x + bias] (mod 2^32)
    uint32_t avail;                            // frame bytes at or past the cursor and
                                               // below avail are in the slot
    uint32_t off, fb;                          // frame's absolute offset; buffer bytes
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ uint32_t at(uint32_t x) const {
        return x < avail ? (uint32_t)base[x + bias] : gbyte(rs, off + x);
    }
    // frame bytes x..x+3 as a little-endian dword: two aligned LDS dwords and a byte
    // align when all four are in the slot, else byte by byte
    __device__ __forceinline__ uint32_t dw(uint32_t x) const {
        if (x + 4u <= avail) {
            const uint32_t y = x + bias, a = y & ~3u;
            return align_bytes(lds32(base, a + 4), lds32(base, a), y & 3u);
        }
        return at(x) | (at(x + 1) << 8) | (at(x + 2) << 16) | (at(x + 3) << 24);
    }
    // big-endian bit field (pktfmt bit order) of `bits` <= 32 at bit offset `ob` of x
    // (cond and length fields are at most 16 bits wide: 4 bytes always cover them)
    __device__ __forceinline__ uint32_t field(uint32_t x, uint32_t ob, uint32_t bits) const {
        const uint32_t v = bswap32(dw(x + (ob >> 3)));
        return (v << (ob & 7u)) >> (32u - bits);
    }
    __device__ __forceinline__ void refill(uint32_t s);
    __device__ __forceinline__ void refill_hi();
};

// Rare paths of the walk, kept out of line so the loop's hot path stays compact in the
// instruction cache: a 16-B chunk straddling the buffer end, a field past the header
// prefix.
__device__ __attribute__((noinline)) u32x4 lay_edge16(__amdgpu_buffer_rsrc_t rs, uint32_t a,
                                                      uint32_t fb) {
    return load16(rs, a, fb);
}
// The slot holds buffer bytes from a 16-B boundary a (frame byte -bias): refill(s) loads
// its first kLayFill chunks from the boundary at or below frame byte s, refill_hi() the
// rest from a + 16 kLayFill (RPKT_LAY_HALF: a refill fetches the 64 B most walks stay in,
// and only a lane whose next header crosses them fetches the second half).  Bytes past
// the buffer read as 0, as gbyte's; at most one chunk straddles its end.
template <int K0, int K1>
__device__ __forceinline__ void lay_load(uint8_t* base, __amdgpu_buffer_rsrc_t rs, uint32_t a,
                                         uint32_t fb) {
    u32x4 d[K1 - K0];
#pragma unroll
    for (int k = K0; k < K1; ++k) d[k - K0] = load16_fast(rs, a + 16u * k);
    uint32_t* w = reinterpret_cast<uint32_t*>(base);
#pragma unroll
    for (int k = K0; k < K1; ++k) {
        w[4 * k] = d[k - K0].x;
        w[4 * k + 1] = d[k - K0].y;
        w[4 * k + 2] = d[k - K0].z;
        w[4 * k + 3] = d[k - K0].w;
    }
    // only the chunk holding the buffer's last byte can straddle its end (chunk
    // (fb - a) / 16, when fb is not on a 16-B boundary): one test, not one per chunk
    const uint32_t rel = fb - a;
    if (__builtin_expect(fb > a && (rel & 15u) != 0 && rel >= 16u * K0 && rel < 16u * K1, 0)) {
        const uint32_t k = rel >> 4;
        const u32x4 v = lay_edge16(rs, a + 16u * k, fb);
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
}
__device__ __forceinline__ void LayerWin::refill(uint32_t s) {
    const uint32_t a = (off + s) & ~15u;
    lay_load<0, kLayFill>(base, rs, a, fb);
    bias = off - a;
    avail = a + 16u * kLayFill - off;
}
__device__ __forceinline__ void LayerWin::refill_hi() {
    if constexpr (kLayFill < kLayChunks) {
        lay_load<kLayFill, kLayChunks>(base, rs, off - bias, fb);
        avail = 16u * kLayChunks - bias;
    }
}
__device__ __attribute__((noinline)) uint32_t lay_far_field(uint8_t* base, uint32_t bias,
                                                            uint32_t avail, uint32_t off,
                                                            __amdgpu_buffer_rsrc_t rs, uint32_t s,
                                                            uint32_t ob, uint32_t bits) {
    const LayerWin Wn{base, bias, avail, off, 0u, rs};     // by value: no address taken
    return Wn.field(s, ob, bits);
}

// The first 20 bytes of a header as frame-relative little-endian dwords, read once per
// layer step: every condition, header_len and payload_len field of the table but one
// (MSTP's, at byte 36) and every dispatch key of lay_next lies in them.
struct LayHdr {
    uint32_t F[5];
};

// `fill`: a header past the slot refills it; without, such a header reads as garbage
// (the caller then never uses it)
__device__ __forceinline__ LayHdr lay_hdr(LayerWin& Wn, uint32_t s, bool fill) {
    const bool out = s + 20u > Wn.avail;
    if (__builtin_expect(out && fill, 0)) {
        // the header still starts in the slot's span and ends in its unfetched half:
        // fetch that half; else the slot moves to the header
        if (kLayFill < kLayChunks && s + 20u <= 16u * kLayChunks - Wn.bias) Wn.refill_hi();
        else Wn.refill(s);
    }
    const uint32_t y = out && !fill ? 0u : s + Wn.bias, a = y & ~3u;
    uint32_t R[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) R[k] = lds32(Wn.base, a + 4 * k);
    LayHdr H;
#pragma unroll
    for (int k = 0; k < 5; ++k) H.F[k] = align_bytes(R[k + 1], R[k], y & 3u);
    return H;
}
// header bytes [x, x + 4), x <= 15
__device__ __forceinline__ uint32_t hdr_dw(const LayHdr& H, uint32_t x) {
    const uint32_t k = x >> 2;
    uint32_t lo = H.F[0], hi = H.F[1];
    lo = k == 1 ? H.F[1] : lo;
    hi = k == 1 ? H.F[2] : hi;
    lo = k == 2 ? H.F[2] : lo;
    hi = k == 2 ? H.F[3] : hi;
    lo = k == 3 ? H.F[3] : lo;
    hi = k == 3 ? H.F[4] : hi;
    return align_bytes(hi, lo, x & 3u);
}
__device__ __forceinline__ uint32_t hdr_be16(const LayHdr& H, uint32_t x) {
    return be16_lo(hdr_dw(H, x));
}

// The walk's LDS image of the table, built from kProtos / kGroups / kMembers at kernel
// start.  A length expression is stored as (x + add) * mul + add2 (pktfmt's five forms
// in the same 32-bit arithmetic), a member's condition as a masked range test on its
// group's key dword (kMembers), the next-layer dispatch as a 16-bit rule.
struct LayProto {
    uint32_t a;               // hdr | hl_kind << 8 | pl_kind << 12 | next rule << 16
    int32_t hl_fixed;
    uint32_t hlf, hl_am;      // header_len: field bit off | bits << 16 ; add | mul << 16
    uint32_t hl_b, plf;       // header_len add2 ; payload field
    uint32_t pl_am, pl_b;
};
struct LayMember {
    uint32_t mask, lo, span, pad;
};
struct __attribute__((aligned(16))) LayGroupRec {
    LayProto p;               // the first member's protocol
    uint32_t g;               // first | count << 8 | cond_bytes << 16 | lut << 24 | key << 28
    uint32_t m0[3];           // member tests of the first two members: mask, lo, span
    uint32_t m1[3];
    uint32_t pad;
};
struct LayTable {
    LayGroupRec gr[RPKT_N_GROUPS];
    LayProto p[RPKT_N_PROTOS];
    LayMember m[RPKT_N_PROTOS + RPKT_MAX_MEMBERS]; // members 2.. read MAX entries
    uint8_t lut[RPKT_N_LUT][256];   // lookup groups: key byte -> member (0xff: none)
    uint32_t et[32];                // EtherType -> group: ethertype << 8 | group at et_slot()
    int8_t ip[256];                 // IP protocol number -> group / kNextEnd / kNextUnknown
};
// a perfect hash of the ten EtherTypes of the walk into 32 slots (empty: ~0u)
__device__ __forceinline__ uint32_t et_slot(uint32_t k16) { return ((k16 * 0x36u) >> 8) & 31u; }
constexpr uint32_t kNoLut = 15;
static_assert(RPKT_N_LUT < kNoLut, "lookup ids fit 4 bits");
static_assert(RPKT_N_PROTOS + RPKT_MAX_MEMBERS <= kWave * kWavesPerBlock, "one fill pass");
static_assert(RPKT_N_GROUPS <= 32, "a rule's fixed group fits 5 bits");

constexpr int kNextEnd = -1, kNextUnknown = -2;

__device__ inline int lay_ethertype(uint32_t et) {
    switch (et) {
        case 0x0800: return RPKT_G_IPV4;
        case 0x86dd: return RPKT_G_IPV6;
        case 0x8100: case 0x88a8: return RPKT_G_VLAN;
        case 0x0806: return RPKT_G_ARP;
        case 0x8847: case 0x8848: return RPKT_G_MPLS;
        case 0x8863: case 0x8864: return RPKT_G_PPPOE;
        case 0x6558: return RPKT_G_ETHER;                    // GRE only (kNxTeb)
        default: return kNextUnknown;
    }
}
__device__ inline int lay_ipproto(uint32_t p) {
    switch (p) {
        case 0: return RPKT_G_IPV6_HOPBYHOP;
        case 1: return RPKT_G_ICMPV4;
        case 4: return RPKT_G_IPV4;
        case 6: return RPKT_G_TCP;
        case 17: return RPKT_G_UDP;
        case 41: return RPKT_G_IPV6;
        case 43: return RPKT_G_IPV6_ROUTING;
        case 44: return RPKT_G_IPV6_FRAGMENT;
        case 47: return RPKT_G_GRE;
        case 51: return RPKT_G_IPV6_AUTH;
        case 59: return kNextEnd;                            // no next header
        case 60: return RPKT_G_IPV6_DESTOPTS;
        default: return kNextUnknown;
    }
}

// The dispatch of include/rpkt_gpu.h (rpkt_layers_t) after each protocol, as a rule:
// kind | key byte << 4 | fixed group << 8 | flags.  lay_next evaluates it.
constexpr uint32_t kNxEnd = 0, kNxFixed = 1, kNxEther = 2, kNxIp = 3, kNxUdp = 4,
                   kNxGtpu = 5, kNxMpls = 6, kNxPpp = 7, kNxLlc = 8;
constexpr uint32_t kNxTeb = 1u << 13;        // GRE: 0x6558 carries Ethernet
constexpr uint32_t kNxV4Frag = 1u << 14;     // IPv4: a non-first fragment ends the walk
constexpr uint32_t kNxV6Frag = 1u << 15;     // IPv6 fragment header: likewise
__device__ inline uint32_t lay_next_rule(uint32_t p) {
    switch (p) {
        case RPKT_P_ETHER_ETHERFRAME: return kNxEther | 12u << 4;
        case RPKT_P_VLAN_VLANFRAME: return kNxEther | 2u << 4;
        case RPKT_P_ETHER_ETHERDOT3FRAME: case RPKT_P_VLAN_VLANDOT3FRAME:
            return kNxFixed | (uint32_t)RPKT_G_LLC << 8;
        case RPKT_P_IPV4_IPV4: return kNxIp | 9u << 4 | kNxV4Frag;
        case RPKT_P_IPV6_IPV6: return kNxIp | 6u << 4;
        case RPKT_P_IPV6_FRAGMENTHEADER: return kNxIp | kNxV6Frag;
        case RPKT_P_IPV6_HOPBYHOPOPTION: case RPKT_P_IPV6_DESTOPTIONS:
        case RPKT_P_IPV6_ROUTINGHEADER: case RPKT_P_IPV6_AUTHENTICATIONHEADER: return kNxIp;
        case RPKT_P_UDP_UDP: return kNxUdp;
        case RPKT_P_GRE_GRE: return kNxEther | 2u << 4 | kNxTeb;
        case RPKT_P_VXLAN_VXLAN: return kNxFixed | (uint32_t)RPKT_G_ETHER << 8;
        case RPKT_P_GTPV1_GTPV1: return kNxGtpu;
        case RPKT_P_MPLS_MPLS: return kNxMpls;
        case RPKT_P_PPPOE_PPPOESESSION: return kNxPpp | 6u << 4;
        case RPKT_P_LLC_LLC: return kNxLlc;
        default: return kNxEnd;
    }
}

// pktfmt UsableAlgExpr (ast/length.rs:244-283): x, x+a, x*a, (x+a)*b, x*a+b as
// (x + add) * mul + add2
__device__ __forceinline__ void lay_expr(const RpktLenExpr& E, uint32_t& f, uint32_t& am,
                                         uint32_t& b) {
    uint32_t add = 0, mul = 1, add2 = 0;
    switch (E.form) {
        case 1: add = E.a; break;
        case 2: mul = E.a; break;
        case 3: add = E.a; mul = E.b; break;
        case 4: mul = E.a; add2 = E.b; break;
        default: break;
    }
    f = E.off | ((E.bits ? (uint32_t)E.bits : 32u) << 16);   // 32: unused, no 32-bit shift
    am = add | (mul << 16);
    b = add2;
}

__device__ __forceinline__ LayProto lay_proto(uint32_t t) {
    const RpktProto& P = kProtos[t];
    LayProto L;
    L.a = P.hdr | ((uint32_t)P.hl_kind << 8) | ((uint32_t)P.pl_kind << 12) | (lay_next_rule(t) << 16);
    L.hl_fixed = P.hl_fixed;
    lay_expr(P.hl, L.hlf, L.hl_am, L.hl_b);
    lay_expr(P.pl, L.plf, L.pl_am, L.pl_b);
    return L;
}

__device__ __forceinline__ void lay_table_fill(LayTable& T) {
    const uint32_t t = threadIdx.x;
    if (t < RPKT_N_PROTOS) T.p[t] = lay_proto(t);
    if (t < RPKT_N_PROTOS + RPKT_MAX_MEMBERS) {
        const RpktMember M = t < RPKT_N_PROTOS ? kMembers[t] : RpktMember{0u, 0u, 0u};
        T.m[t] = LayMember{M.mask, M.lo, M.span, 0u};
    }
    if (t < RPKT_N_GROUPS) {
        const RpktGroup G = kGroups[t];
        LayGroupRec R;
        R.p = lay_proto(G.first);
        R.g = G.first | ((uint32_t)G.count << 8) | ((uint32_t)G.cond_bytes << 16) |
              ((G.lut == 0xffu ? kNoLut : (uint32_t)G.lut) << 24) | ((uint32_t)G.key << 28);
        const RpktMember M0 = kMembers[G.first];
        const RpktMember M1 = G.count > 1 ? kMembers[G.first + 1] : RpktMember{0u, 0u, 0u};
        R.m0[0] = M0.mask, R.m0[1] = M0.lo, R.m0[2] = M0.span;
        R.m1[0] = M1.mask, R.m1[1] = M1.lo, R.m1[2] = M1.span;
        R.pad = 0;
        T.gr[t] = R;
    }
    for (uint32_t k = t; k < RPKT_N_LUT * 64; k += blockDim.x)
        reinterpret_cast<uint32_t*>(T.lut)[k] = reinterpret_cast<const uint32_t*>(kGroupLut)[k];
    if (t < 256) T.ip[t] = (int8_t)lay_ipproto(t);
    if (t < 32) {                   // the EtherType hashing to slot t, if any
        constexpr uint16_t kEt[10] = {0x0800, 0x86dd, 0x8100, 0x88a8, 0x0806,
                                      0x8847, 0x8848, 0x8863, 0x8864, 0x6558};
        uint32_t v = ~0u;
        for (int k = 0; k < 10; ++k)
            if (et_slot(kEt[k]) == t) v = ((uint32_t)kEt[k] << 8) | (uint32_t)lay_ethertype(kEt[k]);
        T.et[t] = v;
    }
}

// the table's length expression at field f of header s
template <bool kFar>
__device__ __forceinline__ uint32_t lay_len(const LayerWin& Wn, const LayHdr& H, uint32_t s,
                                            uint32_t f, uint32_t am, uint32_t b) {
    const uint32_t ob = f & 0xffffu, bits = (f >> 16) & 0xffu;
    uint32_t x;
    if (kFar && __builtin_expect((ob >> 3) > 15u, 0))        // MSTP's, at byte 36
        x = lay_far_field(Wn.base, Wn.bias, Wn.avail, Wn.off, Wn.rs, s, ob, bits);
    else
        x = (bswap32(hdr_dw(H, ob >> 3)) << (ob & 7u)) >> (32u - bits);
    return (x + (am & 0xffffu)) * (am >> 16) + b;
}

__device__ __forceinline__ bool member_hit(uint32_t K, uint32_t mask, uint32_t lo, uint32_t span) {
    return (K & mask) - lo <= span;
}

// group_parse + parse + payload() of group g at cursor [s, e): returns the member
// protocol (< 0 on Err) with its header length, the trimmed packet end and its
// next-layer rule.  Members are tried in order, the first match wins (the generated
// group_parse's order); a group keyed on one byte (ICMPv4 types, PPPoE codes) looks
// its member up.  Every check folds into one `bad` flag.
__device__ __forceinline__ int walk_group(const LayerWin& Wn, const LayHdr& H, const LayTable& T,
                                          uint32_t g, uint32_t s, uint32_t e, uint32_t& hl,
                                          uint32_t& end, uint32_t& rule) {
    const uint32_t r = e - s;
    const LayGroupRec& GR = T.gr[g];
    LayProto P = GR.p;
    const uint32_t G = GR.g;
    const uint32_t first = G & 0xffu, count = (G >> 8) & 0xffu, cond_bytes = (G >> 16) & 0xffu;
    const uint32_t lut = (G >> 24) & 15u;
    const uint32_t K = bswap32(hdr_dw(H, G >> 28));            // the key dword, big-endian
    // (bitwise & and |: no short-circuit, so no branch around the second test)
    const bool hit0 = member_hit(K, GR.m0[0], GR.m0[1], GR.m0[2]);
    const bool hit1 = (count > 1) & member_hit(K, GR.m1[0], GR.m1[1], GR.m1[2]);
    int m = hit0 ? (int)first : (hit1 ? (int)first + 1 : -1);
    if (__builtin_expect(__ballot(m < 0 && count > 2) != 0, 0)) {      // STP's BPDUs
#pragma unroll
        for (uint32_t k = 2; k < RPKT_MAX_MEMBERS; ++k) {
            const LayMember M = T.m[first + k];
            const bool hit = k < count && member_hit(K, M.mask, M.lo, M.span);
            m = (m < 0 && hit) ? (int)(first + k) : m;
        }
    }
    if (__builtin_expect(__ballot(lut != kNoLut) != 0, 0)) {          // ICMPv4, PPPoE
        const uint32_t lm = T.lut[lut < RPKT_N_LUT ? lut : 0u][K >> 24];
        m = lut != kNoLut ? (lm == 0xffu ? -1 : (int)lm) : m;
    }
    if (__builtin_expect(__ballot(m > (int)first) != 0, 0)) {         // not the first member
        // field by field: a select of the whole struct would keep both copies in scratch
        const bool o = m > (int)first;
        const LayProto Q = T.p[o ? (uint32_t)m : first];
        P.a = o ? Q.a : P.a;
        P.hl_fixed = o ? Q.hl_fixed : P.hl_fixed;
        P.hlf = o ? Q.hlf : P.hlf;
        P.hl_am = o ? Q.hl_am : P.hl_am;
        P.hl_b = o ? Q.hl_b : P.hl_b;
        P.plf = o ? Q.plf : P.plf;
        P.pl_am = o ? Q.pl_am : P.pl_am;
        P.pl_b = o ? Q.pl_b : P.pl_b;
    }
    bool bad = (r < cond_bytes) | (m < 0);
    const uint32_t hdr = P.a & 0xffu, hk = (P.a >> 8) & 15u, pk = (P.a >> 12) & 15u;
    bad |= r < hdr;
    const uint32_t ind = hdr_be16(H, 0), b0 = H.F[0] & 0xffu;
    uint32_t h = lay_len<true>(Wn, H, s, P.hlf, P.hl_am, P.hl_b);
    // gre/mod.rs:68-101 (GRE, PPTP), gtpv1.pktfmt / gtpv2.pktfmt header_len
    const uint32_t h_gre = 4u + ((ind & 0xc000u) ? 4u : 0u) + ((ind & 0x2000u) ? 4u : 0u) +
                           ((ind & 0x1000u) ? 4u : 0u);
    const uint32_t h_pptp = 8u + ((ind & 0x1000u) ? 4u : 0u) + ((ind & 0x0080u) ? 4u : 0u);
    h = hk == 2u ? h_gre : h;
    h = hk == 3u ? h_pptp : h;
    h = hk == 4u ? ((b0 & 7u) ? 12u : 8u) : h;
    h = hk == 5u ? ((b0 & 8u) ? 12u : 8u) : h;
    h = hk == 0u ? hdr : h;
    const bool hbad = P.hl_fixed >= 0 ? h != (uint32_t)P.hl_fixed : ((h < hdr) | (h > r));
    bad |= (hk != 0u) & hbad;
    const uint32_t pl = lay_len<false>(Wn, H, s, P.plf, P.pl_am, P.pl_b);
    bad |= (pk == 1u) & ((uint64_t)pl + h > r);              // payload_len
    bad |= (pk == 2u) & ((pl < h) | (pl > r));               // packet_len
    end = pk == 1u ? s + h + pl : (pk == 2u ? s + pl : e);
    hl = h;
    rule = bad ? kNxEnd : P.a >> 16;
    return bad ? -1 : m;
}

// The dispatch after a protocol with rule R whose header H started the step; the cursor
// is now [s, e) and pb is its first byte.  Every candidate is computed and selected by
// the rule's kind; key is the unknown next protocol's number when the result is
// kNextUnknown.
__device__ __forceinline__ int lay_next(const LayHdr& H, const LayTable& T, uint32_t pb, uint32_t R,
                                        uint32_t s, uint32_t e, uint32_t& key) {
    const uint32_t kind = R & 15u;
    const uint32_t k16 = hdr_be16(H, (R >> 4) & 15u), k8 = k16 >> 8;
    const uint32_t b0 = H.F[0] & 0xffu, b1 = (H.F[0] >> 8) & 0xffu, b2 = (H.F[0] >> 16) & 0xffu;
    const bool more = e > s;
    const uint32_t E = T.et[et_slot(k16)];                  // EtherType
    int eg = (E >> 8) == k16 ? (int)(E & 0xffu) : kNextUnknown;
    eg = (k16 == 0x6558u && !(R & kNxTeb)) ? kNextUnknown : eg;
    const uint32_t fv = ((R & kNxV4Frag) ? hdr_be16(H, 6) & 0x1fffu : 0u) |
                        ((R & kNxV6Frag) ? hdr_be16(H, 2) >> 3 : 0u);
    const bool frag = fv != 0u;
    const int ig = frag ? kNextEnd : (int)T.ip[k8];          // IP protocol number
    const uint32_t dp = hdr_be16(H, 2), sp = hdr_be16(H, 0); // UDP: VXLAN / GTP-U / GTP-C
    const bool dpt = (dp == 4789u) | (dp == 2152u) | (dp == 2123u);
    const bool spt = (sp == 4789u) | (sp == 2152u) | (sp == 2123u);
    const uint32_t port = dpt ? dp : (spt ? sp : 0u);
    const uint32_t gv = pb >> 5, iv = pb >> 4;
    const int gtp = gv == 1u ? RPKT_G_GTPV1 : (gv == 2u ? RPKT_G_GTPV2 : kNextUnknown);
    const int ipv = iv == 4u ? RPKT_G_IPV4 : (iv == 6u ? RPKT_G_IPV6 : kNextUnknown);
    const int udp = !port ? kNextEnd : (port == 4789u ? RPKT_G_VXLAN : (more ? gtp : kNextEnd));
    const int gtpu = (((b0 & 4u) != 0u) | (b1 != 255u) | !more) ? kNextEnd : ipv;
    const int mpls = !(b2 & 1u) ? RPKT_G_MPLS : (more ? ipv : kNextEnd);
    const int ppp = k16 == 0x0021u ? RPKT_G_IPV4 : (k16 == 0x0057u ? RPKT_G_IPV6 : kNextUnknown);
    const int llc = ((b0 == 0x42u) & (b1 == 0x42u)) ? RPKT_G_STP : kNextEnd;
    int nx = kNextEnd;
    nx = kind == kNxFixed ? (int)((R >> 8) & 31u) : nx;
    nx = kind == kNxEther ? eg : nx;
    nx = kind == kNxIp ? ig : nx;
    nx = kind == kNxUdp ? udp : nx;
    nx = kind == kNxGtpu ? gtpu : nx;
    nx = kind == kNxMpls ? mpls : nx;
    nx = kind == kNxPpp ? ppp : nx;
    nx = kind == kNxLlc ? llc : nx;
    key = kind == kNxIp ? k8 : (kind == kNxUdp ? gv : ((kind == kNxGtpu || kind == kNxMpls) ? iv : k16));
    return nx;
}

// Every walk starts with the Ethernet group (EtherGroup::group_parse,
// ether/generated.rs:287-302): the table interpreter's first step, specialised.  A
// frame's first step is taken with the frame (when the lane takes it from the pool),
// so the general loop runs one iteration less per frame.  Same results as walk_group +
// lay_next on group RPKT_G_ETHER at s = 0 (the table's Ether rows: members EtherFrame,
// EtherType >= 0x0600, and EtherDot3Frame, length field <= 1500 trimmed as payload_len;
// 14 header bytes; then the EtherType dispatch or LLC).  Returns the stop code (0: go on).
#ifndef RPKT_LAY_ETHER_FIRST
#define RPKT_LAY_ETHER_FIRST 1
#endif
__device__ __forceinline__ uint32_t ether_step(LayerWin& Wn, LayHdr& H, const LayTable& T,
                                               uint32_t len, uint32_t (&o)[16], uint32_t& s,
                                               uint32_t& e, uint32_t& nl, int& g) {
    // the length / EtherType field straight from the slot, and the next header (at 14,
    // used only if the walk goes on) read at once: one LDS round trip after the refill
    const uint32_t y = 12u + Wn.bias, a = y & ~3u;
    const uint32_t et = be16_lo(align_bytes(lds32(Wn.base, a + 4u), lds32(Wn.base, a), y & 3u));
    H = lay_hdr(Wn, 14u, false);
    const bool ef = et >= 0x0600u, d3 = et <= 1500u;
    const bool ok = (len >= 14u) & (ef | d3) & !(d3 & (et + 14u > len));
    const uint32_t p = ef ? (uint32_t)RPKT_P_ETHER_ETHERFRAME : (uint32_t)RPKT_P_ETHER_ETHERDOT3FRAME;
    const uint32_t E = T.et[et_slot(et)];
    int nx = ((E >> 8) == et && et != 0x6558u) ? (int)(E & 0xffu) : kNextUnknown;
    nx = ef ? nx : RPKT_G_LLC;
    const bool unk = ok && nx == kNextUnknown;
    const uint32_t stop = !ok ? (uint32_t)RPKT_L_ERR : unk ? (uint32_t)RPKT_L_UNKNOWN : 0u;
    nl = ok ? 1u : 0u;
    e = ok && d3 ? 14u + et : len;
    s = ok ? 14u : 0u;
    o[4] = ok ? p : 0u;
    o[0] = nl | (stop << 8) | ((unk ? p : 0u) << 24);
    o[1] = s;
    o[2] = e - s;
    o[3] = unk ? et : 0u;
    g = nx;
    return stop;
}

// The straight-line prefix (RPKT_LAY_PREFIX): after the Ethernet step, the layers of the
// common stack -- up to two VLAN tags, IPv4 or IPv6, TCP or UDP -- each as its own
// specialised step (the walk_group + lay_next of those five groups, without the table:
// VlanGroup vlan/generated.rs:312-322, Ipv4::parse ipv4/generated.rs:35-51, Ipv6::parse
// ipv6/generated.rs:40-51, Udp::parse udp/generated.rs:31-42, Tcp::parse
// tcp/generated.rs:34-45), stage by stage for the lanes whose walk is at such a layer; the
// interpreter takes over at the first layer outside the set.  Same records as the
// interpreter (tests/test_gpu_layers.py).  Same process, byte-identical (round 6,
// profiles/r06_lay_prefix/): config 5's walk 304.4 -> 262.2 us, config 2 42.9 -> 37.2 us,
// the capture mix 57.2 -> 57.3 us (its VALU per wave 5375 -> 5585: the many stacks that
// leave the prefix early pay its stages on top of the interpreter's).
#ifndef RPKT_LAY_PREFIX
#define RPKT_LAY_PREFIX 1        // 0: the interpreter from the first layer after Ethernet
#endif
__device__ __forceinline__ void lay_put(uint32_t (&o)[16], uint32_t nl, uint32_t p, uint32_t s) {
    // layer nl <= 4 here: proto bytes in o[4..5], offsets in o[8..10]
    const uint32_t pw = p << (8 * (nl & 3)), sw = s << (16 * (nl & 1));
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) o[4 + k] |= (nl >> 2) == k ? pw : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) o[8 + k] |= (nl >> 1) == k ? sw : 0u;
}
// the record's tail after a prefix layer (p) ended the step with (nx, key)
__device__ __forceinline__ uint32_t lay_after(uint32_t (&o)[16], uint32_t nl, uint32_t p, int nx,
                                              uint32_t key, uint32_t s, uint32_t e) {
    const bool unk = nx == kNextUnknown;
    const uint32_t stop = nx == kNextEnd ? (uint32_t)RPKT_L_END : unk ? (uint32_t)RPKT_L_UNKNOWN : 0u;
    o[0] = nl | (stop << 8) | ((unk ? p : 0u) << 24);
    o[1] = s & 0xffffu;
    o[2] = e - s;
    o[3] = unk ? key : 0u;
    return stop;
}
__device__ __forceinline__ uint32_t lay_bad(uint32_t (&o)[16], uint32_t nl, uint32_t g, uint32_t s,
                                            uint32_t e) {
    o[0] = nl | ((uint32_t)RPKT_L_ERR << 8) | (g << 16);
    o[1] = s & 0xffffu;
    o[2] = e - s;
    o[3] = 0u;
    return RPKT_L_ERR;
}
// EtherType dispatch (lay_next's kNxEther without GRE's 0x6558)
__device__ __forceinline__ int lay_by_et(const LayTable& T, uint32_t et) {
    const uint32_t E = T.et[et_slot(et)];
    return ((E >> 8) == et && et != 0x6558u) ? (int)(E & 0xffu) : kNextUnknown;
}
__device__ __forceinline__ void prefix_walk(LayerWin& Wn, LayHdr& H, const LayTable& T,
                                            uint32_t (&o)[16], uint32_t& s, uint32_t& e,
                                            uint32_t& nl, int& g, uint32_t& pend) {
    // up to two VLAN tags
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        if (pend == 0u && g == RPKT_G_VLAN) {
            const uint32_t r = e - s, et = be16_hi(H.F[0]);
            const bool ef = et >= 0x0600u, d3 = et <= 1500u;
            if ((r < 4u) | !(ef | d3) | (d3 & (et + 4u > r))) {
                pend = lay_bad(o, nl, (uint32_t)g, s, e);
            } else {
                const uint32_t p = ef ? (uint32_t)RPKT_P_VLAN_VLANFRAME : (uint32_t)RPKT_P_VLAN_VLANDOT3FRAME;
                lay_put(o, nl, p, s);
                nl += 1u;
                e = d3 ? s + 4u + et : e;
                s += 4u;
                const int nx = ef ? lay_by_et(T, et) : RPKT_G_LLC;
                pend = lay_after(o, nl, p, nx, et, s, e);
                g = nx;
                H = lay_hdr(Wn, s, true);
            }
        }
    }
    // IPv4 / IPv6
    if (pend == 0u && (g == RPKT_G_IPV4 || g == RPKT_G_IPV6)) {
        const uint32_t r = e - s, F0 = H.F[0], F1 = H.F[1];
        const bool v4 = g == RPKT_G_IPV4;
        const uint32_t ihl = (F0 & 0xfu) * 4u, tot = be16_hi(F0), plen = be16_lo(F1);
        const bool bad = v4 ? ((r < 20u) | (ihl < 20u) | (ihl > r) | (tot < ihl) | (tot > r))
                            : ((r < 40u) | (plen + 40u > r));
        if (bad) {
            pend = lay_bad(o, nl, (uint32_t)g, s, e);
        } else {
            const uint32_t p = v4 ? (uint32_t)RPKT_P_IPV4_IPV4 : (uint32_t)RPKT_P_IPV6_IPV6;
            lay_put(o, nl, p, s);
            nl += 1u;
            e = v4 ? s + tot : s + 40u + plen;
            const uint32_t key = v4 ? (H.F[2] >> 8) & 0xffu : (F1 >> 16) & 0xffu;
            const bool frag = v4 && (be16_hi(F1) & 0x1fffu) != 0u;   // a non-first fragment
            s += v4 ? ihl : 40u;
            const int nx = frag ? kNextEnd : (int)T.ip[key];
            pend = lay_after(o, nl, p, nx, key, s, e);
            g = nx;
            H = lay_hdr(Wn, s, pend == 0u);
        }
    }
    // TCP / UDP
    if (pend == 0u && (g == RPKT_G_TCP || g == RPKT_G_UDP)) {
        const uint32_t r = e - s, F0 = H.F[0];
        const bool udp = g == RPKT_G_UDP;
        const uint32_t ulen = be16_lo(H.F[1]), doff = ((H.F[3] >> 4) & 0xfu) * 4u;
        const bool bad = udp ? ((r < 8u) | (ulen < 8u) | (ulen > r))
                             : ((r < 20u) | (doff < 20u) | (doff > r));
        if (bad) {
            pend = lay_bad(o, nl, (uint32_t)g, s, e);
        } else {
            const uint32_t p = udp ? (uint32_t)RPKT_P_UDP_UDP : (uint32_t)RPKT_P_TCP_TCP;
            lay_put(o, nl, p, s);
            nl += 1u;
            e = udp ? s + ulen : e;
            s += udp ? 8u : doff;
            // UDP: VXLAN / GTP-U / GTP-C by port, the GTP version from the payload's first
            // byte (lay_next's kNxUdp); TCP ends the walk
            const uint32_t dp = be16_hi(F0), sp = be16_lo(F0);
            const bool dpt = (dp == 4789u) | (dp == 2152u) | (dp == 2123u);
            const bool spt = (sp == 4789u) | (sp == 2152u) | (sp == 2123u);
            const uint32_t port = udp ? (dpt ? dp : (spt ? sp : 0u)) : 0u;
            const bool more = e > s;
            const LayHdr H2 = lay_hdr(Wn, s, port != 0u && (port == 4789u || more));
            const uint32_t gv = (H2.F[0] & 0xffu) >> 5;
            const int gtp = gv == 1u ? RPKT_G_GTPV1 : (gv == 2u ? RPKT_G_GTPV2 : kNextUnknown);
            const int nx = !port ? kNextEnd : (port == 4789u ? RPKT_G_VXLAN : (more ? gtp : kNextEnd));
            pend = lay_after(o, nl, p, nx, gv, s, e);
            g = nx;
            H = H2;
        }
    }
}

// Lane L of a wave walks frames base + L + 64 k, k = 0 .. F-1, one after the other: a
// walk's depth varies from frame to frame (the capture mix: 2.6 layers on average, a
// wave's deepest lane 6.8), and a wave runs until its deepest lane ends, so a lane
// that walks several frames in a row evens the depths out over the wave.  The first
// frame's window is staged cooperatively (coalesced 16-B loads).  Records are stored
// per lane (64 B each).
// frames per lane on average: a wave walks a pool of 64 kLayFrames frames, each lane
// taking the next untaken frame when its walk ends (82.9 -> 68.7 us on the capture
// mix vs four fixed frames per lane, profiles/r02_fwd/ablate_layers_c9.log)
constexpr int kLayFrames = 4;
#ifndef RPKT_LAY_RUNTIME_POOL
#define RPKT_LAY_RUNTIME_POOL 0  // 1: block pools sized for one round of resident blocks
#endif
// A lane stores its 64-B record as four 16-B stores when its walk ends, so every store
// instruction writes 16 B into each of up to 64 different records: with the default
// policy L2 merges a record's four pieces into one line write, non-temporal stores do not
// (config 2 walk 60.3 -> 42.2 us, config 5 337.6 -> 312.6 us, capture mix 59.1 -> 58.3 us,
// same process, profiles/r02_ab_recnt).
#ifndef RPKT_LAY_REC_NT
#define RPKT_LAY_REC_NT 0        // 1: record stores non-temporal
#endif
#ifndef RPKT_LAY_BLOCK_POOL
#define RPKT_LAY_BLOCK_POOL 1    // 0: one pool per wave
#endif

// ABL (librpkt_gpu_ablate.so timing only, results not meaningful), bits: 1 = a taken
// frame walks the slot's stale bytes (no refill), 2 = no record stores, 4 = every walk
// ends after its Ethernet step
template <int F, bool DYN = false, int ABL = 0>
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void layers_kernel(const uint8_t* __restrict__ frames, uint32_t fb,
                   const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                   uint32_t n, rpkt_layers_t* __restrict__ out, uint32_t pool) {
    __shared__ __attribute__((aligned(16))) LayScratch scratch[kWavesPerBlock];
    // the protocol table in LDS: lanes walk different protocols, so table reads are
    // per-lane (divergent) loads; from LDS they cost tens of cycles instead of a
    // global-memory round trip per dependent lookup
    __shared__ __attribute__((aligned(16))) LayTable T;
    // DYN with block pooling: the block's 4 waves share one pool of 4 x 64 F frames
    // through an LDS counter, so they end together (per-wave pools differ by +-12 % in
    // work on the capture mix, and a pass of waves lasts as long as its slowest)
    constexpr bool kBlk = DYN && RPKT_LAY_BLOCK_POOL;
    __shared__ uint32_t blk_taken;
    lay_table_fill(T);
    if (threadIdx.x == 0) blk_taken = kWave * kWavesPerBlock;    // the waves' first tiles
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    LayScratch& W = scratch[wid];
    const uint32_t bb = blockIdx.x * pool;                   // the block's frames (kBlk)
    const uint32_t p0 = kBlk ? bb + wid * kWave : (blockIdx.x * kWavesPerBlock + wid) * (kWave * F);
    if (p0 >= n) return;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    constexpr int FR = DYN ? 1 : F;                          // DYN takes later frames as it goes
    Frame fr[FR];
#pragma unroll
    for (int k = 0; k < FR; ++k) fr[k] = spans.get(p0 + lane + kWave * k);
    {
        u32x4 d[kLayFill];
        uint32_t addr[kLayFill];
        uint32_t fix = 0;
#pragma unroll
        for (int k = 0; k < kLayFill; ++k) {
            const int c = k * kWave + lane;
            const int q = c / kLayFill, j = c % kLayFill;
            const uint32_t qo = (uint32_t)__shfl((int)fr[0].off, q, kWave);
            const uint32_t ql = (uint32_t)__shfl((int)fr[0].len, q, kWave);
            const uint32_t a = (qo & ~15u) + 16u * j;
            addr[k] = (a < qo + ql) ? a : fb;
            fix |= (uint32_t)straddles(addr[k], fb) << k;
        }
#pragma unroll
        for (int k = 0; k < kLayFill; ++k) d[k] = load16_fast(rs, addr[k]);
#pragma unroll
        for (int k = 0; k < kLayFill; ++k) {
            const int c = k * kWave + lane;
            u32x4 v = d[k];
            if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
            uint32_t* dst = reinterpret_cast<uint32_t*>(&W.win[(c / kLayFill) * kLaySlot +
                                                              (c % kLayFill) * 16]);
            dst[0] = v.x;
            dst[1] = v.y;
            dst[2] = v.z;
            dst[3] = v.w;
        }
    }
    wave_sync();

    LayerWin Wn{&W.win[lane * kLaySlot], fr[0].off & 15u, (uint32_t)(kLayFill * 16) - (fr[0].off & 15u),
                fr[0].off, fb, rs};
    uint32_t o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0;
    uint32_t i = p0 + lane;                                  // the lane's current frame
    bool active = i < n;
    uint32_t taken = kWave;                                  // DYN: frames of the pool started
    uint32_t fk = 0;                                         // its index in fr[]
    uint32_t s = 0, e = fr[0].len, nl = 0;
    int g = RPKT_G_ETHER;
    LayHdr H = lay_hdr(Wn, 0u, false);                      // in the staged window
    // DYN: a frame's first (Ethernet) step is taken with the frame; pend holds the stop
    // code of a frame that ended there, stored by the next iteration
    constexpr bool kEth = DYN && RPKT_LAY_ETHER_FIRST;
    uint32_t pend = 0;
    if constexpr (kEth) {
        if (active) {
            pend = ether_step(Wn, H, T, e, o, s, e, nl, g);   // H: the header at 14, in the slot
            if constexpr (RPKT_LAY_PREFIX) prefix_walk(Wn, H, T, o, s, e, nl, g, pend);
        }
        if constexpr ((ABL & 4) != 0) pend = active ? (uint32_t)RPKT_L_END : 0u;
    }
    while (__ballot(active)) {
        uint32_t stop = pend;
        if (active && !pend) {
            uint32_t hl = 0, end = 0, rule = 0;
            const int p = walk_group(Wn, H, T, (uint32_t)g, s, e, hl, end, rule);
            const bool ok = p >= 0;
            // proto[nl] at byte 16 + nl, off[nl] at byte 32 + 2 nl (predicated: nl
            // differs per lane, and a runtime register index would be a branch per
            // register)
            {
                const uint32_t pw = (uint32_t)p << (8 * (nl & 3)), sw = s << (16 * (nl & 1));
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) o[4 + k] |= (ok && (nl >> 2) == k) ? pw : 0u;
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) o[8 + k] |= (ok && (nl >> 1) == k) ? sw : 0u;
            }
            nl += ok ? 1u : 0u;
            e = ok ? end : e;
            s = ok ? s + hl : s;
            // the next header (its first byte also keys the GTP / IP version dispatch);
            // a walk that ends here does not refill the slot for it
            const LayHdr H2 = lay_hdr(Wn, s, (rule & 15u) != kNxEnd);
            uint32_t k2 = 0;
            const int nx = lay_next(H, T, H2.F[0] & 0xffu, rule, s, e, k2);
            stop = !ok                    ? (uint32_t)RPKT_L_ERR
                 : nx == kNextEnd         ? (uint32_t)RPKT_L_END
                 : nx == kNextUnknown     ? (uint32_t)RPKT_L_UNKNOWN
                 : nl == RPKT_MAX_LAYERS  ? (uint32_t)RPKT_L_MAX : 0u;
            const uint32_t err_g = ok ? 0u : (uint32_t)g;
            const bool unk = ok && nx == kNextUnknown;
            o[0] = nl | (stop << 8) | (err_g << 16) | ((unk ? (uint32_t)p : 0u) << 24);
            o[1] = s & 0xffffu;
            o[2] = e - s;
            o[3] = unk ? k2 : 0u;
            g = nx;
            H = H2;
        }
        // lanes whose walk ended store their record and move to their next frame: at once
        // (RPKT_LAY_TAKE_MIN 1), or when enough of them ended to share the take path's
        // fixed cost (the ended ones wait with pend set, as after an Ethernet-only walk)
        const uint64_t sm = __ballot(stop != 0);
        bool take = sm != 0;
        if constexpr (RPKT_LAY_TAKE_MIN > 1)
            take = take && ((uint32_t)__builtin_popcountll(sm) >= (uint32_t)RPKT_LAY_TAKE_MIN ||
                            __ballot(active && stop == 0) == 0);
        if (!take) pend = stop;
        if (take) {
            // DYN: the wave's 64 F frames are a pool; a lane that ends a frame takes
            // the next untaken one (rank among this step's finishers), so lanes stay
            // busy until the pool is empty instead of after their own F frames
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
            uint32_t kbase = taken;
            if constexpr (kBlk) {                              // every lane: full EXEC
                uint32_t b0 = 0;
                if (lane == 0) b0 = atomicAdd(&blk_taken, (uint32_t)__builtin_popcountll(sm));
                kbase = (uint32_t)__shfl((int)b0, 0, kWave);
            }
            // Records of the ended walks.  When many walks end together (a uniform
            // batch) they go through their (now free) slots, so that four neighbouring
            // lanes store one record's four 16-B pieces (whole 64-B writes instead of
            // 16-B pieces of 64 records per store instruction); a few at a time are
            // stored by their own lanes.
            const uint32_t m = (uint32_t)__builtin_popcountll(sm);
            const bool staged = RPKT_LAY_STAGE_REC && m >= (uint32_t)RPKT_LAY_STAGE_MIN;
            bool filled = false;
            Frame fq{0u, 0u};
#if RPKT_LAY_STAGE_REC
            if (staged) {
                if (stop) {
                    uint32_t* r = reinterpret_cast<uint32_t*>(Wn.base);
#pragma unroll
                    for (int k = 0; k < 16; ++k) r[k] = o[k];
                    W.emap[rank] = (uint32_t)lane;
                }
                wave_sync();
                if constexpr ((ABL & 2) == 0) {
                    for (uint32_t q0 = 0; q0 < m; q0 += kWave / 4) {   // wave-uniform
                        const uint32_t q = q0 + (uint32_t)(lane >> 2), j = (uint32_t)lane & 3u;
                        const uint32_t src = W.emap[q < m ? q : m - 1u];
                        const uint32_t isrc =
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)i);
                        const uint32_t* pr =
                            reinterpret_cast<const uint32_t*>(&W.win[src * kLaySlot]) + 4u * j;
                        const u32x4 v{pr[0], pr[1], pr[2], pr[3]};
                        if (q < m) reinterpret_cast<u32x4*>(out + isrc)[j] = v;
                    }
                }
                wave_sync();
            }
            // DYN block pools, many walks ended: the new frames (ranks 0..m-1 take frames
            // kbase + rank, consecutive) have their windows loaded cooperatively, each
            // load instruction covering whole windows of 64 / kLayChunks frames, as the
            // first tiles are; the lanes' own refill is skipped
            if constexpr (DYN && kBlk && RPKT_LAY_COOP_FILL && (ABL & 1) == 0) {
                if (staged) {
                    const uint32_t kq = kbase + (uint32_t)lane, iq = bb + kq;
                    if ((uint32_t)lane < m && kq < pool && iq < n) fq = spans.get(iq);
                    u32x4 d[kLayChunks];
                    uint32_t addr[kLayChunks];
                    uint32_t fix = 0;
#pragma unroll
                    for (int k = 0; k < kLayChunks; ++k) {
                        const int c = k * kWave + lane;
                        const int q = c / kLayChunks, j = c % kLayChunks;
                        const uint32_t qo = (uint32_t)__shfl((int)fq.off, q, kWave);
                        const uint32_t ql = (uint32_t)__shfl((int)fq.len, q, kWave);
                        const uint32_t a = (qo & ~15u) + 16u * j;
                        addr[k] = ((uint32_t)q < m && a < qo + ql) ? a : fb;
                        fix |= (uint32_t)straddles(addr[k], fb) << k;
                    }
#pragma unroll
                    for (int k = 0; k < kLayChunks; ++k) d[k] = load16_fast(rs, addr[k]);
#pragma unroll
                    for (int k = 0; k < kLayChunks; ++k) {
                        const int c = k * kWave + lane;
                        const uint32_t q = (uint32_t)(c / kLayChunks);
                        u32x4 v = d[k];
                        if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
                        if (q < m) {
                            uint32_t* dst = reinterpret_cast<uint32_t*>(
                                &W.win[W.emap[q] * kLaySlot + (c % kLayChunks) * 16]);
                            dst[0] = v.x;
                            dst[1] = v.y;
                            dst[2] = v.z;
                            dst[3] = v.w;
                        }
                    }
                    wave_sync();
                    filled = true;
                    // each taking lane's frame from the lane of its rank (full EXEC here)
                    fq.off = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rank << 2), (int)fq.off);
                    fq.len = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rank << 2), (int)fq.len);
                }
            }
#endif
            if (stop) {
                if (!staged) {
                    u32x4* dst = reinterpret_cast<u32x4*>(out + i);
#pragma unroll
                    for (int k = 0; k < ((ABL & 2) ? 0 : 4); ++k) {
#if RPKT_LAY_REC_NT
                        __builtin_nontemporal_store(
                            u32x4{o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]}, &dst[k]);
#else
                        dst[k] = u32x4{o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
#endif
                    }
                }
                Frame f = fr[0];
                if constexpr (DYN) {
                    const uint32_t k = kbase + rank;
                    i = (kBlk ? bb : p0) + k;
                    active = k < (kBlk ? pool : (uint32_t)(kWave * F)) && i < n;
                    if (filled) {
                        f = fq;                               // this rank's, from its lane
                    } else if (active) {
                        f = spans.get(i);
                    }
                } else {
                    fk += 1;
                    i += kWave;
                    active = fk < (uint32_t)F && i < n;
#pragma unroll
                    for (int k = 1; k < FR; ++k) f = fk == (uint32_t)k ? fr[k] : f;
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) o[k] = 0;
                s = 0, e = f.len, nl = 0, g = RPKT_G_ETHER;
                Wn.off = f.off;
                pend = 0;
                if (active) {
                    if constexpr ((ABL & 1) != 0) {
                        Wn.bias = f.off & 15u;
                        Wn.avail = (uint32_t)(kLayFill * 16) - Wn.bias;
                    } else if (filled) {
                        Wn.bias = f.off & 15u;
                        Wn.avail = (uint32_t)(kLayChunks * 16) - Wn.bias;
                    } else {
                        Wn.refill(0u);
                    }
                    if constexpr (kEth) {
                        pend = ether_step(Wn, H, T, e, o, s, e, nl, g);
                        if constexpr (RPKT_LAY_PREFIX) prefix_walk(Wn, H, T, o, s, e, nl, g, pend);
                    } else {
                        H = lay_hdr(Wn, 0u, false);
                    }
                    if constexpr ((ABL & 4) != 0) pend = (uint32_t)RPKT_L_END;
                }
            }
            if constexpr (DYN) taken += (uint32_t)__builtin_popcountll(sm);
        }
    }
}

// Blocks of kernel k resident on the current device at once (CUs x blocks per CU),
// once per device and kernel.
int resident_blocks(const void* k, uint32_t block_threads, uint32_t& out) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, uint32_t> cache;
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev));
    if (rc) return rc;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({dev, k});
    if (it != cache.end()) {
        out = it->second;
        return RPKT_OK;
    }
    int cus = 0, per_cu = 0;
    rc = hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (rc) return rc;
    rc = hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, (int)block_threads, 0));
    if (rc) return rc;
    out = (uint32_t)(cus > 0 ? cus : 1) * (uint32_t)(per_cu > 0 ? per_cu : 1);
    cache[{dev, k}] = out;
    return RPKT_OK;
}

// F = 0: the block pools are sized at run time so that the grid is one round of
// resident blocks (each block walks ceil(n / resident) frames, at least its waves'
// first tiles); F > 0: pools of 64 F frames per wave (kLayFrames, the ablations).
template <int F, bool DYN = false, int ABL = 0>
int launch_layers(const rpkt_batch_t* b, uint32_t flen, rpkt_layers_t* layers_dev, void* stream) {
    const uint32_t per_block = kWave * kWavesPerBlock;
    uint32_t pool = per_block * (F > 0 ? F : 1), grid;
    if constexpr (F == 0) {
        static_assert(DYN, "run-time pools are block pools");
        uint32_t res = 0;
        const int rc = resident_blocks((const void*)layers_kernel<F, DYN, ABL>, per_block, res);
        if (rc) return rc;
        const uint32_t want = (uint32_t)(((uint64_t)b->n + res - 1) / res);
        pool = want > per_block ? want : per_block;
        grid = (uint32_t)(((uint64_t)b->n + pool - 1) / pool);
    } else {
        const uint32_t waves = (uint32_t)((b->n + (uint64_t)kWave * F - 1) / ((uint64_t)kWave * F));
        grid = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    }
    return launch(layers_kernel<F, DYN, ABL>, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  layers_dev, pool);
}

}  // namespace

extern "C" {

int rpkt_gpu_options_batch(const rpkt_batch_t* b, const rpkt_rec_t* recs_dev,
                           rpkt_opts_t* opts_dev, void* stream) {
    if (!b || !recs_dev || !opts_dev) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)opts_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    return launch(options_kernel<false>, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  (const void*)recs_dev, opts_dev);
}

int rpkt_gpu_options_batch_compact(const rpkt_batch_t* b, const rpkt_rec16_t* recs_dev,
                                   rpkt_opts_t* opts_dev, void* stream) {
    if (!b || !recs_dev || !opts_dev) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)opts_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    return launch(options_kernel<true>, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  (const void*)recs_dev, opts_dev);
}

int rpkt_gpu_layers_batch(const rpkt_batch_t* b, rpkt_layers_t* layers_dev, void* stream) {
    if (!b || !layers_dev) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)layers_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
#if RPKT_LAY_RUNTIME_POOL
    return launch_layers<0, true>(b, flen, layers_dev, stream);
#else
    return launch_layers<kLayFrames, true>(b, flen, layers_dev, stream);
#endif
}

#ifdef RPKT_ABLATE
// Development hook (librpkt_gpu_ablate.so only, not part of include/rpkt_gpu.h): the walk
// with F frames per lane
// (1, 2, 4, 8), for timing the choice of kLayFrames.  (Tried and dropped, DESIGN.md:
// prefetching a lane's next frame window into registers, 84 -> 90 us; per-group steps
// specialised at compile time and run one uniform group after another, 84 -> 195 us
// on the capture mix, whose waves hold many groups per step.)
int rpkt_gpu_debug_layers_variant(const rpkt_batch_t* b, rpkt_layers_t* layers_dev, int frames,
                                  void* stream) {
    if (!b || !layers_dev || b->n == 0 || !b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    switch (frames) {
        case 1: return launch_layers<1>(b, flen, layers_dev, stream);
        case 2: return launch_layers<2>(b, flen, layers_dev, stream);
        case 4: return launch_layers<4>(b, flen, layers_dev, stream);
        case 8: return launch_layers<8>(b, flen, layers_dev, stream);
        case 104: return launch_layers<4, true>(b, flen, layers_dev, stream);   // pooled
        case 102: return launch_layers<2, true>(b, flen, layers_dev, stream);
        case 108: return launch_layers<8, true>(b, flen, layers_dev, stream);
        case 201: return launch_layers<4, true, 1>(b, flen, layers_dev, stream);  // ablations
        case 202: return launch_layers<4, true, 2>(b, flen, layers_dev, stream);
        case 203: return launch_layers<4, true, 3>(b, flen, layers_dev, stream);
        case 204: return launch_layers<4, true, 4>(b, flen, layers_dev, stream);
        case 205: return launch_layers<4, true, 5>(b, flen, layers_dev, stream);
        case 206: return launch_layers<4, true, 6>(b, flen, layers_dev, stream);
        case 207: return launch_layers<4, true, 7>(b, flen, layers_dev, stream);
        case 300: return launch_layers<0, true>(b, flen, layers_dev, stream);     // run-time pools
        default: return RPKT_E_INVAL;
    }
}

#endif  // RPKT_ABLATE

}  // extern "C"
