// rpkt_opts.h — the IPv4 / TCP option walks (Ipv4OptionsIter over
// ipv4.var_header_slice(), ipv4/generated.rs:1595-1722; TcpOptionsIter over
// tcp.var_header_slice(), tcp/generated.rs:1357-1484) as lane-per-frame device code over
// option bytes held in LDS.  Shared by the standalone walk over a parsed batch
// (options_kernel, rpkt_walks.hip) and the walk fused into the parse (parse_kernel with
// OPTS, rpkt_parse.hip), which runs it on the header window the parse already holds.
// oracle/rpkt_oracle_opts.c restates the same iterators and cites them line by line.
#pragma once
#include "rpkt_common.h"

#ifndef RPKT_OPT_PAIRED
#define RPKT_OPT_PAIRED 1        // 0: both walks of a frame stepped together (walk_options)
#endif
#ifndef RPKT_OPT_DEFER
#define RPKT_OPT_DEFER 1         // 0: the paired walk with the getters updated every step
#endif
#ifndef RPKT_OPT_STEP2
#define RPKT_OPT_STEP2 1         // 0: a deferred-walk step takes a run OR one TLV option
#endif

namespace {

// Option bytes in LDS: frame byte x of this lane at base[x + bias].
struct OptWin {
    const uint8_t* base;                       // the lane's slot (4-aligned)
    uint32_t bias;
    // frame bytes x..x+3, little-endian: two aligned LDS dwords and a byte align
    __device__ __forceinline__ uint32_t dw(uint32_t x) const {
        const uint32_t y = x + bias, a = y & ~3u;
        return align_bytes(lds32(base, a + 4), lds32(base, a), y & 3u);
    }
    __device__ __forceinline__ uint32_t be32(uint32_t x) const { return bswap32(dw(x)); }
};

// The per-type parse rules of the generated option views, as a table per option type
// read from LDS in the walk (a per-lane type would make a switch divergent): kind
// index (2..7; 0: not an option type of this iterator) | fixed << 3 | x << 4, where the
// option needs n >= x remaining bytes and header_len == x (fixed) or x <= header_len
// <= n.  Types 0 (EOL) and 1 (NOP), kinds 0 and 1 of both iterators, are length-1
// options consumed by opt_run.
__device__ inline uint32_t opt_rule(bool tcp, uint32_t t) {
    if (tcp) {
        switch (t) {
            case 2: return 2u | 8u | 4u << 4;      // Mss
            case 3: return 3u | 8u | 3u << 4;      // WindowScale
            case 4: return 4u | 8u | 2u << 4;      // SackPermitted
            case 5: return 5u | 2u << 4;           // Sack
            case 8: return 6u | 8u | 10u << 4;     // Timestamp
            case 34: return 7u | 2u << 4;          // FastOpen
            default: return 0u;
        }
    }
    switch (t) {
        case 68: return 2u | 4u << 4;              // Timestamp
        case 7: return 3u | 3u << 4;               // RecordRoute
        case 148: return 4u | 8u | 4u << 4;        // RouteAlert
        case 134: return 5u | 6u << 4;             // CommercialSecurity
        case 137: return 6u | 8u | 7u << 4;        // StrictSourceRoute
        case 131: return 7u | 8u | 7u << 4;        // LooseSourceRoute
        default: return 0u;
    }
}

// The same rules computed in registers (no dependent LDS read per step): the kind index
// by compares, then the length and the fixed flag from per-kind nibble / bit tables.
#ifndef RPKT_OPT_RULE_ALU
#define RPKT_OPT_RULE_ALU 0      // 1: opt_rule_alu in the paired walk instead of the LDS table
#endif
__device__ __forceinline__ uint32_t opt_rule_alu(bool tcp, uint32_t t) {
    uint32_t k;
    if (tcp) {
        k = t == 2u ? 2u : t == 3u ? 3u : t == 4u ? 4u : t == 5u ? 5u : t == 8u ? 6u : t == 34u ? 7u : 0u;
    } else {
        k = t == 68u ? 2u : t == 7u ? 3u : t == 148u ? 4u : t == 134u ? 5u : t == 137u ? 6u
          : t == 131u ? 7u : 0u;
    }
    // X per kind index 2..7 (nibble k) and fixed (bit k), as opt_rule's table
    const uint32_t xs = tcp ? 0x2a223400u : 0x77643400u;
    const uint32_t fx = tcp ? 0x5cu : 0xd0u;
    const uint32_t x = (xs >> (4u * k)) & 15u;
    return k == 0u ? 0u : (k | (((fx >> k) & 1u) << 3) | (x << 4));
}

// Both iterators' rule tables (IPv4: [0, 256), TCP: [256, 512)) into the block's LDS;
// the caller synchronises the block before the walks read them.
__device__ __forceinline__ void opt_rules_fill(uint8_t* rules) {
    for (uint32_t t = threadIdx.x; t < 256u; t += blockDim.x) {   // any block size
        rules[t] = (uint8_t)opt_rule(false, t);
        rules[256 + t] = (uint8_t)opt_rule(true, t);
    }
}

// option length (> 0), 0 = the type's parse fails (malformed), -1 = unknown type
__device__ __forceinline__ int opt_len(uint32_t rule, uint32_t d0, uint32_t n, int& kind) {
    const uint32_t hl = n >= 2 ? (d0 >> 8) & 0xffu : 0u;
    const uint32_t x = rule >> 4;
    const bool fixed = (rule & 8u) != 0u;
    const bool ok = (n >= x) & (fixed ? hl == x : (hl >= x) & (hl <= n));
    kind = (int)(rule & 7u);
    return (rule & 7u) == 0u ? -1 : (ok ? (int)(fixed ? x : hl) : 0);
}

// One step of a TLV walk (state of Ipv4OptionsIter / TcpOptionsIter): the two walks of
// a frame are independent, so the kernel steps both in one loop and their LDS round
// trips overlap.
struct OptWalk {
    uint32_t lo, nb, pos, cnt, kinds, stop;
    uint64_t trace;
    bool on;
};

// A run of one-byte options of one type (EOL = kind 0, NOP = kind 1 in both iterators:
// each is an option of length 1 and the walk goes on) is consumed up to four at a
// time from the dword at the cursor: padding runs are most of a walk's steps.
__device__ __forceinline__ bool opt_run(OptWalk& w, uint32_t d0) {
    const uint32_t t0 = d0 & 0xffu;
    if (t0 > 1u) return false;
    const uint32_t x = d0 ^ (t0 ? 0x01010101u : 0u);   // zero bytes: the same type
    uint32_t k = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4u;
    k = k < w.nb - w.pos ? k : w.nb - w.pos;            // >= 1: byte 0 matches
    w.kinds |= 1u << t0;
    if (w.cnt < 16) {
        const uint32_t nib = (t0 ? 0x2222u : 0x1111u) & ((1u << (4 * k)) - 1u);   // k <= 4
        w.trace |= (uint64_t)nib << (4 * w.cnt);
    }
    w.cnt += k;
    w.pos += k;
    w.on = w.pos < w.nb;
    return true;
}

// The option slices of a parsed frame (what the walks read from its record): the IPv4
// slice [l3 + 20, l4) when IPv4 parsed, the TCP slice [l4 + 20, l4 + doff4) when the
// frame parsed OK as TCP (include/rpkt_gpu.h, rpkt_gpu_options_batch).
struct OptSlices {
    bool ip_parsed, tcp;
    uint32_t ip_lo, ip_hi, t_lo, t_hi;
    uint32_t need_lo, need_hi;     // frame bytes both walks read: [need_lo, need_hi)
    bool need;
    bool ip6;                      // IPv6 header parsed: the IPv6 option walk (ip6_walk_row)
    uint32_t l3, l4;               //   over the extension chain [l3 + 40, l4)
    uint32_t nh0;                  // its first next_header (frame byte l3 + 6) when the caller
};                                 //   has it (record word 7), else 256: read from the frame

// is6: an IPv6 record (RPKT_F_IPV6): no IPv4 option slice; its TCP slice as any other
__device__ __forceinline__ OptSlices opt_slices(uint32_t status, uint32_t proto, uint32_t l3,
                                                uint32_t l4, uint32_t doff4, bool is6) {
    OptSlices S;
    S.ip_parsed = !is6 && (status == RPKT_S_OK ||
                           (status >= RPKT_S_L4_OTHER && status <= RPKT_S_TCP_BAD_DOFF) ||
                           status == RPKT_S_ICMP_EMPTY);
    S.tcp = status == RPKT_S_OK && proto == 6u;
    S.ip_lo = l3 + 20u;
    S.ip_hi = S.ip_parsed ? l4 : S.ip_lo;
    S.t_lo = l4 + 20u;
    S.t_hi = S.tcp ? l4 + doff4 : S.t_lo;
    S.need_lo = S.ip_hi > S.ip_lo ? S.ip_lo : S.t_lo;
    S.need_hi = S.t_hi > S.t_lo ? S.t_hi : S.ip_hi;
    S.need = (S.ip_hi > S.ip_lo) || (S.t_hi > S.t_lo);
    S.ip6 = is6 && status != RPKT_S_IP6_SHORT && status != RPKT_S_IP6_BAD_LEN;
    S.l3 = l3;
    S.l4 = l4;
    S.nh0 = 256u;
    return S;
}

// Frame bytes [x, x + 4) of a lane's frame as a little-endian dword for the IPv6 option
// walk: from the lane's LDS slot when they lie in the frame range [lo, hi) the slot holds
// (frame byte x at slot[x + bias]), else from global memory.  An empty range (lo == hi)
// reads everything from memory.
struct OptDw {
    const uint8_t* slot;
    uint32_t bias, lo, hi, fo, fb;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ uint32_t operator()(uint32_t x) const {
        if (x >= lo && x + 4u <= hi) {
            const uint32_t y = x + bias, a = y & ~3u;
            return align_bytes(lds32(slot, a + 4u), lds32(slot, a), y & 3u);
        }
        return gdword(rs, fb, fo + x);
    }
};

// The IPv6 half of a frame's rpkt_opts_t (Ipv6OptionsIter over every HopByHop /
// DestOptions header of [l3 + 40, l4)): words 7..10, the trace (14, 15) and byte 27.
struct Ip6Opts {
    uint32_t w7, w8, w9, w10, tr_lo, tr_hi, end;
};

__device__ __forceinline__ Ip6Opts ip6_walk(const OptDw& dw, uint32_t l3, uint32_t l4, uint32_t nh0) {
    uint32_t nh = nh0 < 256u ? nh0 : (dw(l3 + 4u) >> 16) & 0xffu;  // next_header, byte 6
    uint32_t c = l3 + 40u;
    uint32_t cnt = 0, kinds = 0, stop = RPKT_OPT_NONE, end = 0, ra = 0, gt = 0, gl = 0, gd = 0;
    uint32_t nhdr = 0, first = 0;
    uint64_t trace = 0;
    for (int k = 0; k < RPKT_MAX_IP6_EXT && c < l4; ++k) {
        const uint32_t d0 = dw(c);
        const uint32_t b1 = (d0 >> 8) & 0xffu;
        const uint32_t hl = nh == 44u ? 8u : (nh == 51u ? b1 * 4u + 8u : b1 * 8u + 8u);
        if (nh == 0u || nh == 60u) {
            first = nhdr == 0u ? nh : first;
            nhdr += 1u;
            stop = RPKT_OPT_END;
            const uint32_t s0 = c + 2u, nb = hl - 2u;
            uint32_t pos = 0;
            while (pos < nb) {
                const uint32_t d = dw(s0 + pos);
                const uint32_t t = d & 0xffu, rem = nb - pos;
                if (t == 0u) {                          // a run of Pad0 (up to 4 bytes)
                    uint32_t kz = d ? (uint32_t)__builtin_ctz(d) >> 3 : 4u;
                    kz = kz < rem ? kz : rem;
                    kinds |= 1u;
                    trace |= cnt < 16u ? (uint64_t)(0x1111u & ((1u << (4u * kz)) - 1u)) << (4u * cnt)
                                       : 0ull;
                    cnt += kz;
                    pos += kz;
                    continue;
                }
                const uint32_t ln = ((d >> 8) & 0xffu) + 2u;             // header_len
                const bool ok = t == 5u ? (rem >= 4u && ln == 4u) : (rem >= 2u && ln <= rem);
                if (!ok) {
                    stop = RPKT_OPT_MALFORMED;
                    break;
                }
                const uint32_t kind = t == 1u ? 1u : (t == 5u ? 2u : 3u);
                if (kind == 2u) ra = be16_hi(d);                         // router_alert
                if (kind == 3u) {                                        // Generic: type_,
                    gt = t;                                              // data length, the
                    gl = ln - 2u;                                        // slice's first bytes
                    const uint32_t v = bswap32(dw(s0 + pos + 2u));
                    gd = gl >= 4u ? v : v & ~(0xffffffffu >> (8u * gl));
                }
                kinds |= 1u << kind;
                trace |= cnt < 16u ? (uint64_t)(kind + 1u) << (4u * cnt) : 0ull;
                cnt += 1u;
                pos += ln;
            }
            end = pos;
            if (stop == RPKT_OPT_MALFORMED) break;
        }
        nh = d0 & 0xffu;
        c += hl;
    }
    return Ip6Opts{(cnt & 0xffu) | (stop << 8) | (kinds << 16), ra | (gt << 16) | (gl << 24),
                   nhdr | (first << 8), gd, (uint32_t)trace, (uint32_t)(trace >> 32), end};
}

// One HopByHop / DestOptions header's option walk (the inner loop of ip6_walk) from a
// fresh count: what the frame's walk adds for this header.
struct Ip6Hdr {
    uint32_t cnt, kinds, end, ra, g, gd;        // g: type_ | data length << 8 of a Generic
    uint64_t trace;
    bool mal, has_ra, has_g;
};
// RPKT_IP6_STEP2: a step takes a Pad0 run and the option after it (as the IPv4 / TCP
// walks' step does), instead of one step each.
#ifndef RPKT_IP6_STEP2
#define RPKT_IP6_STEP2 1
#endif
__device__ __forceinline__ Ip6Hdr ip6_hdr_walk(const OptDw& dw, uint32_t c, uint32_t hl) {
    Ip6Hdr R{0u, 0u, 0u, 0u, 0u, 0u, 0ull, false, false, false};
    const uint32_t s0 = c + 2u, nb = hl - 2u;
    uint32_t pos = 0;
    while (pos < nb) {
        uint32_t d = dw(s0 + pos);
        uint32_t t = d & 0xffu, rem = nb - pos;
        if (t == 0u) {                                  // a run of Pad0 (up to 4 bytes)
            uint32_t kz = d ? (uint32_t)__builtin_ctz(d) >> 3 : 4u;
            kz = kz < rem ? kz : rem;
            R.kinds |= 1u;
            R.trace |= R.cnt < 16u ? (uint64_t)(0x1111u & ((1u << (4u * kz)) - 1u)) << (4u * R.cnt)
                                   : 0ull;
            R.cnt += kz;
            pos += kz;
            // a run shorter than 4 that the header does not cut ends at an option
            if (!RPKT_IP6_STEP2 || kz == 4u || pos >= nb) continue;
            d = dw(s0 + pos);
            t = d & 0xffu;
            rem = nb - pos;
        }
        const uint32_t ln = ((d >> 8) & 0xffu) + 2u;                     // header_len
        const bool ok = t == 5u ? (rem >= 4u && ln == 4u) : (rem >= 2u && ln <= rem);
        if (!ok) {
            R.mal = true;
            break;
        }
        const uint32_t kind = t == 1u ? 1u : (t == 5u ? 2u : 3u);
        if (kind == 2u) {                                                // router_alert
            R.ra = be16_hi(d);
            R.has_ra = true;
        }
        if (kind == 3u) {                               // Generic: type_, data length, the
            const uint32_t gl = ln - 2u;                // slice's first bytes
            const uint32_t v = bswap32(dw(s0 + pos + 2u));
            R.g = t | (gl << 8);
            R.gd = gl >= 4u ? v : v & ~(0xffffffffu >> (8u * gl));
            R.has_g = true;
        }
        R.kinds |= 1u << kind;
        R.trace |= R.cnt < 16u ? (uint64_t)(kind + 1u) << (4u * R.cnt) : 0ull;
        R.cnt += 1u;
        pos += ln;
    }
    R.end = pos;
    return R;
}

// The IPv6 walks of the wave's IPv6 frames, while their windows are still in LDS (before
// the rows are staged over them); a frame's bytes outside the window come from memory.
// RPKT_IP6_DIST: a frame's walk is a chain of headers, each HopByHop / DestOptions one an
// option walk of its own, and a wave used to step those option walks frame by frame:
// header k of every frame, as many iterations as the frame with the most options in it
// (config 11: 16.3 iterations per wave, by a count over its frames).  Here each lane first
// walks its frame's header chain alone (one read per header), the wave's option headers
// (19 per wave on config 11) are dealt out one per lane, walked at once (as many
// iterations as the longest one: 5.8), and each frame folds its headers' results in chain
// order -- counts and trace offsets add up, the last RouterAlert / Generic wins, the first
// malformed header ends the walk.  A frame with more than kIp6Dist option headers walks
// them itself, as before.
#ifndef RPKT_IP6_DIST
#define RPKT_IP6_DIST 1
#endif
constexpr uint32_t kIp6Dist = 3;
__device__ __forceinline__ Ip6Opts ip6_walks(const OptSlices& S, const OptDw& dw) {
    Ip6Opts v{0u, 0u, 0u, 0u, 0u, 0u, 0u};
#if !RPKT_IP6_DIST
    if (__ballot(S.ip6) != 0 && S.ip6) v = ip6_walk(dw, S.l3, S.l4, S.nh0);
    return v;
#else
    // frames without extension headers have nothing to walk: their words are zero
    const bool w = S.ip6 && S.l4 > S.l3 + 40u;
    if (__ballot(w) == 0) return v;
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    // the frame's header chain: where its first kIp6Dist option headers start, and their
    // lengths (the same loop as ip6_walk's, without the option steps)
    uint32_t hc0 = 0, hc1 = 0, hc2 = 0, hh0 = 0, hh1 = 0, hh2 = 0, nopt = 0, first = 0;
    if (w) {
        uint32_t nh = S.nh0 < 256u ? S.nh0 : (dw(S.l3 + 4u) >> 16) & 0xffu;
        uint32_t c = S.l3 + 40u;
        for (int k = 0; k < RPKT_MAX_IP6_EXT && c < S.l4; ++k) {
            const uint32_t d0 = dw(c);
            const uint32_t b1 = (d0 >> 8) & 0xffu;
            const uint32_t hl = nh == 44u ? 8u : (nh == 51u ? b1 * 4u + 8u : b1 * 8u + 8u);
            if (nh == 0u || nh == 60u) {
                hc0 = nopt == 0u ? c : hc0;
                hh0 = nopt == 0u ? hl : hh0;
                hc1 = nopt == 1u ? c : hc1;
                hh1 = nopt == 1u ? hl : hh1;
                hc2 = nopt == 2u ? c : hc2;
                hh2 = nopt == 2u ? hl : hh2;
                first = nopt == 0u ? nh : first;
                nopt += 1u;
            }
            nh = d0 & 0xffu;
            c += hl;
        }
    }
    const bool serial = w && nopt > kIp6Dist;
    const uint32_t m = w && !serial ? nopt : 0u;
    // entries: frame l's option headers are P_l .. P_l + m_l - 1 (an exclusive scan of m)
    uint32_t inc = m;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, d, kWave);
        inc += lane >= (uint32_t)d ? y : 0u;
    }
    const uint32_t P = inc - m;
    const uint32_t total = (uint32_t)__shfl((int)inc, kWave - 1, kWave);
    const uint64_t slot = (uint64_t)(uintptr_t)dw.slot;
    uint32_t cnt = 0, kinds = 0, stop = RPKT_OPT_NONE, end = 0, ra = 0, g = 0, gd = 0, nhdr = 0;
    uint64_t trace = 0;
    bool stopped = false;
    for (uint32_t r0 = 0; r0 < total; r0 += (uint32_t)kWave) {          // wave-uniform
        // entry E = r0 + lane: its frame is the last lane l with P_l <= E
        const uint32_t E = r0 + lane;
        uint32_t l = 0;
#pragma unroll
        for (uint32_t st = kWave / 2; st >= 1u; st >>= 1) {
            const uint32_t p = (uint32_t)__shfl((int)P, (int)(l + st), kWave);
            l = p <= E ? l + st : l;
        }
        const uint32_t j = E - (uint32_t)__shfl((int)P, (int)l, kWave);
        const uint32_t c0 = (uint32_t)__shfl((int)hc0, (int)l, kWave);
        const uint32_t c1 = (uint32_t)__shfl((int)hc1, (int)l, kWave);
        const uint32_t c2 = (uint32_t)__shfl((int)hc2, (int)l, kWave);
        const uint32_t h0 = (uint32_t)__shfl((int)hh0, (int)l, kWave);
        const uint32_t h1 = (uint32_t)__shfl((int)hh1, (int)l, kWave);
        const uint32_t h2 = (uint32_t)__shfl((int)hh2, (int)l, kWave);
        OptDw de = dw;                                  // frame l's window and offset
        de.slot = reinterpret_cast<const uint8_t*>(
            (uintptr_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)(slot >> 32), (int)l, kWave) << 32) |
                        (uint32_t)__shfl((int)(uint32_t)slot, (int)l, kWave)));
        de.bias = (uint32_t)__shfl((int)dw.bias, (int)l, kWave);
        de.lo = (uint32_t)__shfl((int)dw.lo, (int)l, kWave);
        de.hi = (uint32_t)__shfl((int)dw.hi, (int)l, kWave);
        de.fo = (uint32_t)__shfl((int)dw.fo, (int)l, kWave);
        Ip6Hdr R{0u, 0u, 0u, 0u, 0u, 0u, 0ull, false, false, false};
        if (E < total)
            R = ip6_hdr_walk(de, j == 0u ? c0 : (j == 1u ? c1 : c2), j == 0u ? h0 : (j == 1u ? h1 : h2));
        // each frame folds its entries of this round, in chain order
        const uint32_t flags = (R.mal ? 1u : 0u) | (R.has_ra ? 2u : 0u) | (R.has_g ? 4u : 0u);
#pragma unroll
        for (uint32_t jj = 0; jj < kIp6Dist; ++jj) {
            const uint32_t Eo = P + jj;
            const bool mine = jj < m && Eo >= r0 && Eo < r0 + (uint32_t)kWave;
            const int src = (int)((Eo - r0) & (uint32_t)(kWave - 1));
            const uint32_t rc = (uint32_t)__shfl((int)R.cnt, src, kWave);
            const uint32_t rk = (uint32_t)__shfl((int)R.kinds, src, kWave);
            const uint32_t re = (uint32_t)__shfl((int)R.end, src, kWave);
            const uint32_t rr = (uint32_t)__shfl((int)R.ra, src, kWave);
            const uint32_t rg = (uint32_t)__shfl((int)R.g, src, kWave);
            const uint32_t rd = (uint32_t)__shfl((int)R.gd, src, kWave);
            const uint32_t rf = (uint32_t)__shfl((int)flags, src, kWave);
            const uint32_t tl = (uint32_t)__shfl((int)(uint32_t)R.trace, src, kWave);
            const uint32_t th = (uint32_t)__shfl((int)(uint32_t)(R.trace >> 32), src, kWave);
            if (mine && !stopped) {
                const uint64_t rt = ((uint64_t)th << 32) | tl;
                trace |= cnt < 16u ? rt << (4u * cnt) : 0ull;
                cnt += rc;
                kinds |= rk;
                ra = (rf & 2u) ? rr : ra;
                g = (rf & 4u) ? rg : g;
                gd = (rf & 4u) ? rd : gd;
                end = re;
                nhdr += 1u;
                stopped = (rf & 1u) != 0u;
                stop = stopped ? (uint32_t)RPKT_OPT_MALFORMED : (uint32_t)RPKT_OPT_END;
            }
        }
    }
    if (w && !serial)
        v = Ip6Opts{(cnt & 0xffu) | (stop << 8) | (kinds << 16), ra | ((g & 0xffu) << 16) | ((g >> 8) << 24),
                    nhdr | (first << 8), gd, (uint32_t)trace, (uint32_t)(trace >> 32), end};
    if (__ballot(serial) != 0 && serial) v = ip6_walk(dw, S.l3, S.l4, S.nh0);
    return v;
#endif
}

// The two walks (Ipv4OptionsIter::next, ipv4/generated.rs:1640-1722;
// TcpOptionsIter::next, tcp/generated.rs:1400-1484), stepped together, into the 16
// words of rpkt_opts_t (include/rpkt_gpu.h).  rules: opt_rules_fill's table.
__device__ __forceinline__ void walk_options(const OptWin& s, const OptSlices& S,
                                             const uint8_t* rules, uint32_t (&o)[16]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0;
    OptWalk ip{S.ip_lo, S.ip_hi - S.ip_lo, 0, 0, 0, RPKT_OPT_END, 0, S.ip_parsed && S.ip_hi > S.ip_lo};
    OptWalk tw{S.t_lo, S.t_hi - S.t_lo, 0, 0, 0, RPKT_OPT_END, 0, S.tcp && S.t_hi > S.t_lo};
    while (ip.on || tw.on) {
        if (ip.on) {
            const uint32_t at = ip.lo + ip.pos;
            const uint32_t d0 = s.dw(at);
            int kind = 0;
            const int used = opt_run(ip, d0) ? -2 : opt_len(rules[d0 & 0xffu], d0, ip.nb - ip.pos, kind);
            if (used == -2) {
            } else if (used <= 0) {
                ip.stop = used < 0 ? RPKT_OPT_UNKNOWN : RPKT_OPT_MALFORMED;
                ip.on = false;
            } else {
                if (kind == 2) o[9] = (o[9] & 0xff000000u) | (d0 >> 8);
                if (kind == 3) o[8] = (o[8] & 0xffffu) | ((d0 >> 8) << 16);
                if (kind == 4) o[8] = (o[8] & 0xffff0000u) | be16_hi(d0);
                if (kind == 5) o[11] = s.be32(at + 2);
                if (kind == 6 || kind == 7) {
                    o[9] = (o[9] & 0x00ffffffu) | ((d0 >> 16) << 24);
                    o[10] = s.be32(at + 3);
                }
                ip.kinds |= 1u << kind;
                if (ip.cnt < 16) ip.trace |= (uint64_t)(kind + 1) << (4 * ip.cnt);
                ip.cnt += 1;
                ip.pos += (uint32_t)used;
                ip.on = ip.pos < ip.nb;
            }
        }
        if (tw.on) {
            const uint32_t at = tw.lo + tw.pos;
            const uint32_t d0 = s.dw(at);
            int kind = 0;
            const int used = opt_run(tw, d0) ? -2 : opt_len(rules[256 + (d0 & 0xffu)], d0, tw.nb - tw.pos, kind);
            if (used == -2) {
            } else if (used <= 0) {
                tw.stop = used < 0 ? RPKT_OPT_UNKNOWN : RPKT_OPT_MALFORMED;
                tw.on = false;
            } else {
                if (kind == 2) o[1] = (o[1] & 0xffffu) | (be16_hi(d0) << 16);
                if (kind == 3) o[0] = (o[0] & 0xff00ffffu) | (((d0 >> 16) & 0xffu) << 16);
                if (kind == 5) {
                    const uint32_t hl = (d0 >> 8) & 0xffu;
                    o[0] = (o[0] & 0x00ffffffu) | (((hl - 2u) / 8u) << 24);
                    o[4] = hl >= 6u ? s.be32(at + 2) : 0u;
                    o[5] = hl >= 10u ? s.be32(at + 6) : 0u;
                }
                if (kind == 6) {
                    o[2] = s.be32(at + 2);
                    o[3] = s.be32(at + 6);
                }
                if (kind == 7) o[6] = (o[6] & 0xffff0000u) | ((d0 >> 8) & 0xffu);
                tw.kinds |= 1u << kind;
                if (tw.cnt < 16) tw.trace |= (uint64_t)(kind + 1) << (4 * tw.cnt);
                tw.cnt += 1;
                tw.pos += (uint32_t)used;
                tw.on = tw.pos < tw.nb;
            }
        }
    }
    if (S.ip_parsed) {
        // word 6: tcp_fo_len | tcp_end << 16 | ip_end << 24; word 7: ip_count | ip_stop << 8 | ip_kinds << 16
        o[6] |= ip.pos << 24;
        o[7] = ip.cnt | (ip.stop << 8) | (ip.kinds << 16);
    }
    if (S.tcp) {
        // word 0: tcp_count | tcp_stop << 8 | wscale << 16 | sack_blocks << 24; word 1: kinds | mss << 16
        o[0] = (o[0] & 0xffff0000u) | tw.cnt | (tw.stop << 8);
        o[1] = (o[1] & 0xffff0000u) | tw.kinds;
        o[6] = (o[6] & 0xff00ffffu) | (tw.pos << 16);
    }
    const uint64_t tcp_trace = tw.trace, ip_trace = ip.trace;
    o[12] = (uint32_t)tcp_trace;
    o[13] = (uint32_t)(tcp_trace >> 32);
    o[14] = (uint32_t)ip_trace;
    o[15] = (uint32_t)(ip_trace >> 32);
}

// The IPv6 half of one frame's row staged in LDS (`row`, 17-dword stride), for lanes whose
// frame is IPv6; the wave synchronises before and after (other lanes wrote the rows).
__device__ __forceinline__ void ip6_patch_rows(uint32_t* st, int lane, const OptSlices& S,
                                               const Ip6Opts& v) {
    if (__ballot(S.ip6) == 0) return;                          // wave-uniform
    wave_sync();
    if (S.ip6) {
        uint32_t* row = st + lane * 17;
        row[7] = v.w7;
        row[8] = v.w8;
        row[9] = v.w9;
        row[10] = v.w10;
        row[11] = 0u;
        row[14] = v.tr_lo;
        row[15] = v.tr_hi;
        reinterpret_cast<uint8_t*>(row)[27] = (uint8_t)v.end;
    }
    wave_sync();
}

// ---- paired walks: one iterator step per lane per iteration ----
// walk_options steps a frame's two walks together, so every loop iteration runs both
// step bodies and a wave runs until its longest walk of either kind ends (config 5: 14.1
// iterations of two bodies per 64-frame wave, 6.6 walk steps per frame).  Here a lane
// runs ONE walk at a time with one step body for both iterators (the kind index carries
// the iterator): first its own frame's TCP walk, then the IPv4 walk of a frame chosen so
// that long TCP slices meet short IPv4 slices -- lanes ranked by TCP slice length
// (descending) take the IPv4 walks ranked by slice length (ascending), the k-th with the
// k-th.  Config 5: 15.3 iterations of one body per wave (a model over its frames), about
// half the step bodies.  Each lane holds its own frame's TCP words and its partner's
// IPv4 words of rpkt_opts_t (disjoint words but word 6); both reach their rows through
// the LDS stage.
//
// rank of this lane's key among the wave's keys (0..10), ascending or descending,
// ties by lane: a permutation of 0..63
__device__ __forceinline__ uint32_t wave_rank11(uint32_t key, bool descending) {
    uint32_t rank = 0, base = 0;
#pragma unroll
    for (uint32_t v = 0; v < 11; ++v) {
        const uint32_t b = descending ? 10u - v : v;
        const uint64_t m = __ballot(key == b);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (key == b) rank = base + below;
        base += (uint32_t)__builtin_popcountll(m);
    }
    return rank;
}

// One iterator's walk over the option bytes at LDS offsets [at, end) of `win`.
struct OptCur {
    uint32_t at, end, base, cnt, kinds, stop;
    uint64_t trace;
};

// Both slices of this lane's frame as LDS offsets in `win` (slot_off + bias + frame
// offset), the TCP walk kept, the IPv4 walk handed to the partner lane.  Results go to
// the stage rows (stride 17 dwords) in `win` once every walk of the wave has ended.
__device__ __forceinline__ void walk_options_paired(uint8_t* win, int lane, uint32_t slot_bias,
                                                    const OptSlices& S, const uint8_t* rules,
                                                    rpkt_opts_t* opts, uint32_t p0, uint32_t n,
                                                    const OptDw& d6) {
    // (a lane past the batch end may hold a zero record: status OK, l4 = 0, so a slice
    // can come out "negative"; it is empty, as walk_options' `on` flags treat it)
    const uint32_t t_nb = S.tcp && S.t_hi > S.t_lo ? S.t_hi - S.t_lo : 0u;
    const uint32_t ip_nb = S.ip_parsed && S.ip_hi > S.ip_lo ? S.ip_hi - S.ip_lo : 0u;
    // the partner frame q of this lane: rank by TCP bytes (desc) == q's rank by IPv4 bytes
    // (asc); slices are at most 40 B (keys 0..10), the clamp keeps the ranks a permutation
    const uint32_t rt = wave_rank11(min(t_nb >> 2, 10u), true);
    const uint32_t ri = wave_rank11(min(ip_nb >> 2, 10u), false);
    const int q = __builtin_amdgcn_ds_bpermute((int)(rt << 2),
                                               __builtin_amdgcn_ds_permute((int)(ri << 2), lane));
    const uint32_t ip_at = (uint32_t)__shfl((int)(slot_bias + S.ip_lo), q, kWave);
    const uint32_t ip_n = (uint32_t)__shfl((int)ip_nb, q, kWave);
    const bool ip_has = __shfl((int)S.ip_parsed, q, kWave) != 0;

    uint32_t o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0;
    uint32_t ip_end = 0;
#if RPKT_OPT_DEFER
    // One branch-free step body: an EOL/NOP run or a TLV option, and the getters deferred:
    // a step records only where the last option of its kind starts (a byte per kind,
    // kinds 2..7: positions 0..3 in P0, 4..5 in P1), and the getters of both walks are
    // read from LDS once, after the loop, at those positions.  The per-kind getter code
    // inside the loop was a divergent branch tree executed every step.
    uint32_t phase = S.tcp ? 0u : (ip_has ? 1u : 2u);
    uint32_t at = phase == 0 ? slot_bias + S.t_lo : ip_at;
    uint32_t base = at, end = at + (phase == 0 ? t_nb : ip_n);
    uint32_t cnt = 0, kinds = 0, stop = RPKT_OPT_END, P0 = 0, P1 = 0, T0 = 0, T1 = 0;
    uint64_t trace = 0;
    uint32_t t_cnt = 0, t_kinds = 0, t_stop = 0, t_pos = 0;
    uint64_t t_trace = 0;
    while (phase < 2u) {
        const bool tcp = phase == 0u;
#if RPKT_OPT_STEP2
        // a step takes an EOL/NOP run (<= 4 of one type) at the cursor AND the TLV option
        // right after it, if one follows: the walks alternate padding and options (config
        // 5: 15.3 -> 13.1 iterations per wave in a model of its frames)
        if (at < end) {
            const uint32_t a4 = at & ~3u, sh = at & 3u;
            const uint32_t R0 = lds32(win, a4), R1 = lds32(win, a4 + 4u), R2 = lds32(win, a4 + 8u);
            const uint32_t d0 = align_bytes(R1, R0, sh), d1 = align_bytes(R2, R1, sh);
            const uint32_t t0 = d0 & 0xffu;
            const uint32_t nrem = end - at;
            const bool run = t0 <= 1u;
            const uint32_t x = d0 ^ (t0 ? 0x01010101u : 0u);
            uint32_t kr = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4u;
            kr = kr < nrem ? kr : nrem;
            const uint32_t k = run ? kr : 0u;                  // run bytes this step
            const uint32_t e0 = k == 4u ? d1 : align_bytes(d1, d0, k);
            const uint32_t at2 = at + k, nrem2 = nrem - k;
            const uint32_t t2 = e0 & 0xffu, hl = (e0 >> 8) & 0xffu;
            const bool tlv = (nrem2 != 0u) & (t2 > 1u);       // a TLV option follows
            const uint32_t rule = rules[(tcp ? 256u : 0u) + t2];
            const uint32_t X = rule >> 4, kind = rule & 7u;
            const bool fixed = (rule & 8u) != 0u;
            const bool ok = (kind != 0u) & (nrem2 >= X) & (hl - X <= (fixed ? 0u : nrem2 - X));
            const bool took = tlv & ok;
            const uint32_t runnib = (t0 + 1u) * (0x1111u & ((1u << (4u * k)) - 1u));
            const uint32_t nibs = runnib | (took ? (kind + 1u) << (4u * k) : 0u);
            kinds |= (run ? 1u << t0 : 0u) | (took ? 1u << kind : 0u);
            trace |= cnt < 16u ? (uint64_t)nibs << (4u * cnt) : 0ull;
            // the TLV's start, as a byte at kind - 2 of P0 / P1 (kinds 2..7)
            const uint32_t kp = kind - 2u, sb = 8u * (kp & 3u);
            const uint32_t v = (at2 - base) << sb, m = 0xffu << sb;
            P0 = (took && kp < 4u) ? (P0 & ~m) | v : P0;
            P1 = (took && kp >= 4u) ? (P1 & ~m) | v : P1;
            cnt += k + (took ? 1u : 0u);
            const bool fail = tlv & !ok;
            stop = fail ? (kind == 0u ? (uint32_t)RPKT_OPT_UNKNOWN : (uint32_t)RPKT_OPT_MALFORMED) : stop;
            end = fail ? at2 : end;
            at = at2 + (took ? (fixed ? X : hl) : 0u);
        }
#else
        if (at < end) {
            const uint32_t a4 = at & ~3u;
            const uint32_t d0 = align_bytes(lds32(win, a4 + 4u), lds32(win, a4), at & 3u);
            const uint32_t t = d0 & 0xffu, hl = (d0 >> 8) & 0xffu;
            const uint32_t nrem = end - at;
            const uint32_t rule = rules[(tcp ? 256u : 0u) + t];
            const bool run = t <= 1u;
            const uint32_t x = d0 ^ (t ? 0x01010101u : 0u);
            uint32_t kr = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4u;
            kr = kr < nrem ? kr : nrem;
            const uint32_t X = rule >> 4, kind = rule & 7u;
            const bool fixed = (rule & 8u) != 0u;
            const bool ok = run | ((kind != 0u) & (nrem >= X) & (hl - X <= (fixed ? 0u : nrem - X)));
            const uint32_t nn = run ? kr : 1u;                 // options this step yields
            const uint32_t code = run ? t + 1u : kind + 1u;   // trace nibble
            const uint32_t nibs = code * (0x1111u & ((1u << (4u * nn)) - 1u));
            const uint32_t kb = run ? t : kind;
            kinds |= ok ? 1u << kb : 0u;
            trace |= (ok && cnt < 16u) ? (uint64_t)nibs << (4u * cnt) : 0ull;
            // the TLV's start, as a byte at kind - 2 of P0 / P1 (kinds 2..7)
            const uint32_t kp = kind - 2u, sh = 8u * (kp & 3u);
            const bool rec = ok & !run;
            const uint32_t v = (at - base) << sh, m = 0xffu << sh;
            P0 = (rec && kp < 4u) ? (P0 & ~m) | v : P0;
            P1 = (rec && kp >= 4u) ? (P1 & ~m) | v : P1;
            cnt += ok ? nn : 0u;
            stop = ok ? stop : (kind == 0u ? (uint32_t)RPKT_OPT_UNKNOWN : (uint32_t)RPKT_OPT_MALFORMED);
            const uint32_t adv = run ? kr : (fixed ? X : hl);
            end = ok ? end : at;
            at = ok ? at + adv : at;
        }
#endif  // RPKT_OPT_STEP2
        if (at >= end) {                                       // this walk ended
            if (tcp) {
                t_cnt = cnt, t_kinds = kinds, t_stop = stop, t_pos = at - base, t_trace = trace;
                T0 = P0, T1 = P1;
                phase = ip_has ? 1u : 2u;
                base = at = ip_at;
                end = ip_at + ip_n;
                cnt = kinds = P0 = P1 = 0;
                stop = RPKT_OPT_END;
                trace = 0;
            } else {
                phase = 2u;
            }
        }
    }
    // the getters of the last option of each kind, from its recorded start: 12 bytes at
    // `a` (the options read at most bytes a .. a + 9)
    auto bytes12 = [&](uint32_t a, uint32_t& d0, uint32_t& d1, uint32_t& d2) {
        const uint32_t a4 = a & ~3u, sh = a & 3u;
        const uint32_t R0 = lds32(win, a4), R1 = lds32(win, a4 + 4u);
        const uint32_t R2 = lds32(win, a4 + 8u), R3 = lds32(win, a4 + 12u);
        d0 = align_bytes(R1, R0, sh);
        d1 = align_bytes(R2, R1, sh);
        d2 = align_bytes(R3, R2, sh);
    };
    const uint32_t tb = slot_bias + S.t_lo;                    // TCP: this lane's frame
    if (S.tcp) {
        // word 0: tcp_count | tcp_stop << 8 | wscale << 16 | sack_blocks << 24;
        // word 1: kinds | mss << 16; word 6: tcp_fo_len | tcp_end << 16
        o[0] = t_cnt | (t_stop << 8);
        o[1] = t_kinds;
        o[6] = t_pos << 16;
        o[12] = (uint32_t)t_trace;
        o[13] = (uint32_t)(t_trace >> 32);
    }
    uint32_t d0, d1, d2;
    if (__ballot(t_kinds & (1u << 2))) {                      // Mss
        bytes12(tb + (T0 & 0xffu), d0, d1, d2);
        if (t_kinds & (1u << 2)) o[1] |= be16_hi(d0) << 16;
    }
    if (__ballot(t_kinds & (1u << 3))) {                      // WindowScale
        bytes12(tb + ((T0 >> 8) & 0xffu), d0, d1, d2);
        if (t_kinds & (1u << 3)) o[0] |= ((d0 >> 16) & 0xffu) << 16;
    }
    if (__ballot(t_kinds & (1u << 5))) {                      // Sack
        bytes12(tb + (T0 >> 24), d0, d1, d2);
        if (t_kinds & (1u << 5)) {
            const uint32_t h = (d0 >> 8) & 0xffu;
            o[0] |= ((h - 2u) >> 3) << 24;
            o[4] = h >= 6u ? bswap32(align_bytes(d1, d0, 2)) : 0u;
            o[5] = h >= 10u ? bswap32(align_bytes(d2, d1, 2)) : 0u;
        }
    }
    if (__ballot(t_kinds & (1u << 6))) {                      // Timestamp
        bytes12(tb + (T1 & 0xffu), d0, d1, d2);
        if (t_kinds & (1u << 6)) {
            o[2] = bswap32(align_bytes(d1, d0, 2));
            o[3] = bswap32(align_bytes(d2, d1, 2));
        }
    }
    if (__ballot(t_kinds & (1u << 7))) {                      // FastOpen
        bytes12(tb + ((T1 >> 8) & 0xffu), d0, d1, d2);
        if (t_kinds & (1u << 7)) o[6] |= (d0 >> 8) & 0xffu;
    }
    if (ip_has) {
        // word 7: ip_count | ip_stop << 8 | ip_kinds << 16; ip_end: byte 27
        ip_end = at - base;
        o[7] = cnt | (stop << 8) | (kinds << 16);
        o[14] = (uint32_t)trace;
        o[15] = (uint32_t)(trace >> 32);
    }
    const uint32_t ib = ip_at;                                 // IPv4: the partner frame
    if (__ballot(kinds & (1u << 2))) {                        // Timestamp
        bytes12(ib + (P0 & 0xffu), d0, d1, d2);
        if (kinds & (1u << 2)) o[9] = d0 >> 8;
    }
    if (__ballot(kinds & (1u << 3))) {                        // RecordRoute
        bytes12(ib + ((P0 >> 8) & 0xffu), d0, d1, d2);
        if (kinds & (1u << 3)) o[8] = (d0 >> 8) << 16;
    }
    if (__ballot(kinds & (1u << 4))) {                        // RouteAlert
        bytes12(ib + ((P0 >> 16) & 0xffu), d0, d1, d2);
        if (kinds & (1u << 4)) o[8] |= be16_hi(d0);
    }
    if (__ballot(kinds & (1u << 5))) {                        // CommercialSecurity
        bytes12(ib + (P0 >> 24), d0, d1, d2);
        if (kinds & (1u << 5)) o[11] = bswap32(align_bytes(d1, d0, 2));
    }
    if (__ballot(kinds & (3u << 6))) {                        // Strict / LooseSourceRoute
        // both kinds set the same getters: the later of the two options wins
        const uint32_t p6 = P1 & 0xffu, p7 = (P1 >> 8) & 0xffu;
        const uint32_t ps = !(kinds & (1u << 6)) ? p7 : (!(kinds & (1u << 7)) ? p6 : max(p6, p7));
        bytes12(ib + ps, d0, d1, d2);
        if (kinds & (3u << 6)) {
            o[9] |= ((d0 >> 16) & 0xffu) << 24;
            o[10] = bswap32(align_bytes(d1, d0, 3));
        }
    }
#else
    // phase 0: this frame's TCP walk; 1: frame q's IPv4 walk; 2: done
    uint32_t phase = S.tcp ? 0u : (ip_has ? 1u : 2u);
    OptCur c;
    c.base = c.at = phase == 0 ? slot_bias + S.t_lo : ip_at;
    c.end = c.at + (phase == 0 ? t_nb : ip_n);
    c.cnt = c.kinds = 0;
    c.stop = RPKT_OPT_END;
    c.trace = 0;
    while (phase < 2u) {
        const bool tcp = phase == 0u;
        if (c.at < c.end) {
            const uint32_t a = c.at & ~3u, sh = c.at & 3u;
            const uint32_t R0 = lds32(win, a), R1 = lds32(win, a + 4u);
            const uint32_t R2 = lds32(win, a + 8u), R3 = lds32(win, a + 12u);
            const uint32_t d0 = align_bytes(R1, R0, sh);
            const uint32_t t = d0 & 0xffu;
            const uint32_t nrem = c.end - c.at;
            if (t <= 1u) {                                     // EOL / NOP run
                const uint32_t x = d0 ^ (t ? 0x01010101u : 0u);
                uint32_t k = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4u;
                k = k < nrem ? k : nrem;
                c.kinds |= 1u << t;
                const uint32_t nib = (t ? 0x2222u : 0x1111u) & ((1u << (4 * k)) - 1u);
                if (c.cnt < 16) c.trace |= (uint64_t)nib << (4 * c.cnt);
                c.cnt += k;
                c.at += k;
            } else {
                const uint32_t rule = RPKT_OPT_RULE_ALU ? opt_rule_alu(tcp, t)
                                                        : rules[(tcp ? 256u : 0u) + t];
                const uint32_t hl = (d0 >> 8) & 0xffu;     // n >= 2 whenever a rule can pass
                const uint32_t X = rule >> 4, kind = rule & 7u;
                const bool fixed = (rule & 8u) != 0u;
                const bool ok = (kind != 0u) & (nrem >= X) & (hl - X <= (fixed ? 0u : nrem - X));
                if (!ok) {
                    c.stop = kind == 0u ? RPKT_OPT_UNKNOWN : RPKT_OPT_MALFORMED;
                    c.end = c.at;
                } else {
                    const uint32_t d1 = align_bytes(R2, R1, sh), d2 = align_bytes(R3, R2, sh);
                    const uint32_t g = kind | (tcp ? 8u : 0u);
                    if (g == 2u) o[9] = (o[9] & 0xff000000u) | (d0 >> 8);
                    if (g == 3u) o[8] = (o[8] & 0xffffu) | ((d0 >> 8) << 16);
                    if (g == 4u) o[8] = (o[8] & 0xffff0000u) | be16_hi(d0);
                    if (g == 5u) o[11] = bswap32(align_bytes(d1, d0, 2));
                    if (g == 6u || g == 7u) {
                        o[9] = (o[9] & 0x00ffffffu) | ((d0 >> 16) << 24);
                        o[10] = bswap32(align_bytes(d1, d0, 3));
                    }
                    if (g == 10u) o[1] = (o[1] & 0xffffu) | (be16_hi(d0) << 16);
                    if (g == 11u) o[0] = (o[0] & 0xff00ffffu) | (((d0 >> 16) & 0xffu) << 16);
                    if (g == 13u) {
                        o[0] = (o[0] & 0x00ffffffu) | (((hl - 2u) >> 3) << 24);
                        o[4] = hl >= 6u ? bswap32(align_bytes(d1, d0, 2)) : 0u;
                        o[5] = hl >= 10u ? bswap32(align_bytes(d2, d1, 2)) : 0u;
                    }
                    if (g == 14u) {
                        o[2] = bswap32(align_bytes(d1, d0, 2));
                        o[3] = bswap32(align_bytes(d2, d1, 2));
                    }
                    if (g == 15u) o[6] = (o[6] & 0xffff0000u) | hl;
                    c.kinds |= 1u << kind;
                    if (c.cnt < 16) c.trace |= (uint64_t)(kind + 1) << (4 * c.cnt);
                    c.cnt += 1;
                    c.at += fixed ? X : hl;
                }
            }
        }
        if (c.at >= c.end) {                                   // this walk ended
            const uint32_t pos = c.at - c.base;
            if (tcp) {
                // word 0: tcp_count | tcp_stop << 8 | wscale << 16 | sack_blocks << 24;
                // word 1: kinds | mss << 16; word 6: tcp_fo_len | tcp_end << 16
                o[0] = (o[0] & 0xffff0000u) | c.cnt | (c.stop << 8);
                o[1] = (o[1] & 0xffff0000u) | c.kinds;
                o[6] = (o[6] & 0xff00ffffu) | (pos << 16);
                o[12] = (uint32_t)c.trace;
                o[13] = (uint32_t)(c.trace >> 32);
                phase = ip_has ? 1u : 2u;
                c.base = c.at = ip_at;
                c.end = ip_at + ip_n;
                c.cnt = c.kinds = 0;
                c.stop = RPKT_OPT_END;
                c.trace = 0;
            } else {
                // word 7: ip_count | ip_stop << 8 | ip_kinds << 16; ip_end: byte 27
                ip_end = pos;
                o[7] = c.cnt | (c.stop << 8) | (c.kinds << 16);
                o[14] = (uint32_t)c.trace;
                o[15] = (uint32_t)(c.trace >> 32);
                phase = 2u;
            }
        }
    }
#endif  // RPKT_OPT_DEFER
    // IPv6 frames' option walks, over the windows before the rows are staged on them
    const Ip6Opts v6 = ip6_walks(S, d6);
    // rows: this frame's TCP words, then frame q's IPv4 words (word 6's top byte last)
    wave_sync();                                               // every walk has ended
    uint32_t* st = reinterpret_cast<uint32_t*>(win);
    uint32_t* me = st + lane * 17;
    uint32_t* pq = st + q * 17;
    me[0] = o[0]; me[1] = o[1]; me[2] = o[2]; me[3] = o[3]; me[4] = o[4]; me[5] = o[5];
    me[6] = o[6]; me[12] = o[12]; me[13] = o[13];
    pq[7] = o[7]; pq[8] = o[8]; pq[9] = o[9]; pq[10] = o[10]; pq[11] = o[11];
    pq[14] = o[14]; pq[15] = o[15];
    reinterpret_cast<uint8_t*>(pq)[27] = (uint8_t)ip_end;
    wave_sync();
    ip6_patch_rows(st, lane, S, v6);                           // IPv6 frames' option walks
    const uint32_t nrow = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* out = reinterpret_cast<u32x4*>(opts + p0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t cidx = k * kWave + lane, r = cidx / 4, pc = cidx % 4;
        const uint32_t* src = st + r * 17 + pc * 4;
        if (r < nrow) __builtin_nontemporal_store(u32x4{src[0], src[1], src[2], src[3]}, &out[cidx]);
    }
}

// A wave's 64 results staged through LDS `st` (stride 17 dwords: conflict-free) and
// stored as 64-B rows, 4 KiB coalesced, with non-temporal stores.  `st` must not be
// read by any lane of the wave after this call begins until it returns.
__device__ __forceinline__ void store_opts(uint32_t* st, int lane, const uint32_t (&o)[16],
                                           rpkt_opts_t* opts, uint32_t p0, uint32_t n,
                                           const OptSlices& S, const OptDw& d6) {
    const Ip6Opts v6 = ip6_walks(S, d6);
    wave_sync();
#pragma unroll
    for (int k = 0; k < 16; ++k) st[lane * 17 + k] = o[k];
    wave_sync();
    ip6_patch_rows(st, lane, S, v6);
    const uint32_t nrow = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* out = reinterpret_cast<u32x4*>(opts + p0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c = k * kWave + lane, r = c / 4, pc = c % 4;
        const uint32_t* src = st + r * 17 + pc * 4;
        if (r < nrow) __builtin_nontemporal_store(u32x4{src[0], src[1], src[2], src[3]}, &out[c]);
    }
}

}  // namespace
