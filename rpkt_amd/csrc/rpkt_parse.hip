// rpkt_parse.hip — receive side: parse_kernel (frame batches), parse_chains_kernel
// (mbuf chains), the flow-counter histogram and reduce, batched checksum::from_slice /
// from_buf, and the streaming references tools/ablate.py times against the parse.
#include "rpkt_common.h"
#include "rpkt_opts.h"

#include <mutex>

namespace {

// The option walks of parse_kernel<.., OPTS>: Ipv4OptionsIter / TcpOptionsIter over the
// slices the parse just located, read from the header window in LDS.  The window holds
// frame bytes [0, kWin - ph); a frame whose option bytes run past it (deep VLAN + IPv4
// options + TCP options: up to byte 142 + 15 of phase) has its slot refilled, by the
// wave's cooperative chunk mapping, with the 128 B from the 16-B chunk of its first
// option byte (both slices span at most ihl4 + 40 <= 100 B); those lines were fetched
// by the window and edge-line loads moments earlier, so the refill mostly hits L2.
// Results leave through the window area (stride 17) before the records are staged
// there.
__device__ __forceinline__ void options_from_window(WaveScratch& W, __amdgpu_buffer_rsrc_t rs,
                                                    uint32_t fb, int lane, Frame fr,
                                                    const LaneRec& L, const uint8_t* rules,
                                                    rpkt_opts_t* opts, uint32_t p0, uint32_t n) {
    const uint32_t* w = L.w;
    const uint32_t l3 = w[16] & 0xffffu, l4 = w[16] >> 16;
    const OptSlices S = opt_slices(L.status, (w[8] >> 8) & 0xffu, l3, l4,
                                   ((w[14] >> 12) & 0xfu) * 4u, L.is6);
    const uint32_t ph = fr.off & 15u;
    // every byte the walks use lies below need_hi (OptWin::dw's dword pair may read up to
    // 7 B past it: window padding or the next slot, never used)
    const bool over = S.need && S.need_hi + ph > (uint32_t)kWin;
    uint32_t bias = ph;
#ifndef RPKT_OPT_ABLATE
#define RPKT_OPT_ABLATE 0        // development: 1 = no walks (zero results), 2 = no refill
#endif
    if (RPKT_OPT_ABLATE != 2 && __builtin_expect(__ballot(over) != 0, 1)) {   // wave-uniform
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        uint32_t fix = 0;
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) {
            const int c = k * kWave + lane;
            const int q = c / kWinChunks, j = c % kWinChunks;
            const uint32_t lo = (uint32_t)__shfl((int)(over ? fr.off + S.need_lo : 0u), q, kWave);
            const uint32_t hi = (uint32_t)__shfl((int)(over ? fr.off + S.need_hi : 0u), q, kWave);
            const uint32_t a = (lo & ~15u) + 16u * j;
            addr[k] = a < hi ? a : fb;
            fix |= (uint32_t)straddles(addr[k], fb) << k;
        }
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) d[k] = load16_fast(rs, addr[k]);
        wave_sync();                                                // the parse's reads are done
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) {
            u32x4 v = d[k];
            if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
            if (addr[k] != fb) put_chunk(W, k * kWave + lane, v);
        }
        wave_sync();
        if (over) bias = ((fr.off + S.need_lo) & 15u) - S.need_lo;
    }
    // the frame bytes the slot holds, for the IPv6 option walk (ip6_walk): the header
    // window [0, kWin - ph), or a refilled slot's loaded chunks from need_lo's phase
    uint32_t wlo = 0u, whi = (uint32_t)kWin - ph;
    if (over) {
        const uint32_t ph2 = (fr.off + S.need_lo) & 15u;
        const uint32_t span = (S.need_hi - S.need_lo + ph2 + 15u) & ~15u;
        wlo = S.need_lo - ph2;
        whi = wlo + (span < (uint32_t)kWin ? span : (uint32_t)kWin);
    }
    const OptDw d6{&W.win[lane * kSlot], bias, wlo, whi, fr.off, fb, rs};
#if RPKT_OPT_ABLATE == 1
    uint32_t o[16] = {};
    store_opts(reinterpret_cast<uint32_t*>(W.win), lane, o, opts, p0, n, S, d6);
#elif RPKT_OPT_PAIRED
    walk_options_paired(W.win, lane, lane * kSlot + bias, S, rules, opts, p0, n, d6);
#else
    const OptWin s{&W.win[lane * kSlot], bias};
    uint32_t o[16];
    walk_options(s, S, rules, o);
    store_opts(reinterpret_cast<uint32_t*>(W.win), lane, o, opts, p0, n, S, d6);
#endif
}

// One wavefront per 64-frame tile: window loads -> LDS, lane-per-frame parse,
// flattened L4 stream, LDS-staged coalesced record stores.  (A persistent variant
// that prefetched the next tile's window into registers measured 1-3 % slower on
// every config: the extra live registers cost more occupancy than the overlap gave.
// Plain loops of 2 or 4 tiles per wave, no prefetch, measured 4-20 % slower:
// profiles/r01_ablate_tiles_per_wave.log.)
// L4: compiled with the L4 checksum stream (RPKT_F_L4_SUM).  V: ablation variant for
// tools/ablate.py (0 = the product kernel; 1 = no parse, 3 = no record stores,
// 8 = plain instead of non-temporal record stores, 21 = nt window loads too,
// 22 = default-policy stream loads, 23 = edge lines streamed first after the parse,
// 24 = never, 25 = after the parse on long tiles, 40 / 41 / 43 = edge lines with the
// window on tiles streaming more than 0 / 16 / 64 KB (the product: 32 KB), 44 = the
// round-1 edge_lines_first pass on tiles streaming more than 64 KB, 45 = default-policy
// window loads without the L4 stream).
// C16: write the 16-byte compact record (rpkt_rec16_t) instead of the 80-byte one:
// kept in registers, one 16-B store per lane (1 KiB contiguous per wave), no LDS stage.
// OPTS: also walk each frame's IPv4 and TCP options (rpkt_gpu_parse_options_batch) from
// the header window the parse holds, between the parse and the L4 stream.
// The tile of frames [p0, p0 + 64) of a batch, by one wave with its scratch W (p0 < n).
#ifndef RPKT_EDGE_JOINT
#define RPKT_EDGE_JOINT 1          // 0: the edge lines in their own pass after the window
#endif
// INWIN: every frame of the batch lies inside its header window (a strided batch of
// short frames, window_fits), so the L4 sums are whole in LDS and step 3 (the edge lines
// and the stream past the window) is compiled out.
template <bool L4, int V, bool C16, bool OPTS, bool INWIN = false>
__device__ __forceinline__ void parse_tile(WaveScratch& W, const uint8_t* opt_rules,
                                           const uint8_t* __restrict__ frames, uint32_t frames_bytes,
                                           const uint32_t* __restrict__ offsets, uint32_t stride,
                                           uint32_t frame_len, uint32_t n, uint32_t flags,
                                           rpkt_rec_t* __restrict__ recs,
                                           uint64_t* __restrict__ flow_ev, uint32_t n_buckets,
                                           rpkt_opts_t* __restrict__ opts, uint32_t p0, int lane) {
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, frames_bytes);
    const SpanSrc spans{offsets, stride, frame_len, frames_bytes, n};

    // 1. header windows -> LDS; on long tiles with the edge lines (window_with_edges)
    const Frame fr = spans.get(i);
    const uint32_t wend = (fr.off & ~15u) + kWin, fend = fr.off + fr.len;
    EdgeLines X{false, 0u, 0u, 0u};
    // header-only batches read each frame line once: non-temporal window loads
    // (config 2: 27.2 -> 26.1 us, profiles/r02_ablate_c2_v21.log); with the L4 stream the
    // window's lines are shared with the stream, and nt there costs +13-30 % (configs 3-5)
    constexpr int kWinAux = (V == 21 || (!L4 && V != 45)) ? 2 : 0;
    constexpr bool kJoint = L4 && !INWIN && RPKT_EDGE_JOINT && (V == 0 || V == 50) && kWinChunks == 8;
    bool joint = false;
    if constexpr (kJoint) {
        // tiles streaming more than 32 KB sum their frames' edge lines with the window
        // (profiles/r02_edge_window: config 5 -9 % read traffic); beyond 64 KB (1500-B
        // frames) loaded together with it: config 3 reads 1.042x -> 1.000x its frame
        // bytes, 269.0 -> 265.7 us, config 11 279.6 -> 275.0 us.  The parse of config 5's
        // 40-60 KB tiles read 3.7 % less that way too but ran 2.3 % slower, so it keeps
        // the separate edge pass; its fused option walks (4-wave blocks) ran 2.7 % faster
        // and take the joint loads from 32 KB (profiles/r04_wpb/ab_joint_*.jsonl)
        constexpr uint32_t kJointMin = OPTS ? kEdgeWindowBytes : kSplitStreamBytes;
        const uint32_t span = (valid && fend > wend) ? fend - wend : 0u;
        joint = wave_sum(span) > kJointMin;                           // wave-uniform
    }
    if (joint) {
        if constexpr (kJoint) X = window_with_edges(rs, frames_bytes, W, lane, fr, valid);
    } else {
        {
            u32x4 d[kWinChunks];
            uint32_t addr[kWinChunks];
            const uint32_t fix = window_issue<kWinAux>(rs, frames_bytes, fr, lane, d, addr);
            window_commit(W, rs, frames_bytes, d, addr, fix, lane);
        }
        // (ablation variants: the edge lines in their own pass after the window, at other
        // thresholds, or the round-1 split)
        if constexpr (L4 && !INWIN && V != 1 && V != 23 && V != 24 && V != 25 && V != 44)
            X = edge_lines_window(rs, frames_bytes, W, lane, fr, valid,
                                  V == 40 ? 0u : V == 41 ? 16384u : V == 43 ? 65536u : kEdgeWindowBytes);
        else if constexpr (L4 && V == 44)
            X = edge_lines_first(rs, frames_bytes, W, lane, valid, wend, fend);
    }
    wave_sync();

    // 2. lane-per-frame parse
    LaneRec L;
    if constexpr (V == 1) {                                       // ablation: window only
        const uint32_t* ww = reinterpret_cast<const uint32_t*>(&W.win[lane * kSlot]);
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < kWin / 4; ++k) x ^= ww[k];
#pragma unroll
        for (int k = 0; k < 20; ++k) L.w[k] = x + k;
        L.status = 0;
    } else {
        parse_lane(W, lane, fr, valid, flags, L, rs, frames_bytes);
    }
    if constexpr (OPTS) options_from_window(W, rs, frames_bytes, lane, fr, L, opt_rules, opts, p0, n);
    if constexpr (V != 3 && !C16) stage_record(W, lane, L.w);

    // 3. L4 bytes beyond the window: flattened chunk stream over the tile.  The stream
    // is read once: non-temporal loads (measured -13 % at 1500 B); the header windows
    // keep the default policy (nt there measured slower).
    if (L4 && V != 1) {
        constexpr int kAux = (V == 22) ? 0 : 2;
        uint32_t sp = 0;
        const uint32_t ss = L.stream_s, se = L.stream_e;
        if constexpr (INWIN) {
            (void)ss, (void)se;
        } else if (V == 23 || (V == 25 && wave_sum(se - ss) > kSplitStreamBytes)) {
            // ablation: the same split taken after the parse
            const uint32_t h1 = min(se, (ss + 127u) & ~127u);
            const uint32_t t0 = max(se & ~127u, h1);
            sp = wave_stream_sum<0>(rs, frames_bytes, ss, h1, W, lane);
            sp += wave_stream_sum<0>(rs, frames_bytes, t0, se, W, lane);
            sp += wave_stream_sum<kAux>(rs, frames_bytes, h1, t0, W, lane);
        } else {
            sp = stream_rest<kAux>(X, rs, frames_bytes, ss, se, wend, fend, W, lane);
        }
        if constexpr (V == 3) {                                   // ablation: 4 B per frame
            uint32_t x = sp;
#pragma unroll
            for (int k = 0; k < 20; ++k) x ^= L.w[k];
            if (valid) reinterpret_cast<uint32_t*>(recs)[i] = x;
            return;
        }
        if (L.want_l4) {
            const uint32_t seg = be_sum(L.l4_part + sp, L.l4_start_abs);
            if constexpr (C16) L.w[18] |= fold16(L.pseudo + seg) << 16;
            else rec_stage(W)[lane * 21 + 18] |= fold16(L.pseudo + seg) << 16;
        }
    }
    if constexpr (V == 3) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 20; ++k) x ^= L.w[k];
        if (valid) reinterpret_cast<uint32_t*>(recs)[i] = x;
        return;
    }

    // 4. records (+ flow events)
    if ((flags & RPKT_F_FLOW_EV) && valid) {
        const uint64_t ev = flow_event(L, C16 ? L.w : rec_stage(W) + lane * 21, n_buckets);
        __builtin_nontemporal_store(ev, &flow_ev[i]);
    }
    if constexpr (C16) {
        if (valid)
            __builtin_nontemporal_store(compact_record(L, flags),
                                        reinterpret_cast<u32x4*>(recs) + i);
    } else {
        flush_records<V != 8>(W, lane, recs, p0, n);
    }
}

// INWIN: see parse_tile.  WPB: waves per block.  A block's slot on its CU is freed only when its last wave
// ends, and a config-2 wave lasts 3.7-7.3 us (tools/launch_stamps.py), so one-wave
// blocks keep more waves in flight: the batch and compact entries launch kParseWPB = 1
// (config 2: 27.0 -> 25.9 and 27.5 -> 26.1 us, compact 15.8 -> 15.5 us, config 3 the
// same; profiles/r04_wpb/).  The fused option walks keep 4 (their 512-B rule table is
// filled per block: 689 -> 701 us with one-wave blocks).
#ifndef RPKT_PARSE_WPB
#define RPKT_PARSE_WPB 1
#endif
constexpr int kParseWPB = RPKT_PARSE_WPB;
template <bool L4, int V, bool C16 = false, bool OPTS = false, int WPB = kWavesPerBlock,
          bool INWIN = false>
__global__ __launch_bounds__(kWave * WPB, 4)    // 4 waves/SIMD: <= 128 VGPRs
void parse_kernel(const uint8_t* __restrict__ frames, uint32_t frames_bytes,
                  const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                  uint32_t n, uint32_t flags, rpkt_rec_t* __restrict__ recs,
                  uint64_t* __restrict__ flow_ev, uint32_t n_buckets,
                  rpkt_opts_t* __restrict__ opts) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[WPB];
    // the option-type rules of both iterators (OPTS; 4 + 4 x 9744 + 512 B: still four
    // blocks per CU)
    __shared__ uint8_t opt_rules[OPTS ? 512 : 4];
    if constexpr (OPTS) {
        opt_rules_fill(opt_rules);
        __syncthreads();
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const uint32_t p0 = (blockIdx.x * WPB + wid) * kWave;
    if (p0 >= n) return;                                          // wave-uniform exit
#ifdef RPKT_ABLATE
    // V == 50 (tools/launch_stamps.py): the wave's start and end on the 100-MHz clock all
    // CUs share, after its stores are acknowledged, and where it ran; flow_ev is the stamp
    // buffer (4 u64 per wave) and the flags carry no RPKT_F_FLOW_EV
    uint64_t t0 = 0;
    if constexpr (V == 50) t0 = __builtin_amdgcn_s_memrealtime();
#endif
    parse_tile<L4, V, C16, OPTS, INWIN>(scratch[wid], opt_rules, frames, frames_bytes, offsets,
                                        stride, frame_len, n, flags, recs, flow_ev, n_buckets,
                                        opts, p0, lane);
#ifdef RPKT_ABLATE
    if constexpr (V == 50) {
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);    // XCC_ID
        if (lane == 0) {
            u32x4* st = reinterpret_cast<u32x4*>(flow_ev) + 2u * (p0 / kWave);
            st[0] = u32x4{(uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32)};
            st[1] = u32x4{hw, xcc, 0u, 0u};
        }
    }
#endif
}

// A receive ring's slots in one launch (rpkt_gpu_parse_ring): wave t takes tile t of the
// ring's tiles, numbered slot after slot (tile0[k] = the first tile of slot k), and
// parses it exactly as parse_kernel parses that tile of the slot's own batch.  The slot
// descriptors are kernel arguments, read with scalar loads.
constexpr uint32_t kRingMax = RPKT_RING_MAX_SLOTS;
struct RingSlot {
    const uint8_t* frames;
    const uint32_t* offsets;
    rpkt_rec_t* recs;
    uint64_t* flow_ev;
    uint32_t frames_bytes, stride, frame_len, n;
};
struct RingArgs {
    uint32_t n_slots;
    uint32_t tile0[kRingMax + 1];
    RingSlot s[kRingMax];
};

// waves per block of the ring launch: one, as the batch entries (8-slot ring of config
// 2: 195.8 -> 193.0 us, compact 109.0 -> 103.2 us; profiles/r04_wpb/ab_ring1.jsonl)
#ifndef RPKT_RING_WPB
#define RPKT_RING_WPB 1
#endif
constexpr int kRingWPB = RPKT_RING_WPB;
template <bool L4, bool C16, bool INWIN = false>
__global__ __launch_bounds__(kWave * kRingWPB, 4)
void parse_ring_kernel(const RingArgs A, uint32_t flags, uint32_t n_buckets) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kRingWPB];
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t t = blockIdx.x * kRingWPB + wid;
    if (t >= A.tile0[A.n_slots]) return;                          // wave-uniform exit
    uint32_t k = 0;                                               // the slot holding tile t
    for (uint32_t j = 1; j < A.n_slots; ++j) k = A.tile0[j] <= t ? j : k;
    const RingSlot& S = A.s[k];
    parse_tile<L4, 0, C16, false, INWIN>(scratch[wid], nullptr, S.frames, S.frames_bytes, S.offsets,
                                    S.stride, S.frame_len, S.n, flags, S.recs, S.flow_ev, n_buckets,
                                    nullptr, (t - A.tile0[k]) * kWave, lane);
}

// ---- mbuf chains: the same parse over rpkt-dpdk's Pbuf ----
// A chain is a list of (offset, data_len) segments of one arena.  Over a Pbuf the
// generic views test header sizes against chunk(), the rest of the segment that holds
// the header's first byte (pbuf.rs:48-57, 86-96), and totals against remaining()
// (pbuf.rs:98-101); trim_off cuts the packet end (pbuf.rs:117-140).  Segment 0 is
// windowed into LDS like a frame, so every header that starts inside it is parsed by
// the window path; a header that starts exactly at segment 0's end (the only way
// past it) is read from global memory byte-wise on a rare path.  The L4 bytes past
// the window are summed by the flattened chunk stream over (chain, segment) items,
// each item's sum brought to segment 0's byte phase before it is added.
struct ChainSrc {
    const uint2* segs;
    uint32_t fb;
    __device__ __forceinline__ Frame seg(uint32_t k) const {
        const uint2 v = segs[k];
        const uint32_t off = v.x < fb ? v.x : fb;
        const uint32_t len = v.y < fb - off ? v.y : fb - off;
        return Frame{off, len};
    }
};

// checksum::from_slice over n bytes at absolute `a` (rpkt/src/checksum.rs:33-62)
__device__ __forceinline__ uint32_t gsum_be(__amdgpu_buffer_rsrc_t rs, uint32_t a, uint32_t n) {
    uint32_t acc = 0, k = 0;
    for (; k + 1 < n; k += 2) acc += (gbyte(rs, a + k) << 8) | gbyte(rs, a + k + 1);
    if (k < n) acc += gbyte(rs, a + k) << 8;
    return fold16(acc);
}

// Chunk at logical cursor c > 0 of segments [a, b) under the packet end `limit`: the
// rest of the first segment whose end passes c (empty segments skipped, as
// advance_common walks), cut at limit.  `abs` = the chunk's first byte.
__device__ __forceinline__ uint32_t chain_chunk(const ChainSrc& S, uint32_t a, uint32_t b,
                                                uint32_t c, uint32_t limit, uint32_t& abs) {
    uint32_t cum = 0;
    for (uint32_t k = a; k < b; ++k) {
        const Frame s = S.seg(k);
        const uint32_t end = cum + s.len;
        if (end > c) {
            abs = s.off + (c - cum);
            return (end < limit ? end : limit) - c;
        }
        cum = end;
    }
    abs = S.fb;
    return 0;
}

// Chain bytes at absolute a..a+3 as a little-endian dword: from segment 0's LDS window
// when they lie in its windowed part (frame bytes [0, lim) of segment 0), else byte-wise
// from global memory.  A header lies inside the chunk it was tested against, i.e. in one
// segment, so its bytes are at consecutive absolute addresses.
struct ChainDw {
    const uint8_t* slot;
    uint32_t ph, off0, lim;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ uint32_t operator()(uint32_t a) const {
        const uint32_t x = a - off0;                           // wraps for other segments
        if (x < lim && lim - x >= 4u) {
            const uint32_t y = ph + x, q = y & ~3u;
            return align_bytes(lds32(slot, q + 4), lds32(slot, q), y & 3u);
        }
        return gbyte(rs, a) | (gbyte(rs, a + 1) << 8) | (gbyte(rs, a + 2) << 16) |
               (gbyte(rs, a + 3) << 24);
    }
};

// parse_ip6 (rpkt_common.h) over a Pbuf: every header size against chunk().len() at its
// first byte (the rest of the segment holding it, cut at the packet end), the payload
// length against remaining() (ipv6/generated.rs:40-92 and the extension headers'
// parses, as oracle/rpkt_oracle_chain.c parse_pbuf_ip6).
__device__ __forceinline__ uint32_t parse_chain_ip6(const ChainDw& dw, uint32_t C, uint32_t pkt,
                                                    const ChainSrc& S, uint32_t a, uint32_t b,
                                                    uint32_t l3, uint32_t* w, uint32_t& l4,
                                                    uint32_t& l4rem, uint32_t& proto,
                                                    uint32_t& paddr) {
    // chunk at logical cursor c under the packet end `lim`, its first byte's address
    auto chunk = [&](uint32_t c, uint32_t lim, uint32_t& abs) -> uint32_t {
        if (c < C) {
            abs = dw.off0 + c;
            return (C < lim ? C : lim) - c;
        }
        abs = S.fb;
        return c < lim ? chain_chunk(S, a, b, c, lim, abs) : 0u;
    };
    uint32_t ab3;
    if (chunk(l3, pkt, ab3) < 40u) return RPKT_S_IP6_SHORT;               // :42
    uint32_t F[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) F[k] = dw(ab3 + 4u * k);
    const uint32_t plen = be16_lo(F[1]);
    if (plen + 40u > pkt - l3) return RPKT_S_IP6_BAD_LEN;                 // :47
    w[6] = bswap32(F[0]);
    w[7] = plen | (F[1] & 0xffff0000u);
    w[9] = bswap32(F[2]) ^ bswap32(F[3]) ^ bswap32(F[4]) ^ bswap32(F[5]);
    w[10] = bswap32(F[6]) ^ bswap32(F[7]) ^ bswap32(F[8]) ^ bswap32(F[9]);
    const uint32_t src_sum = addr_words_sum(F[2], F[3], F[4], F[5]);
    uint32_t pdst_sum = addr_words_sum(F[6], F[7], F[8], F[9]);
    uint32_t pdst_off = l3 + 24u;
    uint32_t c = l3 + 40u;
    const uint32_t end = c + plen;                                        // payload() trim
    uint32_t nh = (F[1] >> 16) & 0xffu, n_ext = 0, status = RPKT_S_OK;
    for (int k = 0; k < RPKT_MAX_IP6_EXT && is_ip6_ext(nh); ++k) {
        const bool fg = nh == 44u, ah = nh == 51u, rt = nh == 43u;
        const uint32_t fixed = (nh == 0u || nh == 60u) ? 2u : (ah ? 12u : 8u);
        uint32_t ax;
        const uint32_t cl = chunk(c, end, ax);
        if (cl < fixed) { status = RPKT_S_IP6_EXT_SHORT; break; }
        const uint32_t d0 = dw(ax);
        const uint32_t b1 = (d0 >> 8) & 0xffu;
        const uint32_t hl = fg ? 8u : (ah ? b1 * 4u + 8u : b1 * 8u + 8u);
        if (!fg && (hl < fixed || hl > cl)) { status = RPKT_S_IP6_EXT_BAD_LEN; break; }
        if (rt && (d0 >> 24) != 0u) {
            const uint32_t type = (d0 >> 16) & 0xffu, n_addr = (hl - 8u) >> 4;
            if (n_addr != 0u && (type == 0u || type == 2u || type == 4u)) {
                const uint32_t r = 8u + (type == 4u ? 0u : 16u * (n_addr - 1u));
                pdst_off = c + r;
                pdst_sum = addr_words_sum(dw(ax + r), dw(ax + r + 4u), dw(ax + r + 8u),
                                          dw(ax + r + 12u));
            }
        }
        nh = d0 & 0xffu;
        c += hl;
        n_ext += 1u;
        if (fg && (be16_hi(d0) & 0xfff9u) != 0u) { status = RPKT_S_IP6_FRAGMENT; break; }
    }
    if (status == RPKT_S_OK && is_ip6_ext(nh)) status = RPKT_S_L4_OTHER;
    w[8] = n_ext | (nh << 8) | (pdst_off << 16);
    l4 = c;
    l4rem = end - c;
    proto = nh;
    paddr = src_sum + pdst_sum;
    return status;
}

// Lane-per-chain parse: parse_lane with the chunk/remaining distinction of a Pbuf.
// C = segment 0's length: headers starting below C are read from the LDS window.
__device__ __forceinline__ void parse_chain_lane(const WaveScratch& W, int lane, Frame s0,
                                                 uint32_t pkt, const ChainSrc& S, uint32_t a,
                                                 uint32_t b, __amdgpu_buffer_rsrc_t rs,
                                                 uint32_t flags, LaneRec& L) {
    const uint32_t ph = s0.off & 15u;
    const uint8_t* slot = &W.win[lane * kSlot];
    uint32_t* w = L.w;
#pragma unroll
    for (int k = 0; k < 20; ++k) w[k] = 0;
    const uint32_t C = s0.len;                                 // Pbuf::new, pbuf.rs:19-34
    L.stream_s = L.stream_e = L.l4_part = L.l4_start_abs = L.pseudo = 0;
    L.want_l4 = false;
    L.is6 = false;
    w[19] = pkt;
    uint32_t status = RPKT_S_OK;

    uint32_t E[6];
    {
        const uint32_t a0 = ph & ~3u, sh = ph & 3u;
        uint32_t R[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) R[k] = lds32(slot, a0 + 4 * k);
#pragma unroll
        for (int k = 0; k < 6; ++k) E[k] = align_bytes(R[k + 1], R[k], sh);
    }
    if (C < 14) {                                              // ether/generated.rs:36
        L.status = RPKT_S_ETH_SHORT;
        w[0] = RPKT_S_ETH_SHORT;
        return;
    }
    w[1] = E[0];
    w[2] = E[1];
    w[3] = E[2];
    const uint32_t eth_et = be16_lo(E[3]);
    uint32_t nvlan = 0, et = eth_et, c = 14;
#pragma unroll
    for (int v = 0; v < RPKT_MAX_VLAN; ++v) {                  // vlan/generated.rs:32-61
        if (!is_tag(et)) break;
        uint32_t T = 0, ck = 0;
        if (c < C) {
            ck = C - c;
            T = v == 0 ? align_bytes(E[4], E[3], 2) : align_bytes(E[5], E[4], 2);
        } else if (c < pkt) {
            uint32_t ab;
            ck = chain_chunk(S, a, b, c, pkt, ab);
            T = gbyte(rs, ab) | (gbyte(rs, ab + 1) << 8) | (gbyte(rs, ab + 2) << 16) |
                (gbyte(rs, ab + 3) << 24);
        }
        if (ck < 4) {
            status = RPKT_S_VLAN_SHORT;
            break;
        }
        et = be16_hi(T);
        w[4] |= be16_lo(T) << (16 * v);
        w[5] |= et << (16 * v);
        nvlan += 1;
        c += 4;
    }
    w[0] = (nvlan << 8) | (eth_et << 16);
    const bool v6 = (flags & RPKT_F_IPV6) && status == RPKT_S_OK && et == 0x86ddu;
    if (status == RPKT_S_OK && et != 0x0800u && !v6) status = RPKT_S_NOT_IPV4;
    if (status != RPKT_S_OK) {
        w[0] |= status;
        L.status = status;
        return;
    }

    const uint32_t l3 = c;
    w[16] = l3;
    uint32_t l4, limit, l4rem, proto, paddr;
    if (v6) {
        L.is6 = true;
        const uint32_t wl = (uint32_t)kWin - ph;
        const ChainDw dw{slot, ph, s0.off, C < wl ? C : wl, rs};
        status = parse_chain_ip6(dw, C, pkt, S, a, b, l3, w, l4, l4rem, proto, paddr);
        if (status != RPKT_S_IP6_SHORT && status != RPKT_S_IP6_BAD_LEN) {
            w[16] |= l4 << 16;
            w[17] = (l4 & 0xffffu) | (l4rem << 16);
        }
        if (status != RPKT_S_OK) {
            w[0] |= status;
            L.status = status;
            return;
        }
        limit = l4 + l4rem;
    } else {
    // Ipv4::parse (ipv4/generated.rs:35-51): chunk vs remaining
    Hdr6 ip;
    uint32_t ck3 = 0, ab3 = 0;
    const bool fast3 = l3 < C;
    if (fast3) {
        ck3 = C - l3;
        read_hdr(slot, ph + l3, ip);
    } else {
        if (l3 < pkt) ck3 = chain_chunk(S, a, b, l3, pkt, ab3);
        gread20(rs, S.fb, ck3 ? ab3 : S.fb, ip.F);
    }
    const uint32_t vhl = ip.F[0] & 0xffu;
    const uint32_t ihl4 = (vhl & 0xfu) * 4u;
    const uint32_t tot = be16_hi(ip.F[0]);
    if (ck3 < 20) status = RPKT_S_IP_SHORT;
    else if (ihl4 < 20) status = RPKT_S_IP_BAD_IHL;
    else if (ihl4 > ck3) status = RPKT_S_IP_IHL_GT_LEN;
    else if (tot < ihl4) status = RPKT_S_IP_TOT_LT_IHL;
    else if (tot > pkt - l3) status = RPKT_S_IP_TOT_GT_LEN;
    if (status != RPKT_S_OK) {
        w[0] |= status;
        L.status = status;
        return;
    }
    proto = (ip.F[2] >> 8) & 0xffu;
    const uint32_t src = bswap32(ip.F[3]), dst = bswap32(ip.F[4]);
    w[6] = (ip.F[0] & 0xffffu) | (tot << 16);
    w[7] = be16_lo(ip.F[1]) | (be16_hi(ip.F[1]) << 16);
    w[8] = (ip.F[2] & 0xffffu) | (be16_hi(ip.F[2]) << 16);
    w[9] = src;
    w[10] = dst;
    if (flags & RPKT_F_IP_SUM)
        w[18] = fast3 ? be_sum(raw_range_sum(slot, ip.R, ip.a0, ph + l3, ph + l3 + ihl4),
                               s0.off + l3)
                      : gsum_be(rs, ab3, ihl4);
    l4 = l3 + ihl4;                                            // Ipv4::payload :115-127
    limit = l3 + tot;
    l4rem = tot - ihl4;
    w[16] |= l4 << 16;
    w[17] = l4 | (l4rem << 16);
    paddr = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu);
    }

    // Udp::parse / Tcp::parse against the chunk at l4 under the trimmed end (an IPv6 L4
    // header past segment 0's window is read from global memory)
    Hdr6 h4;
    uint32_t ck4 = 0, ab4 = 0;
    const bool fast4 = l4 < C && ph + l4 + 20u <= (uint32_t)kWin;
    if (fast4) {
        ck4 = (C < limit ? C : limit) - l4;
        read_hdr(slot, ph + l4, h4);
    } else {
        if (l4 < limit) ck4 = chain_chunk(S, a, b, l4, limit, ab4);
        gread20(rs, S.fb, ck4 ? ab4 : S.fb, h4.F);
    }
    uint32_t l4len = 0;
    bool other_sum = false;                                    // ICMP / GRE (parse_lane)
    if (proto == 17u) {
        const uint32_t ulen = be16_lo(h4.F[1]);
        if (ck4 < 8) status = RPKT_S_UDP_SHORT;
        else if (ulen < 8 || ulen > l4rem) status = RPKT_S_UDP_BAD_LEN;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[14] = ulen;
            w[15] = be16_hi(h4.F[1]);
            w[17] = ((l4 + 8) & 0xffffu) | ((ulen - 8) << 16);
            l4len = ulen;
        }
    } else if (proto == 6u) {
        const uint32_t hl = ((h4.F[3] >> 4) & 0xfu) * 4u;
        if (ck4 < 20) status = RPKT_S_TCP_SHORT;
        else if (hl < 20 || hl > ck4) status = RPKT_S_TCP_BAD_DOFF;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[12] = bswap32(h4.F[1]);
            w[13] = bswap32(h4.F[2]);
            w[14] = be16_lo(h4.F[3]) | (be16_hi(h4.F[3]) << 16);
            w[15] = be16_lo(h4.F[4]) | (be16_hi(h4.F[4]) << 16);
            w[17] = ((l4 + hl) & 0xffffu) | ((l4rem - hl) << 16);
            l4len = l4rem;
        }
    } else {
        // ICMP and GRE-with-checksum sums over the IP payload, as parse_lane (the GRE
        // header's first byte is the first byte of the chunk at l4)
        status = RPKT_S_L4_OTHER;
        if (!v6 && proto == 1u) {
            if (l4rem == 0u) status = RPKT_S_ICMP_EMPTY;
            else other_sum = true;
        } else if (proto == 47u && l4rem >= 4u && (h4.F[0] & 0x80u)) {
            other_sum = true;
        }
        l4len = l4rem;
    }
    w[0] |= status;
    L.status = status;
    if ((status == RPKT_S_OK || other_sum) && (flags & RPKT_F_L4_SUM)) {
        L.want_l4 = true;
        L.pseudo = other_sum ? 0u : paddr + proto + l4len;
        const uint32_t e = l4 + l4len;
        L.l4_start_abs = s0.off + l4;                          // segment 0's byte phase
        if (fast4) {
            const uint32_t win_end = kWin - ph;
            uint32_t e_in = e < win_end ? e : win_end;
            e_in = e_in < C ? e_in : C;
            L.l4_part = raw_range_sum(slot, h4.R, h4.a0, ph + l4, ph + e_in);
            L.stream_s = e_in;
        } else {
            L.stream_s = l4;
        }
        L.stream_e = e;                                        // logical, not absolute
    }
}

// Sum of the logical range [ss, se) of this lane's chain, in segment 0's byte phase,
// for every lane of the wave.  Items (chain, segment intersecting its range) are
// flattened in chain order; each round streams 64 of them with wave_stream_sum.
// An item's logical start is its owner's running cursor plus a segmented prefix sum
// of the round's segment lengths.  Scratch: the window area past the staged records
// (dwords [0, 513) of it; the caller keeps per-lane values at [513, 705)).
__device__ __forceinline__ uint32_t chain_stream(WaveScratch& W, __amdgpu_buffer_rsrc_t rs,
                                                 uint32_t fb, const ChainSrc& S, uint32_t a,
                                                 uint32_t b, uint32_t off0, uint32_t ss,
                                                 uint32_t se, int lane) {
    uint32_t k = 0, fi = 0, ls0 = 0;
    if (se > ss) {
        uint32_t cum = 0;
        for (uint32_t j = a; j < b; ++j) {
            const uint32_t len = S.seg(j).len;
            if (cum + len > ss && cum < se) {
                if (k == 0) {
                    fi = j;
                    ls0 = cum;
                }
                ++k;
            }
            cum += len;
            if (cum >= se) break;
        }
    }
    const uint32_t incl = wave_incl_scan(k);
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    if (T == 0) return 0;                                      // wave-uniform
    uint32_t* X = rec_stage(W) + kWave * 21;
    uint32_t* cb = X;                  // [65] first item of each lane
    uint32_t* cfi = X + 65;            // first segment index
    uint32_t* ccum = X + 129;          // logical start of the lane's next item
    uint32_t* css = X + 193;
    uint32_t* cse = X + 257;
    uint32_t* cacc = X + 321;
    uint32_t* citem = X + 385;         // [128] per-item state held over the stream
    cb[lane] = incl - k;
    if (lane == 63) cb[64] = incl;
    cfi[lane] = fi | (off0 << 31);     // segment 0's byte parity in bit 31
    ccum[lane] = ls0;
    css[lane] = ss;
    cse[lane] = se;
    cacc[lane] = 0;
    wave_sync();
    for (uint32_t r0 = 0; r0 < T; r0 += kWave) {
        const uint32_t g = r0 + lane;
        const bool v = g < T;
        uint32_t q = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1)
            if (cb[q + step] <= g) q += step;
        const uint32_t bq = cb[q];
        const uint32_t t = g - bq;
        const uint32_t fq = cfi[q];
        const Frame sg = v ? S.seg((fq & 0x7fffffffu) + t) : Frame{0, 0};
        const uint32_t x = sg.len;
        const uint32_t inc = wave_incl_scan(x);
        const uint32_t j0 = (bq > r0 ? bq : r0) - r0;          // owner's first lane this round
        const uint32_t base = (uint32_t)__shfl((int)(inc - x), (int)j0, kWave);
        const uint32_t ls = ccum[q] + (inc - x) - base;
        const uint32_t lo = ls > css[q] ? ls : css[q];
        const uint32_t he = ls + x, hi = he < cse[q] ? he : cse[q];
        uint32_t s_abs = 0, e_abs = 0;
        if (v && hi > lo) {
            s_abs = sg.off + (lo - ls);
            e_abs = sg.off + (hi - ls);
        }
        const uint32_t swap = ((sg.off - ls) ^ (fq >> 31)) & 1u;
        const uint32_t last = v && (lane == kWave - 1 || t + 1 == cb[q + 1] - bq);
        citem[lane] = q | (swap << 8) | (last << 9) | ((uint32_t)v << 10);   // kept in LDS
        citem[kWave + lane] = he;                                               // over the stream
        const uint32_t part = wave_stream_sum<2, kChainStreamUnroll>(rs, fb, s_abs, e_abs, W, lane);
        const uint32_t it = citem[lane];
        const uint32_t qq = it & 63u;
        if (it & (1u << 10)) {
            uint32_t c = fold16(part);
            atomicAdd(&cacc[qq], (it & (1u << 8)) ? bswap16(c) : c);
        }
        if (it & (1u << 9)) ccum[qq] = citem[kWave + lane];
        wave_sync();
    }
    return cacc[lane];
}

template <bool L4>
// A long chain makes a wave's item stream long and the grid small (256K 8000-B
// chains = 4096 waves, one per SIMD): the stream keeps kChainStreamUnroll loads per
// lane per batch in flight, and registers, not waves, are the budget (<= 256).
__global__ __launch_bounds__(kWave * kWavesPerBlock, 2)
void parse_chains_kernel(const uint8_t* __restrict__ buf, uint32_t fb,
                         const uint2* __restrict__ segs, uint32_t n_segs,
                         const uint32_t* __restrict__ chain_first, uint32_t n, uint32_t flags,
                         rpkt_rec_t* __restrict__ recs, uint64_t* __restrict__ flow_ev,
                         uint32_t n_buckets) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    WaveScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;                                          // wave-uniform exit
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(buf, fb);
    const ChainSrc S{segs, fb};

    // chain bounds, segment 0 and pkt_len (sum of data_len, saturating)
    uint32_t a = 0, b = 0;
    if (valid) {
        const uint32_t f0 = chain_first[i], f1 = chain_first[i + 1];
        a = f0 < n_segs ? f0 : n_segs;
        b = f1 > a ? f1 : a;
        b = b < n_segs ? b : n_segs;
    }
    Frame s0{0, 0};
    uint32_t pkt = 0;
    for (uint32_t k = a; k < b; ++k) {
        const Frame s = S.seg(k);
        if (k == a) s0 = s;
        pkt = pkt + s.len < pkt ? 0xffffffffu : pkt + s.len;
    }

    // 1. segment 0's header window -> LDS
    {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        const uint32_t fix = window_issue(rs, fb, s0, lane, d, addr);
        window_commit(W, rs, fb, d, addr, fix, lane);
    }
    wave_sync();

    // 2. lane-per-chain parse
    LaneRec L;
    parse_chain_lane(W, lane, s0, pkt, S, a, b, rs, flags, L);
    stage_record(W, lane, L.w);

    // 3. L4 bytes past the window, across segments (the in-window part and the
    //    pseudo header wait in LDS, past chain_stream's scratch)
    if (L4) {
        uint32_t* keep = rec_stage(W) + kWave * 21 + 513;
        keep[lane] = L.l4_part;
        keep[kWave + lane] = L.want_l4 ? (L.pseudo | 0x80000000u) : 0u;
        keep[2 * kWave + lane] = L.l4_start_abs;
        const uint32_t acc = chain_stream(W, rs, fb, S, a, b, s0.off, L.stream_s, L.stream_e, lane);
        const uint32_t ps = keep[kWave + lane];
        if (ps) {
            const uint32_t sum = be_sum(keep[lane] + acc, keep[2 * kWave + lane]);
            rec_stage(W)[lane * 21 + 18] |= fold16((ps & 0x7fffffffu) + sum) << 16;
        }
    }

    // 4. records (+ flow events)
    if ((flags & RPKT_F_FLOW_EV) && valid) {
        const uint64_t ev = flow_event(L, rec_stage(W) + lane * 21, n_buckets);
        __builtin_nontemporal_store(ev, &flow_ev[i]);
    }
    flush_records<true>(W, lane, recs, p0, n);
}

#ifdef RPKT_ABLATE
// Wave-contiguous streaming references (the copy ceiling of bench.py): every wave owns
// one contiguous slice of the input and one of the output, in 1-KiB units (64 lanes x
// 16 B, one dwordx4 per lane per unit), reads its input slice four units at a time and
// writes its output slice in proportion as it goes, so the read and write streams mix
// at the in:out ratio throughout (1:1, or config 2's 64 B read : 80 B written per
// frame).  AUX: load cache policy (2 = non-temporal); NTS: non-temporal stores.
// COPY: the output is the input itself (memcpy; in16 == out16), else a value derived
// from the loads (keeps them live).
template <int AUX, bool NTS, bool COPY>
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void wave_stream_ref_kernel(const uint8_t* __restrict__ in, uint32_t in16,
                            u32x4* __restrict__ out, uint32_t out16) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t gw = blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t in_u = in16 / kWave, out_u = out16 / kWave;
    const uint32_t i0 = (uint32_t)((uint64_t)in_u * gw / nw), i1 = (uint32_t)((uint64_t)in_u * (gw + 1) / nw);
    const uint32_t o0 = (uint32_t)((uint64_t)out_u * gw / nw), o1 = (uint32_t)((uint64_t)out_u * (gw + 1) / nw);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(in, in16 * 16u);
    const uint32_t oob = in16 * 16u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    uint32_t o = o0;
    for (uint32_t i = i0; i < i1; i += 4) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = load16_fast<AUX>(rs, i + u < i1 ? ((i + u) * kWave + lane) * 16u : oob);
        if constexpr (COPY) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i + u < i1) {
                    u32x4* dst = &out[(size_t)(i + u) * kWave + lane];
                    if constexpr (NTS) __builtin_nontemporal_store(x[u], dst);
                    else *dst = x[u];
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= x[u];
            const uint32_t done = i + 4 < i1 ? i + 4 - i0 : i1 - i0;
            const uint32_t due = o0 + (uint32_t)((uint64_t)(o1 - o0) * done / (i1 - i0));
            for (; o < due; ++o) {
                u32x4* dst = &out[(size_t)o * kWave + lane];
                if constexpr (NTS) __builtin_nontemporal_store(acc + o, dst);
                else *dst = acc + o;
            }
        }
    }
    if constexpr (!COPY) {
        for (; o < o1; ++o) {
            u32x4* dst = &out[(size_t)o * kWave + lane];
            if constexpr (NTS) __builtin_nontemporal_store(acc + o, dst);
            else *dst = acc + o;
        }
    }
}

// Streaming reference for the roofline: read `in16` 16-B chunks and write `out16`
// chunks with plain coalesced dwordx4 accesses (what a perfect parse would move).
template <int U, bool NT>
__global__ __launch_bounds__(256)
void copy_ref_kernel(const u32x4* __restrict__ in, uint32_t in16, u32x4* __restrict__ out,
                     uint32_t out16) {
    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    uint32_t i = t;
    for (; i + (U - 1) * T < in16; i += U * T) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = in[i + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
    }
    for (; i < in16; i += T) acc ^= in[i];
    for (uint32_t j = t; j < out16; j += T) {
        if constexpr (NT) __builtin_nontemporal_store(acc + j, &out[j]);
        else out[j] = acc + j;
    }
}

// Read-only streaming reference (what HBM gives a pure 16-B/lane read stream).
__global__ __launch_bounds__(256)
void read_ref_kernel(const u32x4* __restrict__ in, uint32_t in16, uint32_t* __restrict__ out) {
    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    uint32_t i = t;
    for (; i + 7 * T < in16; i += 8 * T) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = in[i + u * T];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u];
    }
    for (; i < in16; i += T) acc ^= in[i];
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x12345678u) out[t] = r;       // keeps the loads live, never taken in practice
}

// Same-traffic reference for the parse: each wave reads its 64-frame tile's bytes as
// one contiguous non-temporal 16-B/lane stream and writes 64 records (80 B each) with
// non-temporal stores, like parse_kernel, but does no parse work.  `tile_bytes` is the
// tile's span (64 x stride); the last tile is clipped.
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void tile_rw_ref_kernel(const uint8_t* __restrict__ frames, uint32_t frames_bytes,
                        const uint32_t* __restrict__ offsets, uint32_t tile_bytes, uint32_t n,
                        u32x4* __restrict__ out) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t t = blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const uint32_t p0 = t * kWave;
    if (p0 >= n) return;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, frames_bytes);
    uint32_t s = t * tile_bytes, e = s + tile_bytes;
    if (offsets) {                                   // packed: the tile's frames' span
        s = offsets[p0];
        e = offsets[p0 + kWave < n ? p0 + kWave : n];
    }
    e = e < frames_bytes ? e : frames_bytes;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (uint32_t a = (s & ~15u) + 16u * lane; a < e; a += 16u * kWave * 8) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = load16_fast<2>(rs, a + 16u * kWave * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u];
    }
    const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t c = k * kWave + lane;
        if (c / 5 < nrec) __builtin_nontemporal_store(acc + c, &out[(size_t)p0 * 5 + c]);
    }
}

#endif  // RPKT_ABLATE

// ---- flow counters: LDS-privatised histogram per workgroup + slab reduce ----
// One workgroup per CU-sized slice of the events; each keeps, per bucket in LDS, a
// u64 {pkts | bytes << 16} (one 64-bit LDS atomic per event; a slice holds at most
// 32768 events, so pkts never carries into bytes, and 48 bits hold the bytes of any
// slice) and a u32 {ip_bad | l4_bad << 16}, writes them once to its slab, and a
// second kernel sums the slabs in a fixed order (bitwise reproducible counters).
// Slab layout: u64[rows] then u32[rows] (3 * rows dwords).
// 16 waves per block, one block per CU (its LDS histogram): 1M events 14.8 -> 12.6 us
// against 8 waves, 8M events 25.2 vs 25.5 us; 4 waves slower at both sizes
// (profiles/r02_ab_flowthreads)
#ifndef RPKT_FLOW_THREADS
#define RPKT_FLOW_THREADS 1024
#endif
constexpr int kFlowThreads = RPKT_FLOW_THREADS;
constexpr uint32_t kFlowLdsMax = 8192;      // buckets (+1 unparsed row) privatised in LDS
constexpr uint32_t kFlowMaxPerBlock = 32768;
constexpr uint32_t kFlowMinBlocks = 256;
constexpr int kFlowUnroll = 8;

// at least 16384 events per slab: below that the slabs' fixed cost (each holds every
// bucket, written once and read by the reduce) outweighs spreading the atomics over
// more CUs (1M events: 256 slabs 21.4 us, 128 17.3, 64 14.8; profiles/r02_ab_flow_small)
#ifndef RPKT_FLOW_MIN_PER_BLOCK
#define RPKT_FLOW_MIN_PER_BLOCK 16384
#endif
__host__ __device__ inline uint32_t flow_blocks(uint32_t n) {
    uint32_t b = (n + kFlowMaxPerBlock - 1) / kFlowMaxPerBlock;
    uint32_t m = (n + RPKT_FLOW_MIN_PER_BLOCK - 1) / RPKT_FLOW_MIN_PER_BLOCK;   // slabs of >= 16384
    uint32_t want = kFlowMinBlocks < m ? kFlowMinBlocks : m;
    return b > want ? b : (want ? want : 1);
}

__global__ __launch_bounds__(kFlowThreads)
void flow_hist_kernel(const uint64_t* __restrict__ ev, uint32_t n, uint32_t per_block,
                      uint32_t n_buckets, uint32_t* __restrict__ slab) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];   // 3 * (n_buckets + 1)
    const uint32_t rows = n_buckets + 1;
    unsigned long long* pb = reinterpret_cast<unsigned long long*>(h);  // pkts | bytes << 16
    uint32_t* bad_h = h + 2 * rows;                                     // ip_bad | l4_bad << 16
    for (uint32_t r = threadIdx.x; r < 3 * rows; r += blockDim.x) h[r] = 0;
    __syncthreads();
    const uint32_t lo = blockIdx.x * per_block;
    const uint32_t hi = min(n, lo + per_block);
    for (uint32_t i0 = lo; i0 < hi; i0 += kFlowThreads * kFlowUnroll) {
        uint64_t e[kFlowUnroll];
#pragma unroll
        for (int u = 0; u < kFlowUnroll; ++u) {
            const uint32_t i = i0 + u * kFlowThreads + threadIdx.x;
            e[u] = i < hi ? ev[i] : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < kFlowUnroll; ++u) {
            if (e[u] == ~0ull) continue;
            uint32_t b = (uint32_t)(e[u] >> 32) & 0xffffu;
            if (b > n_buckets) b = n_buckets;
            atomicAdd(&pb[b], 1ull | ((e[u] & 0xffffffffull) << 16));
            const uint32_t bad =
                (uint32_t)((e[u] >> 48) & 1u) | ((uint32_t)((e[u] >> 49) & 1u) << 16);
            if (bad) atomicAdd(&bad_h[b], bad);
        }
    }
    __syncthreads();
    uint32_t* out = slab + (size_t)blockIdx.x * 3 * rows;
    for (uint32_t r = threadIdx.x; r < 3 * rows; r += blockDim.x) out[r] = h[r];
}

// Slab reduce without atomics: block x owns buckets [64x, 64x + 64); its 16 waves
// split the slabs (wave w sums slabs w, w + 16, ...; lane = bucket, so every load is
// a coalesced 256-B row), the 16 partials meet in LDS, and wave 0 adds the totals to
// the counters.  Each bucket has one writer, and integer sums in a fixed order give
// the same bits every run.  (The earlier form, 16 slab groups per bucket joined by
// u64 atomics, was atomic-bound: 18 us at 8M events; 4 groups 35 us, 64 groups 38 us.)
constexpr uint32_t kReduceWaves = 16;

__global__ __launch_bounds__(kWave * kReduceWaves)
void flow_reduce_kernel(const uint32_t* __restrict__ slab, uint32_t n_slabs,
                        uint32_t n_buckets, unsigned long long* __restrict__ counters) {
    __shared__ uint32_t part[kReduceWaves][5][kWave];     // pk, bytes lo, bytes hi, ipb, l4b
    const uint32_t rows = n_buckets + 1;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const uint32_t b = blockIdx.x * kWave + lane;
    uint32_t pk = 0, ipb = 0, l4b = 0;
    uint64_t by = 0;
    if (b < rows) {
#pragma unroll 4
        for (uint32_t s = w; s < n_slabs; s += kReduceWaves) {
            const uint32_t* sl = slab + (size_t)s * 3 * rows;    // 4-B aligned: two dwords
            const uint64_t v = sl[2 * b] | ((uint64_t)sl[2 * b + 1] << 32);
            pk += (uint32_t)v & 0xffffu;
            by += v >> 16;
            const uint32_t bad = sl[2 * rows + b];
            ipb += bad & 0xffffu;
            l4b += bad >> 16;
        }
    }
    part[w][0][lane] = pk;
    part[w][1][lane] = (uint32_t)by;
    part[w][2][lane] = (uint32_t)(by >> 32);
    part[w][3][lane] = ipb;
    part[w][4][lane] = l4b;
    __syncthreads();
    if (w != 0 || b >= rows) return;
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#pragma unroll
    for (uint32_t k = 0; k < kReduceWaves; ++k) {
        t0 += part[k][0][lane];
        t1 += part[k][1][lane] | ((uint64_t)part[k][2][lane] << 32);
        t2 += part[k][3][lane];
        t3 += part[k][4][lane];
    }
    counters[4 * b + 0] += t0;
    counters[4 * b + 1] += t1;
    counters[4 * b + 2] += t2;
    counters[4 * b + 3] += t3;
}

// n_buckets above the LDS limit: one global atomic set per event.
__global__ void flow_atomic_kernel(const uint64_t* __restrict__ ev, uint32_t n,
                                   uint32_t n_buckets, unsigned long long* counters) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t e = ev[i];
        uint32_t b = (uint32_t)(e >> 32) & 0xffffu;
        if (b > n_buckets) b = n_buckets;
        atomicAdd(&counters[4 * b + 0], 1ull);
        atomicAdd(&counters[4 * b + 1], (unsigned long long)(e & 0xffffffffu));
        if ((e >> 48) & 1u) atomicAdd(&counters[4 * b + 2], 1ull);
        if ((e >> 49) & 1u) atomicAdd(&counters[4 * b + 3], 1ull);
    }
}

// ---- batched checksum::from_slice over ranges ----
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void checksum_ranges_kernel(const uint8_t* __restrict__ buf, uint32_t buf_bytes,
                            const uint32_t* __restrict__ ranges, uint32_t n,
                            uint16_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    uint32_t s = 0, e = 0;
    if (i < n) {
        uint64_t st = ranges[2 * i], ln = ranges[2 * i + 1];
        if (st > buf_bytes) st = buf_bytes;
        if (st + ln > buf_bytes) ln = buf_bytes - st;
        s = (uint32_t)st;
        e = (uint32_t)(st + ln);
    }
    const uint32_t part =
        wave_stream_sum(make_rsrc(buf, buf_bytes), buf_bytes, s, e, scratch[wid], lane);
    if (i < n) out[i] = (uint16_t)be_sum(part, s);
}

// ---- batched checksum::from_buf over segment chains (mbuf chains) ----
// Pass 1: every segment's standalone big-endian sum (the ranges kernel) plus its
// length parity.  Pass 2: lane per chain folds its segments in order; a segment that
// starts at an odd offset of the chain's byte stream contributes its byte-swapped
// sum, which is exactly from_buf's pairing of a chunk's odd tail byte with the next
// chunk's first byte (checksum.rs:13-24, 82-88).
__global__ __launch_bounds__(kWave * kWavesPerBlock)
void segment_sums_kernel(const uint8_t* __restrict__ buf, uint32_t buf_bytes,
                         const uint32_t* __restrict__ segs, uint32_t n,
                         uint32_t* __restrict__ seg_out) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    uint32_t s = 0, e = 0, len = 0;
    if (i < n) {
        uint64_t st = segs[2 * i], ln = segs[2 * i + 1];
        len = (uint32_t)ln;
        if (st > buf_bytes) st = buf_bytes;
        if (st + ln > buf_bytes) ln = buf_bytes - st;
        s = (uint32_t)st;
        e = (uint32_t)(st + ln);
    }
    const uint32_t part =
        wave_stream_sum(make_rsrc(buf, buf_bytes), buf_bytes, s, e, scratch[wid], lane);
    if (i < n) seg_out[i] = be_sum(part, s) | ((len & 1u) << 16);
}

__global__ void chain_fold_kernel(const uint32_t* __restrict__ seg_out,
                                  const uint32_t* __restrict__ first, uint32_t n_chains,
                                  uint32_t n_segs, uint16_t* __restrict__ out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_chains) return;
    uint32_t a = first[p], b = first[p + 1];
    if (b > n_segs) b = n_segs;
    uint32_t acc = 0, odd = 0;
    for (uint32_t i = a; i < b; ++i) {
        const uint32_t v = seg_out[i];
        const uint32_t sum = v & 0xffffu;
        acc += odd ? bswap16(sum) : sum;
        odd ^= v >> 16;
    }
    out[p] = (uint16_t)fold16(acc);
}

// flags the batch / ring / fused-option parses accept
constexpr uint32_t kParseFlags = RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_FLOW_EV | RPKT_F_IPV6;

// every frame of a strided batch inside the header window from its 16-B boundary (the
// frame at i * stride has phase (i * stride) & 15: 0 for strides of 16-B multiples)
inline bool window_fits(const rpkt_batch_t& b, uint32_t win) {
    const uint32_t flen = b.frame_len ? b.frame_len : b.stride;
    if (b.offsets_dev || b.stride == 0 || flen == 0) return false;
    return flen + ((b.stride & 15u) ? 15u : 0u) <= win;
}

// shared checks of the parse entry points
int parse_args_ok(const rpkt_batch_t* b, uint32_t flags, const void* recs_dev,
                         const void* flow_ev_dev, uint32_t n_buckets) {
    if (!b || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~kParseFlags) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0) return RPKT_E_ALIGN;
    if (flags & RPKT_F_FLOW_EV) {
        if (!flow_ev_dev || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS)
            return RPKT_E_INVAL;
        if (((uintptr_t)flow_ev_dev & 7u) != 0) return RPKT_E_ALIGN;
    }
    return 1;
}

template <bool C16>
int parse_options(const rpkt_batch_t* b, uint32_t flags, void* recs_dev, rpkt_opts_t* opts_dev,
                         rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!opts_dev) return RPKT_E_INVAL;
    const int ok = parse_args_ok(b, flags, recs_dev, flow_ev_dev, n_buckets);
    if (ok != 1) return ok;
    if (((uintptr_t)opts_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_F_L4_SUM) ? parse_kernel<true, 0, C16, true>
                                     : parse_kernel<false, 0, C16, true>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  (rpkt_rec_t*)recs_dev, (uint64_t*)flow_ev_dev, n_buckets, opts_dev);
}

template <bool C16>
int parse_ring(const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags,
                      uint32_t n_buckets, void* stream) {
    if (n_slots && !slots) return RPKT_E_INVAL;
    if (flags & ~kParseFlags) return RPKT_E_INVAL;
    const bool fev = (flags & RPKT_F_FLOW_EV) != 0;
    for (uint32_t k = 0; k < n_slots; ++k) {                      // all checked, then launched
        const rpkt_ring_slot_t& q = slots[k];
        const rpkt_batch_t& b = q.batch;
        if (b.n == 0) continue;                // as rpkt_gpu_parse_batch with n == 0: RPKT_OK
        if (fev && (n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS)) return RPKT_E_INVAL;
        if (!b.frames_dev || !q.recs_dev) return RPKT_E_INVAL;
        if (b.frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
        if (!b.offsets_dev && b.stride == 0) return RPKT_E_INVAL;
        if (((uintptr_t)q.recs_dev & 15u) != 0) return RPKT_E_ALIGN;
        if (fev && !q.flow_ev_dev) return RPKT_E_INVAL;
        if (fev && ((uintptr_t)q.flow_ev_dev & 7u) != 0) return RPKT_E_ALIGN;
    }
    bool inwin = (flags & RPKT_F_L4_SUM) != 0;                    // every slot's frames in LDS
    for (uint32_t k = 0; inwin && k < n_slots; ++k)
        inwin = slots[k].batch.n == 0 || window_fits(slots[k].batch, (uint32_t)kWin);
    auto k = !(flags & RPKT_F_L4_SUM) ? parse_ring_kernel<false, C16>
           : inwin                    ? parse_ring_kernel<true, C16, true>
                                      : parse_ring_kernel<true, C16>;
    RingArgs A;
    uint32_t k0 = 0;
    while (k0 < n_slots) {
        A.n_slots = 0;
        A.tile0[0] = 0;
        for (; k0 < n_slots && A.n_slots < kRingMax; ++k0) {
            const rpkt_ring_slot_t& q = slots[k0];
            const rpkt_batch_t& b = q.batch;
            if (b.n == 0) continue;
            RingSlot& S = A.s[A.n_slots];
            S.frames = b.frames_dev;
            S.offsets = b.offsets_dev;
            S.recs = (rpkt_rec_t*)q.recs_dev;
            S.flow_ev = fev ? (uint64_t*)q.flow_ev_dev : nullptr;
            S.frames_bytes = (uint32_t)b.frames_bytes;
            S.stride = b.stride;
            S.frame_len = b.offsets_dev ? 0u : (b.frame_len ? b.frame_len : b.stride);
            S.n = b.n;
            A.tile0[A.n_slots + 1] = A.tile0[A.n_slots] + (b.n + kWave - 1) / kWave;
            ++A.n_slots;
        }
        if (A.n_slots == 0) break;
        const uint32_t waves = A.tile0[A.n_slots];
        const int rc = launch(k, dim3((waves + kRingWPB - 1) / kRingWPB), dim3(kWave * kRingWPB),
                              0, (hipStream_t)stream, A, flags, n_buckets);
        if (rc) return rc;
    }
    return RPKT_OK;
}

}  // namespace

// This unit compiles twice: as is (128-B windows) and with RPKT_PARSE_W64 (RPKT_WIN 64,
// rpkt_amd/build.py), whose only entry points are the hidden
// rpkt_gpu_parse_batch_compact_w64 / rpkt_gpu_parse_ring_compact_w64 the first compile
// hands strided batches (rings of them) of short frames to: every frame lies inside its 64-B window (parse_w64_fits), so the headers
// and the L4 bytes are all in LDS, a wave's LDS drops from 9.7 to 6.5 KB (the window
// area keeps the 64 x 21-dword record stage's 5376 B), and with the 16-B records kept in
// registers the VGPRs, not the LDS, set the waves per SIMD.
#ifndef RPKT_PARSE_W64_ON
#define RPKT_PARSE_W64_ON 1
#endif

extern "C" {

#ifdef RPKT_PARSE_W64
__attribute__((visibility("hidden"))) int rpkt_gpu_parse_ring_compact_w64(
    const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags, uint32_t n_buckets,
    void* stream) {
    return parse_ring<true>(slots, n_slots, flags, n_buckets, stream);
}
__attribute__((visibility("hidden"))) int rpkt_gpu_parse_batch_compact_w64(
    const rpkt_batch_t* b, uint32_t flags, rpkt_rec16_t* recs_dev, rpkt_flow_ev_t* flow_ev_dev,
    uint32_t n_buckets, void* stream) {
    const uint32_t flen = b->frame_len ? b->frame_len : b->stride;
    const uint32_t per_block = kWave * kParseWPB;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    // the caller checked that every frame lies in its 64-B window: in-window L4 sums
    auto k = (flags & RPKT_F_L4_SUM) ? parse_kernel<true, 0, true, false, kParseWPB, true>
                                     : parse_kernel<false, 0, true, false, kParseWPB>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  (rpkt_rec_t*)recs_dev, (uint64_t*)flow_ev_dev, n_buckets,
                  (rpkt_opts_t*)nullptr);
}
// 80-B records with the L4 sum (RPKT_PARSE_W64_FULL): the record stage keeps the
// window area at 5376 B, so a wave needs 6.5 KB of LDS instead of 9.7 KB and the
// in-window L4 instantiation (68 VGPRs) runs 6 waves per SIMD instead of 4
__attribute__((visibility("hidden"))) int rpkt_gpu_parse_batch_l4_w64(
    const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs_dev, rpkt_flow_ev_t* flow_ev_dev,
    uint32_t n_buckets, void* stream) {
    const uint32_t flen = b->frame_len ? b->frame_len : b->stride;
    const uint32_t per_block = kWave * kParseWPB;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_F_L4_SUM) ? parse_kernel<true, 0, false, false, kParseWPB, true>
                                     : parse_kernel<false, 0, false, false, kParseWPB>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  recs_dev, (uint64_t*)flow_ev_dev, n_buckets, (rpkt_opts_t*)nullptr);
}
#else
int rpkt_gpu_parse_batch_compact_w64(const rpkt_batch_t*, uint32_t, rpkt_rec16_t*,
                                     rpkt_flow_ev_t*, uint32_t, void*);
int rpkt_gpu_parse_batch_l4_w64(const rpkt_batch_t*, uint32_t, rpkt_rec_t*, rpkt_flow_ev_t*,
                                uint32_t, void*);
#ifndef RPKT_PARSE_W64_FULL
#define RPKT_PARSE_W64_FULL 1
#endif
int rpkt_gpu_parse_ring_compact_w64(const rpkt_ring_slot_t*, uint32_t, uint32_t, uint32_t, void*);

// every frame of a strided batch inside a 64-B window from its 16-B boundary
static bool parse_w64_fits(const rpkt_batch_t* b, uint32_t flen) {
    if (b->offsets_dev || b->stride == 0 || flen == 0) return false;
    return flen + ((b->stride & 15u) ? 15u : 0u) <= 64u;
}

uint32_t rpkt_flow_hash(uint32_t ip_src, uint32_t ip_dst, uint16_t sp, uint16_t dp,
                        uint8_t proto) {
    uint32_t h = 0x811c9dc5u;
    h = (h ^ ip_src) * 0x01000193u;
    h = (h ^ ip_dst) * 0x01000193u;
    h = (h ^ (((uint32_t)sp << 16) | dp)) * 0x01000193u;
    h = (h ^ proto) * 0x01000193u;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

int rpkt_gpu_parse_batch(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs_dev,
                         rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!b || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~kParseFlags) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0) return RPKT_E_ALIGN;
    if (flags & RPKT_F_FLOW_EV) {
        if (!flow_ev_dev || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS)
            return RPKT_E_INVAL;
        if (((uintptr_t)flow_ev_dev & 7u) != 0) return RPKT_E_ALIGN;
    }
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    if (RPKT_PARSE_W64_ON && RPKT_PARSE_W64_FULL && ((flags & RPKT_F_L4_SUM) || RPKT_PARSE_W64_FULL > 1) &&
        parse_w64_fits(b, flen))
        return rpkt_gpu_parse_batch_l4_w64(b, flags, recs_dev, flow_ev_dev, n_buckets, stream);
    const uint32_t per_block = kWave * kParseWPB;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = !(flags & RPKT_F_L4_SUM)     ? parse_kernel<false, 0, false, false, kParseWPB>
           : window_fits(*b, (uint32_t)kWin) ? parse_kernel<true, 0, false, false, kParseWPB, true>
                                            : parse_kernel<true, 0, false, false, kParseWPB>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  recs_dev, (uint64_t*)flow_ev_dev, n_buckets, (rpkt_opts_t*)nullptr);
}

int rpkt_gpu_parse_ring(const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags,
                        uint32_t n_buckets, void* stream) {
    return parse_ring<false>(slots, n_slots, flags, n_buckets, stream);
}

int rpkt_gpu_parse_ring_compact(const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags,
                                uint32_t n_buckets, void* stream) {
    // a ring whose every slot is a strided batch of short frames goes to the 64-B-window
    // compile, as rpkt_gpu_parse_batch_compact hands such a batch over
    bool w64 = RPKT_PARSE_W64_ON && slots && n_slots;
    for (uint32_t k = 0; w64 && k < n_slots; ++k) {
        const rpkt_batch_t& b = slots[k].batch;
        w64 = b.n == 0 || parse_w64_fits(&b, b.frame_len ? b.frame_len : b.stride);
    }
    return w64 ? rpkt_gpu_parse_ring_compact_w64(slots, n_slots, flags, n_buckets, stream)
               : parse_ring<true>(slots, n_slots, flags, n_buckets, stream);
}

int rpkt_gpu_parse_batch_compact(const rpkt_batch_t* b, uint32_t flags, rpkt_rec16_t* recs_dev,
                                 rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!b || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~kParseFlags) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0) return RPKT_E_ALIGN;
    if (flags & RPKT_F_FLOW_EV) {
        if (!flow_ev_dev || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS)
            return RPKT_E_INVAL;
        if (((uintptr_t)flow_ev_dev & 7u) != 0) return RPKT_E_ALIGN;
    }
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    if (RPKT_PARSE_W64_ON && parse_w64_fits(b, flen))
        return rpkt_gpu_parse_batch_compact_w64(b, flags, recs_dev, flow_ev_dev, n_buckets, stream);
    const uint32_t per_block = kWave * kParseWPB;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = !(flags & RPKT_F_L4_SUM)     ? parse_kernel<false, 0, true, false, kParseWPB>
           : window_fits(*b, (uint32_t)kWin) ? parse_kernel<true, 0, true, false, kParseWPB, true>
                                            : parse_kernel<true, 0, true, false, kParseWPB>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  (rpkt_rec_t*)recs_dev, (uint64_t*)flow_ev_dev, n_buckets,
                  (rpkt_opts_t*)nullptr);
}

int rpkt_gpu_parse_options_batch(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs_dev,
                                 rpkt_opts_t* opts_dev, rpkt_flow_ev_t* flow_ev_dev,
                                 uint32_t n_buckets, void* stream) {
    return parse_options<false>(b, flags, recs_dev, opts_dev, flow_ev_dev, n_buckets, stream);
}

int rpkt_gpu_parse_options_batch_compact(const rpkt_batch_t* b, uint32_t flags,
                                         rpkt_rec16_t* recs_dev, rpkt_opts_t* opts_dev,
                                         rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets,
                                         void* stream) {
    return parse_options<true>(b, flags, recs_dev, opts_dev, flow_ev_dev, n_buckets, stream);
}

int rpkt_gpu_parse_chains(const rpkt_chains_t* c, uint32_t flags, rpkt_rec_t* recs_dev,
                          rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!c || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~kParseFlags) return RPKT_E_INVAL;
    if (c->n_chains == 0) return RPKT_OK;
    if (!c->chain_first_dev || (c->n_segs && (!c->buf_dev || !c->segs_dev))) return RPKT_E_INVAL;
    if (c->buf_bytes > kMaxFrameBytes || c->n_segs >= 0x80000000u) return RPKT_E_TOO_LARGE;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)c->segs_dev & 7u) != 0) return RPKT_E_ALIGN;
    if (flags & RPKT_F_FLOW_EV) {
        if (!flow_ev_dev || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS)
            return RPKT_E_INVAL;
        if (((uintptr_t)flow_ev_dev & 7u) != 0) return RPKT_E_ALIGN;
    }
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (c->n_chains + per_block - 1) / per_block;
    auto k = (flags & RPKT_F_L4_SUM) ? parse_chains_kernel<true> : parse_chains_kernel<false>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, c->buf_dev,
                  (uint32_t)c->buf_bytes, (const uint2*)c->segs_dev, c->n_segs,
                  c->chain_first_dev, c->n_chains, flags, recs_dev, (uint64_t*)flow_ev_dev,
                  n_buckets);
}

#ifdef RPKT_ABLATE
// Development hook (librpkt_gpu_ablate.so only, not part of include/rpkt_gpu.h): the
// parse kernel's ablation variants and the streaming references, for tools/ablate.py,
// tools/variant_check.py and bench.py's copy_ceiling.
int rpkt_gpu_debug_variant(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs, int variant,
                           void* stream) {
    if (!b || !recs || b->n == 0) return RPKT_E_INVAL;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    hipStream_t st = (hipStream_t)stream;
#define RPKT_V(v)                                                                       \
    launch((flags & RPKT_F_L4_SUM) ? parse_kernel<true, v> : parse_kernel<false, v>,   \
           dim3(grid), dim3(per_block), 0, st, b->frames_dev, (uint32_t)b->frames_bytes,   \
           b->offsets_dev, b->stride, flen, b->n, flags, recs, (uint64_t*)nullptr, 0u,      \
           (rpkt_opts_t*)nullptr)
    switch (variant) {
        case 0: return RPKT_V(0);
        case 1: return RPKT_V(1);
        case 3: return RPKT_V(3);
        case 8: return RPKT_V(8);
        case 21: return RPKT_V(21);
        case 22: return RPKT_V(22);
        case 23: return RPKT_V(23);
        case 24: return RPKT_V(24);
        case 25: return RPKT_V(25);
        case 40: return RPKT_V(40);
        case 41: return RPKT_V(41);
        case 42: return RPKT_V(42);
        case 43: return RPKT_V(43);
        case 44: return RPKT_V(44);
        case 45: return RPKT_V(45);
        case 10:
            return launch(copy_ref_kernel<4, false>, dim3(2048), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (u32x4*)recs, b->n * (RPKT_REC_BYTES / 16));
        case 11:
            return launch(copy_ref_kernel<8, false>, dim3(2048), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (u32x4*)recs, b->n * (RPKT_REC_BYTES / 16));
        case 12:
            return launch(copy_ref_kernel<8, true>, dim3(2048), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (u32x4*)recs, b->n * (RPKT_REC_BYTES / 16));
        case 14:
            return launch(read_ref_kernel, dim3(4096), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (uint32_t*)recs);
        case 15:
            return launch(tile_rw_ref_kernel, dim3(grid), dim3(per_block), 0, st, b->frames_dev,
                          (uint32_t)b->frames_bytes, b->offsets_dev, b->stride * kWave, b->n,
                          (u32x4*)recs);
        // wave-contiguous references: 16/17 the read:write mix of the batch (frames read,
        // n x 80 B written) default / non-temporal, 18/19 a memcpy of the frames buffer
        // into recs (frames_bytes of it) default / non-temporal
        case 16: case 17: case 18: case 19: {
            const uint32_t in16 = (uint32_t)(b->frames_bytes / 16);
            const uint32_t out16 = variant >= 18 ? in16 : b->n * (RPKT_REC_BYTES / 16);
            // 16384 waves: tools/copybw.hip's best mixed shape (4096 waves: 5.1-5.4 TB/s)
            const dim3 g(4096), blk(kWave * kWavesPerBlock);
            switch (variant) {
                case 16: return launch(wave_stream_ref_kernel<0, false, false>, g, blk, 0, st,
                                       b->frames_dev, in16, (u32x4*)recs, out16);
                case 17: return launch(wave_stream_ref_kernel<2, true, false>, g, blk, 0, st,
                                       b->frames_dev, in16, (u32x4*)recs, out16);
                case 18: return launch(wave_stream_ref_kernel<0, false, true>, g, blk, 0, st,
                                       b->frames_dev, in16, (u32x4*)recs, out16);
                default: return launch(wave_stream_ref_kernel<2, true, true>, g, blk, 0, st,
                                       b->frames_dev, in16, (u32x4*)recs, out16);
            }
        }
        case 13:
            return launch(copy_ref_kernel<8, false>, dim3(8192), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (u32x4*)recs, b->n * (RPKT_REC_BYTES / 16));
        default: return RPKT_E_INVAL;
    }
#undef RPKT_V
}

// The parse with per-wave clock stamps (variant 50, 32 B per wave of the grid in
// stamps_dev), for tools/launch_stamps.py: where a launch's fixed cost goes.
// wpb: waves per block, 1, 2 or 4 (the product's); stamps_dev may be null (variant 0:
// the product kernel at that block size)
extern "C++" template <int WPB>
int launch_stamps(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs, void* stamps_dev,
                  hipStream_t st) {
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * WPB;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    const bool l4 = (flags & RPKT_F_L4_SUM) != 0;
    auto k = stamps_dev ? (l4 ? parse_kernel<true, 50, false, false, WPB>
                              : parse_kernel<false, 50, false, false, WPB>)
                        : (l4 ? parse_kernel<true, 0, false, false, WPB>
                              : parse_kernel<false, 0, false, false, WPB>);
    return launch(k, dim3(grid), dim3(per_block), 0, st, b->frames_dev, (uint32_t)b->frames_bytes,
                  b->offsets_dev, b->stride, flen, b->n, flags & kParseFlags, recs,
                  (uint64_t*)stamps_dev, 0u, (rpkt_opts_t*)nullptr);
}
int rpkt_gpu_debug_stamps(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* recs,
                          void* stamps_dev, int wpb, void* stream) {
    if (!b || !recs || b->n == 0 || (flags & RPKT_F_FLOW_EV)) return RPKT_E_INVAL;
    switch (wpb) {
        case 1: return launch_stamps<1>(b, flags, recs, stamps_dev, (hipStream_t)stream);
        case 2: return launch_stamps<2>(b, flags, recs, stamps_dev, (hipStream_t)stream);
        case 4: return launch_stamps<4>(b, flags, recs, stamps_dev, (hipStream_t)stream);
        default: return RPKT_E_INVAL;
    }
}

#endif  // RPKT_ABLATE

// The histogram's 98 KB of dynamic LDS needs hipFuncSetAttribute once per device (the
// attribute belongs to the function on the current device).  Host threads may call the
// ABI concurrently and a process may drive several GPUs (examples/flow_reduce.cpp), so
// the flag is per device and set under a lock; a failed attempt is retried next call.
static int flow_hist_attr_once() {
    static std::mutex mu;
    static uint64_t done[4] = {0, 0, 0, 0};          // bit d: device d (up to 256 devices)
    int dev = -1;
    {
        const int rc = hip_check(hipGetDevice(&dev));
        if (rc) return rc;
    }
    auto set = [] {
        return hip_check(hipFuncSetAttribute((const void*)flow_hist_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             3 * (kFlowLdsMax + 1) * sizeof(uint32_t)));
    };
    if (dev < 0 || dev >= 256) return set();         // not cached: set on every call
    std::lock_guard<std::mutex> g(mu);
    if (done[dev >> 6] & (1ull << (dev & 63))) return RPKT_OK;
    const int rc = set();
    if (rc == RPKT_OK) done[dev >> 6] |= 1ull << (dev & 63);
    return rc;
}

size_t rpkt_gpu_flow_workspace_bytes(uint32_t n, uint32_t n_buckets) {
    if (n_buckets > kFlowLdsMax) return 16;
    return (size_t)flow_blocks(n) * 3 * (size_t)(n_buckets + 1) * sizeof(uint32_t);
}

int rpkt_gpu_flow_count(const rpkt_flow_ev_t* ev, uint32_t n, uint32_t n_buckets,
                        uint64_t* counters, void* workspace, void* stream) {
    if (!counters || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS) return RPKT_E_INVAL;
    if (n == 0) return RPKT_OK;
    if (!ev) return RPKT_E_INVAL;
    hipStream_t st = (hipStream_t)stream;
    if (n_buckets > kFlowLdsMax) {
        return launch(flow_atomic_kernel, dim3(1024), dim3(256), 0, st, (const uint64_t*)ev, n,
                      n_buckets, (unsigned long long*)counters);
    }
    if (!workspace) return RPKT_E_INVAL;
    const uint32_t slabs = flow_blocks(n);
    const uint32_t per = (n + slabs - 1) / slabs;
    const size_t lds = 3 * (size_t)(n_buckets + 1) * sizeof(uint32_t);
    {
        const int rc0 = flow_hist_attr_once();
        if (rc0) return rc0;
    }
    int rc = launch(flow_hist_kernel, dim3(slabs), dim3(kFlowThreads), lds, st,
                    (const uint64_t*)ev, n, per, n_buckets, (uint32_t*)workspace);
    if (rc) return rc;
    const uint32_t rows = n_buckets + 1;
    return launch(flow_reduce_kernel, dim3((rows + kWave - 1) / kWave), dim3(kWave * kReduceWaves),
                  0, st, (const uint32_t*)workspace, slabs, n_buckets,
                  (unsigned long long*)counters);
}

int rpkt_gpu_checksum_ranges(const uint8_t* buf, uint64_t buf_bytes, const uint32_t* ranges,
                             uint32_t n, uint16_t* out, void* stream) {
    if (n == 0) return RPKT_OK;
    if (!buf || !ranges || !out) return RPKT_E_INVAL;
    if (buf_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    const uint32_t per_block = kWave * kWavesPerBlock;
    return launch(checksum_ranges_kernel, dim3((n + per_block - 1) / per_block), dim3(per_block),
                  0, (hipStream_t)stream, buf, (uint32_t)buf_bytes, ranges, n, out);
}

size_t rpkt_gpu_checksum_chains_workspace_bytes(uint32_t n_segs) {
    return (size_t)(n_segs ? n_segs : 1) * sizeof(uint32_t);
}

int rpkt_gpu_checksum_chains(const uint8_t* buf, uint64_t buf_bytes, const uint32_t* segs,
                             uint32_t n_segs, const uint32_t* chain_first, uint32_t n_chains,
                             uint16_t* out, void* workspace, void* stream) {
    if (n_chains == 0) return RPKT_OK;
    if (!chain_first || !out || (n_segs && (!buf || !segs || !workspace))) return RPKT_E_INVAL;
    if (buf_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t per_block = kWave * kWavesPerBlock;
    if (n_segs) {
        int rc = launch(segment_sums_kernel, dim3((n_segs + per_block - 1) / per_block),
                        dim3(per_block), 0, st, buf, (uint32_t)buf_bytes, segs, n_segs,
                        (uint32_t*)workspace);
        if (rc) return rc;
    }
    return launch(chain_fold_kernel, dim3((n_chains + 255) / 256), dim3(256), 0, st,
                  (const uint32_t*)workspace, chain_first, n_chains, n_segs, out);
}

#endif  // RPKT_PARSE_W64

}  // extern "C"
