// rpkt_common.h — shared device code of the MI355X (gfx950, CDNA4) batch engine for
// Ether -> (802.1Q/802.1ad)* -> IPv4 -> {TCP, UDP} decode-and-verify path.
//
// One wavefront owns a tile of 64 frames.  The work is split three ways:
//   1. header window: the wave copies the first 128 aligned bytes of each of
//      its 64 frames into LDS with 16-byte buffer loads (8 chunks per frame,
//      one 1 KiB contiguous LDS write per wave-instruction);
//   2. lane-per-frame parse from LDS: the rpkt parse chain (EtherFrame::parse
//      ether/generated.rs:34-41, VlanFrame::parse vlan/generated.rs:32-39,
//      Ipv4::parse ipv4/generated.rs:35-51, Udp::parse udp/generated.rs:31-42,
//      Tcp::parse tcp/generated.rs:34-45) with every getter into registers, the
//      IPv4 header sum and the in-window part of the L4 sum;
//   3. the rest of each L4 segment (frames longer than the window) as ONE
//      flattened stream of 16-byte chunks over the whole tile: consecutive lanes
//      read consecutive chunks (coalesced HBM reads whatever the frame sizes),
//      each chunk's masked word sum enters a wave prefix scan (DPP), and every
//      frame's sum is the scan difference between its last and first chunk.
// All partial sums are taken over absolute-address-aligned little-endian
// 16-bit words; RFC 1071 byte-order independence makes the big-endian sum of a
// range equal to that sum when the range starts at an odd address and to its
// byte swap when it starts at an even one (checksum.rs:33-62 semantics,
// including the odd tail byte << 8 of :57-59).
//
// Loads go through a buffer resource descriptor whose range is frames_bytes, so
// a malformed offset table can only produce wrong records, never a fault.
//
// Everything here is inline in an anonymous namespace: each kernel file (rpkt_parse.hip,
// rpkt_tx.hip, rpkt_walks.hip) includes it and compiles on its own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <tuple>
#include <type_traits>

#include "../../include/rpkt_gpu.h"

namespace rpkt_detail {
// last HIP error seen by this thread (rpkt_gpu_last_hip_error); defined in rpkt_abi.hip
extern thread_local int g_last_hip_error;
}  // namespace rpkt_detail

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;            // lanes per wavefront (CDNA)
constexpr int kWavesPerBlock = 4;    // 256-thread workgroups
#ifndef RPKT_WIN
#define RPKT_WIN 128
#endif
// header window bytes per frame in LDS: 128, or 64 in the TX unit's second compile
// (rpkt_tx.hip with RPKT_TX_W64) for strided batches of frames within 64 bytes
constexpr int kWin = RPKT_WIN;
constexpr int kWinChunks = kWin / 16;
constexpr int kSlot = kWin + 4;      // LDS slot stride: 33 dwords, so lane-strided
                                     // reads of the 64 slots hit 32 distinct banks
constexpr int kStreamUnroll = 4;     // 16-B chunk loads in flight per lane per step
constexpr int kChainStreamUnroll = 8;  // the same in the mbuf-chain kernel
constexpr uint64_t kMaxFrameBytes = 0xffffff00ull;  // voffset + 16 never wraps
constexpr uint32_t kSplitStreamBytes = 65536;  // tile stream above which edge lines go first
constexpr uint32_t kEdgeWindowBytes = 32768;   // tile stream above which the window phase
                                               // sums the edge lines (edge_lines_window)

// the window area also stages a tile's 64 records (stride 21 dwords)
constexpr int kWinArea = kWave * kSlot > kWave * 21 * 4 ? kWave * kSlot : kWave * 21 * 4;
struct WaveScratch {                 // 9744 B per wave at kWin 128: 4 waves x 4 blocks fit a CU
    uint8_t  win[kWinArea];          // header windows, slot stride kWin + 4
    uint32_t s[kWave];               // window phase: frame offset; stream: range start
    uint32_t e[kWave];               // window phase: frame length; stream: range end
    uint32_t pref[kWave + 1];        // stream: exclusive prefix of chunk counts
    uint32_t first[kWave];           // stream: scan value before a range's first chunk
    uint32_t last[kWave];            // stream: scan value at a range's last chunk
};
static_assert(sizeof(WaveScratch) * kWavesPerBlock * 4 <= 160 * 1024, "4 blocks per CU");
static_assert(kWin != 128 || (64 * 21 + 705) * 4 <= kWinArea, "chain scratch fits the window area");

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

// 16 bytes at `off` of a buffer of `limit` bytes: bytes at or past `limit` read as 0.
// A dwordx4 that straddles the range end is dropped whole by the hardware range
// check, so the (at most one per buffer) straddling chunk is read as the last 16
// in-range bytes and shifted down.
__device__ __forceinline__ u32x4 load16_bytes(__amdgpu_buffer_rsrc_t r, uint32_t off,
                                                         uint32_t limit) {
    u32x4 v = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        uint32_t b = off + k < limit
                         ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(off + k), 0, 0)
                         : 0u;
        v[k >> 2] |= b << (8 * (k & 3));
    }
    return v;
}

// Branch-free main-path load: out-of-range and straddling chunks read as zeros (the
// caller patches a straddling chunk with load16_fix on a rare, separate path, so the
// hot loops carry no data-dependent vmcnt waits).
template <int AUX = 0>     // cache-policy bits of the buffer load (2 = nt)
__device__ __forceinline__ u32x4 load16_fast(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
}

__device__ __forceinline__ bool straddles(uint32_t off, uint32_t limit) {
    return off < limit && off + 16u > limit;
}

__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t limit) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (off + 16u <= limit) {
        v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    } else if (off < limit) {
        if (__builtin_expect(limit >= 16u, 1)) {
            u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(limit - 16u), 0, 0);
            unsigned __int128 x = (unsigned __int128)t.x | ((unsigned __int128)t.y << 32) |
                                  ((unsigned __int128)t.z << 64) | ((unsigned __int128)t.w << 96);
            x >>= 8u * (16u - (limit - off));
            v = u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
        } else {
            v = load16_bytes(r, off, limit);
        }
    }
    return v;
}

// Inclusive prefix sum over the 64 lanes (DPP: row shifts then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Inclusive max-scan over the 64 lanes (the same DPP pattern; 0 is the identity).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return __builtin_amdgcn_readlane(wave_incl_scan(x), 63);
}

// propagate_carries (checksum.rs:115-118) for any u32 partial: 0 iff x == 0.
__device__ __forceinline__ uint32_t fold16(uint32_t x) {
    x = (x & 0xffffu) + (x >> 16);
    x = (x & 0xffffu) + (x >> 16);
    return x;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
    return ((x & 0xffu) << 8) | (x >> 8);
}

// Big-endian RFC 1071 sum of a range from its absolute-phase LE partial.
__device__ __forceinline__ uint32_t be_sum(uint32_t le_partial, uint32_t start_abs) {
    uint32_t f = fold16(le_partial);
    return (start_abs & 1u) ? f : bswap16(f);
}

// Keep bytes [lo, hi) of a little-endian dword (lo, hi clamped to 0..4).
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi) {
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    uint32_t mh = (uint32_t)((1ull << (8 * hi)) - 1);
    uint32_t ml = (uint32_t)((1ull << (8 * lo)) - 1);
    return mh & ~ml;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// acc + low half + high half of w, in one v_dot2_u32_u16 against (1, 1)
__device__ __forceinline__ uint32_t hsum(uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), u16x2{1, 1}, acc, false);
}
__device__ __forceinline__ uint32_t halves(uint32_t w) { return hsum(w, 0u); }

// Word sum of bytes [lo, hi) of a 16-byte chunk (absolute phase).
__device__ __forceinline__ uint32_t chunk_sum(u32x4 d, int lo, int hi) {
    if (lo <= 0 && hi >= 16) return hsum(d.w, hsum(d.z, hsum(d.y, hsum(d.x, 0u))));
    uint32_t acc = hsum(d.x & byte_mask(lo, hi), 0u);
    acc = hsum(d.y & byte_mask(lo - 4, hi - 4), acc);
    acc = hsum(d.z & byte_mask(lo - 8, hi - 8), acc);
    return hsum(d.w & byte_mask(lo - 12, hi - 12), acc);
}

// Flattened chunk stream over the tile: lane q owns absolute byte range
// [s_abs, e_abs) (empty allowed); returns that range's absolute-phase word sum.
// The range splits into full 16-byte chunks [ceil16(s), floor16(e)) and at most two
// partial edge chunks.  The full chunks of all 64 ranges are concatenated and read
// by consecutive lanes (coalesced whatever the frame sizes); each chunk's plain word
// sum enters a wave-wide inclusive scan, and a range's sum is the scan value at its
// last chunk minus the value before its first.  The edge chunks are loaded by their
// owner lane alongside the stream and summed under a byte mask once per range, so
// the per-chunk path carries no masking, no clipping and no conditional load.  Loads
// are double-buffered (batch k+1 in flight while batch k is summed) and every load
// issues unconditionally (lanes past the end read the descriptor's out-of-range
// offset: zeros, no traffic), so the vmcnt waits stay exact.  A full chunk ends at or
// before its range end, so it never straddles the end of the buffer; only an edge
// chunk can, and it is re-read exactly after the loop.  `oob` = the descriptor's range.
template <int U>
struct StreamBatch {
    u32x4 d[U];
    uint32_t m[U];                   // owner q | first << 8 | last << 9
};

// Per-lane cursor over the concatenated full chunks: the owner range q of the lane's
// current chunk, its chunk span [p0, p1), and off = ceil16(s_q) - 16 * p0, so chunk c
// of range q is at off + 16 c.  The ranges are in chunk order, so a cursor only moves
// forward: one step to the next range, binary search only for jumps.
// Short ranges (under 64 chunks on average: packed IMIX-like tiles) make most steps
// jump, and a wave then runs the six dependent LDS reads of the search on nearly every
// chunk (config 4: a lane jumps on 71 % of its steps, some lane of the wave on 89 %).
// There the owners come from marks instead (MARKS): each range whose first chunk falls
// in the wave's current 64-chunk window writes its index + 1 at that position of a
// 64-entry LDS row (W.e, free during the stream), every lane reads its position, and an
// inclusive max-scan across the lanes carries each range to the chunks after its start,
// with the last owner of the window before as the floor.  No search, no branch.
struct StreamCursor {
    uint32_t q, p0, p1, off;
    uint32_t my_p0;            // MARKS: this lane's range: first chunk, and
    bool my_has;               //   whether it has any
    uint32_t carry;            // MARKS: owner + 1 of the previous window's last chunk
};
#ifndef RPKT_STREAM_MARKS
#define RPKT_STREAM_MARKS 1      // 0: the cursor with binary search on every tile
#endif

__device__ __forceinline__ void cursor_load(const WaveScratch& W, StreamCursor& k, uint32_t q) {
    k.q = q;
    k.p0 = W.pref[q];
    k.p1 = W.pref[q + 1];
    k.off = W.s[q];
}

template <int AUX, int U, bool MARKS>
__device__ __forceinline__ void stream_issue(__amdgpu_buffer_rsrc_t rs, uint32_t oob,
                                             WaveScratch& W, uint32_t total, uint32_t base,
                                             int lane, StreamCursor& k, StreamBatch<U>& B) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t c = base + u * kWave + lane;
        const bool valid = c < total;
        if constexpr (MARKS) {
            const uint32_t rel = k.my_p0 - (base + u * kWave);     // the window's start: uniform
            if (k.my_has && rel < (uint32_t)kWave) W.e[rel] = (uint32_t)lane + 1u;
            __builtin_amdgcn_wave_barrier();                       // LDS is in order per wave
            const uint32_t mk = W.e[lane];
            W.e[lane] = 0u;                                        // clear for the next window
            uint32_t v = wave_incl_max(mk);
            v = v > k.carry ? v : k.carry;
            k.carry = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
            const uint32_t q = valid ? v - 1u : 0u;
            const uint32_t p0 = W.pref[q], p1 = W.pref[q + 1];
            B.m[u] = q | ((uint32_t)(c == p0) << 8) | ((uint32_t)(c + 1 == p1) << 9);
            B.d[u] = load16_fast<AUX>(rs, valid ? W.s[q] + 16u * c : oob);
            continue;
        }
        if (valid && k.p1 <= c) {
            uint32_t q = k.q + 1;
            if (W.pref[q + 1] <= c) {
                q = 0;
#pragma unroll
                for (int step = 32; step; step >>= 1)
                    if (W.pref[q + step] <= c) q += step;
            }
            cursor_load(W, k, q);
        }
        // lanes past the end never match first/last: c >= total >= p1 > p0
        B.m[u] = k.q | ((uint32_t)(c == k.p0) << 8) | ((uint32_t)(c + 1 == k.p1) << 9);
        B.d[u] = load16_fast<AUX>(rs, valid ? k.off + 16u * c : oob);
    }
}

template <int U>
__device__ __forceinline__ void stream_consume(WaveScratch& W, uint32_t& run,
                                               const StreamBatch<U>& B) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32x4 d = B.d[u];
        const uint32_t v = hsum(d.w, hsum(d.z, hsum(d.y, hsum(d.x, 0u))));
        const uint32_t sc = wave_incl_scan(v) + run;
        run = __builtin_amdgcn_readlane(sc, 63);
        const uint32_t m = B.m[u], q = m & 63u;
        if (m & (1u << 8)) W.first[q] = sc - v;
        if (m & (1u << 9)) W.last[q] = sc;
    }
}

template <int AUX = 0, int U = kStreamUnroll>
__device__ __forceinline__ uint32_t wave_stream_sum(__amdgpu_buffer_rsrc_t rs, uint32_t oob,
                                                    uint32_t s_abs, uint32_t e_abs,
                                                    WaveScratch& W, int lane) {
    const bool ne = e_abs > s_abs;
    if (__ballot(ne) == 0) return 0u;          // uniform: no range in the wave, no loads
    const uint32_t S = (s_abs + 15u) & ~15u, E = e_abs & ~15u;
    // edge chunks: head [s, min(e, S)) in the chunk at floor16(s); tail [max(s, E), e)
    // in the chunk at E when that is not the head chunk
    const uint32_t hs = s_abs & ~15u;
    const bool head = ne && (s_abs & 15u);
    const bool tail = ne && (e_abs & 15u) && E >= S;
    const uint32_t ha = head ? hs : oob, ta = tail ? E : oob;
    const u32x4 hd = load16_fast<AUX>(rs, ha);
    const u32x4 td = load16_fast<AUX>(rs, ta);

    // the edge sums are taken once the first stream batch is in flight, so no edge load
    // is still outstanding when the loop starts (its vmcnt waits then count exactly the
    // stream's own loads)
    auto edges = [&]() -> uint32_t {
        u32x4 h = hd, t = td;
        // a chunk straddling the buffer end was dropped whole by the range check: re-read
        // it as the last 16 in-range bytes (rare path)
        const bool hfix = head && straddles(hs, oob), tfix = tail && straddles(E, oob);
        if (__builtin_expect(__ballot(hfix || tfix) != 0, 0)) {
            if (hfix) h = load16(rs, hs, oob);
            if (tfix) t = load16(rs, E, oob);
        }
        uint32_t x = 0;
        if (head) {
            const uint32_t he = e_abs - hs;
            x = chunk_sum(h, (int)(s_abs - hs), he < 16u ? (int)he : 16);
        }
        if (tail) x += chunk_sum(t, 0, (int)(e_abs - E));
        return x;
    };

    const uint32_t nch = ne && E > S ? (E - S) >> 4 : 0;
    const uint32_t incl = wave_incl_scan(nch);
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
    if (total == 0) return edges();                              // wave-uniform
    W.pref[lane] = incl - nch;
    if (lane == 63) W.pref[64] = incl;
    W.s[lane] = S - 16u * (incl - nch);
    W.e[lane] = 0;
    W.first[lane] = 0;
    W.last[lane] = 0;
    wave_sync();

    constexpr uint32_t kBatch = kWave * U;
    uint32_t run = 0;
    StreamCursor k;
    cursor_load(W, k, 0);
    k.my_p0 = incl - nch;
    k.my_has = nch != 0;
    k.carry = 0;
    StreamBatch<U> A, B;
    uint32_t base = 0;
    // the loop, with the owners from marks (short ranges) or from the cursor
    auto loop = [&](auto marks) -> uint32_t {
        constexpr bool M = decltype(marks)::value;
        stream_issue<AUX, U, M>(rs, oob, W, total, base, lane, k, A);
        const uint32_t edge = edges();
        for (;;) {
            stream_issue<AUX, U, M>(rs, oob, W, total, base + kBatch, lane, k, B);
            stream_consume<U>(W, run, A);
            stream_issue<AUX, U, M>(rs, oob, W, total, base + 2 * kBatch, lane, k, A);
            stream_consume<U>(W, run, B);
            base += 2 * kBatch;
            if (base >= total) break;
        }
        return edge;
    };
    const uint32_t edge = (RPKT_STREAM_MARKS && total < 64u * kWave)            // uniform
                              ? loop(std::integral_constant<bool, true>{})
                              : loop(std::integral_constant<bool, false>{});
    wave_sync();
    return (nch ? W.last[lane] - W.first[lane] : 0) + edge;
}

// Edge lines first (long tiles).  A frame's L4 stream shares a 128-B line with its own
// window (the line the window ends in) and, at its end, with the next frame's window;
// the memory side fetches whole lines.  On a long tile the stream reaches those lines
// tens of microseconds after the window loads, when L2 no longer holds them, so they
// came from HBM twice (+10-14 % traffic at 1500 B).  edge_lines_first sums each
// frame's partial head line [wend, he) and partial tail line [tb, fend) right after
// the window loads land, while those lines are in L2; stream_rest then streams only
// the line-aligned middle [he, tb) of a frame whose stream range is exactly
// [wend, fend), and the whole range of any other frame.
struct EdgeLines {
    bool on;                                 // wave-uniform
    uint32_t sum, mid_s, mid_e;
};

__device__ __forceinline__ EdgeLines edge_lines_first(__amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                                      WaveScratch& W, int lane, bool valid,
                                                      uint32_t wend, uint32_t fend) {
    EdgeLines X{false, 0u, 0u, 0u};
    const uint32_t span = (valid && fend > wend) ? fend - wend : 0u;
    if (wave_sum(span) <= kSplitStreamBytes) return X;            // wave-uniform
    X.on = true;
    const uint32_t he = span ? min((wend + 127u) & ~127u, fend) : 0u;
    const uint32_t tb = span ? max(fend & ~127u, he) : 0u;
    X.sum = wave_stream_sum<0>(rs, fb, span ? wend : 0u, he, W, lane);
    X.sum += wave_stream_sum<0>(rs, fb, tb, span ? fend : 0u, W, lane);
    X.mid_s = he;
    X.mid_e = tb;
    return X;
}

template <int AUX>
__device__ __forceinline__ uint32_t stream_rest(const EdgeLines& X, __amdgpu_buffer_rsrc_t rs,
                                                uint32_t fb, uint32_t ss, uint32_t se,
                                                uint32_t wend, uint32_t fend, WaveScratch& W,
                                                int lane) {
    if (!X.on) return wave_stream_sum<AUX>(rs, fb, ss, se, W, lane);
    const bool fast = se > ss && ss == wend && se == fend;
    const uint32_t sp = wave_stream_sum<AUX>(rs, fb, fast ? X.mid_s : ss, fast ? X.mid_e : se,
                                             W, lane);
    return fast ? sp + X.sum : sp;
}

// one byte at absolute offset a (0 past the descriptor range)
__device__ __forceinline__ uint32_t gbyte(__amdgpu_buffer_rsrc_t rs, uint32_t a) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)a, 0, 0);
}

struct Frame { uint32_t off, len; };

// Edge lines in the window phase (every tile).  The same split as edge_lines_first --
// a frame's partial head line [wend, he) and partial tail line [tb, fend) summed
// early, the stream then covering only [he, tb) -- but the edge chunks are loaded
// with the window, by the same cooperative mapping (chunk k of lane l: piece l % 8 of
// frame 8k + l / 8), and each frame's eight chunk sums are added by three DPP steps
// within its 8 lanes.  No scan, no extra pass: the head line is fetched once with
// the window it shares a line with, the tail line together with the next frame's
// window.  Sums land in W.first / W.last (free until the stream), one per frame.
__device__ __forceinline__ uint32_t sum8_lanes(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0xb1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x4e, 0xf, 0xf, false);   // quad_perm 2,3,0,1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xf, 0xf, false);  // row_half_mirror
    return x;                                                          // lane 8m: the sum
}

__device__ __forceinline__ void edge_spans(uint32_t qo, uint32_t ql, uint32_t& wend,
                                           uint32_t& fend, uint32_t& he, uint32_t& tb) {
    wend = (qo & ~15u) + kWin;
    fend = qo + ql;
    const bool has = fend > wend;
    he = has ? min((wend + 127u) & ~127u, fend) : 0u;
    tb = has ? max(fend & ~127u, he) : 0u;
}

template <int AUX = 0>
__device__ __forceinline__ EdgeLines edge_lines_window(__amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                                       WaveScratch& W, int lane, Frame fr,
                                                       bool valid, uint32_t min_tile_stream) {
    // the cooperative mapping below gives each frame 8 lanes for kWinChunks passes, so it
    // covers all 64 frames only with 128-B windows (8 chunks); the 64-B-window compiles
    // take only batches whose frames lie inside their windows (nothing streams), so they
    // never need the edge lines
    if constexpr (kWinChunks != 8) return EdgeLines{false, 0u, 0u, 0u};
    {
        const uint32_t wend = (fr.off & ~15u) + kWin, fend = fr.off + fr.len;
        const uint32_t span = (valid && fend > wend) ? fend - wend : 0u;
        if (wave_sum(span) <= min_tile_stream) return EdgeLines{false, 0u, 0u, 0u};  // uniform
    }
    const int j = lane & 7;
    u32x4 d[kWinChunks];
    uint32_t lim[kWinChunks], a0[kWinChunks];
    // head chunks, then tail chunks: 8 loads in flight per pass
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) {
            const int q = (k * kWave + lane) >> 3;
            const uint32_t qo = (uint32_t)__shfl((int)fr.off, q, kWave);
            const uint32_t ql = (uint32_t)__shfl((int)(valid ? fr.len : 0u), q, kWave);
            uint32_t wend, fend, he, tb;
            edge_spans(qo, ql, wend, fend, he, tb);
            const uint32_t a = pass == 0 ? wend + 16u * j : tb + 16u * j;
            const uint32_t e = pass == 0 ? he : fend;
            const bool in = a < e && (pass == 0 || tb < fend);
            a0[k] = a;
            lim[k] = in ? (e - a < 16u ? e - a : 16u) : 0u;
            d[k] = load16_fast<AUX>(rs, in ? a : fb);
        }
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) {
            u32x4 v = d[k];
            if (__builtin_expect(lim[k] != 0 && straddles(a0[k], fb), 0)) v = load16(rs, a0[k], fb);
            const uint32_t x = sum8_lanes(lim[k] ? chunk_sum(v, 0, (int)lim[k]) : 0u);
            if (j == 0) (pass == 0 ? W.first : W.last)[(k * kWave + lane) >> 3] = x;
        }
    }
    wave_sync();
    uint32_t wend, fend, he, tb;
    edge_spans(fr.off, valid ? fr.len : 0u, wend, fend, he, tb);
    return EdgeLines{true, W.first[lane] + W.last[lane], he, tb};
}


__device__ __forceinline__ Frame frame_span(const uint32_t* offsets, uint32_t stride,
                                            uint32_t frame_len, uint32_t frames_bytes,
                                            uint32_t i) {
    uint64_t off, len;
    if (offsets) {
        uint32_t a = offsets[i], b = offsets[i + 1];
        off = a;
        len = b >= a ? b - a : 0;
    } else {
        off = (uint64_t)i * stride;
        len = frame_len;
    }
    if (off > frames_bytes) off = frames_bytes;
    if (off + len > frames_bytes) len = frames_bytes - off;
    return Frame{(uint32_t)off, (uint32_t)len};
}

__device__ __forceinline__ uint32_t flow_hash(uint32_t src, uint32_t dst, uint32_t sp,
                                              uint32_t dp, uint32_t proto) {
    uint32_t h = 0x811c9dc5u;
    h = (h ^ src) * 0x01000193u;
    h = (h ^ dst) * 0x01000193u;
    h = (h ^ ((sp << 16) | dp)) * 0x01000193u;
    h = (h ^ proto) * 0x01000193u;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

// ---- per-frame parse state (registers) ----
struct LaneRec {
    uint32_t w[20];                  // the 80-byte rpkt_rec_t as 20 little-endian words
    uint32_t status;
    uint32_t stream_s, stream_e;     // absolute L4 bytes past the LDS window
    uint32_t l4_part;                // in-window part of the L4 word sum
    uint32_t l4_start_abs, pseudo;
    bool want_l4;
    bool is6;                        // dispatched to Ipv6::parse (RPKT_F_IPV6): the IPv6 block
};

// Window loads of one tile into registers: chunk c = k*64 + lane is piece c%8 of
// frame c/8; a frame's offset/length come from its owning lane by ds_bpermute.
// Returns a bit per k whose chunk straddles the end of the frames buffer.
template <int AUX = 0>
__device__ __forceinline__ uint32_t window_issue(__amdgpu_buffer_rsrc_t rs, uint32_t fb, Frame fr,
                                                 int lane, u32x4 (&d)[kWinChunks],
                                                 uint32_t (&addr)[kWinChunks]) {
    uint32_t fix = 0;
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) {
        const int c = k * kWave + lane;
        const int q = c / kWinChunks, j = c % kWinChunks;
        const uint32_t qo = (uint32_t)__shfl((int)fr.off, q, kWave);
        const uint32_t ql = (uint32_t)__shfl((int)fr.len, q, kWave);
        const uint32_t a = (qo & ~15u) + 16u * j;
        addr[k] = (a < qo + ql) ? a : fb;
        fix |= (uint32_t)straddles(addr[k], fb) << k;
    }
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) d[k] = load16_fast<AUX>(rs, addr[k]);
    return fix;
}

__device__ __forceinline__ void put_chunk(WaveScratch& W, int c, u32x4 v) {
    uint32_t* dst =
        reinterpret_cast<uint32_t*>(&W.win[(c / kWinChunks) * kSlot + (c % kWinChunks) * 16]);
    dst[0] = v.x;
    dst[1] = v.y;
    dst[2] = v.z;
    dst[3] = v.w;
}

// Registers -> LDS window slots (slot stride 132 B, so 4-byte stores).  A chunk that
// straddles the buffer end (at most one per buffer) is then re-read exactly and
// overwritten in LDS: the registers themselves are never modified conditionally.
__device__ __forceinline__ void window_commit(WaveScratch& W, __amdgpu_buffer_rsrc_t rs,
                                              uint32_t fb, const u32x4 (&d)[kWinChunks],
                                              const uint32_t (&addr)[kWinChunks], uint32_t fix,
                                              int lane) {
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) put_chunk(W, k * kWave + lane, d[k]);
    if (__builtin_expect(__ballot(fix != 0) != 0, 0)) {
        for (int k = 0; k < kWinChunks; ++k)
            if (fix & (1u << k)) put_chunk(W, k * kWave + lane, load16(rs, addr[k], fb));
    }
}

// The window and the edge lines issued together (long tiles).  A frame's head edge
// line is the line its window ends in, and its tail edge line the line the next frame's
// window starts in; loaded in separate passes (edge_lines_window after window_commit),
// the second touch of such a line comes microseconds after the first, when 512 waves
// per XCD streaming their tiles have pushed it out of the 4-MB L2, and it is fetched
// twice (config 3: reads 1.042x the frame bytes at stride 1500, 1.000x at stride 1536
// where no line is shared; profiles/r04_fp/).  Here each load instruction group covers
// eight frames' window, head and tail chunks at once (the same cooperative mapping:
// chunk k of lane l is piece l % 8 of frame 8k + l / 8), in two halves of 12 loads.
// Returns the same EdgeLines as edge_lines_window; the window lands in LDS as
// window_commit leaves it.
template <int AUX = 0>
__device__ __forceinline__ EdgeLines window_with_edges(__amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                                       WaveScratch& W, int lane, Frame fr,
                                                       bool valid) {
    static_assert(kWinChunks == 8, "the 128-B window compile");
    const int j = lane & 7;
    constexpr int kHalf = kWinChunks / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32x4 dw[kHalf], dh[kHalf], dt[kHalf];
        uint32_t aw[kHalf], ah[kHalf], at[kHalf], lh[kHalf], lt[kHalf];
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int k = h * kHalf + i;
            const int q = (k * kWave + lane) >> 3;
            const uint32_t qo = (uint32_t)__shfl((int)fr.off, q, kWave);
            const uint32_t qn = (uint32_t)__shfl((int)fr.len, q, kWave);
            const uint32_t ql = (uint32_t)__shfl((int)(valid ? fr.len : 0u), q, kWave);
            const uint32_t a = (qo & ~15u) + 16u * j;                // window_issue's chunk
            aw[i] = (a < qo + qn) ? a : fb;
            uint32_t wend, fend, he, tb;
            edge_spans(qo, ql, wend, fend, he, tb);
            const uint32_t x = wend + 16u * j, y = tb + 16u * j;
            const bool hin = x < he, tin = y < fend && tb < fend;
            ah[i] = hin ? x : fb;
            at[i] = tin ? y : fb;
            lh[i] = hin ? (he - x < 16u ? he - x : 16u) : 0u;
            lt[i] = tin ? (fend - y < 16u ? fend - y : 16u) : 0u;
        }
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            dw[i] = load16_fast<0>(rs, aw[i]);
            dh[i] = load16_fast<AUX>(rs, ah[i]);
            dt[i] = load16_fast<AUX>(rs, at[i]);
        }
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int k = h * kHalf + i;
            u32x4 v = dw[i], vh = dh[i], vt = dt[i];
            if (__builtin_expect(straddles(aw[i], fb), 0)) v = load16(rs, aw[i], fb);
            if (__builtin_expect(lh[i] != 0 && straddles(ah[i], fb), 0)) vh = load16(rs, ah[i], fb);
            if (__builtin_expect(lt[i] != 0 && straddles(at[i], fb), 0)) vt = load16(rs, at[i], fb);
            put_chunk(W, k * kWave + lane, v);
            const uint32_t xh = sum8_lanes(lh[i] ? chunk_sum(vh, 0, (int)lh[i]) : 0u);
            const uint32_t xt = sum8_lanes(lt[i] ? chunk_sum(vt, 0, (int)lt[i]) : 0u);
            if (j == 0) {
                W.first[(k * kWave + lane) >> 3] = xh;
                W.last[(k * kWave + lane) >> 3] = xt;
            }
        }
    }
    wave_sync();
    uint32_t wend, fend, he, tb;
    edge_spans(fr.off, valid ? fr.len : 0u, wend, fend, he, tb);
    return EdgeLines{true, W.first[lane] + W.last[lane], he, tb};
}

// ---- dword-granular LDS access for the parse ----
// Frame byte x of this lane lives at LDS offset ph + x of its slot (ph = frame
// offset & 15, the absolute 16-byte phase), so aligned LDS dwords are aligned in
// absolute address too: the raw dwords feed the checksum sums directly, and
// v_alignbyte turns them into frame-relative little-endian dwords for the getters.
__device__ __forceinline__ uint32_t lds32(const uint8_t* slot, uint32_t a) {
    return *reinterpret_cast<const uint32_t*>(slot + a);
}
__device__ __forceinline__ uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
// big-endian u16 from little-endian bytes 0,1 / 2,3 of a dword
__device__ __forceinline__ uint32_t be16_lo(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c0c0001u); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c0c0203u); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

// Read the 6 aligned LDS dwords covering frame bytes [x, x + 20) (any phase): raw
// dwords R (absolute-aligned, for sums) and frame-relative dwords F (for getters).
struct Hdr6 {
    uint32_t a0;            // LDS offset of R[0]
    uint32_t R[6];
    uint32_t F[5];
};
__device__ __forceinline__ void read_hdr(const uint8_t* slot, uint32_t ldsx, Hdr6& h) {
    h.a0 = ldsx & ~3u;
    const uint32_t sh = ldsx & 3u;
#pragma unroll
    for (int k = 0; k < 6; ++k) h.R[k] = lds32(slot, h.a0 + 4 * k);
#pragma unroll
    for (int k = 0; k < 5; ++k) h.F[k] = align_bytes(h.R[k + 1], h.R[k], sh);
}

// Word sum of LDS bytes [s, e) using the already-read raw dwords R[0..N) at
// a0 = s & ~3, continuing with LDS reads past them (IPv4 options, long in-window L4
// spans).  Whole dwords [a0, ceil4(e)) are summed unmasked, then the bytes of the
// first dword below s and of the last dword from e on are subtracted (exact: they
// were added): two masks per range instead of one per dword.
__device__ __forceinline__ uint32_t low_bytes(uint32_t x, uint32_t n) {   // bytes [0, n), n <= 3
    return x & ((1u << (8u * n)) - 1u);
}
template <int N>
__device__ __forceinline__ uint32_t raw_range_sum(const uint8_t* slot, const uint32_t (&R)[N],
                                                  uint32_t a0, uint32_t s, uint32_t e) {
    if (e <= s) return 0u;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) acc = hsum(a0 + 4 * k < e ? R[k] : 0u, acc);
    // four reads in flight per round trip (a long in-window L4 span is up to ~24 dwords)
    uint32_t a = a0 + 4 * N;
    for (; a + 12u < e; a += 16u) {
        const uint32_t x0 = lds32(slot, a), x1 = lds32(slot, a + 4u);
        const uint32_t x2 = lds32(slot, a + 8u), x3 = lds32(slot, a + 12u);
        acc = hsum(x3, hsum(x2, hsum(x1, hsum(x0, acc))));
    }
    for (; a < e; a += 4) acc = hsum(lds32(slot, a), acc);
    acc -= halves(low_bytes(R[0], s & 3u));
    if (e & 3u) acc -= halves(lds32(slot, e & ~3u) & ~((1u << (8u * (e & 3u))) - 1u));
    return acc;
}

__device__ __forceinline__ bool is_tag(uint32_t et) { return et == 0x8100u || et == 0x88a8u; }

// Buffer bytes a..a+3 as a little-endian dword: two aligned dword loads and a byte
// align (bytes past the buffer read as 0, as gbyte's: the buffer's last, partial dword
// byte-wise)
__device__ __forceinline__ uint32_t gdword(__amdgpu_buffer_rsrc_t rs, uint32_t fb, uint32_t a) {
    const uint32_t a4 = a & ~3u;
    auto ld = [&](uint32_t x) -> uint32_t {
        if (__builtin_expect(x + 4u <= fb, 1))
            return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)x, 0, 0);
        return gbyte(rs, x) | (gbyte(rs, x + 1u) << 8) | (gbyte(rs, x + 2u) << 16) |
               (gbyte(rs, x + 3u) << 24);
    };
    return align_bytes(ld(a4 + 4u), ld(a4), a & 3u);
}

// 20 bytes at absolute `a` as frame-relative little-endian dwords (Hdr6::F layout): the
// rare paths whose header lies outside the LDS window.  Six aligned dword loads in one
// round trip; near the buffer's end, bytes.
__device__ __forceinline__ void gread20(__amdgpu_buffer_rsrc_t rs, uint32_t fb, uint32_t a,
                                        uint32_t (&F)[5]) {
    const uint32_t a4 = a & ~3u, sh = a & 3u;
    uint32_t R[6];
    if (__builtin_expect(a4 + 24u <= fb, 1)) {
#pragma unroll
        for (int k = 0; k < 6; ++k)
            R[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a4 + 4u * k), 0, 0);
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t x = a4 + 4u * k;
            R[k] = gbyte(rs, x) | (gbyte(rs, x + 1) << 8) | (gbyte(rs, x + 2) << 16) |
                   (gbyte(rs, x + 3) << 24);
        }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) F[k] = align_bytes(R[k + 1], R[k], sh);
}

// Frame bytes x..x+3 of a lane's frame as a little-endian dword: from its LDS window
// slot when they lie in the window, else from global memory (IPv6 extension headers
// past the window; bytes past the buffer read as 0).
struct FrameDw {
    const uint8_t* slot;
    uint32_t ph, off, fb;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ uint32_t operator()(uint32_t x) const {
        if (__builtin_expect(ph + x + 4u <= (uint32_t)kWin, 1)) {
            const uint32_t y = ph + x, a = y & ~3u;
            return align_bytes(lds32(slot, a + 4), lds32(slot, a), y & 3u);
        }
        return gdword(rs, fb, off + x);
    }
};

// RFC 1071 word sum of a 16-byte address given as frame-relative LE dwords: the four
// host-order words' 16-bit halves (big-endian words, as the pseudo header sums them)
__device__ __forceinline__ uint32_t addr_words_sum(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return halves(bswap32(a)) + halves(bswap32(b)) + halves(bswap32(c)) + halves(bswap32(d));
}

__device__ __forceinline__ bool is_ip6_ext(uint32_t nh) {
    return nh == 0u || nh == 43u || nh == 44u || nh == 60u || nh == 51u;
}

// The IPv6 part of the parse (RPKT_F_IPV6, include/rpkt_gpu.h documents the record's
// IPv6 block): Ipv6::parse (ipv6/generated.rs:40-51) and getters (:57-80, 194-205),
// Ipv6::payload (:83-92: trim to 40 + payload_len, advance 40), then the extension
// headers: each type's generated parse (DestOptions :241-252, HopByHopOption :384-395,
// RoutingHeader :528-539, FragmentHeader :696-703, AuthenticationHeader :850-861) and
// payload() = advance(header_len).  The 40-byte header always lies in the window (it
// ends by frame byte 62); extension headers past it are read from global memory.
// Returns the status; on OK: l4 (frame offset of the upper-layer header), its
// remaining bytes, the protocol and the pseudo header's address sum.
__device__ __forceinline__ uint32_t parse_ip6(const uint8_t* slot, uint32_t ph, Frame fr,
                                              __amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                              uint32_t l3, uint32_t rem,
                                              uint32_t* w, uint32_t& l4, uint32_t& l4rem,
                                              uint32_t& proto, uint32_t& paddr) {
    if (rem < 40u) return RPKT_S_IP6_SHORT;                               // :42
    uint32_t F[10];
    {
        const uint32_t x = ph + l3, a0 = x & ~3u, sh = x & 3u;
        uint32_t R[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) R[k] = lds32(slot, a0 + 4 * k);
#pragma unroll
        for (int k = 0; k < 10; ++k) F[k] = align_bytes(R[k + 1], R[k], sh);
    }
    const uint32_t plen = be16_lo(F[1]);                                  // payload_len :77-79
    if (plen + 40u > rem) return RPKT_S_IP6_BAD_LEN;                      // :47
    w[6] = bswap32(F[0]);                                                 // version, tc, flow
    w[7] = plen | (F[1] & 0xffff0000u);                                   // next_header, hop_limit
    w[9] = bswap32(F[2]) ^ bswap32(F[3]) ^ bswap32(F[4]) ^ bswap32(F[5]);    // src fold
    w[10] = bswap32(F[6]) ^ bswap32(F[7]) ^ bswap32(F[8]) ^ bswap32(F[9]);   // dst fold
    const uint32_t src_sum = addr_words_sum(F[2], F[3], F[4], F[5]);
    uint32_t pdst_sum = addr_words_sum(F[6], F[7], F[8], F[9]);
    uint32_t pdst_off = l3 + 24u;
    const FrameDw dw{slot, ph, fr.off, fb, rs};
    uint32_t c = l3 + 40u;
    const uint32_t end = c + plen;
    uint32_t nh = (F[1] >> 16) & 0xffu, n_ext = 0, status = RPKT_S_OK;
    for (int k = 0; k < RPKT_MAX_IP6_EXT && is_ip6_ext(nh); ++k) {
        const bool fg = nh == 44u, ah = nh == 51u, rt = nh == 43u;
        const uint32_t fixed = (nh == 0u || nh == 60u) ? 2u : (ah ? 12u : 8u);
        const uint32_t cl = end - c;                                      // chunk_len
        if (cl < fixed) { status = RPKT_S_IP6_EXT_SHORT; break; }
        const uint32_t d0 = dw(c);                 // next_header, len, (type, segments_left)
        const uint32_t b1 = (d0 >> 8) & 0xffu;
        const uint32_t hl = fg ? 8u : (ah ? b1 * 4u + 8u : b1 * 8u + 8u);    // header_len
        if (!fg && (hl < fixed || hl > cl)) { status = RPKT_S_IP6_EXT_BAD_LEN; break; }
        if (rt && (d0 >> 24) != 0u) {
            // segments_left > 0: the pseudo header's destination is the final address
            // (RFC 8200 section 8.1): the last of the list (types 0, 2), Segment List[0] (4)
            const uint32_t type = (d0 >> 16) & 0xffu, n_addr = (hl - 8u) >> 4;
            if (n_addr != 0u && (type == 0u || type == 2u || type == 4u)) {
                const uint32_t a = c + 8u + (type == 4u ? 0u : 16u * (n_addr - 1u));
                pdst_off = a;
                pdst_sum = addr_words_sum(dw(a), dw(a + 4u), dw(a + 8u), dw(a + 12u));
            }
        }
        nh = d0 & 0xffu;
        c += hl;
        n_ext += 1u;
        // offset (:717-719) != 0 or more_frag (:725-727): a fragment, not reassembled here
        if (fg && (be16_hi(d0) & 0xfff9u) != 0u) { status = RPKT_S_IP6_FRAGMENT; break; }
    }
    if (status == RPKT_S_OK && is_ip6_ext(nh)) status = RPKT_S_L4_OTHER;   // chain too long
    w[8] = n_ext | (nh << 8) | (pdst_off << 16);
    l4 = c;
    l4rem = end - c;
    proto = nh;
    paddr = src_sum + pdst_sum;
    return status;
}

// Lane-per-frame parse from the LDS window: the rpkt chain with every getter, the
// IPv4 header sum and the in-window part of the L4 sum.  Three dependent rounds of
// LDS dword reads: link layer (bytes 0..23), IPv4 header at l3, L4 header at l4.
// start_et != 0 (rpkt_gpu_parse_tunnel_batch's inner packets): the frame starts at its IP
// header, dispatched as ethertype start_et (Ipv4|Ipv6::parse on the whole buffer); base:
// added to every offset the record holds (the inner frame's position in the outer one).
// Both are compile-time 0 for the other callers.
__device__ __forceinline__ void parse_lane(const WaveScratch& W, int lane, Frame fr, bool valid,
                                           uint32_t flags, LaneRec& L,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                           uint32_t start_et = 0u, uint32_t base = 0u) {
    const uint32_t ph = fr.off & 15u;
    const uint8_t* slot = &W.win[lane * kSlot];
    uint32_t* w = L.w;
#pragma unroll
    for (int k = 0; k < 20; ++k) w[k] = 0;
    const uint32_t len = valid ? fr.len : 0u;
    L.stream_s = L.stream_e = L.l4_part = L.l4_start_abs = L.pseudo = 0;
    L.want_l4 = false;
    L.is6 = false;
    w[19] = len;
    uint32_t status = RPKT_S_OK;

    uint32_t nvlan = 0, et = start_et;
    if (start_et == 0u) {
        // round 1: Ethernet + up to two 802.1Q/802.1ad tags, frame bytes [0, 24)
        uint32_t E[6];
        {
            const uint32_t a0 = ph & ~3u, sh = ph & 3u;
            uint32_t R[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) R[k] = lds32(slot, a0 + 4 * k);
#pragma unroll
            for (int k = 0; k < 6; ++k) E[k] = align_bytes(R[k + 1], R[k], sh);
        }
        if (len < 14) {                                        // ether/generated.rs:36
            L.status = RPKT_S_ETH_SHORT;
            w[0] = RPKT_S_ETH_SHORT;
            return;
        }
        w[1] = E[0];                                           // dst_addr, src_addr
        w[2] = E[1];                                           //   ether/generated.rs:47-54
        w[3] = E[2];
        const uint32_t eth_et = be16_lo(E[3]);                 // ethertype :55-59
        // VLAN walk (vlan/generated.rs:32-61), at most RPKT_MAX_VLAN tags
        et = eth_et;
        if (is_tag(et)) {
            if (len - 14 < 4) {
                status = RPKT_S_VLAN_SHORT;
            } else {
                et = be16_lo(E[4]);
                w[4] = be16_hi(E[3]);
                w[5] = et;
                nvlan = 1;
                if (is_tag(et)) {
                    if (len - 18 < 4) {
                        status = RPKT_S_VLAN_SHORT;
                    } else {
                        et = be16_lo(E[5]);
                        w[4] |= be16_hi(E[4]) << 16;
                        w[5] |= et << 16;
                        nvlan = 2;
                    }
                }
            }
        }
        w[0] = (nvlan << 8) | (eth_et << 16);
    } else {
        w[0] = start_et << 16;                                 // the tunnel's dispatch value
    }
    // EtherType::IPV6 (ether/mod.rs), ipv6_test.rs:25: with RPKT_F_IPV6 only
    const bool v6 = (flags & RPKT_F_IPV6) && status == RPKT_S_OK && et == 0x86ddu;
    if (status == RPKT_S_OK && et != 0x0800u && !v6) status = RPKT_S_NOT_IPV4;
    if (status != RPKT_S_OK) {
        w[0] |= status;
        L.status = status;
        return;
    }

    const uint32_t l3 = start_et ? 0u : 14u + 4u * nvlan, rem = len - l3;
    w[16] = base + l3;
    uint32_t l4, l4rem, proto, paddr;
    if (v6) {
        // round 2 (IPv6): the header, the extension headers, the pseudo header's addresses
        L.is6 = true;
        status = parse_ip6(slot, ph, fr, rs, fb, l3, rem, w, l4, l4rem, proto, paddr);
        if (status != RPKT_S_IP6_SHORT && status != RPKT_S_IP6_BAD_LEN) {
            w[16] |= (base + l4) << 16;
            w[17] = ((base + l4) & 0xffffu) | (l4rem << 16);
            w[8] += base << 16;                                // ip6_pdst_off
        }
        if (status != RPKT_S_OK) {
            w[0] |= status;
            L.status = status;
            return;
        }
    } else {
        // round 2: Ipv4::parse (ipv4/generated.rs:35-51) and getters (:61-112, 269-288)
        Hdr6 ip;
        read_hdr(slot, ph + l3, ip);
        const uint32_t vhl = ip.F[0] & 0xffu;
        const uint32_t ihl4 = (vhl & 0xfu) * 4u;
        const uint32_t tot = be16_hi(ip.F[0]);
        if (rem < 20) status = RPKT_S_IP_SHORT;
        else if (ihl4 < 20) status = RPKT_S_IP_BAD_IHL;
        else if (ihl4 > rem) status = RPKT_S_IP_IHL_GT_LEN;
        else if (tot < ihl4) status = RPKT_S_IP_TOT_LT_IHL;
        else if (tot > rem) status = RPKT_S_IP_TOT_GT_LEN;
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
            w[18] = be_sum(raw_range_sum(slot, ip.R, ip.a0, ph + l3, ph + l3 + ihl4), fr.off + l3);
        l4 = l3 + ihl4;                                        // Ipv4::payload :115-127
        l4rem = tot - ihl4;
        w[16] |= (base + l4) << 16;
        w[17] = (base + l4) | (l4rem << 16);
        // pseudo header (smoltcp pseudo_header_v4): src, dst
        paddr = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu);
    }

    // round 3: Udp::parse (udp/generated.rs:31-42) / Tcp::parse (tcp/generated.rs:34-45).
    // An IPv4 L4 header always lies in the window (l4 <= 82); an IPv6 one past its
    // extension headers may not: its fields are then read from global memory, and the
    // in-window part of its sum is whatever of it the window holds.
    Hdr6 h4;
    read_hdr(slot, v6 && ph + l4 > (uint32_t)kWin ? (uint32_t)kWin : ph + l4, h4);
    // (a UDP header needs only its 8 bytes in the window: the 64-B-window compile keeps
    // an untagged IPv6/UDP frame's header, bytes 54..61, in LDS)
    if (v6 && __builtin_expect(ph + l4 + (proto == 17u ? 8u : 20u) > (uint32_t)kWin, 0))
        gread20(rs, fb, fr.off + l4, h4.F);
    uint32_t l4len = 0;
    bool other_sum = false;                                    // ICMP / GRE: no pseudo header
    if (proto == 17u) {
        const uint32_t ulen = be16_lo(h4.F[1]);
        if (l4rem < 8) status = RPKT_S_UDP_SHORT;
        else if (ulen < 8 || ulen > l4rem) status = RPKT_S_UDP_BAD_LEN;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[14] = ulen;
            w[15] = be16_hi(h4.F[1]);
            w[17] = ((base + l4 + 8) & 0xffffu) | ((ulen - 8) << 16);   // Udp::payload :66-76
            l4len = ulen;
        }
    } else if (proto == 6u) {
        const uint32_t hl = ((h4.F[3] >> 4) & 0xfu) * 4u;
        if (l4rem < 20) status = RPKT_S_TCP_SHORT;
        else if (hl < 20 || hl > l4rem) status = RPKT_S_TCP_BAD_DOFF;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[12] = bswap32(h4.F[1]);
            w[13] = bswap32(h4.F[2]);
            w[14] = be16_lo(h4.F[3]) | (be16_hi(h4.F[3]) << 16);
            w[15] = be16_lo(h4.F[4]) | (be16_hi(h4.F[4]) << 16);
            w[17] = ((base + l4 + hl) & 0xffffu) | ((l4rem - hl) << 16);   // Tcp::payload :125-131
            l4len = l4rem;
        }
    } else {
        status = RPKT_S_L4_OTHER;
        // ICMP (IPv4 protocol 1; calculate_icmp_checksum, icmpv4/generated.rs:2678-2701, is
        // the complement of this sum; an empty payload panics there: ICMP_EMPTY) and GRE
        // with checksum_present (gre/generated.rs:55; RFC 2784 section 2.5): the sum over
        // the whole IP payload, no pseudo header (include/rpkt_gpu.h, l4_sum)
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
        // pseudo header: addresses, protocol, length (smoltcp pseudo_header_v4 / _v6; the
        // v6 u32 length is < 2^16 here, so one word)
        L.pseudo = other_sum ? 0u : paddr + proto + l4len;
        const uint32_t win_end = kWin - ph;                    // frame offset where LDS ends
        const uint32_t e = l4 + l4len;
        const uint32_t e_in = e < win_end ? e : win_end;
        L.l4_part = raw_range_sum(slot, h4.R, h4.a0, ph + l4, ph + e_in);
        L.l4_start_abs = fr.off + l4;
        if (e > win_end) {
            L.stream_s = fr.off + (l4 > win_end ? l4 : win_end);
            L.stream_e = fr.off + e;
        }
    }
}

// Flow event of a parsed frame (include/rpkt_gpu.h, rpkt_flow_ev_t) from its record
// words w (registers or the LDS stage).
__device__ __forceinline__ uint64_t flow_event(const LaneRec& L, const uint32_t* w,
                                               uint32_t n_buckets) {
    uint64_t ev = w[19];
    uint32_t bucket = n_buckets;
    const uint32_t proto = (w[8] >> 8) & 0xffu;
    const bool ip4_parsed = !L.is6 && (L.status == RPKT_S_OK ||
                                       (L.status >= RPKT_S_L4_OTHER && L.status <= RPKT_S_TCP_BAD_DOFF) ||
                                       L.status == RPKT_S_ICMP_EMPTY);
    // words 9 / 10: the IPv4 addresses, or the IPv6 address folds
    if (L.status == RPKT_S_OK)
        bucket = flow_hash(w[9], w[10], w[11] & 0xffffu, w[11] >> 16, proto) % n_buckets;
    ev |= (uint64_t)bucket << 32;
    if (ip4_parsed && (w[18] & 0xffffu) != 0xffffu) ev |= 1ull << 48;
    if (L.status == RPKT_S_OK && (w[18] >> 16) != 0xffffu &&
        !(!L.is6 && proto == 17u && (w[15] & 0xffffu) == 0))
        ev |= 1ull << 49;
    return ev;
}

// The 16-byte compact record (rpkt_rec16_t) of a parsed frame, from the record words
// (the projection of rpkt_rec_t documented in include/rpkt_gpu.h).
__device__ __forceinline__ u32x4 compact_record(const LaneRec& L, uint32_t flags) {
    const uint32_t* w = L.w;
    const uint32_t proto = (w[8] >> 8) & 0xffu;
    uint32_t verdict = 0;
    // IPv6: no header checksum; bit 0 = the IPv6 header parsed
    const bool ip_ok = L.is6 ? (L.status != RPKT_S_IP6_SHORT && L.status != RPKT_S_IP6_BAD_LEN)
                             : (w[18] & 0xffffu) == 0xffffu;
    if ((flags & RPKT_F_IP_SUM) && ip_ok) verdict |= 1u;
    if ((flags & RPKT_F_L4_SUM) && L.status == RPKT_S_OK &&
        ((w[18] >> 16) == 0xffffu || (!L.is6 && proto == 17u && (w[15] & 0xffffu) == 0)))
        verdict |= 2u;
    if (L.is6) verdict |= 4u;
    return u32x4{(w[0] & 0xffffu) | (proto << 16) | (verdict << 24), w[16], w[17], w[18]};
}

// Records of the tile are staged through LDS (the window area, free once the parse
// is done; stride 21 dwords: conflict-free) and stored as wave-instructions of 1 KiB
// contiguous each, with non-temporal stores (measured -12 % at 64 B, -2 % at 1500 B
// vs plain).  Staging right after the parse keeps the 20 record words out of the
// registers of the L4 stream.
__device__ __forceinline__ uint32_t* rec_stage(WaveScratch& W) {
    return reinterpret_cast<uint32_t*>(W.win);
}

__device__ __forceinline__ void stage_record(WaveScratch& W, int lane, const uint32_t (&w)[20]) {
    wave_sync();                                     // every lane done reading the window
    uint32_t* rl = rec_stage(W) + lane * 21;
#pragma unroll
    for (int k = 0; k < 20; ++k) rl[k] = w[k];
}

template <bool NT>
__device__ __forceinline__ void flush_records(WaveScratch& W, int lane, rpkt_rec_t* recs,
                                              uint32_t p0, uint32_t n) {
    wave_sync();
    const uint32_t* rl = rec_stage(W);
    const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* out = reinterpret_cast<u32x4*>(recs + p0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t c = k * kWave + lane, r = c / 5, pc = c % 5;
        const uint32_t* src = rl + r * 21 + pc * 4;
        const u32x4 v = {src[0], src[1], src[2], src[3]};
        if (r < nrec) {
            if constexpr (NT) __builtin_nontemporal_store(v, &out[c]);
            else out[c] = v;
        }
    }
}

struct SpanSrc {
    const uint32_t* offsets;
    uint32_t stride, frame_len, fb, n;
    __device__ __forceinline__ Frame get(uint32_t i) const {
        if (i >= n) return Frame{0, 0};
        return frame_span(offsets, stride, frame_len, fb, i);
    }
};


inline int hip_check(hipError_t e) {
    if (e != hipSuccess) {
        rpkt_detail::g_last_hip_error = (int)e;
        return RPKT_E_HIP;
    }
    return RPKT_OK;
}

// Launch and report THIS launch's status (hipGetLastError would also return
// errors other libraries in the process left behind).
template <typename... KArgs, typename... Args>
int launch(void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t st,
           Args... args) {
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel arity");
    auto packed = std::tuple<KArgs...>(static_cast<KArgs>(args)...);
    void* argv[sizeof...(KArgs)];
    std::apply([&](auto&... a) {
        int k = 0;
        ((argv[k++] = (void*)&a), ...);
    }, packed);
    return hip_check(hipLaunchKernel((const void*)kernel, grid, block, argv, lds, st));
}

}  // namespace
