// rpkt_gpu.hip — MI355X (gfx950, CDNA4) batch engine for rpkt's
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
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <tuple>

#include "../../include/rpkt_gpu.h"
#include "rpkt_proto_table.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;            // lanes per wavefront (CDNA)
constexpr int kWavesPerBlock = 4;    // 256-thread workgroups
constexpr int kWin = 128;            // header window bytes per frame in LDS
constexpr int kWinChunks = kWin / 16;
constexpr int kSlot = kWin + 4;      // LDS slot stride: 33 dwords, so lane-strided
                                     // reads of the 64 slots hit 32 distinct banks
constexpr int kStreamUnroll = 4;     // 16-B chunk loads in flight per lane per step
constexpr int kChainStreamUnroll = 8;  // the same in the mbuf-chain kernel
constexpr uint64_t kMaxFrameBytes = 0xffffff00ull;  // voffset + 16 never wraps
constexpr uint32_t kSplitStreamBytes = 65536;  // tile stream above which edge lines go first

struct WaveScratch {                 // 9744 B per wave: 4 waves x 4 blocks fit a CU
    uint8_t  win[kWave * kSlot];     // header windows, slot stride 132 B
    uint32_t s[kWave];               // window phase: frame offset; stream: range start
    uint32_t e[kWave];               // window phase: frame length; stream: range end
    uint32_t pref[kWave + 1];        // stream: exclusive prefix of chunk counts
    uint32_t first[kWave];           // stream: scan value before a range's first chunk
    uint32_t last[kWave];            // stream: scan value at a range's last chunk
};
static_assert(sizeof(WaveScratch) * kWavesPerBlock * 4 <= 160 * 1024, "4 blocks per CU");
static_assert((64 * 21 + 705) * 4 <= 64 * 132, "chain scratch fits the window area");

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
struct StreamCursor { uint32_t q, p0, p1, off; };

__device__ __forceinline__ void cursor_load(const WaveScratch& W, StreamCursor& k, uint32_t q) {
    k.q = q;
    k.p0 = W.pref[q];
    k.p1 = W.pref[q + 1];
    k.off = W.s[q];
}

template <int AUX, int U>
__device__ __forceinline__ void stream_issue(__amdgpu_buffer_rsrc_t rs, uint32_t oob,
                                             const WaveScratch& W, uint32_t total, uint32_t base,
                                             int lane, StreamCursor& k, StreamBatch<U>& B) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t c = base + u * kWave + lane;
        const bool valid = c < total;
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
    W.first[lane] = 0;
    W.last[lane] = 0;
    wave_sync();

    constexpr uint32_t kBatch = kWave * U;
    uint32_t run = 0;
    StreamCursor k;
    cursor_load(W, k, 0);
    StreamBatch<U> A, B;
    uint32_t base = 0;
    stream_issue<AUX, U>(rs, oob, W, total, base, lane, k, A);
    const uint32_t edge = edges();
    for (;;) {
        stream_issue<AUX, U>(rs, oob, W, total, base + kBatch, lane, k, B);
        stream_consume<U>(W, run, A);
        stream_issue<AUX, U>(rs, oob, W, total, base + 2 * kBatch, lane, k, A);
        stream_consume<U>(W, run, B);
        base += 2 * kBatch;
        if (base >= total) break;
    }
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

struct Frame { uint32_t off, len; };

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
    for (uint32_t a = a0 + 4 * N; a < e; a += 4) acc = hsum(lds32(slot, a), acc);
    acc -= halves(low_bytes(R[0], s & 3u));
    if (e & 3u) acc -= halves(lds32(slot, e & ~3u) & ~((1u << (8u * (e & 3u))) - 1u));
    return acc;
}

__device__ __forceinline__ bool is_tag(uint32_t et) { return et == 0x8100u || et == 0x88a8u; }

// Lane-per-frame parse from the LDS window: the rpkt chain with every getter, the
// IPv4 header sum and the in-window part of the L4 sum.  Three dependent rounds of
// LDS dword reads: link layer (bytes 0..23), IPv4 header at l3, L4 header at l4.
__device__ __forceinline__ void parse_lane(const WaveScratch& W, int lane, Frame fr, bool valid,
                                           uint32_t flags, LaneRec& L) {
    const uint32_t ph = fr.off & 15u;
    const uint8_t* slot = &W.win[lane * kSlot];
    uint32_t* w = L.w;
#pragma unroll
    for (int k = 0; k < 20; ++k) w[k] = 0;
    const uint32_t len = valid ? fr.len : 0u;
    L.stream_s = L.stream_e = L.l4_part = L.l4_start_abs = L.pseudo = 0;
    L.want_l4 = false;
    w[19] = len;
    uint32_t status = RPKT_S_OK;

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
    if (len < 14) {                                            // ether/generated.rs:36
        L.status = RPKT_S_ETH_SHORT;
        w[0] = RPKT_S_ETH_SHORT;
        return;
    }
    w[1] = E[0];                                               // dst_addr, src_addr
    w[2] = E[1];                                               //   ether/generated.rs:47-54
    w[3] = E[2];
    const uint32_t eth_et = be16_lo(E[3]);                     // ethertype :55-59
    // VLAN walk (vlan/generated.rs:32-61), at most RPKT_MAX_VLAN tags
    uint32_t nvlan = 0, et = eth_et;
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
    if (status == RPKT_S_OK && et != 0x0800u) status = RPKT_S_NOT_IPV4;
    if (status != RPKT_S_OK) {
        w[0] |= status;
        L.status = status;
        return;
    }

    // round 2: Ipv4::parse (ipv4/generated.rs:35-51) and getters (:61-112, 269-288)
    const uint32_t l3 = 14u + 4u * nvlan, rem = len - l3;
    w[16] = l3;
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
    const uint32_t proto = (ip.F[2] >> 8) & 0xffu;
    const uint32_t src = bswap32(ip.F[3]), dst = bswap32(ip.F[4]);
    w[6] = (ip.F[0] & 0xffffu) | (tot << 16);
    w[7] = be16_lo(ip.F[1]) | (be16_hi(ip.F[1]) << 16);
    w[8] = (ip.F[2] & 0xffffu) | (be16_hi(ip.F[2]) << 16);
    w[9] = src;
    w[10] = dst;
    if (flags & RPKT_F_IP_SUM)
        w[18] = be_sum(raw_range_sum(slot, ip.R, ip.a0, ph + l3, ph + l3 + ihl4), fr.off + l3);
    const uint32_t l4 = l3 + ihl4;                             // Ipv4::payload :115-127
    const uint32_t l4rem = tot - ihl4;
    w[16] |= l4 << 16;
    w[17] = l4 | (l4rem << 16);

    // round 3: Udp::parse (udp/generated.rs:31-42) / Tcp::parse (tcp/generated.rs:34-45)
    Hdr6 h4;
    read_hdr(slot, ph + l4, h4);
    uint32_t l4len = 0;
    if (proto == 17u) {
        const uint32_t ulen = be16_lo(h4.F[1]);
        if (l4rem < 8) status = RPKT_S_UDP_SHORT;
        else if (ulen < 8 || ulen > l4rem) status = RPKT_S_UDP_BAD_LEN;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[14] = ulen;
            w[15] = be16_hi(h4.F[1]);
            w[17] = (l4 + 8) | ((ulen - 8) << 16);             // Udp::payload :66-76
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
            w[17] = (l4 + hl) | ((l4rem - hl) << 16);          // Tcp::payload :125-131
            l4len = l4rem;
        }
    } else {
        status = RPKT_S_L4_OTHER;
    }
    w[0] |= status;
    L.status = status;
    if (status == RPKT_S_OK && (flags & RPKT_F_L4_SUM)) {
        L.want_l4 = true;
        // pseudo header (smoltcp pseudo_header_v4): src, dst, proto, length
        L.pseudo = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu) + proto + l4len;
        const uint32_t win_end = kWin - ph;                    // frame offset where LDS ends
        const uint32_t e = l4 + l4len;
        const uint32_t e_in = e < win_end ? e : win_end;
        L.l4_part = raw_range_sum(slot, h4.R, h4.a0, ph + l4, ph + e_in);
        L.l4_start_abs = fr.off + l4;
        if (e > win_end) {
            L.stream_s = fr.off + win_end;
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
    const bool ip_parsed = L.status == RPKT_S_OK || L.status >= RPKT_S_L4_OTHER;
    if (L.status == RPKT_S_OK)
        bucket = flow_hash(w[9], w[10], w[11] & 0xffffu, w[11] >> 16, proto) % n_buckets;
    ev |= (uint64_t)bucket << 32;
    if (ip_parsed && (w[18] & 0xffffu) != 0xffffu) ev |= 1ull << 48;
    if (L.status == RPKT_S_OK && (w[18] >> 16) != 0xffffu &&
        !(proto == 17u && (w[15] & 0xffffu) == 0))
        ev |= 1ull << 49;
    return ev;
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

// One wavefront per 64-frame tile: window loads -> LDS, lane-per-frame parse,
// flattened L4 stream, LDS-staged coalesced record stores.  (A persistent variant
// that prefetched the next tile's window into registers measured 1-3 % slower on
// every config: the extra live registers cost more occupancy than the overlap gave.)
// L4: compiled with the L4 checksum stream (RPKT_F_L4_SUM).  V: ablation variant for
// tools/ablate.py (0 = the product kernel; 1 = no parse, 3 = no record stores,
// 8 = plain instead of non-temporal record stores, 21 = nt window loads too,
// 22 = default-policy stream loads, 23 = edge lines streamed first after the parse,
// 24 = never, 25 = after the parse on long tiles).
template <bool L4, int V>
__global__ __launch_bounds__(kWave * kWavesPerBlock, 4)    // 4 waves/SIMD: <= 128 VGPRs
void parse_kernel(const uint8_t* __restrict__ frames, uint32_t frames_bytes,
                  const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                  uint32_t n, uint32_t flags, rpkt_rec_t* __restrict__ recs,
                  uint64_t* __restrict__ flow_ev, uint32_t n_buckets) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    WaveScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;                                          // wave-uniform exit
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, frames_bytes);
    const SpanSrc spans{offsets, stride, frame_len, frames_bytes, n};

    // 1. header windows -> LDS (then, on long tiles, the edge lines: edge_lines_first)
    const Frame fr = spans.get(i);
    const uint32_t wend = (fr.off & ~15u) + kWin, fend = fr.off + fr.len;
    {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        const uint32_t fix = window_issue<(V == 21) ? 2 : 0>(rs, frames_bytes, fr, lane, d, addr);
        window_commit(W, rs, frames_bytes, d, addr, fix, lane);
    }
    EdgeLines X{false, 0u, 0u, 0u};
    if constexpr (L4 && V != 1 && V != 23 && V != 24 && V != 25)
        X = edge_lines_first(rs, frames_bytes, W, lane, valid, wend, fend);
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
        parse_lane(W, lane, fr, valid, flags, L);
    }
    if constexpr (V != 3) stage_record(W, lane, L.w);

    // 3. L4 bytes beyond the window: flattened chunk stream over the tile.  The stream
    // is read once: non-temporal loads (measured -13 % at 1500 B); the header windows
    // keep the default policy (nt there measured slower).
    if (L4 && V != 1) {
        constexpr int kAux = (V == 22) ? 0 : 2;
        uint32_t sp;
        const uint32_t ss = L.stream_s, se = L.stream_e;
        if (V == 23 || (V == 25 && wave_sum(se - ss) > kSplitStreamBytes)) {
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
            rec_stage(W)[lane * 21 + 18] |= fold16(L.pseudo + seg) << 16;
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
        const uint64_t ev = flow_event(L, rec_stage(W) + lane * 21, n_buckets);
        __builtin_nontemporal_store(ev, &flow_ev[i]);
    }
    flush_records<V != 8>(W, lane, recs, p0, n);
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

__device__ __forceinline__ uint32_t gbyte(__amdgpu_buffer_rsrc_t rs, uint32_t a) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)a, 0, 0);
}
// 20 bytes at absolute `a` as frame-relative little-endian dwords (Hdr6::F layout)
__device__ __forceinline__ void gread20(__amdgpu_buffer_rsrc_t rs, uint32_t a, uint32_t (&F)[5]) {
#pragma unroll
    for (int k = 0; k < 5; ++k)
        F[k] = gbyte(rs, a + 4 * k) | (gbyte(rs, a + 4 * k + 1) << 8) |
               (gbyte(rs, a + 4 * k + 2) << 16) | (gbyte(rs, a + 4 * k + 3) << 24);
}
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
    if (status == RPKT_S_OK && et != 0x0800u) status = RPKT_S_NOT_IPV4;
    if (status != RPKT_S_OK) {
        w[0] |= status;
        L.status = status;
        return;
    }

    // Ipv4::parse (ipv4/generated.rs:35-51): chunk vs remaining
    const uint32_t l3 = c;
    w[16] = l3;
    Hdr6 ip;
    uint32_t ck3 = 0, ab3 = 0;
    const bool fast3 = l3 < C;
    if (fast3) {
        ck3 = C - l3;
        read_hdr(slot, ph + l3, ip);
    } else {
        if (l3 < pkt) ck3 = chain_chunk(S, a, b, l3, pkt, ab3);
        gread20(rs, ck3 ? ab3 : S.fb, ip.F);
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
    const uint32_t proto = (ip.F[2] >> 8) & 0xffu;
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
    const uint32_t l4 = l3 + ihl4, limit = l3 + tot;           // Ipv4::payload :115-127
    const uint32_t l4rem = tot - ihl4;
    w[16] |= l4 << 16;
    w[17] = l4 | (l4rem << 16);

    // Udp::parse / Tcp::parse against the chunk at l4 under the trimmed end
    Hdr6 h4;
    uint32_t ck4 = 0, ab4 = 0;
    const bool fast4 = l4 < C;
    if (fast4) {
        ck4 = (C < limit ? C : limit) - l4;
        read_hdr(slot, ph + l4, h4);
    } else {
        if (l4 < limit) ck4 = chain_chunk(S, a, b, l4, limit, ab4);
        gread20(rs, ck4 ? ab4 : S.fb, h4.F);
    }
    uint32_t l4len = 0;
    if (proto == 17u) {
        const uint32_t ulen = be16_lo(h4.F[1]);
        if (ck4 < 8) status = RPKT_S_UDP_SHORT;
        else if (ulen < 8 || ulen > l4rem) status = RPKT_S_UDP_BAD_LEN;
        else {
            w[11] = be16_lo(h4.F[0]) | (be16_hi(h4.F[0]) << 16);
            w[14] = ulen;
            w[15] = be16_hi(h4.F[1]);
            w[17] = (l4 + 8) | ((ulen - 8) << 16);
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
            w[17] = (l4 + hl) | ((l4rem - hl) << 16);
            l4len = l4rem;
        }
    } else {
        status = RPKT_S_L4_OTHER;
    }
    w[0] |= status;
    L.status = status;
    if (status == RPKT_S_OK && (flags & RPKT_F_L4_SUM)) {
        L.want_l4 = true;
        L.pseudo = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu) + proto + l4len;
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

// ---- TX side: header build and the loopback_rx forward rewrite ----
// Both compose the fixed header bytes of a frame from an rpkt_rec_t in the frame's
// LDS slot (slot byte x <-> absolute (off & ~15) + x, as for the parse window) and
// write them back with wave-cooperative 16-B chunk stores: a chunk wholly inside a
// frame's written ranges is one dwordx4 store, a partial one (at most the first and
// last of each range) is stored byte by byte, so no byte outside the frame's own
// header ranges is ever written (neighbouring frames are rewritten concurrently).
__device__ __forceinline__ void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
__device__ __forceinline__ void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

// Fixed header bytes from record words (include/rpkt_gpu.h layout): Ethernet, n_vlan
// tags, the 20 IPv4 bytes at l3, the UDP header or the 20 TCP bytes at l4.  These
// are exactly the bytes prepend_header + setters write (ether/generated.rs:71-88,
// vlan/generated.rs:73-100, ipv4/generated.rs:130-206, udp/generated.rs:79-104,
// tcp/generated.rs:135-224); option bytes are not touched.
__device__ __forceinline__ void emit_headers(uint8_t* s, const uint32_t (&w)[20], uint32_t nv,
                                             uint32_t l3, uint32_t l4, uint32_t proto,
                                             uint32_t ip_len, uint32_t udp_len, uint32_t ip_ck,
                                             uint32_t l4_ck) {
#pragma unroll
    for (int k = 0; k < 12; ++k) s[k] = (uint8_t)(w[1 + k / 4] >> (8 * (k % 4)));
    put_be16(s + 12, w[0] >> 16);
#pragma unroll
    for (uint32_t v = 0; v < RPKT_MAX_VLAN; ++v) {
        if (v < nv) {
            put_be16(s + 14 + 4 * v, w[4] >> (16 * v));
            put_be16(s + 16 + 4 * v, w[5] >> (16 * v));
        }
    }
    uint8_t* ip = s + l3;
    ip[0] = (uint8_t)w[6];
    ip[1] = (uint8_t)(w[6] >> 8);
    put_be16(ip + 2, ip_len);
    put_be16(ip + 4, w[7]);
    put_be16(ip + 6, w[7] >> 16);
    ip[8] = (uint8_t)w[8];
    ip[9] = (uint8_t)(w[8] >> 8);
    put_be16(ip + 10, ip_ck);
    put_be32(ip + 12, w[9]);
    put_be32(ip + 16, w[10]);
    uint8_t* t = s + l4;
    if (proto == 17u) {
        put_be16(t, w[11]);
        put_be16(t + 2, w[11] >> 16);
        put_be16(t + 4, udp_len);
        put_be16(t + 6, l4_ck);
    } else if (proto == 6u) {
        put_be16(t, w[11]);
        put_be16(t + 2, w[11] >> 16);
        put_be32(t + 4, w[12]);
        put_be32(t + 8, w[13]);
        put_be16(t + 12, w[14]);
        put_be16(t + 14, w[14] >> 16);
        put_be16(t + 16, l4_ck);
        put_be16(t + 18, w[15] >> 16);
    }
}

// Absolute-phase word sum of LDS slot bytes [s, e) (any alignment): whole dwords,
// minus the bytes of the first dword below s and of the last dword from e on.
__device__ __forceinline__ uint32_t lds_range_sum(const uint8_t* slot, uint32_t s, uint32_t e) {
    if (e <= s) return 0u;
    uint32_t acc = 0;
    for (uint32_t a = s & ~3u; a < e; a += 4) acc = hsum(lds32(slot, a), acc);
    acc -= halves(low_bytes(lds32(slot, s & ~3u), s & 3u));
    if (e & 3u) acc -= halves(lds32(slot, e & ~3u) & ~((1u << (8u * (e & 3u))) - 1u));
    return acc;
}

// Store frame bytes [0, r1) (frame-relative, per owning lane) from the tile's LDS
// slots.  The range lies inside the LDS window (r1 <= kWin - phase).  Each owner lane
// publishes its frame offset and r1 (W.pref / W.s: free once the stream is done);
// the lane that stores chunk c = k*64 + lane (piece j = lane & 7 of frame k*8 +
// lane/8) reads those two words and clips the chunk against the range itself.  A
// full chunk is one dwordx4, a full dword one dword, the rest byte by byte.
__device__ __forceinline__ void write_back(uint8_t* frames, WaveScratch& W, int lane,
                                           uint32_t off, uint32_t r1) {
    W.pref[lane] = off;
    W.s[lane] = r1;
    wave_sync();
    const int j = lane & (kWinChunks - 1);
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) {
        const int q = k * (kWave / kWinChunks) + lane / kWinChunks;
        const uint32_t oq = W.pref[q], rq = W.s[q];
        const int lo = (int)(oq & 15u) - 16 * j;          // chunk-relative frame start
        const int hi = lo + (int)rq;                       // chunk-relative range end
        if (rq == 0 || hi <= 0) continue;
        const uint32_t base = (oq & ~15u) + 16u * j;       // chunk's absolute address
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&W.win[q * kSlot + 16 * j]);
        if (lo <= 0 && hi >= 16) {
            *reinterpret_cast<u32x4*>(frames + base) = u32x4{src[0], src[1], src[2], src[3]};
            continue;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int dl = lo - 4 * d, dh = hi - 4 * d;     // dword-relative range
            if (dh <= 0 || dl >= 4) continue;
            if (dl <= 0 && dh >= 4) {
                *reinterpret_cast<uint32_t*>(frames + base + 4 * d) = src[d];
            } else {
                const uint32_t v = src[d];
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (b >= dl && b < dh) frames[base + 4 * d + b] = (uint8_t)(v >> (8 * b));
            }
        }
    }
}

// Records of the tile, coalesced: 5 dwordx4 per lane over the tile's contiguous
// 5 KiB, staged through the window area (stride 21 dwords), then each lane takes its
// own 20 words.  Must run before the window is committed to LDS.
__device__ __forceinline__ void load_records_tile(const rpkt_rec_t* recs, uint32_t p0, uint32_t n,
                                                  WaveScratch& W, int lane, uint32_t (&w)[20]) {
    const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    const u32x4* in = reinterpret_cast<const u32x4*>(recs + p0);
    u32x4 v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t c = k * kWave + lane;
        v[k] = (c / 5 < nrec) ? in[c] : u32x4{0u, 0u, 0u, 0u};
    }
    uint32_t* st = rec_stage(W);
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
#pragma unroll
    for (int k = 0; k < 20; ++k) w[k] = st[lane * 21 + k];
    wave_sync();
}

// End (frame-relative) of the range to write back for headers ending at `hdr_end`:
// extended, with the window's original bytes, to the end of the 128-B cache line
// (partially written lines cost the memory side a read-modify-write), clipped to the
// frame and to the LDS window.
__device__ __forceinline__ uint32_t line_end(Frame fr, uint32_t hdr_end) {
    const uint32_t ph = fr.off & 15u;
    const uint32_t line = ((fr.off + hdr_end + 127u) & ~127u) - fr.off;
    uint32_t e = line < fr.len ? line : fr.len;
    return e < kWin - ph ? e : kWin - ph;
}

// rpkt_gpu_build_batch: window -> headers composed in LDS -> checksums (IPv4 over the
// slot; L4 over the slot plus the payload stream past the window) -> write-back.
template <bool L4FILL>
__global__ __launch_bounds__(kWave * kWavesPerBlock, 4)
void build_kernel(uint8_t* __restrict__ frames, uint32_t fb, const uint32_t* __restrict__ offsets,
                  uint32_t stride, uint32_t frame_len, uint32_t n,
                  const rpkt_rec_t* __restrict__ recs, uint32_t flags, uint8_t* __restrict__ built) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    WaveScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    const Frame fr = spans.get(i);
    uint32_t w[20];
    {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        const uint32_t fix = window_issue(rs, fb, fr, lane, d, addr);
        load_records_tile(recs, p0, n, W, lane, w);             // window loads in flight
        window_commit(W, rs, fb, d, addr, fix, lane);
    }
    const uint32_t wend = (fr.off & ~15u) + kWin, fend = fr.off + fr.len;
    EdgeLines X{false, 0u, 0u, 0u};
    if constexpr (L4FILL) X = edge_lines_first(rs, fb, W, lane, valid, wend, fend);
    wave_sync();

    const uint32_t ph = fr.off & 15u, len = fr.len;
    uint8_t* slot = &W.win[lane * kSlot];
    const uint32_t nv = (w[0] >> 8) & 0xffu;
    const uint32_t l3 = 14u + 4u * nv;
    const uint32_t ihl4 = (w[6] & 0xfu) * 4u;
    const uint32_t l4 = l3 + ihl4;
    const uint32_t proto = (w[8] >> 8) & 0xffu;
    const uint32_t doff4 = ((w[14] >> 12) & 0xfu) * 4u;
    const uint32_t l4hdr = proto == 17u ? 8u : (proto == 6u ? doff4 : 0u);
    const uint32_t fixed4 = proto == 17u ? 8u : (proto == 6u ? 20u : 0u);
    const bool ok = valid && nv <= RPKT_MAX_VLAN && ihl4 >= 20u && !(proto == 6u && doff4 < 20u) &&
                    len >= l4 + l4hdr && len - l3 <= 65535u &&
                    !(proto == 17u && len - l4 > 65535u);
    const bool fill_ip = ok && (flags & RPKT_BUILD_IP_CSUM);
    const bool fill_l4 = L4FILL && ok && fixed4;
    if (ok)
        emit_headers(slot + ph, w, nv, l3, l4, proto, len - l3, len - l4,
                     fill_ip ? 0u : (w[8] >> 16), fill_l4 ? 0u : (w[15] & 0xffffu));
    if (fill_ip) {
        const uint32_t s = be_sum(lds_range_sum(slot, ph + l3, ph + l4), fr.off + l3);
        put_be16(slot + ph + l3 + 10, ~s & 0xffffu);
    }
    if constexpr (L4FILL) {
        // everything the checksum needs after the stream is packed into the slot's
        // spare dword (bytes 128..131) and two registers, so the stream keeps its
        // registers: pseudo header sum, in-window part, and
        // info = fill | udp << 1 | l4 slot offset << 8
        uint32_t part = 0, ss = 0, se = 0, pseudo = 0;
        const uint32_t win_end = kWin - ph;
        if (fill_l4) {
            const uint32_t e_in = len < win_end ? len : win_end;
            part = lds_range_sum(slot, ph + l4, ph + e_in);
            if (len > e_in) {
                ss = fr.off + e_in;
                se = fr.off + len;
            }
            const uint32_t src = w[9], dst = w[10];
            pseudo = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu) + proto +
                     (len - l4);
        }
        *reinterpret_cast<uint32_t*>(slot + kWin) =
            (uint32_t)fill_l4 | ((uint32_t)(proto == 17u) << 1) | ((ph + l4) << 8);
        const uint32_t sp = stream_rest<2>(X, rs, fb, ss, se, wend, fend, W, lane);
        const uint32_t info = *reinterpret_cast<const uint32_t*>(slot + kWin);
        if (info & 1u) {
            const uint32_t at = info >> 8;                      // slot offset of the L4 header
            const uint32_t sum = fold16(pseudo + be_sum(part + sp, (fr.off & ~15u) + at));
            uint32_t ck = ~sum & 0xffffu;
            const bool udp = info & 2u;
            if (udp && ck == 0u) ck = 0xffffu;                  // RFC 768
            put_be16(slot + at + (udp ? 6u : 16u), ck);
        }
    }
    wave_sync();
    // the window holds the original bytes around the headers: round the written range
    // up to whole 16-B chunks inside the frame (dwordx4 stores instead of byte stores)
    const uint32_t r1 = ok ? line_end(fr, l4 + fixed4) : 0u;
    write_back(frames, W, lane, fr.off, r1);
    if (built && valid) built[i] = ok ? 1 : 0;
}

// rpkt_gpu_forward_batch: the loopback_rx loop fused into one pass per frame: header
// window -> parse (both sums) -> RX verdict -> rewrite in the LDS window -> write-back.
// Checksums are updated from the verify sums (RFC 1624): swapping addresses and
// ports leaves every one's-complement sum unchanged, so only the TTL word and the
// zeroed checksum field move it; both sums are of non-zero data, hence equal to a
// full recompute bit for bit (the oracle recomputes in full).  The written range is
// rounded up to whole 16-B chunks inside the frame (the window holds the original
// payload bytes), so a 64-B frame is rewritten with three dwordx4 stores.
// V: ablation variant for tools/ablate.py (0 = the product kernel; 1 = no write-back,
// 2 = parse without the L4 sum, 3 = window + write-back of the whole frame only).
template <int V>
__global__ __launch_bounds__(kWave * kWavesPerBlock, 4)
void forward_kernel(uint8_t* __restrict__ frames, uint32_t fb, const uint32_t* __restrict__ offsets,
                    uint32_t stride, uint32_t frame_len, uint32_t n, rpkt_fwd_t fwd,
                    uint8_t* __restrict__ keep) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    WaveScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    const Frame fr = spans.get(i);
    {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        const uint32_t fix = window_issue(rs, fb, fr, lane, d, addr);
        window_commit(W, rs, fb, d, addr, fix, lane);
    }
    wave_sync();
    if constexpr (V == 3) {
        write_back(frames, W, lane, fr.off, valid ? line_end(fr, 0u) : 0u);
        if (valid) keep[i] = 1;
        return;
    }
    LaneRec L;
    parse_lane(W, lane, fr, valid, V == 2 ? RPKT_F_IP_SUM : (RPKT_F_IP_SUM | RPKT_F_L4_SUM), L);
    uint8_t* slot = &W.win[lane * kSlot];
    uint8_t* s = slot + (fr.off & 15u);
    {
        // loopback_rx.rs:99-106 before the L4 sum is known: Ok chain, untagged IPv4
        // (w0 = status | n_vlan << 8 | ethertype << 16), IP checksum good, UDP.  The
        // rewrite that does not depend on the L4 sum is done in the window now
        // (written back only if the frame is kept); what the rest needs waits in the
        // slot's spare dword: pre | l4 << 8 | udp checksum << 16.
        const uint32_t w0 = L.w[0], w8 = L.w[8], w9 = L.w[9], w10 = L.w[10], w11 = L.w[11];
        const uint32_t ip_sum = L.w[18] & 0xffffu, l4 = L.w[16] >> 16;
        const bool pre = valid && (w0 & 0xffffu) == RPKT_S_OK && (w0 >> 16) == 0x0800u &&
                         ip_sum == 0xffffu && ((w8 >> 8) & 0xffu) == 17u;
        if (pre) {                                              // loopback_rx.rs:120-133
            const uint32_t ttl = w8 & 0xffu;
            const uint32_t old_w = (ttl << 8) | 17u, new_w = (((ttl - 1u) & 0xffu) << 8) | 17u;
            const uint32_t ip_ck = ~fold16(ip_sum + (~(w8 >> 16) & 0xffffu) +
                                           (~old_w & 0xffffu) + new_w) & 0xffffu;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                s[k] = fwd.dmac[k];
                s[6 + k] = fwd.smac[k];
            }
            s[22] = (uint8_t)(ttl - 1u);
            put_be16(s + 24, ip_ck);
            put_be32(s + 26, w10);
            put_be32(s + 30, w9);
            put_be16(s + l4, w11 >> 16);
            put_be16(s + l4 + 2, w11);
        }
        *reinterpret_cast<uint32_t*>(slot + kWin) =
            (uint32_t)pre | (l4 << 8) | ((L.w[15] & 0xffffu) << 16);
    }
    const uint32_t sp = wave_stream_sum<2>(rs, fb, L.stream_s, L.stream_e, W, lane);
    const uint32_t l4_sum =
        L.want_l4 ? fold16(L.pseudo + be_sum(L.l4_part + sp, L.l4_start_abs)) : 0u;
    const uint32_t info = *reinterpret_cast<const uint32_t*>(slot + kWin);
    const uint32_t l4 = (info >> 8) & 0xffu, udp_ck = info >> 16;
    bool fwd_ok = (info & 1u) && (l4_sum == 0xffffu || udp_ck == 0u);   // :107 L4 good
    if (fwd.n_forbid) {                                         // :111-118, sorted list
        // up to 128 addresses are searched in LDS (W.s and W.e, contiguous, free once
        // the stream is done), a longer list in global memory
        const bool in_lds = fwd.n_forbid <= 2u * kWave;
        const uint32_t* list = fwd.forbid_dev;
        if (in_lds) {
            uint32_t* t = W.s;
            if ((uint32_t)lane < fwd.n_forbid) t[lane] = fwd.forbid_dev[lane];
            if ((uint32_t)lane + kWave < fwd.n_forbid) t[lane + kWave] = fwd.forbid_dev[lane + kWave];
            wave_sync();
            list = t;
        }
        if (fwd_ok) {
            const uint32_t src = ((uint32_t)s[30] << 24) | ((uint32_t)s[31] << 16) |
                                 ((uint32_t)s[32] << 8) | s[33];   // swapped: old source
            uint32_t lo = 0, hi = fwd.n_forbid;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (list[mid] < src) lo = mid + 1; else hi = mid;
            }
            if (lo < fwd.n_forbid && list[lo] == src) fwd_ok = false;
        }
        wave_sync();
    }
    uint32_t r1 = 0;
    if (fwd_ok) {
        uint32_t u_ck = ~fold16(l4_sum + (~udp_ck & 0xffffu)) & 0xffffu;
        if (u_ck == 0u) u_ck = 0xffffu;                         // RFC 768
        put_be16(s + l4 + 6, u_ck);
        r1 = line_end(fr, l4 + 8u);
    }
    wave_sync();
    if constexpr (V != 1) write_back(frames, W, lane, fr.off, r1);
    if (valid) keep[i] = fwd_ok ? 1 : 0;
}

// ---- option iterators: TcpOptionsIter / Ipv4OptionsIter over a parsed batch ----
// One wave per 64 frames.  The records give each frame's option slices; only the
// 16-B chunks that overlap a slice are loaded (frames without options cost their
// record read and the 64-B output only).  Lane-per-frame walk over LDS bytes with
// the per-type parse rules of the generated option views (oracle/rpkt_oracle_opts.c
// cites them); results staged through LDS and stored as 4 KiB of coalesced rows.
constexpr int kOptChunks = 8;                  // 128 B from the 16-B phase of the first
constexpr int kOptSlot = 132;                  // option byte: both slices span at most
                                               // ihl4 + 40 <= 100 B, + 15 of phase
struct OptScratch {
    uint8_t win[kWave * kOptSlot];             // 8448 B (stride 33 dwords: conflict-free),
};                                             // so four blocks (16 waves) fit a CU
static_assert(kWave * 21 * 4 <= kWave * kOptSlot, "record stage fits the option window");

// Option bytes in LDS: frame byte x of this lane at base[x + bias] (bias = the window's
// phase minus the first option byte's frame offset; only x >= that offset is read).
struct OptWin {
    const uint8_t* base;                       // the lane's slot (4-aligned)
    uint32_t bias;
    __device__ __forceinline__ uint32_t b(uint32_t x) const { return base[x + bias]; }
    // frame bytes x..x+3, little-endian: two aligned LDS dwords and a byte align
    __device__ __forceinline__ uint32_t dw(uint32_t x) const {
        const uint32_t y = x + bias, a = y & ~3u;
        return align_bytes(lds32(base, a + 4), lds32(base, a), y & 3u);
    }
    __device__ __forceinline__ uint32_t be16(uint32_t x) const { return be16_lo(dw(x)); }
    __device__ __forceinline__ uint32_t be32(uint32_t x) const { return bswap32(dw(x)); }
};

// returns option length (> 0), 0 = the type's parse fails (malformed), -1 = unknown;
// d0 = the option's first four bytes (type, length, ...)
__device__ __forceinline__ int tcp_opt_len(uint32_t d0, uint32_t n, int& kind) {
    const uint32_t t = d0 & 0xffu, hl = n >= 2 ? (d0 >> 8) & 0xffu : 0u;
    switch (t) {
        case 0: kind = 0; return 1;
        case 1: kind = 1; return 1;
        case 2: kind = 2; return (n >= 4 && hl == 4) ? 4 : 0;
        case 3: kind = 3; return (n >= 3 && hl == 3) ? 3 : 0;
        case 4: kind = 4; return (n >= 2 && hl == 2) ? 2 : 0;
        case 5: kind = 5; return (n >= 2 && hl >= 2 && hl <= n) ? (int)hl : 0;
        case 8: kind = 6; return (n >= 10 && hl == 10) ? 10 : 0;
        case 34: kind = 7; return (n >= 2 && hl >= 2 && hl <= n) ? (int)hl : 0;
        default: return -1;
    }
}
__device__ __forceinline__ int ip_opt_len(uint32_t d0, uint32_t n, int& kind) {
    const uint32_t t = d0 & 0xffu, hl = n >= 2 ? (d0 >> 8) & 0xffu : 0u;
    switch (t) {
        case 0: kind = 0; return 1;
        case 1: kind = 1; return 1;
        case 68: kind = 2; return (n >= 4 && hl >= 4 && hl <= n) ? (int)hl : 0;
        case 7: kind = 3; return (n >= 3 && hl >= 3 && hl <= n) ? (int)hl : 0;
        case 148: kind = 4; return (n >= 4 && hl == 4) ? 4 : 0;
        case 134: kind = 5; return (n >= 6 && hl >= 6 && hl <= n) ? (int)hl : 0;
        case 137: kind = 6; return (n >= 7 && hl == 7) ? 7 : 0;
        case 131: kind = 7; return (n >= 7 && hl == 7) ? 7 : 0;
        default: return -1;
    }
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

__global__ __launch_bounds__(kWave * kWavesPerBlock)
void options_kernel(const uint8_t* __restrict__ frames, uint32_t fb,
                    const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                    uint32_t n, const rpkt_rec_t* __restrict__ recs, rpkt_opts_t* __restrict__ opts) {
    __shared__ __attribute__((aligned(16))) OptScratch scratch[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    OptScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    const Frame fr = spans.get(i);

    // records of the tile (coalesced), keep the four words the walks need
    uint32_t w0, w8, w14, w16;
    {
        const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
        const u32x4* in = reinterpret_cast<const u32x4*>(recs + p0);
        u32x4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t c = k * kWave + lane;
            v[k] = (c / 5 < nrec) ? in[c] : u32x4{0u, 0u, 0u, 0u};
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
        w0 = st[lane * 21 + 0];
        w8 = st[lane * 21 + 8];
        w14 = st[lane * 21 + 14];
        w16 = st[lane * 21 + 16];
        wave_sync();
    }
    const uint32_t status = w0 & 0xffu;
    const bool ip_parsed = status == RPKT_S_OK || status >= RPKT_S_L4_OTHER;
    const bool tcp = status == RPKT_S_OK && ((w8 >> 8) & 0xffu) == 6u;
    const uint32_t l3 = w16 & 0xffffu, l4 = w16 >> 16;
    const uint32_t ip_lo = l3 + 20u, ip_hi = ip_parsed ? l4 : ip_lo;
    const uint32_t t_lo = l4 + 20u, t_hi = tcp ? l4 + ((w14 >> 12) & 0xfu) * 4u : t_lo;
    // option bytes needed: [lo, hi) of the frame (both slices); chunks outside it skip
    const uint32_t need_lo = ip_hi > ip_lo ? ip_lo : t_lo;
    const uint32_t need_hi = t_hi > t_lo ? t_hi : ip_hi;
    const bool need = (ip_hi > ip_lo) || (t_hi > t_lo);

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
        for (int k = 0; k < kOptChunks; ++k) d[k] = load16_fast(rs, addr[k]);
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

    // the two walks (Ipv4OptionsIter::next, ipv4/generated.rs:1640-1722;
    // TcpOptionsIter::next, tcp/generated.rs:1400-1484), stepped together
    const OptWin s{&W.win[lane * kOptSlot], ((fr.off + need_lo) & 15u) - need_lo};
    uint32_t o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0;
    OptWalk ip{ip_lo, ip_hi - ip_lo, 0, 0, 0, RPKT_OPT_END, 0, ip_parsed && ip_hi > ip_lo};
    OptWalk tw{t_lo, t_hi - t_lo, 0, 0, 0, RPKT_OPT_END, 0, tcp && t_hi > t_lo};
    while (ip.on || tw.on) {
        if (ip.on) {
            const uint32_t at = ip.lo + ip.pos;
            const uint32_t d0 = s.dw(at);
            int kind = 0;
            const int used = opt_run(ip, d0) ? -2 : ip_opt_len(d0, ip.nb - ip.pos, kind);
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
            const int used = opt_run(tw, d0) ? -2 : tcp_opt_len(d0, tw.nb - tw.pos, kind);
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
    if (ip_parsed) {
        // word 6: tcp_fo_len | tcp_end << 16 | ip_end << 24; word 7: ip_count | ip_stop << 8 | ip_kinds << 16
        o[6] |= ip.pos << 24;
        o[7] = ip.cnt | (ip.stop << 8) | (ip.kinds << 16);
    }
    if (tcp) {
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

    // stage (stride 17 dwords) and store 64 rows of 64 B coalesced
    wave_sync();
    uint32_t* st = reinterpret_cast<uint32_t*>(W.win);
#pragma unroll
    for (int k = 0; k < 16; ++k) st[lane * 17 + k] = o[k];
    wave_sync();
    const uint32_t nrow = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* out = reinterpret_cast<u32x4*>(opts + p0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c = k * kWave + lane, r = c / 4, pc = c % 4;
        const uint32_t* src = st + r * 17 + pc * 4;
        if (r < nrow) __builtin_nontemporal_store(u32x4{src[0], src[1], src[2], src[3]}, &out[c]);
    }
}

// ---- protocol layer walk: the pktfmt-derived table interpreted per frame ----
// kProtos / kGroups (rpkt_proto_table.h, generated by tools/pktfmt_table.py from the
// reference's pktfmt specs) hold, per protocol, exactly what its generated parse /
// payload / group_parse are functions of; walk_group interprets them with the
// pktfmt codegen rules (pktfmt/src/codegen/parse.rs:138-244, payload.rs:23-87).
// One lane per frame over a 128-B LDS window (deeper bytes, about 1 % of the walks of
// the capture mix, from global memory).  128 B keeps the block at 37 KB of LDS, so four
// blocks (16 waves) fit a CU: the walk is a chain of dependent LDS round trips, and
// occupancy is what hides them.
constexpr int kLayChunks = 8;                  // 128 B window from the 16-B phase
constexpr int kLaySlot = 132;                  // 33 dwords: conflict-free lanes
struct LayScratch {
    uint8_t win[kWave * kLaySlot];             // 8448 B
};

struct LayerWin {
    const uint8_t* base;                       // the lane's slot; frame byte x at ph + x
    uint32_t ph;                               // frame offset & 15
    uint32_t avail;                            // frame bytes held in LDS
    uint32_t off;                              // frame's absolute offset
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ uint32_t at(uint32_t x) const {
        return x < avail ? (uint32_t)base[ph + x] : gbyte(rs, off + x);
    }
    // frame bytes x..x+3 as a little-endian dword: two aligned LDS dwords and a byte
    // align when all four are in the window, else byte by byte
    __device__ __forceinline__ uint32_t dw(uint32_t x) const {
        if (x + 4u <= avail) {
            const uint32_t y = ph + x, a = y & ~3u;
            return align_bytes(lds32(base, a + 4), lds32(base, a), y & 3u);
        }
        return at(x) | (at(x + 1) << 8) | (at(x + 2) << 16) | (at(x + 3) << 24);
    }
    __device__ __forceinline__ uint32_t be16(uint32_t x) const { return be16_lo(dw(x)); }
    // big-endian bit field (pktfmt bit order) of `bits` <= 32 at bit offset `ob` of x
    // (cond and length fields are at most 16 bits wide: 4 bytes always cover them)
    __device__ __forceinline__ uint32_t field(uint32_t x, uint32_t ob, uint32_t bits) const {
        const uint32_t v = bswap32(dw(x + (ob >> 3)));
        return (v << (ob & 7u)) >> (32u - bits);
    }
};

// The first 20 bytes of the current header as frame-relative little-endian dwords,
// read once per layer step: every condition, header_len and payload_len field of the
// table but one (MSTP's, at byte 36) and every dispatch key of lay_next lies in them,
// so a step costs one round of LDS reads instead of a dependent read per field.
struct LayHdr {
    uint32_t F[5];
};

__device__ __forceinline__ LayHdr lay_hdr(const LayerWin& Wn, uint32_t s) {
    LayHdr H;
    if (s + 20u <= Wn.avail) {
        const uint32_t y = Wn.ph + s, a = y & ~3u;
        uint32_t R[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) R[k] = lds32(Wn.base, a + 4 * k);
#pragma unroll
        for (int k = 0; k < 5; ++k) H.F[k] = align_bytes(R[k + 1], R[k], y & 3u);
    } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) H.F[k] = Wn.dw(s + 4 * k);
    }
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
__device__ __forceinline__ uint32_t hdr_at(const LayHdr& H, uint32_t x) {
    return hdr_dw(H, x) & 0xffu;
}
// the big-endian bit field of the table at bit offset ob of header s (Wn.field's rule)
__device__ __forceinline__ uint32_t hdr_field(const LayerWin& Wn, const LayHdr& H, uint32_t s,
                                              uint32_t ob, uint32_t bits) {
    if (__builtin_expect((ob >> 3) > 15u, 0)) return Wn.field(s, ob, bits);
    return (bswap32(hdr_dw(H, ob >> 3)) << (ob & 7u)) >> (32u - bits);
}

// The walk's LDS image of the table, repacked from kProtos / kGroups at kernel start
// so that a protocol's scalars are two 16-B reads and a condition one: per protocol
// 32 B, five 16-B condition slots, one dword per group.
struct LayProto {
    uint32_t a;               // hdr | hl_kind << 16 | pl_kind << 24
    int32_t hl_fixed;
    uint32_t hl0, hl1;        // expression: off | bits << 16 | form << 24 ; a | b << 16
    uint32_t pl0, pl1;
    uint32_t n_cond, pad;
};
struct LayCond {
    uint32_t f;               // off | bits << 16 | n << 24
    uint32_t lo01, hi01;      // lo[0] | lo[1] << 16 ; hi[0] | hi[1] << 16
    uint32_t r2;              // lo[2] | hi[2] << 16
};
struct LayTable {
    LayProto p[RPKT_N_PROTOS];
    LayCond c[RPKT_N_PROTOS][5];
    uint32_t g[RPKT_N_GROUPS];    // first | count << 8 | cond_bytes << 16 | lut << 24
    uint32_t lutf[RPKT_N_LUT];    // lookup groups: the keyed field, off | bits << 16
    uint8_t lut[RPKT_N_LUT][256]; // field value -> member (0xff: none)
};

__device__ __forceinline__ void lay_table_fill(LayTable& T) {
    for (uint32_t t = threadIdx.x; t < RPKT_N_PROTOS * 5; t += blockDim.x) {
        const uint32_t id = t / 5, k = t % 5;
        const RpktCond& C = kProtos[id].cond[k];
        T.c[id][k] = LayCond{C.off | ((uint32_t)C.bits << 16) | ((uint32_t)C.n << 24),
                             C.lo[0] | ((uint32_t)C.lo[1] << 16), C.hi[0] | ((uint32_t)C.hi[1] << 16),
                             C.lo[2] | ((uint32_t)C.hi[2] << 16)};
        if (k == 0) {
            const RpktProto& P = kProtos[id];
            T.p[id] = LayProto{P.hdr | ((uint32_t)P.hl_kind << 16) | ((uint32_t)P.pl_kind << 24),
                               P.hl_fixed,
                               P.hl.off | ((uint32_t)P.hl.bits << 16) | ((uint32_t)P.hl.form << 24),
                               P.hl.a | ((uint32_t)P.hl.b << 16),
                               P.pl.off | ((uint32_t)P.pl.bits << 16) | ((uint32_t)P.pl.form << 24),
                               P.pl.a | ((uint32_t)P.pl.b << 16), P.n_cond, 0u};
        }
    }
    if (threadIdx.x < RPKT_N_GROUPS) {
        const RpktGroup G = kGroups[threadIdx.x];
        T.g[threadIdx.x] = G.first | ((uint32_t)G.count << 8) | ((uint32_t)G.cond_bytes << 16) |
                           ((uint32_t)G.lut << 24);
    }
    if (threadIdx.x < RPKT_N_LUT) T.lutf[threadIdx.x] = kGroupLutField[threadIdx.x];
    for (uint32_t t = threadIdx.x; t < RPKT_N_LUT * 64; t += blockDim.x)
        reinterpret_cast<uint32_t*>(T.lut)[t] = reinterpret_cast<const uint32_t*>(kGroupLut)[t];
}

// pktfmt UsableAlgExpr (ast/length.rs:244-283) of the field at expression e0/e1
__device__ __forceinline__ uint32_t lay_len(const LayerWin& Wn, const LayHdr& H, uint32_t s,
                                            uint32_t e0, uint32_t e1) {
    const uint32_t x = hdr_field(Wn, H, s, e0 & 0xffffu, (e0 >> 16) & 0xffu);
    const uint32_t a = e1 & 0xffffu, b = e1 >> 16;
    switch (e0 >> 24) {
        case 0: return x;
        case 1: return x + a;
        case 2: return x * a;
        case 3: return (x + a) * b;
        default: return x * a + b;
    }
}

// group_parse + parse + payload() of group g at cursor [s, e): returns the member
// protocol (< 0 on Err) with its header length and the trimmed packet end.  A group
// whose members have no conditions (cond_bytes 0: every group but Ether, VLAN, ICMPv4,
// GRE, PPPoE and STP) takes its first member without entering the member loop; a
// group keyed on one byte (ICMPv4 types, PPPoE codes) looks its member up.
__device__ __forceinline__ int walk_group(const LayerWin& Wn, const LayHdr& H, const LayTable& T,
                                          uint32_t g, uint32_t s, uint32_t e, uint32_t& hl,
                                          uint32_t& end) {
    const uint32_t r = e - s;
    const uint32_t G = T.g[g];
    const uint32_t first = G & 0xffu, count = (G >> 8) & 0xffu, cond_bytes = (G >> 16) & 0xffu;
    const uint32_t lut = G >> 24;
    if (r < cond_bytes) return -1;
    int m = (int)first;
    if (lut != 0xffu) {                                      // one keyed field: table lookup
        const uint32_t f = T.lutf[lut];
        const uint32_t mm = T.lut[lut][hdr_field(Wn, H, s, f & 0xffffu, f >> 16)];
        if (mm == 0xffu) return -1;
        m = (int)mm;
    } else if (cond_bytes) {
        m = -1;
        for (uint32_t k = 0; k < count && m < 0; ++k) {
            const uint32_t id = first + k;
            const uint32_t nc = T.p[id].n_cond;
            bool ok = true;
            for (uint32_t c = 0; c < nc && ok; ++c) {
                const LayCond C = T.c[id][c];
                const uint32_t v = hdr_field(Wn, H, s, C.f & 0xffffu, (C.f >> 16) & 0xffu);
                const uint32_t n = C.f >> 24;
                bool in = v >= (C.lo01 & 0xffffu) && v <= (C.hi01 & 0xffffu);
                if (n > 1) in |= v >= (C.lo01 >> 16) && v <= (C.hi01 >> 16);
                if (n > 2) in |= v >= (C.r2 & 0xffffu) && v <= (C.r2 >> 16);
                ok = in;
            }
            if (ok) m = (int)id;
        }
        if (m < 0) return -1;
    }
    const LayProto P = T.p[m];
    const uint32_t hdr = P.a & 0xffffu, hk = (P.a >> 16) & 0xffu, pk = P.a >> 24;
    if (r < hdr) return -1;
    uint32_t h = hdr;
    if (hk == 1) {
        h = lay_len(Wn, H, s, P.hl0, P.hl1);
    } else if (hk == 2 || hk == 3) {                        // gre/mod.rs:68-101
        const uint32_t ind = hdr_be16(H, 0);
        h = hk == 2 ? 4u + ((ind & 0xc000u) ? 4u : 0u) + ((ind & 0x2000u) ? 4u : 0u) +
                          ((ind & 0x1000u) ? 4u : 0u)
                    : 8u + ((ind & 0x1000u) ? 4u : 0u) + ((ind & 0x0080u) ? 4u : 0u);
    } else if (hk == 4) {                                   // gtpv1.pktfmt header_len
        h = (hdr_at(H, 0) & 7u) ? 12u : 8u;
    } else if (hk == 5) {                                   // gtpv2.pktfmt header_len
        h = (hdr_at(H, 0) & 8u) ? 12u : 8u;
    }
    if (hk) {
        if (P.hl_fixed >= 0) {
            if (h != (uint32_t)P.hl_fixed) return -1;
        } else if (h < hdr || h > r) {
            return -1;
        }
    }
    end = e;
    if (pk == 1) {                                          // payload_len
        const uint32_t pay = lay_len(Wn, H, s, P.pl0, P.pl1);
        if ((uint64_t)pay + h > r) return -1;
        end = s + h + pay;
    } else if (pk == 2) {                                   // packet_len
        const uint32_t pkt = lay_len(Wn, H, s, P.pl0, P.pl1);
        if (pkt < h || pkt > r) return -1;
        end = s + pkt;
    }
    hl = h;
    return m;
}

constexpr int kNextEnd = -1, kNextUnknown = -2;

__device__ __forceinline__ int lay_ethertype(uint32_t et) {
    switch (et) {
        case 0x0800: return RPKT_G_IPV4;
        case 0x86dd: return RPKT_G_IPV6;
        case 0x8100: case 0x88a8: return RPKT_G_VLAN;
        case 0x0806: return RPKT_G_ARP;
        case 0x8847: case 0x8848: return RPKT_G_MPLS;
        case 0x8863: case 0x8864: return RPKT_G_PPPOE;
        default: return kNextUnknown;
    }
}
__device__ __forceinline__ int lay_ipproto(uint32_t p) {
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
        case 59: return kNextEnd;
        case 60: return RPKT_G_IPV6_DESTOPTS;
        default: return kNextUnknown;
    }
}

// The dispatch of include/rpkt_gpu.h (rpkt_layers_t) after protocol p whose header
// starts at h; the cursor is now [s, e).
__device__ __forceinline__ int lay_next(const LayerWin& Wn, const LayHdr& H, int p, uint32_t s,
                                        uint32_t e, uint32_t& key) {
    switch (p) {
        case RPKT_P_ETHER_ETHERFRAME: key = hdr_be16(H, 12); return lay_ethertype(key);
        case RPKT_P_VLAN_VLANFRAME: key = hdr_be16(H, 2); return lay_ethertype(key);
        case RPKT_P_ETHER_ETHERDOT3FRAME: case RPKT_P_VLAN_VLANDOT3FRAME: return RPKT_G_LLC;
        case RPKT_P_IPV4_IPV4:
            if (hdr_be16(H, 6) & 0x1fffu) return kNextEnd;          // non-first fragment
            key = hdr_at(H, 9);
            return lay_ipproto(key);
        case RPKT_P_IPV6_IPV6: key = hdr_at(H, 6); return lay_ipproto(key);
        case RPKT_P_IPV6_FRAGMENTHEADER:
            if (hdr_be16(H, 2) >> 3) return kNextEnd;
            key = hdr_at(H, 0);
            return lay_ipproto(key);
        case RPKT_P_IPV6_HOPBYHOPOPTION: case RPKT_P_IPV6_DESTOPTIONS:
        case RPKT_P_IPV6_ROUTINGHEADER: case RPKT_P_IPV6_AUTHENTICATIONHEADER:
            key = hdr_at(H, 0);
            return lay_ipproto(key);
        case RPKT_P_UDP_UDP: {
            const uint32_t dp = hdr_be16(H, 2), sp = hdr_be16(H, 0);
            const uint32_t port = (dp == 4789u || dp == 2152u || dp == 2123u) ? dp
                                : ((sp == 4789u || sp == 2152u || sp == 2123u) ? sp : 0u);
            if (!port) return kNextEnd;
            key = port;
            if (port == 4789u) return RPKT_G_VXLAN;
            if (e <= s) return kNextEnd;
            key = Wn.at(s) >> 5;                                    // GTP version
            return key == 1u ? RPKT_G_GTPV1 : (key == 2u ? RPKT_G_GTPV2 : kNextUnknown);
        }
        case RPKT_P_GRE_GRE:
            key = hdr_be16(H, 2);
            return key == 0x6558u ? RPKT_G_ETHER : lay_ethertype(key);
        case RPKT_P_VXLAN_VXLAN: return RPKT_G_ETHER;
        case RPKT_P_GTPV1_GTPV1:
            if ((hdr_at(H, 0) & 4u) || hdr_at(H, 1) != 255u) return kNextEnd;
            if (e <= s) return kNextEnd;
            key = Wn.at(s) >> 4;
            return key == 4u ? RPKT_G_IPV4 : (key == 6u ? RPKT_G_IPV6 : kNextUnknown);
        case RPKT_P_MPLS_MPLS:
            if (!(hdr_at(H, 2) & 1u)) return RPKT_G_MPLS;
            if (e <= s) return kNextEnd;
            key = Wn.at(s) >> 4;
            return key == 4u ? RPKT_G_IPV4 : (key == 6u ? RPKT_G_IPV6 : kNextUnknown);
        case RPKT_P_PPPOE_PPPOESESSION:
            key = hdr_be16(H, 6);
            return key == 0x0021u ? RPKT_G_IPV4 : (key == 0x0057u ? RPKT_G_IPV6 : kNextUnknown);
        case RPKT_P_LLC_LLC:
            return (hdr_at(H, 0) == 0x42u && hdr_at(H, 1) == 0x42u) ? RPKT_G_STP : kNextEnd;
        default: return kNextEnd;
    }
}

__global__ __launch_bounds__(kWave * kWavesPerBlock)
void layers_kernel(const uint8_t* __restrict__ frames, uint32_t fb,
                   const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                   uint32_t n, rpkt_layers_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) LayScratch scratch[kWavesPerBlock];
    // the protocol table in LDS: lanes walk different protocols, so table reads are
    // per-lane (divergent) loads; from LDS they cost tens of cycles instead of a
    // global-memory round trip per dependent lookup
    __shared__ __attribute__((aligned(16))) LayTable T;
    lay_table_fill(T);
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    LayScratch& W = scratch[wid];
    const uint32_t p0 = (blockIdx.x * kWavesPerBlock + wid) * kWave;
    if (p0 >= n) return;
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    const Frame fr = spans.get(i);
    {
        u32x4 d[kLayChunks];
        uint32_t addr[kLayChunks];
        uint32_t fix = 0;
#pragma unroll
        for (int k = 0; k < kLayChunks; ++k) {
            const int c = k * kWave + lane;
            const int q = c / kLayChunks, j = c % kLayChunks;
            const uint32_t qo = (uint32_t)__shfl((int)fr.off, q, kWave);
            const uint32_t ql = (uint32_t)__shfl((int)fr.len, q, kWave);
            const uint32_t a = (qo & ~15u) + 16u * j;
            addr[k] = (a < qo + ql) ? a : fb;
            fix |= (uint32_t)straddles(addr[k], fb) << k;
        }
#pragma unroll
        for (int k = 0; k < kLayChunks; ++k) d[k] = load16_fast(rs, addr[k]);
#pragma unroll
        for (int k = 0; k < kLayChunks; ++k) {
            const int c = k * kWave + lane;
            u32x4 v = d[k];
            if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
            uint32_t* dst = reinterpret_cast<uint32_t*>(&W.win[(c / kLayChunks) * kLaySlot +
                                                              (c % kLayChunks) * 16]);
            dst[0] = v.x;
            dst[1] = v.y;
            dst[2] = v.z;
            dst[3] = v.w;
        }
    }
    wave_sync();

    const uint32_t ph = fr.off & 15u;
    const LayerWin Wn{&W.win[lane * kLaySlot], ph, (uint32_t)(kLayChunks * 16) - ph, fr.off, rs};
    uint32_t o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0;
    uint32_t s = 0, e = valid ? fr.len : 0u, nl = 0, stop = 0, err_g = 0, key = 0, key_p = 0;
    int g = RPKT_G_ETHER;
    for (;;) {
        if (nl == RPKT_MAX_LAYERS) {
            stop = RPKT_L_MAX;
            break;
        }
        uint32_t hl = 0, end = 0;
        const LayHdr H = lay_hdr(Wn, s);
        const int p = walk_group(Wn, H, T, (uint32_t)g, s, e, hl, end);
        if (p < 0) {
            stop = RPKT_L_ERR;
            err_g = (uint32_t)g;
            break;
        }
        // proto[nl] at byte 16 + nl, off[nl] at byte 32 + 2 nl (predicated: nl differs
        // per lane, and a runtime register index would be a branch per register)
        {
            const uint32_t pw = (uint32_t)p << (8 * (nl & 3)), sw = s << (16 * (nl & 1));
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) o[4 + k] |= (nl >> 2) == k ? pw : 0u;
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) o[8 + k] |= (nl >> 1) == k ? sw : 0u;
        }
        nl += 1;
        e = end;
        s += hl;
        uint32_t k2 = 0;
        const int nx = lay_next(Wn, H, p, s, e, k2);
        if (nx == kNextEnd) {
            stop = RPKT_L_END;
            break;
        }
        if (nx == kNextUnknown) {
            stop = RPKT_L_UNKNOWN;
            key = k2;
            key_p = (uint32_t)p;
            break;
        }
        g = nx;
    }
    o[0] = nl | (stop << 8) | (err_g << 16) | (key_p << 24);
    o[1] = s & 0xffffu;
    o[2] = e - s;
    o[3] = key;

    wave_sync();
    uint32_t* st = reinterpret_cast<uint32_t*>(W.win);
#pragma unroll
    for (int k = 0; k < 16; ++k) st[lane * 17 + k] = o[k];
    wave_sync();
    const uint32_t nrow = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* dst = reinterpret_cast<u32x4*>(out + p0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c = k * kWave + lane, r = c / 4, pc = c % 4;
        const uint32_t* src = st + r * 17 + pc * 4;
        if (r < nrow) __builtin_nontemporal_store(u32x4{src[0], src[1], src[2], src[3]}, &dst[c]);
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

// ---- flow counters: LDS-privatised histogram per workgroup + slab reduce ----
// One workgroup per CU-sized slice of the events; each keeps {pkts, bytes,
// ip_bad | l4_bad << 16} per bucket in LDS (u32; a slice holds < 65536 events,
// so no field can overflow), writes it once to its slab, and a second kernel
// sums the slabs in a fixed order (bitwise reproducible counters).
constexpr int kFlowThreads = 512;
constexpr uint32_t kFlowLdsMax = 8192;      // buckets (+1 unparsed row) privatised in LDS
constexpr uint32_t kFlowMaxPerBlock = 32768;
constexpr uint32_t kFlowMinBlocks = 256;
constexpr int kFlowUnroll = 8;

__host__ __device__ inline uint32_t flow_blocks(uint32_t n) {
    uint32_t b = (n + kFlowMaxPerBlock - 1) / kFlowMaxPerBlock;
    uint32_t m = (n + kFlowThreads - 1) / kFlowThreads;   // >= one event per thread
    uint32_t want = kFlowMinBlocks < m ? kFlowMinBlocks : m;
    return b > want ? b : (want ? want : 1);
}

__global__ __launch_bounds__(kFlowThreads)
void flow_hist_kernel(const uint64_t* __restrict__ ev, uint32_t n, uint32_t per_block,
                      uint32_t n_buckets, uint32_t* __restrict__ slab) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];   // 3 * (n_buckets + 1)
    const uint32_t rows = n_buckets + 1;
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
            atomicAdd(&h[b], 1u);
            atomicAdd(&h[rows + b], (uint32_t)e[u]);
            const uint32_t bad =
                (uint32_t)((e[u] >> 48) & 1u) | ((uint32_t)((e[u] >> 49) & 1u) << 16);
            if (bad) atomicAdd(&h[2 * rows + b], bad);
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
            const uint32_t* sl = slab + (size_t)s * 3 * rows;
            pk += sl[b];
            by += sl[rows + b];
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

thread_local int g_last_hip_error = 0;

inline int hip_check(hipError_t e) {
    if (e != hipSuccess) {
        g_last_hip_error = (int)e;
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

extern "C" {

uint32_t rpkt_gpu_abi_version(void) { return RPKT_ABI_VERSION; }

#ifndef RPKT_SRC_HASH
#define RPKT_SRC_HASH "dev"
#endif
const char* rpkt_gpu_build_info(void) {
    return "rpkt_gpu src=" RPKT_SRC_HASH " gfx950; rec=80B; tile=64 frames/wave; win=128B";
}

const char* rpkt_gpu_status_name(int s) {
    static const char* names[] = {"OK", "ETH_SHORT", "VLAN_SHORT", "NOT_IPV4", "IP_SHORT",
                                  "IP_BAD_IHL", "IP_IHL_GT_LEN", "IP_TOT_LT_IHL",
                                  "IP_TOT_GT_LEN", "L4_OTHER", "UDP_SHORT", "UDP_BAD_LEN",
                                  "TCP_SHORT", "TCP_BAD_DOFF"};
    return (s >= 0 && s < (int)(sizeof(names) / sizeof(names[0]))) ? names[s] : "?";
}

int rpkt_gpu_last_hip_error(void) { return g_last_hip_error; }

int rpkt_gpu_device_info(char* buf, size_t len) {
    int count = 0, dev = -1;
    hipError_t e1 = hipGetDeviceCount(&count);
    hipError_t e2 = hipGetDevice(&dev);
    hipDeviceProp_t p;
    memset(&p, 0, sizeof(p));
    hipError_t e3 = dev >= 0 ? hipGetDeviceProperties(&p, dev) : hipErrorInvalidDevice;
    int rv = 0;
    if (hipRuntimeGetVersion(&rv) != hipSuccess) rv = -1;
    if (buf && len)
        snprintf(buf, len, "hip_runtime=%d devices=%d(err %d) current=%d(err %d) name=%s arch=%s "
                 "cus=%d (err %d)", rv, count, (int)e1, dev, (int)e2, p.name, p.gcnArchName,
                 p.multiProcessorCount, (int)e3);
    return (e1 == hipSuccess && count > 0) ? RPKT_OK : RPKT_E_HIP;
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
    if (flags & ~(uint32_t)(RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_FLOW_EV)) return RPKT_E_INVAL;
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
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_F_L4_SUM) ? parse_kernel<true, 0> : parse_kernel<false, 0>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags,
                  recs_dev, (uint64_t*)flow_ev_dev, n_buckets);
}

int rpkt_gpu_parse_chains(const rpkt_chains_t* c, uint32_t flags, rpkt_rec_t* recs_dev,
                          rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!c || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~(uint32_t)(RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_FLOW_EV)) return RPKT_E_INVAL;
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

int rpkt_gpu_build_batch(const rpkt_batch_t* b, const rpkt_rec_t* recs_dev, uint32_t flags,
                         uint8_t* built_dev, void* stream) {
    if (!b || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~(uint32_t)(RPKT_BUILD_IP_CSUM | RPKT_BUILD_L4_CSUM)) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)b->frames_dev & 15u) != 0)
        return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_BUILD_L4_CSUM) ? build_kernel<true> : build_kernel<false>;
    return launch(k, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,
                  b->stride, flen, b->n, recs_dev, flags, built_dev);
}

int rpkt_gpu_forward_batch(const rpkt_batch_t* b, const rpkt_fwd_t* fwd, uint8_t* keep_dev,
                           void* stream) {
    if (!b || !fwd || !keep_dev) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev || (fwd->n_forbid && !fwd->forbid_dev)) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)b->frames_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    return launch(forward_kernel<0>, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,
                  b->stride, flen, b->n, *fwd, keep_dev);
}

// Development hook (not part of include/rpkt_gpu.h): forward_kernel ablation variants.
int rpkt_gpu_debug_forward_variant(const rpkt_batch_t* b, const rpkt_fwd_t* fwd, uint8_t* keep_dev,
                                   int variant, void* stream) {
    if (!b || !fwd || !keep_dev || b->n == 0) return RPKT_E_INVAL;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
#define RPKT_FV(v)                                                                          \
    launch(forward_kernel<v>, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,          \
           const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,  \
           b->stride, flen, b->n, *fwd, keep_dev)
    switch (variant) {
        case 0: return RPKT_FV(0);
        case 1: return RPKT_FV(1);
        case 2: return RPKT_FV(2);
        case 3: return RPKT_FV(3);
        default: return RPKT_E_INVAL;
    }
#undef RPKT_FV
}

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
    return launch(options_kernel, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  recs_dev, opts_dev);
}

int rpkt_gpu_layers_batch(const rpkt_batch_t* b, rpkt_layers_t* layers_dev, void* stream) {
    if (!b || !layers_dev) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)layers_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    return launch(layers_kernel, dim3(grid), dim3(per_block), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  layers_dev);
}

// Development hook (not part of include/rpkt_gpu.h): ablation variants of the parse
// kernel and the streaming-copy roofline reference, for tools/ablate.py.
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
           b->offsets_dev, b->stride, flen, b->n, flags, recs, (uint64_t*)nullptr, 0u)
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
        case 13:
            return launch(copy_ref_kernel<8, false>, dim3(8192), dim3(256), 0, st,
                          (const u32x4*)b->frames_dev, (uint32_t)(b->frames_bytes / 16),
                          (u32x4*)recs, b->n * (RPKT_REC_BYTES / 16));
        default: return RPKT_E_INVAL;
    }
#undef RPKT_V
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
    static bool attr_set = false;
    if (!attr_set) {
        int rc0 = hip_check(hipFuncSetAttribute((const void*)flow_hist_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                3 * (kFlowLdsMax + 1) * sizeof(uint32_t)));
        if (rc0) return rc0;
        attr_set = true;
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

}  // extern "C"
