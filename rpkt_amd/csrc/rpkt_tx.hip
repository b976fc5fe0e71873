// rpkt_tx.hip — transmit side: build_kernel (prepend_header + setters + checksum fill)
// and forward_kernel (the loopback_rx firewall loop fused into one pass).
#include "rpkt_common.h"

namespace {

#ifndef RPKT_BUILD_WIN_AUX
#define RPKT_BUILD_WIN_AUX 0     // cache policy of build_kernel's window loads (2 = nt)
#endif
#ifndef RPKT_BUILD_REC_NT
#define RPKT_BUILD_REC_NT 1      // build_kernel's record loads non-temporal (read once)
#endif
#ifndef RPKT_TX_W64_ON
#define RPKT_TX_W64_ON 1         // hand short strided batches to the 64-B-window compile
#endif
// The 64-B-window compile serves only batches where every frame lies inside its window
// (tx_w64_fits, checked on the host before the hand-over): no frame has bytes past the
// window, so the edge lines and the payload stream of the L4 sums are compiled out.
// With the stream gone the kernels need 60 / 39 VGPRs and the LDS (26.6 KB per block)
// sets the occupancy: 6 blocks (6 waves per SIMD) per CU.  Dynamic LDS caps it at
// RPKT_TX_W64_BLOCKS: 8 rotated batches, same process, 5 blocks vs 6: build 2 41.6 vs
// 42.6 us, forward 2 28.0 vs 28.5 us; 4 blocks 41.9 / 28.8 (profiles/r02_txw64/).
#ifndef RPKT_TX_WHOLE
#define RPKT_TX_WHOLE 1          // 0: keep the stream code (ablation)
#endif
#ifndef RPKT_TX_W64_BLOCKS
#define RPKT_TX_W64_BLOCKS 5     // blocks per CU of the 64-B-window kernels (0: no cap)
#endif
#ifdef RPKT_TX_W64
constexpr uint32_t kCuLds = 160 * 1024;
__host__ __device__ constexpr uint32_t lds_pad_for(uint32_t blocks, uint32_t block_lds) {
    // the least dynamic LDS so that blocks + 1 no longer fit a CU
    return blocks == 0 || kCuLds / (blocks + 1) + 1 <= block_lds ? 0u
                                                                 : kCuLds / (blocks + 1) + 1 - block_lds;
}
constexpr bool kWholeFrame = RPKT_TX_WHOLE;
constexpr uint32_t kTxLdsPad =
    lds_pad_for(RPKT_TX_W64_BLOCKS, (uint32_t)sizeof(WaveScratch) * kWavesPerBlock);
static_assert(RPKT_TX_W64_BLOCKS == 0 ||
              RPKT_TX_W64_BLOCKS * (sizeof(WaveScratch) * kWavesPerBlock + kTxLdsPad) <= kCuLds,
              "the capped block count still fits a CU");
#else
constexpr bool kWholeFrame = false;
constexpr uint32_t kTxLdsPad = 0;
#endif

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
// tags, the 20 IPv4 bytes at l3 (or the IPv6 header's first 8 bytes), the UDP header or
// the 20 TCP bytes at l4.  These are exactly the bytes prepend_header + setters write
// (ether/generated.rs:71-88, vlan/generated.rs:73-100, ipv4/generated.rs:130-206,
// ipv6/generated.rs:94-135, udp/generated.rs:79-104, tcp/generated.rs:135-224); option
// bytes, IPv6 addresses and extension headers are not touched.
__device__ __forceinline__ void emit_link(uint8_t* s, const uint32_t (&w)[20], uint32_t nv) {
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
}
__device__ __forceinline__ void emit_ip4(uint8_t* ip, const uint32_t (&w)[20], uint32_t ip_len,
                                         uint32_t ip_ck) {
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
}
// Ipv6::prepend_header + setters: version / traffic class / flow label (ip6_vtcfl),
// payload_len = remaining() after the header, next_header, hop_limit
__device__ __forceinline__ void emit_ip6(uint8_t* ip, const uint32_t (&w)[20], uint32_t plen) {
    put_be32(ip, w[6]);
    put_be16(ip + 4, plen);
    ip[6] = (uint8_t)(w[7] >> 16);
    ip[7] = (uint8_t)(w[7] >> 24);
}
// `t` is the LDS slot, or global memory for an IPv6 L4 header past the window
__device__ __forceinline__ void emit_l4(uint8_t* t, const uint32_t (&w)[20], uint32_t proto,
                                        uint32_t udp_len, uint32_t l4_ck) {
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
// The word sum of the L4 header emit_l4 writes, with its checksum field 0 (big-endian
// words from the record's host-order values)
__device__ __forceinline__ uint32_t l4_hdr_sum(const uint32_t (&w)[20], uint32_t proto,
                                               uint32_t udp_len) {
    const uint32_t ports = halves(w[11]);
    return proto == 17u ? ports + udp_len
                        : ports + halves(w[12]) + halves(w[13]) + halves(w[14]) + (w[15] >> 16);
}

// Absolute-phase word sum of LDS slot bytes [s, e) (any alignment): whole dwords,
// minus the bytes of the first dword below s and of the last dword from e on.
__device__ __forceinline__ uint32_t lds_range_sum(const uint8_t* slot, uint32_t s, uint32_t e) {
    if (e <= s) return 0u;
    uint32_t acc = 0;
    uint32_t a = s & ~3u;
    for (; a + 12u < e; a += 16u) {                  // four reads in flight per round trip
        const uint32_t x0 = lds32(slot, a), x1 = lds32(slot, a + 4u);
        const uint32_t x2 = lds32(slot, a + 8u), x3 = lds32(slot, a + 12u);
        acc = hsum(x3, hsum(x2, hsum(x1, hsum(x0, acc))));
    }
    for (; a < e; a += 4) acc = hsum(lds32(slot, a), acc);
    acc -= halves(low_bytes(lds32(slot, s & ~3u), s & 3u));
    if (e & 3u) acc -= halves(lds32(slot, e & ~3u) & ~((1u << (8u * (e & 3u))) - 1u));
    return acc;
}

// Store frame bytes [0, r1) (frame-relative, per owning lane) from the tile's LDS
// slots.  The range lies inside the LDS window (r1 <= kWin - phase).  Each owner lane
// publishes its frame offset and r1 (W.pref / W.s: free once the stream is done);
// the lane that stores chunk c = k*64 + lane (piece j = lane & 7 of frame k*8 +
// lane/8) reads those two words and clips the chunk against the range itself.
// A chunk wholly inside the range is one dwordx4 buffer store, issued by every lane:
// a lane with nothing to store points it past the buffer's range, where the hardware
// drops it, so the common case has no branch.  Chunks the range cuts (a frame's
// first chunk at a nonzero 16-B phase, an end inside a chunk) are collected in a mask
// and stored dword by dword, byte by byte at the cut, behind one wave-uniform branch:
// bytes outside the range belong to neighbouring frames, which other lanes may be
// rewriting.
constexpr uint32_t kDropOffset = 0xffffffe0u;   // past any buffer's range; + 16 does not wrap
static_assert(kMaxFrameBytes <= kDropOffset, "a dropped store stays out of range");
// AUX: cache policy bits of the dwordx4 stores (forward: 3 = sc0 | nt; build: default).
template <int AUX = 0>
__device__ __forceinline__ void write_back(__amdgpu_buffer_rsrc_t rs, uint8_t* frames,
                                           WaveScratch& W, int lane, uint32_t off, uint32_t r1) {
    W.pref[lane] = off;
    W.s[lane] = r1;
    wave_sync();
    const int j = lane & (kWinChunks - 1);
    uint32_t cut = 0;
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) {
        const int q = k * (kWave / kWinChunks) + lane / kWinChunks;
        const uint32_t oq = W.pref[q], rq = W.s[q];
        const int lo = (int)(oq & 15u) - 16 * j;          // chunk-relative frame start
        const int hi = lo + (int)rq;                       // chunk-relative range end
        const bool any = rq != 0 && hi > 0;
        const bool full = any && lo <= 0 && hi >= 16;
        const uint32_t base = (oq & ~15u) + 16u * j;       // chunk's absolute address
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&W.win[q * kSlot + 16 * j]);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{src[0], src[1], src[2], src[3]}, rs,
                                               (int)(full ? base : kDropOffset), 0, AUX);
        cut |= (uint32_t)(any && !full) << k;
    }
    if (__builtin_expect(__ballot(cut != 0) != 0, 0)) {
#pragma unroll
        for (int k = 0; k < kWinChunks; ++k) {
            if (!(cut & (1u << k))) continue;
            const int q = k * (kWave / kWinChunks) + lane / kWinChunks;
            const uint32_t oq = W.pref[q], rq = W.s[q];
            const int lo = (int)(oq & 15u) - 16 * j;
            const int hi = lo + (int)rq;
            const uint32_t base = (oq & ~15u) + 16u * j;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(&W.win[q * kSlot + 16 * j]);
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
        v[k] = (c / 5 < nrec) ? (RPKT_BUILD_REC_NT ? __builtin_nontemporal_load(&in[c]) : in[c])
                              : u32x4{0u, 0u, 0u, 0u};
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

// End (frame-relative) of the 16-B chunk holding header byte hdr_end - 1: the least
// whole-chunk range covering the rewritten bytes, clipped to the frame and the window.
__device__ __forceinline__ uint32_t chunk_end(Frame fr, uint32_t hdr_end) {
    const uint32_t ph = fr.off & 15u;
    const uint32_t c = ((fr.off + hdr_end + 15u) & ~15u) - fr.off;
    uint32_t e = c < fr.len ? c : fr.len;
    return e < kWin - ph ? e : kWin - ph;
}

// The tunnel header rpkt_gpu_build_tunnel_batch writes (t: its first byte in the slot; tw
// the rpkt_tun_t words; tail = the frame's bytes from the header on): the prepend_header
// template + setters of Vxlan (vxlan/generated.rs:99-150: bytes 0-1 flags, group_id,
// vni; byte 7 the template's 0), Gtpv1 (gtpv1/generated.rs:110-170: flags, message
// type, length = remaining - 8, teid; a 12-B header's sequence, bytes 10-11 left as the
// buffer holds them) or Gre (gre/generated.rs:95-230: flags, version, protocol_type; the
// checksum word when C or R, 0 when the fill computes it; the key when K; offset and
// sequence left as the buffer holds them).
__device__ __forceinline__ uint32_t tun_hdr_len(uint32_t kind, uint32_t h0) {
    return kind == RPKT_TUN_VXLAN ? 8u
         : kind == RPKT_TUN_GTPU ? ((h0 & 7u) ? 12u : 8u)
         : 4u + ((h0 & 0xc0u) ? 4u : 0u) + ((h0 & 0x20u) ? 4u : 0u) + ((h0 & 0x10u) ? 4u : 0u);
}
__device__ __forceinline__ void emit_tunnel(uint8_t* t, uint32_t kind, uint32_t tw1, uint32_t tw2,
                                            uint32_t tw3, uint32_t tail, bool zero_ck) {
    t[0] = (uint8_t)tw3;
    t[1] = (uint8_t)(tw3 >> 8);
    if (kind == RPKT_TUN_VXLAN) {
        put_be16(t + 2, tw3 >> 16);                             // set_group_id
        t[4] = (uint8_t)(tw2 >> 16);                            // set_vni
        t[5] = (uint8_t)(tw2 >> 8);
        t[6] = (uint8_t)tw2;
        t[7] = 0u;
    } else if (kind == RPKT_TUN_GTPU) {
        put_be16(t + 2, tail - 8u);                             // set_packet_len(remaining)
        put_be32(t + 4, tw2);                                   // set_teid
        if (tw3 & 7u) put_be16(t + 8, tw3 >> 16);               // set_sequence
    } else {
        put_be16(t + 2, tw1 >> 16);                             // set_protocol_type
        const uint32_t cr = (tw3 & 0xc0u) ? 4u : 0u;
        if (cr) put_be16(t + 4, zero_ck ? 0u : tw3 >> 16);      // set_checksum
        if (tw3 & 0x20u) put_be32(t + 4 + cr, tw2);             // set_key
    }
}

// rpkt_gpu_build_batch: window -> headers composed in LDS -> checksums (IPv4 over the
// slot; L4 over the slot plus the payload stream past the window) -> write-back.
// TUN (rpkt_gpu_build_tunnel_batch): a tunnel header from tun[i] composed in the slot too,
// before the sums (the outer UDP checksum covers it); a GRE checksum filled like an L4 one
// with no pseudo header.
#ifndef RPKT_BUILD_MINW
#define RPKT_BUILD_MINW 3        // waves per SIMD the build compiles for: 3 (132 VGPRs, no
                                 // spill) beat 4 (128, 12 B of scratch with the tunnel stage)
#endif
template <bool L4FILL, bool TUN = false>
__global__ __launch_bounds__(kWave * kWavesPerBlock, RPKT_BUILD_MINW)
void build_kernel(uint8_t* __restrict__ frames, uint32_t fb, const uint32_t* __restrict__ offsets,
                  uint32_t stride, uint32_t frame_len, uint32_t n,
                  const rpkt_rec_t* __restrict__ recs, uint32_t flags, uint8_t* __restrict__ built,
                  const rpkt_tun_t* __restrict__ tun) {
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
        const uint32_t fix = window_issue<RPKT_BUILD_WIN_AUX>(rs, fb, fr, lane, d, addr);
        load_records_tile(recs, p0, n, W, lane, w);             // window loads in flight
        window_commit(W, rs, fb, d, addr, fix, lane);
    }
    const uint32_t wend = (fr.off & ~15u) + kWin, fend = fr.off + fr.len;
    EdgeLines X{false, 0u, 0u, 0u};
    if constexpr (L4FILL && !kWholeFrame) X = edge_lines_first(rs, fb, W, lane, valid, wend, fend);
    wave_sync();

    const uint32_t ph = fr.off & 15u, len = fr.len;
    uint8_t* slot = &W.win[lane * kSlot];
    const uint32_t nv = (w[0] >> 8) & 0xffu;
    const uint32_t l3 = 14u + 4u * nv;
    // an IPv6 record (RPKT_F_IPV6 parse: dispatched on 0x86DD) is built with the IPv6
    // header; its l4 is the record's (after the extension headers)
    const uint32_t st = w[0] & 0xffu;
    const uint32_t det = nv == 0u ? w[0] >> 16 : (nv == 1u ? w[5] & 0xffffu : w[5] >> 16);
    const bool rec6 = det == 0x86ddu && st != RPKT_S_ETH_SHORT && st != RPKT_S_VLAN_SHORT &&
                      st != RPKT_S_NOT_IPV4;
    const uint32_t ihl4 = (w[6] & 0xfu) * 4u;
    const uint32_t l4 = rec6 ? w[16] >> 16 : l3 + ihl4;
    const uint32_t proto = (w[8] >> 8) & 0xffu;                 // byte 33 in both layouts
    const uint32_t doff4 = ((w[14] >> 12) & 0xfu) * 4u;
    const uint32_t l4hdr = proto == 17u ? 8u : (proto == 6u ? doff4 : 0u);
    const uint32_t fixed4 = proto == 17u ? 8u : (proto == 6u ? 20u : 0u);
    const bool fits = valid && nv <= RPKT_MAX_VLAN && !(proto == 6u && doff4 < 20u) &&
                      len >= l4 + l4hdr && !(proto == 17u && len - l4 > 65535u);
    // the tunnel: VXLAN / GTP-U in the UDP payload (l4 + 8), GRE at l4 (protocol 47); the
    // header must lie in the frame and in the LDS window, else the frame is not built
    uint32_t tw1 = 0u, tw2 = 0u, tw3 = 0u, tkind = 0u, ts = 0u, thl = 0u;
    bool tun_ok = true;
    if constexpr (TUN) {
        if (valid) {
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(tun) + i);
            tkind = t.x & 0xffu;
            tw1 = t.y;
            tw2 = t.z;
            tw3 = t.w;
        }
        if (tkind != RPKT_TUN_NONE) {
            ts = tkind == RPKT_TUN_GRE ? l4 : l4 + 8u;
            thl = tun_hdr_len(tkind, tw3 & 0xffu);
            tun_ok = tkind <= RPKT_TUN_GRE && proto == (tkind == RPKT_TUN_GRE ? 47u : 17u) &&
                     len >= ts + thl && ts + thl <= RPKT_TUN_BUILD_MAX_END &&
                     !(tkind == RPKT_TUN_GTPU && len - ts > 65543u);   // gtpv1/generated.rs:116
        }
    }
    const bool ok = fits && tun_ok && (rec6 ? l4 >= l3 + 40u && len - l3 - 40u <= 65535u
                                            : ihl4 >= 20u && len - l3 <= 65535u);
    // an IPv6 L4 header that does not lie whole in the window is written to global memory
    // by its lane (extension headers can push it past the window), never from the slot
    const bool far = ok && rec6 && fixed4 != 0u && ph + l4 + fixed4 > (uint32_t)kWin;
    const bool fill_ip = ok && !rec6 && (flags & RPKT_BUILD_IP_CSUM);
    const bool fill_l4 = L4FILL && ok && fixed4;
    // the GRE checksum (checksum_present) with the L4 fill: RFC 2784 over the GRE header
    // and payload, no pseudo header
    const bool fill_gre = TUN && L4FILL && ok && tkind == RPKT_TUN_GRE && (tw3 & 0x80u);
    if (ok) {
        if constexpr (TUN) {
            if (tkind != RPKT_TUN_NONE) emit_tunnel(slot + ph + ts, tkind, tw1, tw2, tw3, len - ts, fill_gre);
        }
        emit_l4(far ? frames + fr.off + l4 : slot + ph + l4, w, proto, len - l4,
                fill_l4 ? 0u : (w[15] & 0xffffu));
        if (rec6) emit_ip6(slot + ph + l3, w, len - l3 - 40u);
        else emit_ip4(slot + ph + l3, w, len - l3, fill_ip ? 0u : (w[8] >> 16));
        emit_link(slot + ph, w, nv);
    }
    if (fill_ip) {
        const uint32_t s = be_sum(lds_range_sum(slot, ph + l3, ph + l4), fr.off + l3);
        put_be16(slot + ph + l3 + 10, ~s & 0xffffu);
    }
    // the write-back's end, taken before the stream so the header layout is not held
    // across it: the window holds the original bytes around the headers, so the written
    // range is rounded up to whole 16-B chunks inside the frame (dwordx4 stores)
    uint32_t hdr_end = far ? l3 + 8u : l4 + fixed4;
    if (TUN && tkind != RPKT_TUN_NONE && ts + thl > hdr_end) hdr_end = ts + thl;
    uint32_t r1 = ok ? line_end(fr, hdr_end) : 0u;
    r1 = far && r1 > l4 ? l4 : r1;                          // the L4 header went to memory
    if constexpr (L4FILL) {
        // everything the checksum needs after the stream is packed into the slot's
        // spare dword (bytes 128..131) and two registers, so the stream keeps its
        // registers: pseudo header sum, in-window part, and
        // info = fill | udp << 1 | far << 2 | l4 slot offset << 8
        uint32_t part = 0, ss = 0, se = 0, pseudo = 0;
        const uint32_t win_end = kWin - ph;
        if (fill_l4 || fill_gre) {
            // the summed range starts at the L4 header, or past it (far: the header's
            // sum comes from the record's values); the in-window part, then the stream
            const uint32_t ps = far ? l4 + fixed4 : l4;
            const uint32_t e_in = len < win_end ? len : win_end;
            part = ps < e_in ? lds_range_sum(slot, ph + ps, ph + e_in) : 0u;
            const uint32_t s0 = ps > e_in ? ps : e_in;
            if (len > s0) {
                ss = fr.off + s0;
                se = fr.off + len;
            }
            if (fill_gre) {
                pseudo = 0u;            // GRE: the header and payload alone
            } else if (rec6) {          // pseudo_v6: src, the final destination, length, nh
                const FrameDw dw{slot, ph, fr.off, fb, rs};
                uint32_t pd = w[8] >> 16;
                if (pd < l3 + 24u || pd + 16u > l4) pd = l3 + 24u;   // as the oracle
                pseudo = addr_words_sum(dw(l3 + 8u), dw(l3 + 12u), dw(l3 + 16u), dw(l3 + 20u)) +
                         addr_words_sum(dw(pd), dw(pd + 4u), dw(pd + 8u), dw(pd + 12u));
            } else {
                const uint32_t src = w[9], dst = w[10];
                pseudo = (src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu);
            }
            if (!fill_gre) pseudo += proto + (len - l4) + (far ? l4_hdr_sum(w, proto, len - l4) : 0u);
        }
        *reinterpret_cast<uint32_t*>(slot + kWin) = (uint32_t)(fill_l4 || fill_gre) |
            ((uint32_t)(proto == 17u) << 1) | ((uint32_t)far << 2) | ((uint32_t)fill_gre << 3) |
            ((ph + l4) << 8);
        uint32_t sp = 0;
        if constexpr (!kWholeFrame) sp = stream_rest<2>(X, rs, fb, ss, se, wend, fend, W, lane);
        const uint32_t info = *reinterpret_cast<const uint32_t*>(slot + kWin);
        if (info & 1u) {
            const uint32_t at = info >> 8;                      // slot offset of the L4 header
            // (far: the summed range starts fixed4 bytes later, an even offset: same phase)
            const uint32_t sum = fold16(pseudo + be_sum(part + sp, (fr.off & ~15u) + at));
            uint32_t ck = ~sum & 0xffffu;
            const bool udp = info & 2u, gre = info & 8u;
            if (ck == 0u && udp && !gre) ck = 0xffffu;          // RFC 768 / RFC 8200 8.1
            uint8_t* t = (info & 4u) ? frames + (fr.off & ~15u) + at : slot + at;
            put_be16(t + (gre ? 4u : (udp ? 6u : 16u)), ck);
        }
    }
    wave_sync();
    write_back(rs, frames, W, lane, fr.off, r1);
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
// 2 = parse without the L4 sum, 3 = window + write-back of the whole frame only,
// 4 = default-policy window loads).
#ifndef RPKT_FWD_WB_AUX
#define RPKT_FWD_WB_AUX 3        // forward's write-back stores: sc0 | nt
#endif
#ifndef RPKT_FWD_WB_CHUNKS
#define RPKT_FWD_WB_CHUNKS 0     // 1: write back only the 16-B chunks holding rewritten bytes
#endif
#ifndef RPKT_FWD_WAVES_W64
#define RPKT_FWD_WAVES_W64 5     // 64-B windows: LDS allows 6 waves per SIMD; 5 -> <= 96 VGPRs
#endif
#ifdef RPKT_TX_W64
#define RPKT_FWD_WAVES RPKT_FWD_WAVES_W64
#else
#define RPKT_FWD_WAVES 4
#endif
template <int V>
__global__ __launch_bounds__(kWave * kWavesPerBlock, RPKT_FWD_WAVES)
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
    // the forbidden-source list (up to 128 addresses, searched in LDS) is loaded with
    // the window, not after the parse: one memory round trip per wave instead of two
    const bool list_in_lds = fwd.n_forbid != 0 && fwd.n_forbid <= 2u * kWave;
    uint32_t fl0 = 0, fl1 = 0;
    if (list_in_lds) {
        if ((uint32_t)lane < fwd.n_forbid) fl0 = fwd.forbid_dev[lane];
        if ((uint32_t)lane + kWave < fwd.n_forbid) fl1 = fwd.forbid_dev[lane + kWave];
    }
    {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        // non-temporal window loads: 32.1 -> 31.0 us on 64-B frames (profiles/r02_fwd)
        const uint32_t fix = window_issue<V == 4 ? 0 : 2>(rs, fb, fr, lane, d, addr);
        window_commit(W, rs, fb, d, addr, fix, lane);
    }
    wave_sync();
    if constexpr (V == 3) {
        write_back(rs, frames, W, lane, fr.off, valid ? line_end(fr, 0u) : 0u);
        if (valid) keep[i] = 1;
        return;
    }
    LaneRec L;
    parse_lane(W, lane, fr, valid,
               (V == 2 ? RPKT_F_IP_SUM : (RPKT_F_IP_SUM | RPKT_F_L4_SUM)) | (fwd.flags & RPKT_F_IPV6),
               L, rs, fb);
    uint8_t* slot = &W.win[lane * kSlot];
    uint8_t* s = slot + (fr.off & 15u);
    const uint32_t l4 = L.w[16] >> 16;
    uint32_t delta = 0;                 // IPv6 pseudo header change (one's-complement add)
    bool far = false;                   // IPv6: UDP header not whole in the window
    {
        // loopback_rx.rs:99-106 before the L4 sum is known: Ok chain, untagged IPv4
        // (w0 = status | n_vlan << 8 | ethertype << 16), IP checksum good, UDP.  The
        // rewrite that does not depend on the L4 sum is done in the window now
        // (written back only if the frame is kept); what the rest needs waits in the
        // slot's spare dword: pre | far << 1 | udp checksum << 16.
        const uint32_t w0 = L.w[0], w8 = L.w[8], w9 = L.w[9], w10 = L.w[10], w11 = L.w[11];
        const uint32_t ip_sum = L.w[18] & 0xffffu;
        const bool pre4 = valid && !L.is6 && (w0 & 0xffffu) == RPKT_S_OK && (w0 >> 16) == 0x0800u &&
                          ip_sum == 0xffffu && ((w8 >> 8) & 0xffu) == 17u;
        // the IPv6 counterpart (fwd.flags & RPKT_F_IPV6): untagged (the record's n_vlan 0,
        // ethertype 0x86DD), parsed OK to UDP; there is no header checksum
        const bool pre6 = valid && L.is6 && (w0 & 0xffffu) == RPKT_S_OK && ((w8 >> 8) & 0xffu) == 17u;
        if (pre4 || pre6) {                                     // loopback_rx.rs:120-133
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                s[k] = fwd.dmac[k];
                s[6 + k] = fwd.smac[k];
            }
        }
        if (pre4) {
            const uint32_t ttl = w8 & 0xffu;
            const uint32_t old_w = (ttl << 8) | 17u, new_w = (((ttl - 1u) & 0xffu) << 8) | 17u;
            const uint32_t ip_ck = ~fold16(ip_sum + (~(w8 >> 16) & 0xffffu) +
                                           (~old_w & 0xffffu) + new_w) & 0xffffu;
            s[22] = (uint8_t)(ttl - 1u);
            put_be16(s + 24, ip_ck);
            put_be32(s + 26, w10);
            put_be32(s + 30, w9);
            put_be16(s + l4, w11 >> 16);
            put_be16(s + l4 + 2, w11);
        } else if (pre6) {
            // hop_limit - 1, the addresses swapped (bytes 8..39 of the header, 54 at most:
            // in the window), the ports swapped in the window or, past it, after the stream
            constexpr uint32_t l3 = 14u;
            s[l3 + 7] = (uint8_t)(s[l3 + 7] - 1u);
            uint32_t a[4], b[4];
            const FrameDw dw{slot, fr.off & 15u, fr.off, fb, rs};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[k] = dw(l3 + 8u + 4u * k);
                b[k] = dw(l3 + 24u + 4u * k);
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                s[l3 + 8 + k] = (uint8_t)(b[k / 4] >> (8 * (k % 4)));
                s[l3 + 24 + k] = (uint8_t)(a[k / 4] >> (8 * (k % 4)));
            }
            // the pseudo header's destination is the final address of a routing header
            // when there is one (record ip6_pdst_off != dst_addr): the swap then moves the
            // old dst into the source slot only, a change of S(dst) - S(src)
            if ((w8 >> 16) != l3 + 24u) {
                const uint32_t sa = fold16(addr_words_sum(a[0], a[1], a[2], a[3]));
                const uint32_t sb = fold16(addr_words_sum(b[0], b[1], b[2], b[3]));
                delta = sb + (~sa & 0xffffu);
            }
            far = (fr.off & 15u) + l4 + 8u > (uint32_t)kWin;
            if (!far) {
                put_be16(s + l4, w11 >> 16);
                put_be16(s + l4 + 2, w11);
            }
        }
        *reinterpret_cast<uint32_t*>(slot + kWin) =
            (uint32_t)(pre4 || pre6) | ((uint32_t)far << 1) | ((L.w[15] & 0xffffu) << 16);
    }
    uint32_t sp = 0;
    if constexpr (!kWholeFrame) sp = wave_stream_sum<2>(rs, fb, L.stream_s, L.stream_e, W, lane);
    const uint32_t l4_sum =
        L.want_l4 ? fold16(L.pseudo + be_sum(L.l4_part + sp, L.l4_start_abs)) : 0u;
    const uint32_t info = *reinterpret_cast<const uint32_t*>(slot + kWin);
    const uint32_t udp_ck = info >> 16;
    // :107 L4 good (over IPv6 a zero UDP checksum is not "not computed", RFC 8200 8.1)
    bool fwd_ok = (info & 1u) && (l4_sum == 0xffffu || (udp_ck == 0u && !L.is6));
    if (fwd.n_forbid) {                                         // :111-118, sorted list
        // up to 128 addresses are searched in LDS (W.s and W.e, contiguous, free once
        // the stream is done), a longer list in global memory
        const uint32_t* list = fwd.forbid_dev;
        if (list_in_lds) {
            uint32_t* t = W.s;
            t[lane] = fl0;
            t[lane + kWave] = fl1;
            wave_sync();
            list = t;
        }
        // the list holds IPv4 addresses: an IPv6 source never matches it
        if (fwd_ok && !L.is6) {
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
        uint32_t u_ck = ~fold16(l4_sum + (~udp_ck & 0xffffu) + delta) & 0xffffu;
        if (u_ck == 0u) u_ck = 0xffffu;                         // RFC 768
        if (info & 2u) {
            // IPv6 UDP header past the window: ports and checksum stored by the lane (the
            // stream that read those bytes is done), the write-back stops before them
            uint8_t* g = frames + fr.off + l4;
            put_be16(g, L.w[11] >> 16);
            put_be16(g + 2, L.w[11]);
            put_be16(g + 6, u_ck);
            r1 = line_end(fr, 54u);
            r1 = r1 > l4 ? l4 : r1;
        } else {
            put_be16(s + l4 + 6, u_ck);
            r1 = RPKT_FWD_WB_CHUNKS ? chunk_end(fr, l4 + 8u) : line_end(fr, l4 + 8u);
        }
    }
    wave_sync();
    // the rewritten lines are not read again: streaming stores (forward 2: 27.8 -> 26.2 us
    // same process; build keeps the default policy, build 3 +2.5 % with it,
    // profiles/r02_ab_wb)
    if constexpr (V != 1) write_back<RPKT_FWD_WB_AUX>(rs, frames, W, lane, fr.off, r1);
    if (valid) keep[i] = fwd_ok ? 1 : 0;
}

}  // namespace

// This unit compiles twice: as is (128-B windows) and with RPKT_TX_W64 (RPKT_WIN 64,
// rpkt_amd/build.py), whose entry points are the hidden *_w64 functions the first
// compile hands strided batches of short frames to: a 64-B frame needs only a 64-B
// window, so a wave's LDS drops from 9.7 to 6.7 KB and the block from 38.9 to 26.6 KB,
// and the VGPRs, not the LDS, set the waves per SIMD.
#ifdef RPKT_TX_W64
#define RPKT_TX_FN(name) __attribute__((visibility("hidden"))) name##_w64
#else
#define RPKT_TX_FN(name) name
#endif

extern "C" {

#ifndef RPKT_TX_W64
int rpkt_gpu_build_batch_w64(const rpkt_batch_t*, const rpkt_rec_t*, uint32_t, uint8_t*, void*);
int rpkt_gpu_forward_batch_w64(const rpkt_batch_t*, const rpkt_fwd_t*, uint8_t*, void*);
#ifdef RPKT_ABLATE
int rpkt_gpu_debug_forward_variant_w64(const rpkt_batch_t*, const rpkt_fwd_t*, uint8_t*, int, void*);
#endif
#endif

#ifndef RPKT_TX_W64
// strided, every frame within 64 bytes of its 16-B boundary: the 64-B-window compile
static bool tx_w64_fits(const rpkt_batch_t* b, uint32_t flen) {
    if (b->offsets_dev || b->stride == 0 || flen == 0) return false;
    return flen + ((b->stride & 15u) ? 15u : 0u) <= 64u;
}
#endif

int RPKT_TX_FN(rpkt_gpu_build_batch)(const rpkt_batch_t* b, const rpkt_rec_t* recs_dev,
                                     uint32_t flags, uint8_t* built_dev, void* stream) {
    if (!b || !recs_dev) return RPKT_E_INVAL;
    if (flags & ~(uint32_t)(RPKT_BUILD_IP_CSUM | RPKT_BUILD_L4_CSUM)) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)b->frames_dev & 15u) != 0)
        return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
#ifndef RPKT_TX_W64
    if (RPKT_TX_W64_ON && tx_w64_fits(b, flen))
        return rpkt_gpu_build_batch_w64(b, recs_dev, flags, built_dev, stream);
#endif
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_BUILD_L4_CSUM) ? build_kernel<true> : build_kernel<false>;
    return launch(k, dim3(grid), dim3(per_block), kTxLdsPad, (hipStream_t)stream,
                  const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,
                  b->stride, flen, b->n, recs_dev, flags, built_dev,
                  static_cast<const rpkt_tun_t*>(nullptr));
}

#ifndef RPKT_TX_W64
// The encapsulation build (always the 128-B-window compile: a tunnel frame is longer than
// a 64-B window).
int rpkt_gpu_build_tunnel_batch(const rpkt_batch_t* b, const rpkt_rec_t* recs_dev,
                                const rpkt_tun_t* tun_dev, uint32_t flags, uint8_t* built_dev,
                                void* stream) {
    if (!b || !recs_dev || !tun_dev) return RPKT_E_INVAL;
    if (flags & ~(uint32_t)(RPKT_BUILD_IP_CSUM | RPKT_BUILD_L4_CSUM)) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)recs_dev & 15u) != 0 || ((uintptr_t)tun_dev & 15u) != 0 ||
        ((uintptr_t)b->frames_dev & 15u) != 0)
        return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    auto k = (flags & RPKT_BUILD_L4_CSUM) ? build_kernel<true, true> : build_kernel<false, true>;
    return launch(k, dim3(grid), dim3(per_block), kTxLdsPad, (hipStream_t)stream,
                  const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,
                  b->stride, flen, b->n, recs_dev, flags, built_dev, tun_dev);
}
#endif

int RPKT_TX_FN(rpkt_gpu_forward_batch)(const rpkt_batch_t* b, const rpkt_fwd_t* fwd,
                                       uint8_t* keep_dev, void* stream) {
    if (!b || !fwd || !keep_dev) return RPKT_E_INVAL;
    // unknown bits (a caller that left the old `reserved` field uninitialised) are refused,
    // as rpkt_gpu_build_batch refuses unknown build flags
    if (fwd->flags & ~(uint32_t)RPKT_F_IPV6) return RPKT_E_INVAL;
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev || (fwd->n_forbid && !fwd->forbid_dev)) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)b->frames_dev & 15u) != 0) return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
#ifndef RPKT_TX_W64
    if (RPKT_TX_W64_ON && tx_w64_fits(b, flen))
        return rpkt_gpu_forward_batch_w64(b, fwd, keep_dev, stream);
#endif
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
    return launch(forward_kernel<0>, dim3(grid), dim3(per_block), kTxLdsPad, (hipStream_t)stream,
                  const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,
                  b->stride, flen, b->n, *fwd, keep_dev);
}

#ifdef RPKT_ABLATE
// Development hook (librpkt_gpu_ablate.so only, not part of include/rpkt_gpu.h):
// forward_kernel ablation variants for tools/ablate_fwd.py.
int RPKT_TX_FN(rpkt_gpu_debug_forward_variant)(const rpkt_batch_t* b, const rpkt_fwd_t* fwd,
                                               uint8_t* keep_dev, int variant, void* stream) {
    if (!b || !fwd || !keep_dev || b->n == 0) return RPKT_E_INVAL;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
#ifndef RPKT_TX_W64
    if (variant >= 10) {                          // the 64-B-window compile's variants
        if (!tx_w64_fits(b, flen)) return RPKT_E_INVAL;
        return rpkt_gpu_debug_forward_variant_w64(b, fwd, keep_dev, variant - 10, stream);
    }
    if (variant == 9) {                           // the product path of this compile only
        const uint32_t per_block = kWave * kWavesPerBlock;
        return launch(forward_kernel<0>, dim3((b->n + per_block - 1) / per_block), dim3(per_block), kTxLdsPad,
                      (hipStream_t)stream, const_cast<uint8_t*>(b->frames_dev),
                      (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, *fwd,
                      keep_dev);
    }
#endif
    const uint32_t per_block = kWave * kWavesPerBlock;
    const uint32_t grid = (b->n + per_block - 1) / per_block;
#define RPKT_FV(v)                                                                          \
    launch(forward_kernel<v>, dim3(grid), dim3(per_block), kTxLdsPad, (hipStream_t)stream,          \
           const_cast<uint8_t*>(b->frames_dev), (uint32_t)b->frames_bytes, b->offsets_dev,  \
           b->stride, flen, b->n, *fwd, keep_dev)
    switch (variant) {
        case 0: return RPKT_FV(0);
        case 1: return RPKT_FV(1);
        case 2: return RPKT_FV(2);
        case 3: return RPKT_FV(3);
        case 4: return RPKT_FV(4);
        default: return RPKT_E_INVAL;
    }
#undef RPKT_FV
}

#endif  // RPKT_ABLATE

}  // extern "C"
