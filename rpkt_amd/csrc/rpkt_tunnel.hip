// rpkt_tunnel.hip — rpkt_gpu_parse_tunnel_batch: the outer parse, one tunnel level
// (VXLAN, GTP-U with its extension headers, GRE) and the parse of the inner frame, with
// every sum of both levels, in one pass per 64-frame tile (include/rpkt_gpu.h documents
// the records and the dispatch; oracle/rpkt_oracle_tunnel.c restates it on the CPU).
//
// One wavefront per tile, as parse_kernel: the outer header windows go to LDS (on long
// tiles together with each frame's tail line, whose sum is taken there and then) and each
// lane runs parse_lane on its frame; the lane then decodes the tunnel header(s) from the
// same window (FrameDw: global memory past it).  The outer record waits in registers (its
// words 0..11 in LDS past the inner record's stage once that is written: 128 VGPRs and
// 9.7 KB of LDS per wave, 16 waves per CU), and the inner frame's window is made from the
// outer one: the chunks they share move down the lane's slot and only the chunks past the
// outer window are loaded.  parse_lane runs again from the inner frame's first byte (its
// IP header for GTP-U and GRE).  One flattened chunk stream (rpkt_common.h) then sums each
// lane's main range -- the inner L4 bytes past the inner window, or the outer L4 range
// without a tunnel -- and the outer L4 sum (UDP, or GRE with its checksum), whose range
// contains the inner one, is composed from the outer window's part, the inner window's
// part (LDS), the main stream's sum when the rest of the two ranges is the same, and a
// rare stream for bytes before the inner window or a trailer after the inner packet.
// Each payload byte leaves HBM about once for all four sums (config 13: reads 1.09x the
// frame bytes, the excess the line the outer window ends in).
#include "rpkt_common.h"

namespace {

struct Tunnel {
    uint32_t w[4];      // rpkt_tun_t as 4 little-endian words
    uint32_t is, ie;    // the inner frame, frame offsets [is, ie)
    uint32_t start_et;  // the inner frame's first header: 0 Ethernet, 0x0800, 0x86DD
    bool ok;
};

__device__ __forceinline__ void tun_set(Tunnel& T, uint32_t kind, uint32_t status, uint32_t tun_off,
                                        uint32_t inner_off, uint32_t inner_type) {
    T.w[0] = kind | (status << 8) | (tun_off << 16);
    T.w[1] = (inner_off & 0xffffu) | (inner_type << 16);
}

// The inner packet of a GTP-U T-PDU or a GRE payload by its first header's type:
// 0x0800 IPv4, 0x86DD IPv6 (with RPKT_F_IPV6), 0x6558 Ethernet; anything else is
// INNER_UNKNOWN.
__device__ __forceinline__ void tun_inner(Tunnel& T, uint32_t kind, uint32_t ts, uint32_t is,
                                          uint32_t ie, uint32_t type, uint32_t flags) {
    const bool eth = type == 0x6558u, ip4 = type == 0x0800u;
    const bool ip6 = type == 0x86ddu && (flags & RPKT_F_IPV6);
    T.ok = eth || ip4 || ip6;
    T.start_et = eth ? 0u : type;
    T.is = is;
    T.ie = ie;
    tun_set(T, kind, T.ok ? RPKT_T_OK : RPKT_T_INNER_UNKNOWN, ts, is, type);
}

// The tunnel of one parsed frame (L: its outer record; dw: its bytes, frame offsets).
// Every byte read lies inside the span its parse tested ([ts, te) and the headers in it).
__device__ __forceinline__ Tunnel decode_tunnel(const LaneRec& L, const FrameDw& dw,
                                                uint32_t flags) {
    Tunnel T;
    T.w[0] = RPKT_TUN_NONE | (RPKT_T_NONE << 8);
    T.w[1] = T.w[2] = T.w[3] = 0u;
    T.is = T.ie = T.start_et = 0u;
    T.ok = false;
    const uint32_t* w = L.w;
    const uint32_t proto = (w[8] >> 8) & 0xffu;              // ip_protocol (IPv4 and IPv6)
    uint32_t kind = RPKT_TUN_NONE, ts = 0u, te = 0u;
    if (L.status == RPKT_S_OK && proto == 17u) {
        // Udp::payload() (udp/generated.rs:66-76): [payload_off, + payload_len)
        const uint32_t dp = w[11] >> 16, sp = w[11] & 0xffffu;
        const uint32_t port = (dp == 4789u || dp == 2152u) ? dp
                            : ((sp == 4789u || sp == 2152u) ? sp : 0u);
        if (port != 0u) {
            kind = port == 4789u ? RPKT_TUN_VXLAN : RPKT_TUN_GTPU;
            ts = w[17] & 0xffffu;
            te = ts + (w[17] >> 16);
        }
    } else if (L.status == RPKT_S_L4_OTHER && proto == 47u &&
               (L.is6 || ((w[7] >> 16) & 0x1fffu) == 0u)) {
        // Ipv4|Ipv6::payload() of a first (or only) fragment: [l4_off, + payload_len)
        kind = RPKT_TUN_GRE;
        ts = w[16] >> 16;
        te = ts + (w[17] >> 16);
    }
    if (kind == RPKT_TUN_NONE) return T;
    const uint32_t cl = te - ts;                             // chunk() == remaining()
    tun_set(T, kind, RPKT_T_BAD, ts, 0u, 0u);
    if (kind == RPKT_TUN_VXLAN) {
        // Vxlan::parse (vxlan/generated.rs:32-39): chunk_len >= 8; getters :44-87;
        // payload() :91-96 advance 8 -> EtherFrame::parse (vlan_mpls_tests.rs:250)
        if (cl < 8u) return T;
        const uint32_t d0 = dw(ts), d1 = dw(ts + 4u);
        T.w[2] = bswap32(d1) >> 8;                            // vni, bytes 4..6
        T.w[3] = (d0 & 0xffffu) | (be16_hi(d0) << 16);        // flags bytes 0, 1; group_id
        tun_inner(T, kind, ts, ts + 8u, te, 0x6558u, flags);
        return T;
    }
    if (kind == RPKT_TUN_GTPU) {
        // Gtpv1::parse (gtpv1/generated.rs:33-49): chunk_len >= 8, header_len (8, or 12
        // with any of E/S/PN, :239-250) <= chunk_len, header_len <= packet_len (length +
        // 8, :81-84) <= remaining
        if (cl < 8u) return T;
        const uint32_t d0 = dw(ts);
        const uint32_t b0 = d0 & 0xffu, msg = (d0 >> 8) & 0xffu;
        const uint32_t hl = (b0 & 7u) ? 12u : 8u;
        const uint32_t plen = be16_hi(d0) + 8u;
        if (hl > cl || plen < hl || plen > cl) return T;
        const uint32_t d2 = hl == 12u ? dw(ts + 8u) : 0u;
        T.w[2] = bswap32(dw(ts + 4u));                        // teid :74-76
        T.w[3] = (d0 & 0xffffu) | (be16_lo(d2) << 16);        // byte 0, message_type; sequence
        // payload() :98-108: trim to packet_len, advance header_len
        uint32_t c = ts + hl;
        const uint32_t end = ts + plen;
        if ((b0 >> 5) != 1u || msg != 255u) {                 // not a GTPv1 G-PDU
            tun_set(T, kind, RPKT_T_NOT_TPDU, ts, c, 0u);
            return T;
        }
        // the extension headers (gtpv1_test.rs:222-229, 306-318, 494-503): the type named
        // by the previous header's next_extention_header (Gtpv1::next_extention_header
        // :275-278 reads byte 11), each its parse, header_len and payload() (advance)
        uint32_t nx = (b0 & 4u) ? (d2 >> 24) : 0u;
        for (int k = 0; k < RPKT_MAX_GTP_EXT && nx != 0u; ++k) {
            const uint32_t rem = end - c, x = dw(c);
            const uint32_t e0 = x & 0xffu, t = (x >> 12) & 0xfu;
            uint32_t need, mn, ehl;
            if (nx == 0x40u || nx == 0xc0u || nx == 0x20u) {
                need = 4u; mn = 4u; ehl = 4u;                 // ExtUdpPort :336-341,
            } else if (nx == 0x03u || nx == 0x82u) {          //   ExtPduNumber :461-466,
                need = 8u; mn = 8u; ehl = 8u;                 //   ExtServiceClassIndicator
            } else if (nx == 0x81u || nx == 0x83u) {          //   :747-752; ExtLongPduNumber
                need = 1u; mn = 1u; ehl = e0 * 4u;            //   :587-592; ExtContainer
            } else if (nx == 0x84u && t <= 2u) {              //   :880-892 (header_len :902);
                need = 2u; mn = t == 0u ? 6u : (t == 1u ? 7u : 3u); ehl = e0 * 4u;  // NrUp
            } else if (nx == 0x85u && t <= 1u) {              //   :2308-2320; PduSessionUp
                need = 2u; mn = 3u; ehl = e0 * 4u;            //   :1507-1518
            } else {
                need = ~0u; mn = 0u; ehl = 0u;                // unknown type / group Err
            }
            if (rem < need || rem < mn || ehl < mn || ehl > rem) {
                tun_set(T, kind, RPKT_T_EXT_BAD, ts, c, 0u);
                return T;
            }
            nx = dw(c + ehl - 1u) & 0xffu;                    // next_extention_header: last byte
            c += ehl;
        }
        if (nx != 0u) {
            tun_set(T, kind, RPKT_T_EXT_BAD, ts, c, 0u);
            return T;
        }
        // the T-PDU: Ipv4 / Ipv6 by its version nibble (gtpv1_test.rs:229)
        const uint32_t v = c < end ? (dw(c) >> 4) & 0xfu : 0u;
        tun_inner(T, kind, ts, c, end, v == 4u ? 0x0800u : (v == 6u ? 0x86ddu : 0u), flags);
        return T;
    }
    // GreGroup::group_parse (gre/generated.rs:800-820): chunk >= 4; (C, R, K, version,
    // protocol_type) == (0, 0, 1, 1, 0x880B) -> GreForPPTP::parse (:371-386), version 0 ->
    // Gre::parse (:33-44, header_len gre/mod.rs:68-85), else Err
    // (a header that fails its parse leaves id / hdr0 / hdr1 / aux 0)
    if (cl < 4u) return T;
    const uint32_t d0 = dw(ts);
    const uint32_t b0 = d0 & 0xffu, b1 = (d0 >> 8) & 0xffu, pt = be16_hi(d0), ver = b1 & 7u;
    if ((b0 & 0xe0u) == 0x20u && ver == 1u && pt == 0x880bu) {
        if (cl < 8u) return T;
        const uint32_t d1 = dw(ts + 4u);
        const uint32_t phl = 8u + ((b0 & 0x10u) ? 4u : 0u) + ((b1 & 0x80u) ? 4u : 0u);
        if (phl > cl || be16_lo(d1) + phl > cl) return T;     // payload_len + header_len
        T.w[2] = bswap32(d1);                                 // payload_len, call_id
        T.w[3] = d0 & 0xffffu;
        tun_set(T, kind, RPKT_T_INNER_UNKNOWN, ts, ts + phl, pt);   // PPP, not IP
        return T;
    }
    if (ver != 0u) return T;
    const uint32_t cr = (b0 & 0xc0u) ? 4u : 0u;
    const uint32_t hl = 4u + cr + ((b0 & 0x20u) ? 4u : 0u) + ((b0 & 0x10u) ? 4u : 0u);
    if (hl > cl) return T;
    T.w[3] = (d0 & 0xffffu) | (cr ? be16_lo(dw(ts + 4u)) << 16 : 0u);   // checksum :236-241
    if (b0 & 0x20u) T.w[2] = bswap32(dw(ts + 4u + cr));        // key :260-267
    tun_inner(T, kind, ts, ts + hl, te, pt, flags);           // payload() advance header_len
    return T;
}

// Records staged at rl (stride 21 dwords) -> recs[p0 .. p0 + 64), 1-KiB wave stores.
__device__ __forceinline__ void flush_stage(const uint32_t* rl, int lane, rpkt_rec_t* recs,
                                            uint32_t p0, uint32_t n) {
    wave_sync();
    const uint32_t nrec = n - p0 < (uint32_t)kWave ? n - p0 : (uint32_t)kWave;
    u32x4* out = reinterpret_cast<u32x4*>(recs + p0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t c = k * kWave + lane, r = c / 5, pc = c % 5;
        const uint32_t* src = rl + r * 21 + pc * 4;
        if (r < nrec) __builtin_nontemporal_store(u32x4{src[0], src[1], src[2], src[3]}, &out[c]);
    }
}

// Absolute-phase word sum of LDS slot bytes [s, e) (slot byte 0 on a 16-B boundary).
__device__ __forceinline__ uint32_t slot_range_sum(const uint8_t* slot, uint32_t s, uint32_t e) {
    if (e <= s) return 0u;
    uint32_t acc = 0;
    uint32_t a = s & ~3u;
    for (; a + 12u < e; a += 16u) {
        const uint32_t x0 = lds32(slot, a), x1 = lds32(slot, a + 4u);
        const uint32_t x2 = lds32(slot, a + 8u), x3 = lds32(slot, a + 12u);
        acc = hsum(x3, hsum(x2, hsum(x1, hsum(x0, acc))));
    }
    for (; a < e; a += 4) acc = hsum(lds32(slot, a), acc);
    acc -= halves(low_bytes(lds32(slot, s & ~3u), s & 3u));
    if (e & 3u) acc -= halves(lds32(slot, e & ~3u) & ~((1u << (8u * (e & 3u))) - 1u));
    return acc;
}

// The outer header windows, and with them (joint) each frame's tail line [tb, fend): the
// line the next frame's window starts in, fetched in the same load group as that window
// (the cooperative mapping of window_with_edges: chunk k of lane l is piece l % 8 of frame
// 8 k + l / 8), so the stream never fetches it a second time.  Returns this lane's tail sum.
__device__ __forceinline__ uint32_t outer_window_tail(__amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                                      WaveScratch& W, int lane, Frame fr,
                                                      uint32_t tb, uint32_t fend) {
    const int j = lane & 7;
    constexpr int kHalf = kWinChunks / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32x4 dw[kHalf], dt[kHalf];
        uint32_t aw[kHalf], at[kHalf], lt[kHalf];
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int k = h * kHalf + i;
            const int q = (k * kWave + lane) >> 3;
            const uint32_t qo = (uint32_t)__shfl((int)fr.off, q, kWave);
            const uint32_t qn = (uint32_t)__shfl((int)fr.len, q, kWave);
            const uint32_t qt = (uint32_t)__shfl((int)tb, q, kWave);
            const uint32_t qe = (uint32_t)__shfl((int)fend, q, kWave);
            const uint32_t a = (qo & ~15u) + 16u * j, y = qt + 16u * j;
            aw[i] = a < qo + qn ? a : fb;
            const bool tin = y < qe;
            at[i] = tin ? y : fb;
            lt[i] = tin ? (qe - y < 16u ? qe - y : 16u) : 0u;
        }
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            dw[i] = load16_fast<0>(rs, aw[i]);
            dt[i] = load16_fast<0>(rs, at[i]);
        }
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int k = h * kHalf + i;
            u32x4 v = dw[i], vt = dt[i];
            if (__builtin_expect(straddles(aw[i], fb), 0)) v = load16(rs, aw[i], fb);
            if (__builtin_expect(lt[i] != 0 && straddles(at[i], fb), 0)) vt = load16(rs, at[i], fb);
            put_chunk(W, k * kWave + lane, v);
            const uint32_t xt = sum8_lanes(lt[i] ? chunk_sum(vt, 0, (int)lt[i]) : 0u);
            if (j == 0) W.last[(k * kWave + lane) >> 3] = xt;
        }
    }
    wave_sync();
    return W.last[lane];
}

// The inner window from the outer one: a lane whose inner frame starts d chunks into its
// outer window moves chunks d.. of its slot down to 0.. (its own slot: no other lane reads
// it), then the wave loads only the chunks past the outer window (cooperatively, the
// window_issue mapping) and writes them into the slots.  Lanes without a tunnel keep
// their outer window.
__device__ __forceinline__ void inner_window_reuse(__amdgpu_buffer_rsrc_t rs, uint32_t fb,
                                                   WaveScratch& W, int lane, uint32_t a1,
                                                   uint32_t keep, uint32_t lim) {
    u32x4 d[kWinChunks];
    uint32_t addr[kWinChunks];
    uint32_t fix = 0;
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) {
        const int c = k * kWave + lane;
        const int q = c / kWinChunks, j = c % kWinChunks;
        const uint32_t qa = (uint32_t)__shfl((int)a1, q, kWave);
        const uint32_t qk = (uint32_t)__shfl((int)keep, q, kWave);
        const uint32_t ql = (uint32_t)__shfl((int)lim, q, kWave);
        const uint32_t a = qa + 16u * j;
        addr[k] = ((uint32_t)j >= qk && a < ql) ? a : fb;
        fix |= (uint32_t)straddles(addr[k], fb) << k;
    }
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) d[k] = load16_fast<0>(rs, addr[k]);
    const uint32_t sh = (uint32_t)kWinChunks - keep;              // chunks moved down
    if (keep != (uint32_t)kWinChunks && keep != 0u) {
        uint32_t* sl = reinterpret_cast<uint32_t*>(&W.win[lane * kSlot]);
        for (uint32_t j = 0; j < keep; ++j) {
            const uint32_t x0 = sl[4 * (j + sh)], x1 = sl[4 * (j + sh) + 1];
            const uint32_t x2 = sl[4 * (j + sh) + 2], x3 = sl[4 * (j + sh) + 3];
            sl[4 * j] = x0;
            sl[4 * j + 1] = x1;
            sl[4 * j + 2] = x2;
            sl[4 * j + 3] = x3;
        }
    }
    wave_sync();                                      // every slot moved before the writes
#pragma unroll
    for (int k = 0; k < kWinChunks; ++k) {
        if (addr[k] == fb) continue;
        u32x4 v = d[k];
        if (__builtin_expect(fix & (1u << k), 0)) v = load16(rs, addr[k], fb);
        put_chunk(W, k * kWave + lane, v);
    }
    wave_sync();
}

// The flow event of a record from its words alone (its status is byte 0; the IPv6 block
// is used when the dispatch ethertype -- the last tag's, or the frame's, or an inner IP
// packet's start type -- is 0x86DD and the IPv6 header was reached), as flow_event forms it.
template <typename WordsT>
__device__ __forceinline__ uint64_t record_event(const WordsT& w, uint32_t n_buckets) {
    LaneRec R;
    R.status = w[0] & 0xffu;
    const uint32_t nv = (w[0] >> 8) & 0xffu;
    const uint32_t det = nv == 0u ? w[0] >> 16 : (nv == 1u ? w[5] & 0xffffu : w[5] >> 16);
    R.is6 = det == 0x86ddu && R.status != RPKT_S_ETH_SHORT && R.status != RPKT_S_VLAN_SHORT &&
            R.status != RPKT_S_NOT_IPV4;
    uint32_t x[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) x[k] = w[k];
    return flow_event(R, x, n_buckets);
}

// chunk loads in flight per lane in the main stream (2: 1-2 % faster than 3 and 4, the
// fewer lines in flight the fewer window lines evicted before their reuse; 6 and 8: no gain,
// and 8 costs occupancy)
#ifndef RPKT_TUN_UNROLL
#define RPKT_TUN_UNROLL 2
#endif
constexpr int kTunUnroll = RPKT_TUN_UNROLL;

template <bool L4>
__device__ __forceinline__ void tunnel_tile(WaveScratch& W,
                                            const uint8_t* __restrict__ frames, uint32_t fb,
                                            const uint32_t* __restrict__ offsets, uint32_t stride,
                                            uint32_t frame_len, uint32_t n, uint32_t flags,
                                            rpkt_rec_t* __restrict__ outer, rpkt_tun_t* __restrict__ tun,
                                            rpkt_rec_t* __restrict__ inner,
                                            uint64_t* __restrict__ flow_ev, uint32_t n_buckets,
                                            uint32_t p0, int lane) {
    const uint32_t i = p0 + lane;
    const bool valid = i < n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, fb);
    const SpanSrc spans{offsets, stride, frame_len, fb, n};
    // header-only batches read each line once: non-temporal window loads (as parse_tile)
    constexpr int kWinAux = L4 ? 0 : 2;

    // 1. the outer header windows -> LDS (with the frames' tail lines on long tiles), the
    // outer parse
    const Frame fr = spans.get(i);
    const uint32_t a0 = fr.off & ~15u, fend = fr.off + (valid ? fr.len : 0u);
    [[maybe_unused]] uint32_t tb = fend, tail_sum = 0u;
    bool joint = false;
    if constexpr (L4) {
        const uint32_t wend0 = a0 + kWin;
        if (fend > wend0) tb = max(fend & ~127u, wend0);
        joint = wave_sum(fend > wend0 ? fend - wend0 : 0u) > kEdgeWindowBytes;   // uniform
    }
    if (joint) {
        tail_sum = outer_window_tail(rs, fb, W, lane, fr, tb, fend);
    } else {
        u32x4 d[kWinChunks];
        uint32_t addr[kWinChunks];
        const uint32_t fix = window_issue<kWinAux>(rs, fb, fr, lane, d, addr);
        window_commit(W, rs, fb, d, addr, fix, lane);
        wave_sync();
    }
    LaneRec L;
    parse_lane(W, lane, fr, valid, flags, L, rs, fb);

    // 2. the tunnel, from the outer window
    const Tunnel T = decode_tunnel(L, FrameDw{&W.win[lane * kSlot], fr.off & 15u, fr.off, fb, rs},
                                   flags);

    // 3. the outer record in registers through the inner parse (a second LDS stage for it
    // held the kernel at 10 waves per CU), its L4 sum state kept for the streams
    uint32_t ow[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) ow[k] = L.w[k];
    [[maybe_unused]] const uint32_t o_ss = L.stream_s, o_se = L.stream_e, o_part = L.l4_part;
    [[maybe_unused]] const uint32_t o_abs = L.l4_start_abs, o_pseudo = L.pseudo;
    [[maybe_unused]] const bool o_want = L.want_l4;

    // 4. the inner header windows -> LDS (the outer ones are no longer read), inner parse
    const Frame fi = T.ok ? Frame{fr.off + T.is, T.ie - T.is} : Frame{0u, 0u};
    const uint32_t a1 = T.ok ? fi.off & ~15u : a0;
    const uint32_t dch = (a1 - a0) >> 4;
    const uint32_t keep = dch < (uint32_t)kWinChunks ? (uint32_t)kWinChunks - dch : 0u;
    // (chunks loaded up to the outer frame's end: the outer L4 range's part in this window
    // is summed from it below, and it can run past the inner frame)
    inner_window_reuse(rs, fb, W, lane, a1, T.ok ? keep : (uint32_t)kWinChunks, fend);
    parse_lane(W, lane, fi, T.ok, flags, L, rs, fb, T.start_et, T.is);
    if (!T.ok) {
#pragma unroll
        for (int k = 0; k < 20; ++k) L.w[k] = 0u;
        L.w[0] = RPKT_S_NO_INNER;
        L.want_l4 = false;
        L.stream_s = L.stream_e = 0u;
    }
    // the outer L4 range's bytes the inner window holds: [max(o_ss, a1), min(o_se, a1 + 128))
    [[maybe_unused]] uint32_t o_lds = 0u;
    if constexpr (L4) {
        if (T.ok && o_want) {
            const uint32_t ls = o_ss > a1 ? o_ss : a1, le = o_se < a1 + kWin ? o_se : a1 + kWin;
            o_lds = slot_range_sum(&W.win[lane * kSlot], ls - a1, le > ls ? le - a1 : ls - a1);
        }
    }
    stage_record(W, lane, L.w);
    // the outer record's words 0..11 wait in the window area past the inner stage (free
    // now: 3072 B, word-major), so the streams hold 8 of its words in registers, not 20
    static_assert(kWave * 21 * 4 + 12 * kWave * 4 <= kWinArea, "parked words fit past the stage");
    uint32_t* park = reinterpret_cast<uint32_t*>(&W.win[kWave * 21 * 4]);
#pragma unroll
    for (int k = 0; k < 12; ++k) park[k * kWave + lane] = ow[k];

    // 5. L4 bytes past the windows: the inner stream, then the outer range's other bytes
    if constexpr (L4) {
        // one main stream per lane: the inner L4 range (the outer one without a tunnel),
        // less the tail line summed with the windows when the range runs to the frame end
        const uint32_t ms = T.ok ? L.stream_s : (o_want ? o_ss : 0u);
        const uint32_t me = T.ok ? L.stream_e : (o_want ? o_se : 0u);
        const bool use_tail = joint && me > ms && me == fend && tb < fend && tb >= ms;
        const uint32_t sp_m = wave_stream_sum<2, kTunUnroll>(rs, fb, ms, use_tail ? tb : me, W, lane) +
                              (use_tail ? tail_sum : 0u);
        // the outer range of a tunnel frame: [o_ss, a1) streamed (an inner window past the
        // outer one), the inner window's part from LDS, [a1 + 128, o_se) the main stream when
        // it is the same range, else streamed
        const uint32_t w1 = a1 + kWin;
        const uint32_t p3s = o_ss > w1 ? o_ss : w1;
        const bool shared = T.ok && o_want && p3s == ms && o_se == me && me > ms;
        const bool rest = T.ok && o_want;
        uint32_t sp_o = wave_stream_sum<2>(rs, fb, rest ? o_ss : 0u,
                                           rest ? (o_se < a1 ? o_se : a1) : 0u, W, lane);
        sp_o += wave_stream_sum<2>(rs, fb, rest && !shared ? p3s : 0u,
                                   rest && !shared ? o_se : 0u, W, lane);
        sp_o += T.ok ? o_lds + (shared ? sp_m : 0u) : sp_m;
        if (L.want_l4)
            rec_stage(W)[lane * 21 + 18] |= fold16(L.pseudo + be_sum(L.l4_part + sp_m, L.l4_start_abs)) << 16;
        if (o_want) ow[18] |= fold16(o_pseudo + be_sum(o_part + sp_o, o_abs)) << 16;
    }

    // 6. records: the inner one, then the outer one staged where it was (1-KiB wave stores),
    // the tunnel record (16 B per lane); the flow event from the inner record when the
    // tunnel decoded, else from the outer one (include/rpkt_gpu.h)
    const bool ev = (flags & RPKT_F_FLOW_EV) && valid;
    if (ev && T.ok) __builtin_nontemporal_store(record_event(rec_stage(W) + lane * 21, n_buckets),
                                                &flow_ev[i]);
    flush_stage(rec_stage(W), lane, inner, p0, n);
#pragma unroll
    for (int k = 0; k < 12; ++k) ow[k] = park[k * kWave + lane];
    if (ev && !T.ok) __builtin_nontemporal_store(record_event(ow, n_buckets), &flow_ev[i]);
    stage_record(W, lane, ow);
    flush_stage(rec_stage(W), lane, outer, p0, n);
    if (valid) __builtin_nontemporal_store(u32x4{T.w[0], T.w[1], T.w[2], T.w[3]},
                                           reinterpret_cast<u32x4*>(tun) + i);
}

// One wave per workgroup (as the parse: a CU slot frees when its wave ends); 9.7 KB of LDS
// and 128 VGPRs per wave: 16 waves per CU
template <bool L4>
__global__ __launch_bounds__(kWave, 2)
void tunnel_kernel(const uint8_t* __restrict__ frames, uint32_t fb,
                   const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len,
                   uint32_t n, uint32_t flags, rpkt_rec_t* __restrict__ outer,
                   rpkt_tun_t* __restrict__ tun, rpkt_rec_t* __restrict__ inner,
                   uint64_t* __restrict__ flow_ev, uint32_t n_buckets) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t p0 = blockIdx.x * kWave;
    if (p0 >= n) return;                                          // wave-uniform exit
    tunnel_tile<L4>(scratch, frames, fb, offsets, stride, frame_len, n, flags, outer, tun,
                    inner, flow_ev, n_buckets, p0, lane);
}

// A ring of tunnelled bursts in one launch (rpkt_gpu_parse_tunnel_ring): wave t takes
// tile t of the ring's tiles, numbered slot after slot (tile0[k] = the first tile of slot
// k), and parses it exactly as tunnel_kernel parses that tile of the slot's own batch.  The
// slot descriptors are kernel arguments (2.2 KB), read with scalar loads.
constexpr uint32_t kTunRingMax = RPKT_RING_MAX_SLOTS;
struct TunRingSlot {
    const uint8_t* frames;
    const uint32_t* offsets;
    rpkt_rec_t* outer;
    rpkt_tun_t* tun;
    rpkt_rec_t* inner;
    uint64_t* flow_ev;
    uint32_t frames_bytes, stride, frame_len, n;
};
struct TunRingArgs {
    uint32_t n_slots;
    uint32_t tile0[kTunRingMax + 1];
    TunRingSlot s[kTunRingMax];
};

template <bool L4>
__global__ __launch_bounds__(kWave, 2)
void tunnel_ring_kernel(const TunRingArgs A, uint32_t flags, uint32_t n_buckets) {
    __shared__ __attribute__((aligned(16))) WaveScratch scratch;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t t = blockIdx.x;
    if (t >= A.tile0[A.n_slots]) return;                         // wave-uniform exit
    uint32_t k = 0;                                               // the slot holding tile t
    for (uint32_t j = 1; j < A.n_slots; ++j) k = A.tile0[j] <= t ? j : k;
    const TunRingSlot& S = A.s[k];
    tunnel_tile<L4>(scratch, S.frames, S.frames_bytes, S.offsets, S.stride, S.frame_len, S.n,
                    flags, S.outer, S.tun, S.inner, S.flow_ev, n_buckets,
                    (t - A.tile0[k]) * kWave, lane);
}

constexpr uint32_t kTunFlags = RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_IPV6 | RPKT_F_FLOW_EV;

// one batch's argument checks (rpkt_gpu_parse_tunnel_batch's, and each slot's of a ring):
// 1 = launch it, else the status to return
int tunnel_args_ok(const rpkt_batch_t& b, uint32_t flags, const void* outer, const void* tun,
                   const void* inner, const void* flow_ev, uint32_t n_buckets) {
    if (flags & RPKT_F_FLOW_EV) {
        if (!flow_ev || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS) return RPKT_E_INVAL;
        if (((uintptr_t)flow_ev & 7u) != 0) return RPKT_E_ALIGN;
    }
    if (b.n == 0) return RPKT_OK;
    if (!b.frames_dev || !outer || !tun || !inner) return RPKT_E_INVAL;
    if (b.frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b.offsets_dev && b.stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)outer | (uintptr_t)tun | (uintptr_t)inner) & 15u) return RPKT_E_ALIGN;
    return 1;
}

}  // namespace

extern "C" {

int rpkt_gpu_parse_tunnel_batch(const rpkt_batch_t* b, uint32_t flags, rpkt_rec_t* outer_dev,
                                rpkt_tun_t* tun_dev, rpkt_rec_t* inner_dev,
                                rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream) {
    if (!b) return RPKT_E_INVAL;
    if (flags & ~kTunFlags) return RPKT_E_INVAL;
    const int ok = tunnel_args_ok(*b, flags, outer_dev, tun_dev, inner_dev, flow_ev_dev, n_buckets);
    if (ok != 1) return ok;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t grid = (b->n + kWave - 1) / kWave;
    auto k = (flags & RPKT_F_L4_SUM) ? tunnel_kernel<true> : tunnel_kernel<false>;
    return launch(k, dim3(grid), dim3(kWave), 0, (hipStream_t)stream, b->frames_dev,
                  (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n, flags, outer_dev,
                  tun_dev, inner_dev, (uint64_t*)flow_ev_dev, n_buckets);
}

int rpkt_gpu_parse_tunnel_ring(const rpkt_tun_ring_slot_t* slots, uint32_t n_slots,
                               uint32_t flags, uint32_t n_buckets, void* stream) {
    if (n_slots && !slots) return RPKT_E_INVAL;
    if (flags & ~kTunFlags) return RPKT_E_INVAL;
    for (uint32_t k = 0; k < n_slots; ++k) {                      // all checked, then launched
        const rpkt_tun_ring_slot_t& q = slots[k];
        if (q.batch.n == 0) continue;
        const int ok = tunnel_args_ok(q.batch, flags, q.outer_dev, q.tun_dev, q.inner_dev,
                                      q.flow_ev_dev, n_buckets);
        if (ok != 1) return ok;
    }
    const bool fev = (flags & RPKT_F_FLOW_EV) != 0;
    auto kern = (flags & RPKT_F_L4_SUM) ? tunnel_ring_kernel<true> : tunnel_ring_kernel<false>;
    TunRingArgs A;
    uint32_t k0 = 0;
    while (k0 < n_slots) {
        A.n_slots = 0;
        A.tile0[0] = 0;
        for (; k0 < n_slots && A.n_slots < kTunRingMax; ++k0) {
            const rpkt_tun_ring_slot_t& q = slots[k0];
            const rpkt_batch_t& b = q.batch;
            if (b.n == 0) continue;
            TunRingSlot& S = A.s[A.n_slots];
            S.frames = b.frames_dev;
            S.offsets = b.offsets_dev;
            S.outer = q.outer_dev;
            S.tun = q.tun_dev;
            S.inner = q.inner_dev;
            S.flow_ev = fev ? (uint64_t*)q.flow_ev_dev : nullptr;
            S.frames_bytes = (uint32_t)b.frames_bytes;
            S.stride = b.stride;
            S.frame_len = b.offsets_dev ? 0u : (b.frame_len ? b.frame_len : b.stride);
            S.n = b.n;
            A.tile0[A.n_slots + 1] = A.tile0[A.n_slots] + (b.n + kWave - 1) / kWave;
            ++A.n_slots;
        }
        if (A.n_slots == 0) break;
        const int rc = launch(kern, dim3(A.tile0[A.n_slots]), dim3(kWave), 0, (hipStream_t)stream,
                              A, flags, n_buckets);
        if (rc) return rc;
    }
    return RPKT_OK;
}

}  // extern "C"
