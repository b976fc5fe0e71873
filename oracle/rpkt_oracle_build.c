/*
 * rpkt_oracle_build.c — CPU restatement of rpkt's build (TX) side and of the
 * loopback_rx forwarding rewrite.  TEST INFRASTRUCTURE ONLY (tests/, bench.py's
 * cpu_baseline leg); the product (librpkt_gpu.so) never links it.
 *
 * Build: benches/rpkt/rpkt_build.rs:9-28 and rpkt-dpdk/examples/loopback_tx.rs:70-99
 * build a frame inside-out on a cursor that starts at the payload:
 *   Udp|Tcp::prepend_header(template) + setters, Ipv4::prepend_header(template)
 *   + setters, [VlanFrame::prepend_header + setters]*, EtherFrame::prepend_header
 *   + setters.
 * prepend_header moves the cursor back by the header length, copies the 20/8/4/14-B
 * template and sets the length fields from remaining() (ipv4/generated.rs:130-140,
 * udp/generated.rs:79-88, tcp/generated.rs:135-141, vlan/generated.rs:73-78,
 * ether/generated.rs:71-76).  Option bytes (IHL/doff above 5) are not written by
 * prepend_header: they stay as the buffer holds them.  The setter values come from
 * an rpkt_rec_t (the parse record layout), so build(parse(frame)) reproduces a frame.
 * Checksums are filled the way the NIC's TX offload requested by the reference
 * (loopback_rx.rs:133, PKT_TX_IP_CKSUM | PKT_TX_UDP_CKSUM) computes them: the field
 * zeroed, the complement of checksum::from_slice / combine (rpkt/src/checksum.rs:33-74)
 * over the header (IPv4) or pseudo header + segment (UDP/TCP); a UDP result of 0 is
 * sent as 0xffff (RFC 768).
 *
 * IPv6 records (the record's IPv6 block, include/rpkt_gpu.h) are built the same way
 * with Ipv6::prepend_header + setters (rpkt/src/ipv6/generated.rs:94-135) in place of
 * the IPv4 ones: the 40-B template, payload_len = remaining() after the header
 * (:96-105), set_version/traffic_class/flow_label from ip6_vtcfl (:107-123),
 * set_next_header (:125), set_hop_limit (:129).  The record holds the addresses only
 * folded, so the 32 address bytes are left as the buffer holds them (like option bytes),
 * and so are the extension headers between the IPv6 header and l4_off (their own
 * prepend_headers, :282, :425, :581, :743, are the caller's, as the IPv4 options are).
 * The L4 checksum uses the IPv6 pseudo header (src, the address at ip6_pdst_off, u32
 * upper-layer length, next header); a UDP result of 0 is sent as 0xffff, which over IPv6
 * is mandatory (RFC 8200 section 8.1: a zero UDP checksum is never emitted).
 *
 * Forward: rpkt-dpdk/examples/loopback_rx.rs:96-140 per frame, with the NIC's RX
 * checksum verdict bits (:99, :103, :108) replaced by the verify composition (the
 * record's ip_sum / l4_sum) and its TX checksum offload by a full recompute here.
 * With ip6 set (rpkt_fwd_t.flags = RPKT_F_IPV6) an untagged IPv6/UDP frame is forwarded
 * the same way: parsed OK, L4 sum valid (a zero UDP checksum is invalid over IPv6),
 * source not forbidden (the list holds IPv4 addresses: an IPv6 source never matches);
 * addresses and ports swapped, hop_limit - 1 (wrapping), MACs set, UDP checksum
 * recomputed over the IPv6 pseudo header.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include "../include/rpkt_gpu.h"

uint16_t oracle_from_slice(const uint8_t* data, size_t len);
int oracle_rec_is_ip6(const rpkt_rec_t* r);
uint16_t oracle_combine(const uint16_t* checksums, size_t n);
uint16_t oracle_pseudo_header_v4(const uint8_t* src4, const uint8_t* dst4, uint8_t proto,
                                 uint16_t length);
uint16_t oracle_pseudo_header_v6(const uint8_t* src16, const uint8_t* dst16, uint8_t proto,
                                 uint32_t length);

static void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* Templates, rpkt/src/{udp,tcp,ipv4,vlan,ether}/generated.rs:11-15 */
static const uint8_t UDP_T[8] = {0, 0, 0, 0, 0, 8, 0, 0};
static const uint8_t TCP_T[20] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x50, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t IPV4_T[20] = {0x45, 0, 0, 0x14, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t VLAN_T[4] = {0x00, 0x01, 0x08, 0x00};
static const uint8_t ETHER_T[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x08, 0x00};
/* rpkt/src/ipv6/generated.rs:16-20 */
static const uint8_t IPV6_T[40] = {0x60, 0, 0, 0, 0, 0, 0x04, 0};

/* The IPv6 block of a record (include/rpkt_gpu.h: bytes 24..43 of an IPv6 record) */
static uint32_t rec_u32(const rpkt_rec_t* r, int at) {
    uint32_t v;
    memcpy(&v, (const uint8_t*)r + at, 4);
    return v;
}
static uint16_t rec_u16(const rpkt_rec_t* r, int at) {
    uint16_t v;
    memcpy(&v, (const uint8_t*)r + at, 2);
    return v;
}

/* Udp|Tcp::prepend_header + setters at f + l4 (the L4 header bytes of the record) */
static void emit_l4(uint8_t* f, uint32_t len, uint32_t l4, const rpkt_rec_t* r) {
    if (r->ip_protocol == 17) {                             /* Udp::prepend_header :79-88 */
        uint8_t* u = f + l4;
        memcpy(u, UDP_T, 8);
        put16(u + 4, len - l4);                             /* set_packet_len(remaining) */
        put16(u + 0, r->src_port);                          /* set_src_port :90 */
        put16(u + 2, r->dst_port);                          /* set_dst_port :94 */
        put16(u + 6, r->l4_checksum);                       /* set_checksum */
    } else if (r->ip_protocol == 6) {                       /* Tcp::prepend_header :135-141 */
        uint8_t* t = f + l4;
        memcpy(t, TCP_T, 20);
        put16(t + 0, r->src_port);                          /* :148-155 */
        put16(t + 2, r->dst_port);
        put32(t + 4, r->tcp_seq);                           /* set_seq_num :156 */
        put32(t + 8, r->tcp_ack);                           /* set_ack_num :160 */
        put16(t + 12, r->l4_word6);                         /* header_len, reserved, flags :164-224 */
        put16(t + 14, r->tcp_window);                       /* set_window_size :209 */
        put16(t + 16, r->l4_checksum);                      /* set_checksum :213 */
        put16(t + 18, r->tcp_urgent);                       /* set_urgent_pointer :217 */
    }
}

/* [VlanFrame::prepend_header + setters]*, EtherFrame::prepend_header + setters */
static void emit_link(uint8_t* f, uint32_t nv, const rpkt_rec_t* r) {
    for (int k = (int)nv - 1; k >= 0; k--) {                /* VlanFrame::prepend_header :73-78 */
        uint8_t* v = f + 14 + 4 * k;
        memcpy(v, VLAN_T, 4);
        put16(v, r->vlan_tci[k]);                           /* priority / dei / vlan_id */
        put16(v + 2, r->vlan_ethertype[k]);                 /* set_ethertype */
    }
    memcpy(f, ETHER_T, 14);                                 /* EtherFrame::prepend_header :71-76 */
    memcpy(f, r->dst_addr, 6);                              /* set_dst_addr :78 */
    memcpy(f + 6, r->src_addr, 6);                          /* set_src_addr :82 */
    put16(f + 12, r->ethertype);                            /* set_ethertype :86 */
}

/* The IPv6 record's build (Ipv6::prepend_header + setters, ipv6/generated.rs:94-135). */
static int build_one6(uint8_t* f, uint32_t len, const rpkt_rec_t* r, uint32_t flags) {
    uint32_t nv = r->n_vlan;
    uint32_t l3 = 14 + 4 * nv;
    uint32_t l4 = r->l4_off;
    uint32_t proto = r->ip_protocol;
    uint32_t l4hdr = proto == 17 ? 8 : (proto == 6 ? (uint32_t)(r->l4_word6 >> 12) * 4 : 0);
    if (l4 < l3 + 40) return 0;                             /* no IPv6 header parsed */
    if (proto == 6 && l4hdr < 20) return 0;                 /* tcp/generated.rs:137 */
    if (len < l4 + l4hdr) return 0;                         /* chunk_headroom asserts */
    if (len - l3 - 40 > 65535) return 0;                    /* ipv6/generated.rs:99 */
    if (proto == 17 && len - l4 > 65535) return 0;          /* udp/generated.rs:83 */
    emit_l4(f, len, l4, r);
    uint8_t* ip = f + l3;                                   /* Ipv6::prepend_header :96-105 */
    uint8_t addrs[32];
    memcpy(addrs, ip + 8, 32);                              /* the buffer's addresses */
    memcpy(ip, IPV6_T, 40);
    memcpy(ip + 8, addrs, 32);
    put16(ip + 4, len - l3 - 40);                           /* set_payload_len(remaining) */
    put32(ip, rec_u32(r, 24));                              /* version, traffic_class, flow_label */
    ip[6] = ((const uint8_t*)r)[30];                        /* set_next_header :125 */
    ip[7] = ((const uint8_t*)r)[31];                        /* set_hop_limit :129 */
    emit_link(f, nv, r);
    if ((flags & RPKT_BUILD_L4_CSUM) && (proto == 17 || proto == 6)) {
        uint32_t pdst = rec_u16(r, 34);
        /* an address the parse can report lies between dst_addr and the L4 header;
         * any other value (a record no parse produced) falls back to dst_addr */
        if (pdst < l3 + 24 || pdst + 16 > l4) pdst = l3 + 24;
        uint32_t ck_off = proto == 17 ? 6 : 16;
        uint32_t seg = len - l4;
        put16(f + l4 + ck_off, 0);
        uint16_t parts[2] = {oracle_pseudo_header_v6(ip + 8, f + pdst, (uint8_t)proto, seg),
                             oracle_from_slice(f + l4, seg)};
        uint16_t ck = (uint16_t)~oracle_combine(parts, 2);
        if (proto == 17 && ck == 0) ck = 0xffff;            /* RFC 8200 section 8.1 */
        put16(f + l4 + ck_off, ck);
    }
    return 1;
}

/* Build one frame of `len` bytes in place.  Returns 1 if written, 0 if the frame
 * cannot hold the headers the record asks for (where the reference's
 * prepend_header would assert) — the frame is then left untouched. */
int oracle_build_one(uint8_t* f, uint32_t len, const rpkt_rec_t* r, uint32_t flags) {
    uint32_t nv = r->n_vlan;
    if (nv > RPKT_MAX_VLAN) return 0;
    if (oracle_rec_is_ip6(r)) return build_one6(f, len, r, flags);
    uint32_t l3 = 14 + 4 * nv;
    uint32_t ihl4 = (uint32_t)(r->ip_vhl & 0xf) * 4;
    uint32_t l4 = l3 + ihl4;
    uint32_t proto = r->ip_protocol;
    uint32_t l4hdr = proto == 17 ? 8 : (proto == 6 ? (uint32_t)(r->l4_word6 >> 12) * 4 : 0);
    if (ihl4 < 20) return 0;                                /* ipv4/generated.rs:132 */
    if (proto == 6 && l4hdr < 20) return 0;                 /* tcp/generated.rs:137 */
    if (len < l4 + l4hdr) return 0;                         /* chunk_headroom asserts */
    if (len - l3 > 65535) return 0;                         /* ipv4/generated.rs:135 */
    if (proto == 17 && len - l4 > 65535) return 0;          /* udp/generated.rs:83 */

    /* cursor = l4 + l4hdr (the payload); build inside-out */
    emit_l4(f, len, l4, r);
    uint8_t* ip = f + l3;                                   /* Ipv4::prepend_header :130-140 */
    memcpy(ip, IPV4_T, 20);
    ip[0] = r->ip_vhl;                                      /* set_version / set_header_len */
    put16(ip + 2, len - l3);                                /* set_packet_len(remaining) */
    ip[1] = r->ip_tos;                                      /* set_dscp / set_ecn */
    put16(ip + 4, r->ip_ident);                             /* set_ident */
    put16(ip + 6, r->ip_frag);                              /* flags + set_frag_offset */
    ip[8] = r->ip_ttl;                                      /* set_ttl */
    ip[9] = r->ip_protocol;                                 /* set_protocol */
    put16(ip + 10, r->ip_checksum);                         /* set_checksum */
    put32(ip + 12, r->ip_src);                              /* set_src_addr */
    put32(ip + 16, r->ip_dst);                              /* set_dst_addr */
    emit_link(f, nv, r);

    if (flags & RPKT_BUILD_IP_CSUM) {                       /* TX IP checksum offload */
        put16(ip + 10, 0);
        put16(ip + 10, (uint16_t)~oracle_from_slice(ip, ihl4));
    }
    if ((flags & RPKT_BUILD_L4_CSUM) && (proto == 17 || proto == 6)) {
        uint32_t ck_off = proto == 17 ? 6 : 16;
        uint32_t seg = len - l4;
        put16(f + l4 + ck_off, 0);
        uint16_t parts[2] = {oracle_pseudo_header_v4(ip + 12, ip + 16, (uint8_t)proto,
                                                     (uint16_t)seg),
                             oracle_from_slice(f + l4, seg)};
        uint16_t ck = (uint16_t)~oracle_combine(parts, 2);
        if (proto == 17 && ck == 0) ck = 0xffff;
        put16(f + l4 + ck_off, ck);
    }
    return 1;
}

/* The encapsulation build (rpkt_gpu_build_tunnel_batch): the tunnel header written first
 * at the outer UDP payload (VXLAN, GTP-U) or at l4 (GRE), as the reference's build tests
 * prepend it before the outer headers (vlan_mpls_tests.rs:254-300, gtpv1_test.rs:236-282,
 * gre_test.rs:213-278), then oracle_build_one (whose UDP checksum fill covers it), then a
 * GRE checksum fill.  Templates: VXLAN_HEADER_TEMPLATE all zero (vxlan/generated.rs:12),
 * GTPV1_HEADER_TEMPLATE, the GRE template; the setter values from the rpkt_tun_t. */
int oracle_build_tunnel_one(uint8_t* f, uint32_t len, const rpkt_rec_t* r, const rpkt_tun_t* t,
                            uint32_t flags) {
    if (t->kind == RPKT_TUN_NONE) return oracle_build_one(f, len, r, flags);
    if (t->kind > RPKT_TUN_GRE || r->n_vlan > RPKT_MAX_VLAN) return 0;
    const uint32_t l3 = 14 + 4 * (uint32_t)r->n_vlan;
    const uint32_t l4 = oracle_rec_is_ip6(r) ? r->l4_off : l3 + (uint32_t)(r->ip_vhl & 0xf) * 4;
    const uint32_t h0 = t->hdr0;
    uint32_t ts, hl;
    if (t->kind == RPKT_TUN_GRE) {
        if (r->ip_protocol != 47) return 0;
        ts = l4;
        hl = 4 + ((h0 & 0xc0) ? 4 : 0) + ((h0 & 0x20) ? 4 : 0) + ((h0 & 0x10) ? 4 : 0);  /* gre/mod.rs:68-85 */
    } else {
        if (r->ip_protocol != 17) return 0;
        ts = l4 + 8;                                        /* Udp::payload */
        hl = t->kind == RPKT_TUN_VXLAN ? 8 : ((h0 & 7) ? 12 : 8);   /* Gtpv1::header_len :239-250 */
    }
    if (ts + hl > len || ts + hl > RPKT_TUN_BUILD_MAX_END) return 0;
    if (t->kind == RPKT_TUN_GTPU && len - ts > 65543) return 0;     /* gtpv1/generated.rs:116 */
    uint8_t tmp[65536 + 16];
    if (len > sizeof(tmp)) return 0;
    memcpy(tmp, f, len);
    uint8_t* h = tmp + ts;
    const int gre_fill = t->kind == RPKT_TUN_GRE && (flags & RPKT_BUILD_L4_CSUM) && (h0 & 0x80);
    if (t->kind == RPKT_TUN_VXLAN) {
        memset(h, 0, 8);                                    /* Vxlan::prepend_header :99-105 */
        h[0] = t->hdr0;                                     /* set_gbp_extention, set_vni_present .. */
        h[1] = t->hdr1;                                     /* set_dont_learn, set_policy_applied .. */
        put16(h + 2, t->aux);                               /* set_group_id */
        h[4] = (uint8_t)(t->id >> 16); h[5] = (uint8_t)(t->id >> 8); h[6] = (uint8_t)t->id;  /* set_vni */
    } else if (t->kind == RPKT_TUN_GTPU) {
        h[0] = t->hdr0;                                     /* Gtpv1::prepend_header :112-122: */
        h[1] = t->hdr1;                                     /*   the 8-B header given, then */
        put16(h + 2, len - ts - 8);                         /*   set_packet_len(remaining) */
        put32(h + 4, t->id);                                /* set_teid :160 */
        if (hl == 12) put16(h + 8, t->aux);                 /* set_sequence :287-290 */
    } else {
        h[0] = t->hdr0;                                     /* Gre::prepend_header + flag setters */
        h[1] = t->hdr1;
        put16(h + 2, t->inner_type);                        /* set_protocol_type */
        const uint32_t cr = (h0 & 0xc0) ? 4 : 0;
        if (cr) put16(h + 4, gre_fill ? 0 : t->aux);        /* set_checksum */
        if (h0 & 0x20) put32(h + 4 + cr, t->id);            /* set_key */
    }
    if (!oracle_build_one(tmp, len, r, flags)) return 0;
    if (gre_fill) put16(tmp + ts + 4, (uint16_t)~oracle_from_slice(tmp + ts, len - ts));
    memcpy(f, tmp, len);
    return 1;
}

static void span(uint64_t frames_bytes, const uint32_t* offsets, uint32_t stride,
                 uint32_t frame_len, uint32_t i, uint64_t* off, uint64_t* len) {
    if (offsets) {
        *off = offsets[i];
        *len = offsets[i + 1] >= offsets[i] ? offsets[i + 1] - offsets[i] : 0;
    } else {
        *off = (uint64_t)i * stride;
        *len = frame_len ? frame_len : stride;
    }
    if (*off > frames_bytes) *off = frames_bytes;
    if (*off + *len > frames_bytes) *len = frames_bytes - *off;
}

void oracle_build_batch(uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                        uint32_t stride, uint32_t frame_len, uint32_t n, const rpkt_rec_t* recs,
                        uint32_t flags, uint8_t* built) {
    for (uint32_t i = 0; i < n; i++) {
        uint64_t off, len;
        span(frames_bytes, offsets, stride, frame_len, i, &off, &len);
        int b = oracle_build_one(frames + off, (uint32_t)len, &recs[i], flags);
        if (built) built[i] = (uint8_t)b;
    }
}

/* The IPv6 counterpart of the loopback_rx rewrite (rpkt_fwd_t.flags & RPKT_F_IPV6):
 * an untagged IPv6/UDP frame that parsed OK with a valid L4 sum. */
static int forward_one6(uint8_t* f, uint32_t len, const rpkt_rec_t* r, const uint8_t* dmac,
                        const uint8_t* smac) {
    if (r->n_vlan) return 0;                               /* :101 ethertype() == IPV6 */
    if (r->ip_protocol != 17) return 0;                    /* :106 next header UDP */
    if (r->l4_sum != 0xffff) return 0;                     /* :107 L4 good (no 0 exemption) */
    uint32_t l3 = r->l3_off, l4 = r->l4_off;
    if (len < l4 + 8) return 0;
    uint8_t* ip = f + l3;
    uint8_t* u = f + l4;
    uint8_t a[16];
    put16(u + 0, r->dst_port);                             /* swap ports */
    put16(u + 2, r->src_port);
    memcpy(a, ip + 8, 16);                                 /* swap addresses */
    memcpy(ip + 8, ip + 24, 16);
    memcpy(ip + 24, a, 16);
    ip[7] = (uint8_t)(ip[7] - 1);                          /* hop_limit - 1 (wrapping) */
    memcpy(f, dmac, 6);
    memcpy(f + 6, smac, 6);
    uint32_t pdst = rec_u16(r, 34);                        /* final address (routing header) */
    uint32_t seg = (uint32_t)r->l4_word6;                  /* the UDP datagram (length field) */
    put16(u + 6, 0);
    uint16_t parts[2] = {oracle_pseudo_header_v6(ip + 8, f + pdst, 17, seg),
                         oracle_from_slice(u, seg)};
    uint16_t ck = (uint16_t)~oracle_combine(parts, 2);
    put16(u + 6, ck == 0 ? 0xffff : ck);
    return 1;
}

/* loopback_rx.rs:96-140 over one parsed frame.  Returns 1 when the frame is
 * forwarded (rewritten in place), 0 when the reference would drop it.  ip6: also
 * forward IPv6 frames (records of an RPKT_F_IPV6 parse). */
int oracle_forward_one(uint8_t* f, uint32_t len, const rpkt_rec_t* r, const uint8_t* dmac,
                       const uint8_t* smac, const uint32_t* forbid, uint32_t n_forbid, int ip6) {
    if (r->status != RPKT_S_OK) return 0;                  /* every parse Ok */
    if (ip6 && oracle_rec_is_ip6(r)) return forward_one6(f, len, r, dmac, smac);
    if (r->ethertype != 0x0800 || r->n_vlan) return 0;     /* :101 ethertype() == IPV4 */
    if (r->ip_sum != 0xffff) return 0;                     /* :101 rx_offload IP good */
    if (r->ip_protocol != 17) return 0;                    /* :106 protocol() == UDP */
    if (r->l4_sum != 0xffff && r->l4_checksum != 0) return 0;   /* :107 rx_offload L4 good */
    for (uint32_t k = 0; k < n_forbid; k++)                /* :111-118 forbidden source */
        if (forbid[k] == r->ip_src) return 0;
    uint32_t l3 = r->l3_off, l4 = r->l4_off, ihl4 = l4 - l3;
    if (len < l4 + 8) return 0;
    uint8_t* ip = f + l3;
    uint8_t* u = f + l4;
    put16(u + 0, r->dst_port);                             /* :122-124 swap ports */
    put16(u + 2, r->src_port);
    put32(ip + 12, r->ip_dst);                             /* :126-129 swap addresses */
    put32(ip + 16, r->ip_src);
    ip[8] = (uint8_t)(r->ip_ttl - 1);                      /* :130 ttl - 1 (wrapping) */
    memcpy(f, dmac, 6);                                    /* :132-133 */
    memcpy(f + 6, smac, 6);
    /* TX offload (:135): IP and UDP checksums recomputed over the rewritten bytes */
    put16(ip + 10, 0);
    put16(ip + 10, (uint16_t)~oracle_from_slice(ip, ihl4));
    uint32_t seg = (uint32_t)r->l4_word6;                  /* the UDP datagram (length field) */
    put16(u + 6, 0);
    uint16_t parts[2] = {oracle_pseudo_header_v4(ip + 12, ip + 16, 17, (uint16_t)seg),
                         oracle_from_slice(u, seg)};
    uint16_t ck = (uint16_t)~oracle_combine(parts, 2);
    put16(u + 6, ck == 0 ? 0xffff : ck);
    return 1;
}

void oracle_forward_batch(uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                          uint32_t stride, uint32_t frame_len, uint32_t n, const rpkt_rec_t* recs,
                          const uint8_t* dmac, const uint8_t* smac, const uint32_t* forbid,
                          uint32_t n_forbid, uint8_t* keep, uint32_t fwd_flags) {
    for (uint32_t i = 0; i < n; i++) {
        uint64_t off, len;
        span(frames_bytes, offsets, stride, frame_len, i, &off, &len);
        keep[i] = (uint8_t)oracle_forward_one(frames + off, (uint32_t)len, &recs[i], dmac, smac,
                                              forbid, n_forbid,
                                              (fwd_flags & RPKT_F_IPV6) != 0);
    }
}

void oracle_build_tunnel_batch(uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                               uint32_t stride, uint32_t frame_len, uint32_t n,
                               const rpkt_rec_t* recs, const rpkt_tun_t* tun, uint32_t flags,
                               uint8_t* built) {
    for (uint32_t i = 0; i < n; i++) {
        uint64_t off, len;
        span(frames_bytes, offsets, stride, frame_len, i, &off, &len);
        int b = oracle_build_tunnel_one(frames + off, (uint32_t)len, &recs[i], &tun[i], flags);
        if (built) built[i] = (uint8_t)b;
    }
}
