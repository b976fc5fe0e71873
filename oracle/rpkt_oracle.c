/*
 * rpkt_oracle.c — CPU restatement of rpkt's Ether/VLAN/IPv4/{TCP,UDP} parse and
 * RFC 1071 checksum path.  TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load this as the checker; the product path
 * (rpkt_amd/, librpkt_gpu.so) never links or calls it.
 *
 * The reference is Rust and cannot be compiled in this image (no cargo/rustc),
 * so this file restates it line by line.  Parity is pinned by the reference's
 * own fixtures (rpkt/tests/packet_examples/NAME.dat, copied to tests/golden/) and
 * the getter values its tests assert (tests/golden/expected.json), plus the
 * checksum fields real network stacks stored in those captures (a correctly
 * computed sum over a frame with a valid stored checksum is 0xffff).
 *
 * Every function cites the reference lines it follows.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>

#include "../include/rpkt_gpu.h"

/* ------------------------------------------------------------------------- */
/* checksum.rs                                                                */
/* ------------------------------------------------------------------------- */

/* propagate_carries, rpkt/src/checksum.rs:115-118 */
uint16_t oracle_propagate_carries(uint32_t word) {
    uint32_t sum = (word >> 16) + (word & 0xffff);
    return (uint16_t)((uint16_t)(sum >> 16) + (uint16_t)sum);
}

/* from_slice, rpkt/src/checksum.rs:33-62 (32-byte chunk loop kept as written) */
uint16_t oracle_from_slice(const uint8_t* data, size_t len) {
    uint32_t accum = 0;
    const size_t CHUNK_SIZE = 32;
    while (len >= CHUNK_SIZE) {                       /* :38 */
        const uint8_t* d = data;
        size_t dl = CHUNK_SIZE;
        while (dl >= 2) {                             /* :41-44 */
            accum += ((uint32_t)d[0] << 8) | d[1];
            d += 2;
            dl -= 2;
        }
        data += CHUNK_SIZE;                           /* :46 */
        len -= CHUNK_SIZE;
    }
    while (len >= 2) {                                /* :51-54 */
        accum += ((uint32_t)data[0] << 8) | data[1];
        data += 2;
        len -= 2;
    }
    if (len == 1) {                                   /* :57-59 */
        accum += (uint32_t)data[0] << 8;
    }
    return oracle_propagate_carries(accum);                  /* :61 */
}

/* combine, rpkt/src/checksum.rs:68-74 */
uint16_t oracle_combine(const uint16_t* checksums, size_t n) {
    uint32_t accum = 0;
    for (size_t i = 0; i < n; i++) accum += checksums[i];
    return oracle_propagate_carries(accum);
}

/* from_slice_with_tail_byte, rpkt/src/checksum.rs:77-111.
 * tail_in < 0 means None.  Returns the new tail byte or -1 (None). */
int oracle_from_slice_with_tail_byte(const uint8_t* data, size_t len, uint32_t* accum,
                                     int tail_in) {
    if (tail_in >= 0) {                               /* :82-88 */
        *accum += ((uint32_t)(uint8_t)tail_in << 8) | data[0];
        data += 1;
        len -= 1;
    }
    const size_t CHUNK_SIZE = 32;
    while (len >= CHUNK_SIZE) {                       /* :92-101 */
        for (size_t i = 0; i < CHUNK_SIZE; i += 2)
            *accum += ((uint32_t)data[i] << 8) | data[i + 1];
        data += CHUNK_SIZE;
        len -= CHUNK_SIZE;
    }
    while (len >= 2) {                                /* :105-108 */
        *accum += ((uint32_t)data[0] << 8) | data[1];
        data += 2;
        len -= 2;
    }
    return len == 1 ? data[0] : -1;                   /* :110 */
}

/* from_buf over a multi-segment buffer, rpkt/src/checksum.rs:8-27.
 * Segments are (ptr, len) pairs; `len` limits the total (Buf::take, :9). */
uint16_t oracle_from_buf(const uint8_t* const* segs, const size_t* seg_lens, size_t n_segs,
                         size_t len) {
    uint32_t accum = 0;
    int tail = -1;
    for (size_t s = 0; s < n_segs && len > 0; s++) {  /* :13-20 */
        size_t cl = seg_lens[s] < len ? seg_lens[s] : len;
        if (cl == 0) continue;
        tail = oracle_from_slice_with_tail_byte(segs[s], cl, &accum, tail);
        len -= cl;
    }
    if (tail >= 0) accum += (uint32_t)tail << 8;      /* :22-24 */
    return oracle_propagate_carries(accum);
}

/* ------------------------------------------------------------------------- */
/* cursors.rs: Cursor = [start, end) view over one frame                     */
/* ------------------------------------------------------------------------- */

typedef struct cursor {
    const uint8_t* base; /* Cursor::start_addr, cursors.rs:34-37 */
    size_t start;        /* cursor(), cursors.rs:56-59            */
    size_t end;          /* start + chunk.len()                   */
} cursor_t;

static size_t cur_remaining(const cursor_t* c) { return c->end - c->start; } /* :65-68 */
static const uint8_t* cur_chunk(const cursor_t* c) { return c->base + c->start; } /* :70-73 */

static void cur_advance(cursor_t* c, size_t cnt) {   /* cursors.rs:75-78 */
    if (cnt > cur_remaining(c)) { fprintf(stderr, "oracle: advance past end\n"); abort(); }
    c->start += cnt;
}
static void cur_trim_off(cursor_t* c, size_t cnt) {  /* cursors.rs:94-98 */
    if (cnt > cur_remaining(c)) { fprintf(stderr, "oracle: trim past end\n"); abort(); }
    c->end -= cnt;
}

static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* smoltcp pseudo_header_v4 as used by the verify composition:
 * combine(&[data(src), data(dst), data(&[0, proto, len_hi, len_lo])]).
 * smoltcp is the documented origin of checksum.rs (rpkt/src/checksum.rs:3). */
uint16_t oracle_pseudo_header_v4(const uint8_t* src4, const uint8_t* dst4, uint8_t proto,
                                 uint16_t length) {
    uint8_t proto_len[4] = {0, proto, (uint8_t)(length >> 8), (uint8_t)length};
    uint16_t parts[3] = {oracle_from_slice(src4, 4), oracle_from_slice(dst4, 4),
                         oracle_from_slice(proto_len, 4)};
    return oracle_combine(parts, 3);
}

/* smoltcp pseudo_header_v6 (the same origin; RFC 8200 section 8.1):
 * combine(&[data(src), data(dst), data(&(length as u32).to_be_bytes()),
 * data(&[0, 0, 0, next_header])]). */
uint16_t oracle_pseudo_header_v6(const uint8_t* src16, const uint8_t* dst16, uint8_t proto,
                                 uint32_t length) {
    uint8_t len_be[4] = {(uint8_t)(length >> 24), (uint8_t)(length >> 16), (uint8_t)(length >> 8),
                         (uint8_t)length};
    uint8_t nh[4] = {0, 0, 0, proto};
    uint16_t parts[4] = {oracle_from_slice(src16, 16), oracle_from_slice(dst16, 16),
                         oracle_from_slice(len_be, 4), oracle_from_slice(nh, 4)};
    return oracle_combine(parts, 4);
}

/* ------------------------------------------------------------------------- */
/* The decode chain for one frame                                             */
/* ------------------------------------------------------------------------- */

/* Udp::parse / Tcp::parse on the cursor the IP layer's payload() returned, getters,
 * the L4 sum with the pseudo header of the IP version (addresses src/dst, 4 or 16
 * bytes) and payload().  Shared by the IPv4 and IPv6 chains. */
static void oracle_parse_l4(cursor_t* buf, uint8_t proto, const uint8_t* src, const uint8_t* dst,
                            int v6, uint32_t flags, rpkt_rec_t* rec) {
    if (proto == 17) {
        /* Udp::parse, udp/generated.rs:31-42 */
        if (cur_remaining(buf) < 8) { rec->status = RPKT_S_UDP_SHORT; return; }
        const uint8_t* u = cur_chunk(buf);
        size_t ulen = be16(u + 4);                    /* packet_len :59-62 */
        if (ulen < 8 || ulen > cur_remaining(buf)) { rec->status = RPKT_S_UDP_BAD_LEN; return; }
        rec->src_port = be16(u);                      /* :48-51 */
        rec->dst_port = be16(u + 2);                  /* :52-55 */
        rec->l4_word6 = (uint16_t)ulen;
        rec->l4_checksum = be16(u + 6);               /* :56-58 */
        if (flags & RPKT_F_L4_SUM) {
            uint16_t parts[2] = {v6 ? oracle_pseudo_header_v6(src, dst, 17, (uint32_t)ulen)
                                    : oracle_pseudo_header_v4(src, dst, 17, (uint16_t)ulen),
                                 oracle_from_slice(u, ulen)};
            rec->l4_sum = oracle_combine(parts, 2);
        }
        /* Udp::payload, udp/generated.rs:66-76: trim to len, advance 8 */
        size_t ts = cur_remaining(buf) - ulen;
        if (ts > 0) cur_trim_off(buf, ts);
        cur_advance(buf, 8);
        rec->payload_off = (uint16_t)buf->start;
        rec->payload_len = (uint16_t)cur_remaining(buf);
        rec->status = RPKT_S_OK;
    } else if (proto == 6) {
        /* Tcp::parse, tcp/generated.rs:34-45 */
        size_t cl = cur_remaining(buf);
        if (cl < 20) { rec->status = RPKT_S_TCP_SHORT; return; }
        const uint8_t* t = cur_chunk(buf);
        size_t hl = (size_t)(t[12] >> 4) * 4;         /* header_len :119-121 */
        if (hl < 20 || hl > cl) { rec->status = RPKT_S_TCP_BAD_DOFF; return; }
        rec->src_port = be16(t);                      /* :55-62 */
        rec->dst_port = be16(t + 2);
        rec->tcp_seq = be32(t + 4);                   /* :63-66 */
        rec->tcp_ack = be32(t + 8);                   /* :67-70 */
        rec->l4_word6 = be16(t + 12);                 /* header_len/reserved/flags :71-106 */
        rec->tcp_window = be16(t + 14);               /* :107-110 */
        rec->l4_checksum = be16(t + 16);              /* :111-114 */
        rec->tcp_urgent = be16(t + 18);               /* :115-118 */
        if (flags & RPKT_F_L4_SUM) {
            uint16_t parts[2] = {v6 ? oracle_pseudo_header_v6(src, dst, 6, (uint32_t)cl)
                                    : oracle_pseudo_header_v4(src, dst, 6, (uint16_t)cl),
                                 oracle_from_slice(t, cl)};
            rec->l4_sum = oracle_combine(parts, 2);
        }
        cur_advance(buf, hl);                         /* Tcp::payload :125-131 (no trim) */
        rec->payload_off = (uint16_t)buf->start;
        rec->payload_len = (uint16_t)cur_remaining(buf);
        rec->status = RPKT_S_OK;
    } else {
        rec->status = RPKT_S_L4_OTHER;
        size_t n = cur_remaining(buf);
        const uint8_t* p = cur_chunk(buf);
        if (!v6 && proto == 1) {
            /* ICMP: calculate_icmp_checksum (icmpv4/generated.rs:2678-2701) over the IPv4
             * payload is the complement of from_slice over it (oracle_icmp_checksum below,
             * tests/test_oracle_golden.py); its `icmp_data.len() - 1` (:2684) panics on an
             * empty payload: that is a status here */
            if (n == 0) { rec->status = RPKT_S_ICMP_EMPTY; return; }
            if (flags & RPKT_F_L4_SUM) rec->l4_sum = oracle_from_slice(p, n);
        } else if (proto == 47 && n >= 4 && (p[0] & 0x80)) {
            /* GRE with checksum_present (gre/generated.rs:55): RFC 2784 section 2.5, the
             * sum over the GRE header and payload (Gre::checksum :239) */
            if (flags & RPKT_F_L4_SUM) rec->l4_sum = oracle_from_slice(p, n);
        }
    }
}

/* rpkt/src/icmpv4/generated.rs:2678-2701 calculate_icmp_checksum, restated line by line
 * (big-endian words, odd byte << 8, `while (checksum >> 16) != 0` fold, `!checksum as
 * u16`); returns -1 for the empty slice, where the reference's `len() - 1` panics. */
int oracle_icmp_checksum(const uint8_t* d, size_t len) {
    if (len == 0) return -1;
    uint32_t checksum = 0;
    size_t i = 0;
    while (i < len - 1) {
        checksum += ((uint32_t)d[i] << 8) | d[i + 1];
        i += 2;
    }
    if (i < len) checksum += (uint32_t)d[i] << 8;
    while ((checksum >> 16) != 0) checksum = (checksum & 0xFFFF) + (checksum >> 16);
    return (uint16_t)~checksum;
}

static uint32_t fold_be32x4(const uint8_t* a) {
    return be32(a) ^ be32(a + 4) ^ be32(a + 8) ^ be32(a + 12);
}

/* The IPv6 chain from the cursor at the IPv6 header (RPKT_F_IPV6; include/rpkt_gpu.h
 * documents the record's IPv6 block).  Ipv6::parse ipv6/generated.rs:40-51, getters
 * :57-80 and :194-205, Ipv6::payload :83-92; then the extension headers a receive loop
 * steps through (ipv6_test.rs:27-76, 137-178, 233-269, 327-352, 397-421): each is the
 * generated parse of its type and payload() = advance(header_len), until the next
 * header is not an extension type. */
static void oracle_parse_ip6(cursor_t* buf, uint32_t flags, rpkt_rec_t* rec) {
    rec->l3_off = (uint16_t)buf->start;
    size_t chunk_len = cur_remaining(buf);
    if (chunk_len < 40) { rec->status = RPKT_S_IP6_SHORT; return; }          /* :42 */
    const uint8_t* ip = cur_chunk(buf);
    size_t payload_len = be16(ip + 4);                                        /* :77-79 */
    if (payload_len + 40 > cur_remaining(buf)) { rec->status = RPKT_S_IP6_BAD_LEN; return; } /* :47 */
    /* record block: ip_vhl..ip_dst reinterpreted (rpkt_rec_t bytes 24..43) */
    uint8_t* blk = (uint8_t*)rec + 24;
    uint32_t vtcfl = be32(ip);                       /* version :57-59, traffic_class :61-63,
                                                        flow_label :65-67 */
    uint16_t pl = (uint16_t)payload_len;
    uint16_t pdst_off = (uint16_t)(buf->start + 24);
    uint32_t sf = fold_be32x4(ip + 8), df = fold_be32x4(ip + 24);   /* src/dst :196-204 */
    memcpy(blk + 0, &vtcfl, 4);
    memcpy(blk + 4, &pl, 2);
    blk[6] = ip[6];                                  /* next_header :69-71 */
    blk[7] = ip[7];                                  /* hop_limit :73-75 */
    memcpy(blk + 12, &sf, 4);
    memcpy(blk + 16, &df, 4);
    const uint8_t* pdst = ip + 24;

    /* Ipv6::payload, :83-92: trim to 40 + payload_len, advance 40 */
    size_t trim_size = cur_remaining(buf) - (40 + payload_len);
    if (trim_size > 0) cur_trim_off(buf, trim_size);
    cur_advance(buf, 40);

    uint8_t nh = ip[6];
    uint8_t n_ext = 0;
    int stop = 0;
    for (; n_ext < RPKT_MAX_IP6_EXT; n_ext++) {
        size_t cl = cur_remaining(buf);
        const uint8_t* h = cur_chunk(buf);
        size_t hl;
        if (nh == 0 || nh == 60) {
            /* HopByHopOption::parse :384-395 / DestOptions::parse :241-252:
             * chunk_len >= 2, header_len = b1 * 8 + 8 (:410-412, :267-269) <= chunk_len */
            if (cl < 2) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (size_t)h[1] * 8 + 8;
            if (hl < 2 || hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
        } else if (nh == 43) {
            /* RoutingHeader::parse :528-539, header_len :566-568 */
            if (cl < 8) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (size_t)h[1] * 8 + 8;
            if (hl < 8 || hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
            /* segments_left :558-560 > 0: the pseudo header's destination is the final
             * address (RFC 8200 section 8.1); type_ :554-556 */
            if (h[3] > 0) {
                size_t n_addr = (hl - 8) / 16;
                if (h[2] == 4 && n_addr >= 1) pdst = h + 8;                        /* SRH */
                else if ((h[2] == 0 || h[2] == 2) && n_addr >= 1) pdst = h + 8 + 16 * (n_addr - 1);
                if (pdst != ip + 24) pdst_off = (uint16_t)(buf->start + (size_t)(pdst - h));
            }
        } else if (nh == 44) {
            /* FragmentHeader::parse :696-703 (chunk_len >= 8), offset :717-719,
             * more_frag :725-727, payload :735-739 (advance 8) */
            if (cl < 8) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = 8;
            uint16_t off = (uint16_t)(be16(h + 2) >> 3);
            int more = h[3] & 1;
            if (off != 0 || more) {
                nh = h[0];
                cur_advance(buf, hl);
                n_ext++;
                stop = RPKT_S_IP6_FRAGMENT;
                break;
            }
        } else if (nh == 51) {
            /* AuthenticationHeader::parse :850-861, header_len = b1 * 4 + 8 :888-890 */
            if (cl < 12) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (size_t)h[1] * 4 + 8;
            if (hl < 12 || hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
        } else {
            break;                                   /* the upper-layer header */
        }
        nh = h[0];                                   /* next_header of every type */
        cur_advance(buf, hl);                        /* payload(): advance(header_len) */
    }
    blk[8] = n_ext;
    blk[9] = nh;                                     /* ip_protocol */
    memcpy(blk + 10, &pdst_off, 2);
    rec->l4_off = (uint16_t)buf->start;
    rec->payload_off = (uint16_t)buf->start;
    rec->payload_len = (uint16_t)cur_remaining(buf);
    if (stop) { rec->status = (uint8_t)stop; return; }
    if (nh == 0 || nh == 43 || nh == 44 || nh == 60 || nh == 51) {
        rec->status = RPKT_S_L4_OTHER;               /* RPKT_MAX_IP6_EXT reached */
        return;
    }
    oracle_parse_l4(buf, nh, ip + 8, pdst, 1, flags, rec);
}

static inline void oracle_parse_ip4(cursor_t* buf, uint32_t flags, rpkt_rec_t* rec);

/* Parse one frame exactly as the reference chain would, filling `rec`.
 * Chain: benches/rpkt/rpkt_parse.rs:62-80 (Ether -> IPv4 -> UDP) generalised
 * with the VLAN/QinQ walk of rpkt/tests/vlan_mpls_tests.rs:96-108 and the TCP
 * branch of rpkt/tests/tcp_test.rs:17-27. */
void oracle_parse_one(const uint8_t* frame, uint32_t frame_len, uint32_t flags,
                      rpkt_rec_t* rec) {
    memset(rec, 0, sizeof(*rec));
    rec->frame_len = frame_len;
    cursor_t buf = {frame, 0, frame_len};             /* Cursor::new, cursors.rs:42-47 */

    /* EtherFrame::parse, ether/generated.rs:34-41: chunk_len >= 14, no ethertype check */
    if (cur_remaining(&buf) < 14) { rec->status = RPKT_S_ETH_SHORT; return; }
    const uint8_t* e = cur_chunk(&buf);
    memcpy(rec->dst_addr, e + 0, 6);                  /* dst_addr  :47-50 */
    memcpy(rec->src_addr, e + 6, 6);                  /* src_addr  :51-54 */
    uint16_t et = be16(e + 12);                       /* ethertype :55-59 */
    rec->ethertype = et;
    cur_advance(&buf, 14);                            /* payload   :63-67 */

    /* VLAN / QinQ walk (caller-side dispatch, vlan_mpls_tests.rs:96-108):
     * VlanFrame::parse vlan/generated.rs:32-39 (chunk_len >= 4), getters :45-61,
     * payload :65-69 (advance 4).  EtherType consts ether/mod.rs:22-24. */
    while ((et == 0x8100 || et == 0x88a8) && rec->n_vlan < RPKT_MAX_VLAN) {
        if (cur_remaining(&buf) < 4) { rec->status = RPKT_S_VLAN_SHORT; return; }
        const uint8_t* v = cur_chunk(&buf);
        rec->vlan_tci[rec->n_vlan] = be16(v);         /* priority/dei/vlan_id :45-56 */
        et = be16(v + 2);                             /* ethertype :57-61 */
        rec->vlan_ethertype[rec->n_vlan] = et;
        rec->n_vlan++;
        cur_advance(&buf, 4);
    }
    if (et == 0x86dd && (flags & RPKT_F_IPV6)) {     /* EtherType::IPV6, ipv6_test.rs:25 */
        oracle_parse_ip6(&buf, flags, rec);
        return;
    }
    if (et != 0x0800) { rec->status = RPKT_S_NOT_IPV4; return; }   /* rpkt_parse.rs:66 */
    oracle_parse_ip4(&buf, flags, rec);
}

/* The IPv4 chain from the cursor at the IPv4 header, advanced in place (a copy of the
 * cursor here went through the stack as one 16-B store and 8-B reloads: config 1's
 * packet_l4 loop ran ~25 % slower). */
static inline void oracle_parse_ip4(cursor_t* buf, uint32_t flags, rpkt_rec_t* rec) {
    /* Ipv4::parse, ipv4/generated.rs:35-51 */
    rec->l3_off = (uint16_t)buf->start;
    size_t chunk_len = cur_remaining(buf);
    if (chunk_len < 20) { rec->status = RPKT_S_IP_SHORT; return; }
    const uint8_t* ip = cur_chunk(buf);
    size_t header_len = (size_t)(ip[0] & 0xf) * 4;    /* header_len :106-108 */
    size_t packet_len = be16(ip + 2);                 /* packet_len :110-112 */
    if (header_len < 20) { rec->status = RPKT_S_IP_BAD_IHL; return; }
    if (header_len > chunk_len) { rec->status = RPKT_S_IP_IHL_GT_LEN; return; }
    if (packet_len < header_len) { rec->status = RPKT_S_IP_TOT_LT_IHL; return; }
    if (packet_len > cur_remaining(buf)) { rec->status = RPKT_S_IP_TOT_GT_LEN; return; }

    rec->ip_vhl = ip[0];                              /* version :61-63, header_len */
    rec->ip_tos = ip[1];                              /* dscp/ecn :65-72 */
    rec->ip_packet_len = (uint16_t)packet_len;
    rec->ip_ident = be16(ip + 4);                     /* ident :74-76 */
    rec->ip_frag = be16(ip + 6);                      /* flags/frag_offset :78-92 */
    rec->ip_ttl = ip[8];                              /* ttl :94-96 */
    rec->ip_protocol = ip[9];                         /* protocol :98-100 */
    rec->ip_checksum = be16(ip + 10);                 /* checksum :102-104 */
    rec->ip_src = be32(ip + 12);                      /* src_addr :269-277 */
    rec->ip_dst = be32(ip + 16);                      /* dst_addr :279-287 */
    if (flags & RPKT_F_IP_SUM)
        rec->ip_sum = oracle_from_slice(ip, header_len);   /* A12: from_slice(hdr[0..ihl4]) */

    /* Ipv4::payload, ipv4/generated.rs:115-127: trim to packet_len, advance ihl */
    size_t trim_size = cur_remaining(buf) - packet_len;
    if (trim_size > 0) cur_trim_off(buf, trim_size);
    cur_advance(buf, header_len);
    rec->l4_off = (uint16_t)buf->start;
    rec->payload_off = (uint16_t)buf->start;
    rec->payload_len = (uint16_t)cur_remaining(buf);

    oracle_parse_l4(buf, ip[9], ip + 12, ip + 16, 0, flags, rec);
}

/* A frame that starts at its IP header (a tunnel's inner packet: GTP-U T-PDU, GRE over
 * IPv4 / IPv6): Ipv4::parse or Ipv6::parse on the whole buffer, as gtpv1_test.rs:229 and
 * gre_test.rs:44 call them.  The record is oracle_parse_one's with ethertype = et (the
 * tunnel's dispatch value), no link layer (n_vlan 0, MACs 0), l3_off 0. */
void oracle_parse_at_ip(const uint8_t* frame, uint32_t frame_len, uint32_t flags, uint16_t et,
                        rpkt_rec_t* rec) {
    memset(rec, 0, sizeof(*rec));
    rec->frame_len = frame_len;
    rec->ethertype = et;
    cursor_t buf = {frame, 0, frame_len};
    if (et == 0x86dd && (flags & RPKT_F_IPV6)) { oracle_parse_ip6(&buf, flags, rec); return; }
    if (et != 0x0800) { rec->status = RPKT_S_NOT_IPV4; return; }
    oracle_parse_ip4(&buf, flags, rec);
}

/* The dispatch ethertype (the one Ipv4/Ipv6::parse was chosen on) and whether the
 * record is an IPv6 record (include/rpkt_gpu.h: the IPv6 block). */
static uint16_t rec_dispatch_et(const rpkt_rec_t* r) {
    return r->n_vlan ? r->vlan_ethertype[r->n_vlan - 1] : r->ethertype;
}
int oracle_rec_is_ip6(const rpkt_rec_t* r) {
    return r->status != RPKT_S_ETH_SHORT && r->status != RPKT_S_VLAN_SHORT &&
           r->status != RPKT_S_NOT_IPV4 && rec_dispatch_et(r) == 0x86dd;
}
/* IPv4 header parsed (its sum and fields are valid) */
int oracle_rec_ip4_parsed(const rpkt_rec_t* r) {
    return !oracle_rec_is_ip6(r) &&
           (r->status == RPKT_S_OK || (r->status >= RPKT_S_L4_OTHER && r->status <= RPKT_S_TCP_BAD_DOFF) ||
            r->status == RPKT_S_ICMP_EMPTY);
}

/* 5-tuple flow hash (shared definition with the device: include/rpkt_gpu.h). */
uint32_t oracle_flow_hash(uint32_t ip_src, uint32_t ip_dst, uint16_t sp, uint16_t dp,
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

/* Flow event of one record (include/rpkt_gpu.h, rpkt_flow_ev_t). */
uint64_t oracle_flow_event(const rpkt_rec_t* r, uint32_t n_buckets) {
    uint64_t ev = r->frame_len;
    uint32_t bucket = n_buckets;
    const int v6 = oracle_rec_is_ip6(r);
    /* ip_src / ip_dst hold ip6_src_fold / ip6_dst_fold in an IPv6 record */
    if (r->status == RPKT_S_OK)
        bucket = oracle_flow_hash(r->ip_src, r->ip_dst, r->src_port, r->dst_port,
                                  r->ip_protocol) % n_buckets;
    ev |= (uint64_t)bucket << 32;
    if (oracle_rec_ip4_parsed(r) && r->ip_sum != 0xffff) ev |= 1ull << 48;
    if (r->status == RPKT_S_OK && r->l4_sum != 0xffff &&
        !(!v6 && r->ip_protocol == 17 && r->l4_checksum == 0))
        ev |= 1ull << 49;
    return ev;
}

/* Batch driver over the same descriptor as rpkt_gpu_parse_batch (host memory). */
void oracle_parse_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                        uint32_t stride, uint32_t frame_len, uint32_t n, uint32_t flags,
                        uint32_t n_buckets, rpkt_rec_t* recs, uint64_t* flow_ev) {
    for (uint32_t i = 0; i < n; i++) {
        uint64_t off, len;
        if (offsets) {
            off = offsets[i];
            len = offsets[i + 1] >= offsets[i] ? offsets[i + 1] - offsets[i] : 0;
        } else {
            off = (uint64_t)i * stride;
            len = frame_len ? frame_len : stride;
        }
        if (off > frames_bytes) off = frames_bytes;
        if (off + len > frames_bytes) len = frames_bytes - off;
        oracle_parse_one(frames + off, (uint32_t)len, flags, &recs[i]);
        if (flow_ev) flow_ev[i] = oracle_flow_event(&recs[i], n_buckets);
    }
}

/* Flow counters from flow events: u64[(n_buckets+1)*4] += ... */
void oracle_flow_count(const uint64_t* ev, uint32_t n, uint32_t n_buckets, uint64_t* counters) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t b = (uint32_t)(ev[i] >> 32) & 0xffff;
        if (b > n_buckets) b = n_buckets;
        uint64_t* row = counters + (size_t)b * 4;
        row[0] += 1;
        row[1] += ev[i] & 0xffffffffu;
        row[2] += (ev[i] >> 48) & 1;
        row[3] += (ev[i] >> 49) & 1;
    }
}

/* benches/rpkt/rpkt_parse.rs:62-80 `packet_l4` restated over one frame: the
 * CPU-baseline harness of config 1.  Returns 0 when every assert would hold. */
int oracle_packet_l4(const uint8_t* frame, uint32_t len, uint32_t want_src, uint32_t want_dst,
                     uint16_t want_ip_ck, uint16_t want_ident, uint16_t want_sport,
                     uint16_t want_dport, uint16_t want_ulen, uint16_t want_udp_ck) {
    rpkt_rec_t r;
    oracle_parse_one(frame, len, 0, &r);
    if (r.status != RPKT_S_OK || r.ethertype != 0x0800 || r.ip_protocol != 17) return 1;
    if (r.ip_src != want_src || r.ip_dst != want_dst) return 2;
    if (r.ip_checksum != want_ip_ck || r.ip_ident != want_ident) return 3;
    if (r.src_port != want_sport || r.dst_port != want_dport) return 4;
    if (r.l4_word6 != want_ulen || r.l4_checksum != want_udp_ck) return 5;
    return 0;
}

/* Config 1's timed loop: `reps` passes of packet_l4 over n frames at `stride`
 * (criterion's b.iter body, benches/rpkt/rpkt_parse.rs:108-140, once per frame).
 * Returns the number of frames whose asserts failed (summed over reps). */
uint64_t oracle_packet_l4_loop(const uint8_t* frames, uint32_t n, uint32_t stride, uint32_t len,
                               uint32_t reps, uint32_t want_src, uint32_t want_dst,
                               uint16_t want_ip_ck, uint16_t want_ident, uint16_t want_sport,
                               uint16_t want_dport, uint16_t want_ulen, uint16_t want_udp_ck) {
    uint64_t bad = 0;
    for (uint32_t r = 0; r < reps; r++)
        for (uint32_t i = 0; i < n; i++) {
            const uint8_t* f = frames + (size_t)i * stride;
            __asm__ volatile("" : : "r"(f) : "memory");   /* no hoisting across reps */
            bad += oracle_packet_l4(f, len, want_src, want_dst, want_ip_ck, want_ident,
                                    want_sport, want_dport, want_ulen, want_udp_ck) != 0;
        }
    return bad;
}
