/*
 * rpkt_oracle_chain.c — CPU restatement of rpkt's parse chain over a multi-segment
 * packet buffer (rpkt-dpdk's Pbuf over an mbuf chain).  TEST INFRASTRUCTURE ONLY:
 * tests/ and bench.py's cpu_baseline leg load it as the checker; the product path
 * (librpkt_gpu.so) never links or calls it.
 *
 * Pbuf is restated field for field (rpkt-dpdk/src/pbuf.rs:8-16): the current
 * segment, the chunk [chunk_start, chunk_start + chunk_len) inside it and segs_len,
 * the bytes of all segments up to and including the current one.  The mbuf chain
 * is the caller's segment list; Mbuf::truncate_to (rpkt-dpdk/src/mbuf.rs:346-382),
 * which Pbuf::trim_off calls, is applied to a private copy of the segment lengths,
 * so the caller's list is never modified.  The walker is pinned by the assertions
 * of rpkt-dpdk/tests/pbuf.rs, replayed through oracle_pbuf_script
 * (tests/test_oracle_chain.py).
 *
 * The header views (EtherFrame/VlanFrame/Ipv4/Udp/Tcp ::parse) are generic over
 * `T: Buf` and test header lengths against `chunk().len()` and total lengths
 * against `remaining()`; over a Pbuf those differ, which is the whole point of this
 * file.  Lengths are 64-bit here (pkt_len is u32 and data_len u16 in DPDK).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>

#include "../include/rpkt_gpu.h"

uint16_t oracle_from_slice(const uint8_t* data, size_t len);
uint16_t oracle_combine(const uint16_t* checksums, size_t n);
uint16_t oracle_propagate_carries(uint32_t word);
int oracle_from_slice_with_tail_byte(const uint8_t* data, size_t len, uint32_t* accum,
                                     int tail_in);
uint16_t oracle_pseudo_header_v4(const uint8_t* src4, const uint8_t* dst4, uint8_t proto,
                                 uint16_t length);
uint16_t oracle_pseudo_header_v6(const uint8_t* src16, const uint8_t* dst16, uint8_t proto,
                                 uint32_t length);
uint64_t oracle_flow_event(const rpkt_rec_t* r, uint32_t n_buckets);

/* ------------------------------------------------------------------------- */
/* The mbuf chain and Pbuf                                                    */
/* ------------------------------------------------------------------------- */

typedef struct mchain {
    const uint8_t* base;     /* arena holding every segment */
    uint64_t* off;           /* data_addr of segment k, as an arena offset */
    uint64_t* len;           /* data_len of segment k (mutable: truncate_to) */
    uint32_t nb_segs;        /* segments still linked (seg k->next == NULL iff k+1 == nb_segs) */
    uint64_t pkt_len;        /* Mbuf::pkt_len, mbuf.rs:250-252 */
} mchain_t;

typedef struct pbuf {
    mchain_t* m;             /* mbuf_head */
    uint32_t cur;            /* mbuf_cur */
    uint64_t chunk_start;    /* arena offset */
    uint64_t chunk_len;
    uint64_t segs_len;
} pbuf_t;

static void die(const char* what) {
    fprintf(stderr, "oracle: %s (the reference panics here)\n", what);
    abort();
}

static int has_next(const pbuf_t* p) { return p->cur + 1 < p->m->nb_segs; }

/* Pbuf::new, pbuf.rs:19-34 */
static void pbuf_new(pbuf_t* p, mchain_t* m) {
    p->m = m;
    p->cur = 0;
    p->chunk_len = m->nb_segs ? m->len[0] : 0;
    p->chunk_start = m->nb_segs ? m->off[0] : 0;
    p->segs_len = p->chunk_len;
}

/* Pbuf::cursor, pbuf.rs:41-44 */
static uint64_t pbuf_cursor(const pbuf_t* p) { return p->segs_len - p->chunk_len; }

/* Pbuf::advance_common, pbuf.rs:48-57 */
static void pbuf_advance_common(pbuf_t* p, uint64_t target) {
    while (p->segs_len <= target && has_next(p)) {
        p->cur += 1;
        p->segs_len += p->m->len[p->cur];
    }
    p->chunk_len = p->segs_len - target;
    p->chunk_start = p->m->off[p->cur] + p->m->len[p->cur] - p->chunk_len;
}

/* Buf::remaining, pbuf.rs:98-101 */
static uint64_t pbuf_remaining(const pbuf_t* p) { return p->m->pkt_len - pbuf_cursor(p); }

/* Buf::advance, pbuf.rs:86-96 (slow path :59-64) */
static void pbuf_advance(pbuf_t* p, uint64_t cnt) {
    if (cnt >= p->chunk_len) {
        if (cnt > pbuf_remaining(p)) die("advance past end");
        pbuf_advance_common(p, pbuf_cursor(p) + cnt);
    } else {
        p->chunk_start += cnt;
        p->chunk_len -= cnt;
    }
}

/* PktBufMut::chunk_headroom, pbuf.rs:146-149 */
static uint64_t pbuf_headroom(const pbuf_t* p) { return p->m->len[p->cur] - p->chunk_len; }

/* Mbuf::truncate_to, mbuf.rs:346-382 */
static void mbuf_truncate_to(mchain_t* m, uint64_t new_size) {
    if (new_size > m->pkt_len) die("truncate_to past pkt_len");
    uint32_t cur = 0;
    uint64_t remaining = new_size;
    while (m->len[cur] < remaining) {
        remaining -= m->len[cur];
        cur += 1;
    }
    if (cur + 1 < m->nb_segs) m->nb_segs = cur + 1;   /* free the trailing segments */
    m->len[cur] = remaining;
    m->pkt_len = new_size;
}

/* PktBuf::trim_off, pbuf.rs:117-140 */
static void pbuf_trim_off(pbuf_t* p, uint64_t cnt) {
    uint64_t cursor = pbuf_cursor(p);
    if (cnt > pbuf_remaining(p)) die("trim_off past end");
    uint64_t new_len = p->m->pkt_len - cnt;
    if (cursor == new_len && pbuf_headroom(p) == 0) {
        mbuf_truncate_to(p->m, new_len);
        p->cur = 0;
        p->segs_len = p->m->len[0];
        pbuf_advance_common(p, cursor);
    } else {
        mbuf_truncate_to(p->m, new_len);
        if (new_len < p->segs_len) {
            p->chunk_len = new_len - cursor;
            p->segs_len = new_len;
        }
    }
}

static const uint8_t* pbuf_chunk(const pbuf_t* p) { return p->m->base + p->chunk_start; }

/* checksum::from_buf(buf, len), rpkt/src/checksum.rs:8-27, over a Pbuf (Buf::take) */
static uint16_t pbuf_from_buf(pbuf_t buf, uint64_t len) {
    uint32_t accum = 0;
    int tail = -1;
    uint64_t limit = len < pbuf_remaining(&buf) ? len : pbuf_remaining(&buf);
    while (limit > 0) {                                /* has_remaining, :13 */
        uint64_t cl = buf.chunk_len < limit ? buf.chunk_len : limit;
        if (cl == 0 && tail >= 0) die("from_slice_with_tail_byte on an empty chunk");
        if (cl) tail = oracle_from_slice_with_tail_byte(pbuf_chunk(&buf), cl, &accum, tail);
        pbuf_advance(&buf, cl);                        /* :19 */
        limit -= cl;
    }
    if (tail >= 0) accum += (uint32_t)tail << 8;       /* :22-24 */
    return oracle_propagate_carries(accum);
}

static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* ------------------------------------------------------------------------- */
/* The decode chain over a Pbuf                                               */
/* ------------------------------------------------------------------------- */

/* Udp::parse / Tcp::parse over the Pbuf the IP layer's payload() returned (header
 * sizes against chunk().len(), the UDP length against remaining()), getters, the L4
 * sum with the pseudo header of the IP version, payload().  Shared by both chains. */
static void parse_pbuf_l4(pbuf_t* bufp, uint8_t proto, const uint8_t* src, const uint8_t* dst,
                          int v6, uint32_t flags, rpkt_rec_t* rec) {
    pbuf_t buf = *bufp;
    if (proto == 17) {
        /* Udp::parse, udp/generated.rs:31-42 */
        if (buf.chunk_len < 8) { rec->status = RPKT_S_UDP_SHORT; return; }
        const uint8_t* u = pbuf_chunk(&buf);
        uint64_t ulen = be16(u + 4);
        if (ulen < 8 || ulen > pbuf_remaining(&buf)) { rec->status = RPKT_S_UDP_BAD_LEN; return; }
        rec->src_port = be16(u);
        rec->dst_port = be16(u + 2);
        rec->l4_word6 = (uint16_t)ulen;
        rec->l4_checksum = be16(u + 6);
        if (flags & RPKT_F_L4_SUM) {
            uint16_t parts[2] = {v6 ? oracle_pseudo_header_v6(src, dst, 17, (uint32_t)ulen)
                                    : oracle_pseudo_header_v4(src, dst, 17, (uint16_t)ulen),
                                 pbuf_from_buf(buf, ulen)};
            rec->l4_sum = oracle_combine(parts, 2);
        }
        /* Udp::payload, udp/generated.rs:66-76 */
        uint64_t ts = pbuf_remaining(&buf) - ulen;
        if (ts > 0) pbuf_trim_off(&buf, ts);
        pbuf_advance(&buf, 8);
        rec->payload_off = (uint16_t)pbuf_cursor(&buf);
        rec->payload_len = (uint16_t)pbuf_remaining(&buf);
        rec->status = RPKT_S_OK;
    } else if (proto == 6) {
        /* Tcp::parse, tcp/generated.rs:34-45 */
        uint64_t cl = buf.chunk_len;
        if (cl < 20) { rec->status = RPKT_S_TCP_SHORT; return; }
        const uint8_t* t = pbuf_chunk(&buf);
        uint64_t hl = (uint64_t)(t[12] >> 4) * 4;
        if (hl < 20 || hl > cl) { rec->status = RPKT_S_TCP_BAD_DOFF; return; }
        rec->src_port = be16(t);
        rec->dst_port = be16(t + 2);
        rec->tcp_seq = be32(t + 4);
        rec->tcp_ack = be32(t + 8);
        rec->l4_word6 = be16(t + 12);
        rec->tcp_window = be16(t + 14);
        rec->l4_checksum = be16(t + 16);
        rec->tcp_urgent = be16(t + 18);
        uint64_t l4len = pbuf_remaining(&buf);        /* TCP length comes from the IP layer */
        if (flags & RPKT_F_L4_SUM) {
            uint16_t parts[2] = {v6 ? oracle_pseudo_header_v6(src, dst, 6, (uint32_t)l4len)
                                    : oracle_pseudo_header_v4(src, dst, 6, (uint16_t)l4len),
                                 pbuf_from_buf(buf, l4len)};
            rec->l4_sum = oracle_combine(parts, 2);
        }
        pbuf_advance(&buf, hl);                       /* Tcp::payload :125-131 */
        rec->payload_off = (uint16_t)pbuf_cursor(&buf);
        rec->payload_len = (uint16_t)pbuf_remaining(&buf);
        rec->status = RPKT_S_OK;
    } else {
        /* ICMP / GRE-with-checksum sums over the IP payload (rpkt_oracle.c
         * oracle_parse_l4), here from_buf over the segments */
        rec->status = RPKT_S_L4_OTHER;
        uint64_t n = pbuf_remaining(&buf);
        if (!v6 && proto == 1) {
            if (n == 0) { rec->status = RPKT_S_ICMP_EMPTY; return; }
            if (flags & RPKT_F_L4_SUM) rec->l4_sum = pbuf_from_buf(buf, n);
        } else if (proto == 47 && n >= 4 && (pbuf_chunk(&buf)[0] & 0x80)) {
            if (flags & RPKT_F_L4_SUM) rec->l4_sum = pbuf_from_buf(buf, n);
        }
    }
}

static uint32_t fold_be32x4(const uint8_t* a) {
    return be32(a) ^ be32(a + 4) ^ be32(a + 8) ^ be32(a + 12);
}

/* The IPv6 chain over a Pbuf (RPKT_F_IPV6): oracle_parse_ip6 (rpkt_oracle.c) with every
 * header size tested against chunk().len() and the payload length against
 * remaining(): Ipv6::parse ipv6/generated.rs:40-51, payload :83-92, then each
 * extension header's generated parse (DestOptions :241-252, HopByHopOption :384-395,
 * RoutingHeader :528-539, FragmentHeader :696-703, AuthenticationHeader :850-861) and
 * payload() = advance(header_len). */
static void parse_pbuf_ip6(pbuf_t* bufp, uint32_t flags, rpkt_rec_t* rec) {
    pbuf_t buf = *bufp;
    rec->l3_off = (uint16_t)pbuf_cursor(&buf);
    if (buf.chunk_len < 40) { rec->status = RPKT_S_IP6_SHORT; return; }       /* :42 */
    const uint8_t* ip = pbuf_chunk(&buf);            /* the header lies inside the chunk */
    uint64_t payload_len = be16(ip + 4);
    if (payload_len + 40 > pbuf_remaining(&buf)) { rec->status = RPKT_S_IP6_BAD_LEN; return; }
    uint8_t* blk = (uint8_t*)rec + 24;
    uint32_t vtcfl = be32(ip);
    uint16_t pl = (uint16_t)payload_len;
    uint16_t pdst_off = (uint16_t)(pbuf_cursor(&buf) + 24);
    uint32_t sf = fold_be32x4(ip + 8), df = fold_be32x4(ip + 24);
    memcpy(blk + 0, &vtcfl, 4);
    memcpy(blk + 4, &pl, 2);
    blk[6] = ip[6];
    blk[7] = ip[7];
    memcpy(blk + 12, &sf, 4);
    memcpy(blk + 16, &df, 4);
    const uint8_t* pdst = ip + 24;

    /* Ipv6::payload, :83-92 */
    uint64_t trim_size = pbuf_remaining(&buf) - (40 + payload_len);
    if (trim_size > 0) pbuf_trim_off(&buf, trim_size);
    pbuf_advance(&buf, 40);

    uint8_t nh = ip[6];
    uint8_t n_ext = 0;
    int stop = 0;
    for (; n_ext < RPKT_MAX_IP6_EXT; n_ext++) {
        uint64_t cl = buf.chunk_len;
        const uint8_t* h = pbuf_chunk(&buf);
        uint64_t hl;
        if (nh == 0 || nh == 60) {
            if (cl < 2) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (uint64_t)h[1] * 8 + 8;
            if (hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
        } else if (nh == 43) {
            if (cl < 8) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (uint64_t)h[1] * 8 + 8;
            if (hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
            if (h[3] > 0) {                          /* segments_left: the final address */
                uint64_t n_addr = (hl - 8) / 16;
                const uint8_t* q = pdst;
                if (h[2] == 4 && n_addr >= 1) q = h + 8;
                else if ((h[2] == 0 || h[2] == 2) && n_addr >= 1) q = h + 8 + 16 * (n_addr - 1);
                if (q != pdst) {
                    pdst = q;
                    pdst_off = (uint16_t)(pbuf_cursor(&buf) + (uint64_t)(q - h));
                }
            }
        } else if (nh == 44) {
            if (cl < 8) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = 8;
            uint16_t off = (uint16_t)(be16(h + 2) >> 3);
            if (off != 0 || (h[3] & 1)) {
                nh = h[0];
                pbuf_advance(&buf, hl);
                n_ext++;
                stop = RPKT_S_IP6_FRAGMENT;
                break;
            }
        } else if (nh == 51) {
            if (cl < 12) { stop = RPKT_S_IP6_EXT_SHORT; break; }
            hl = (uint64_t)h[1] * 4 + 8;
            if (hl < 12 || hl > cl) { stop = RPKT_S_IP6_EXT_BAD_LEN; break; }
        } else {
            break;
        }
        nh = h[0];
        pbuf_advance(&buf, hl);
    }
    blk[8] = n_ext;
    blk[9] = nh;
    memcpy(blk + 10, &pdst_off, 2);
    rec->l4_off = (uint16_t)pbuf_cursor(&buf);
    rec->payload_off = rec->l4_off;
    rec->payload_len = (uint16_t)pbuf_remaining(&buf);
    if (stop) { rec->status = (uint8_t)stop; return; }
    if (nh == 0 || nh == 43 || nh == 44 || nh == 60 || nh == 51) {
        rec->status = RPKT_S_L4_OTHER;
        return;
    }
    parse_pbuf_l4(&buf, nh, ip + 8, pdst, 1, flags, rec);
}

/* Same chain and record as oracle_parse_one (rpkt_oracle.c), with every length
 * test taken exactly as the generic views take it: header sizes against
 * chunk().len(), IPv4/UDP totals against remaining(). */
static void parse_pbuf(mchain_t* m, uint32_t flags, rpkt_rec_t* rec) {
    memset(rec, 0, sizeof(*rec));
    rec->frame_len = m->pkt_len > 0xffffffffull ? 0xffffffffu : (uint32_t)m->pkt_len;
    pbuf_t buf;
    pbuf_new(&buf, m);

    /* EtherFrame::parse, ether/generated.rs:34-41 */
    if (buf.chunk_len < 14) { rec->status = RPKT_S_ETH_SHORT; return; }
    const uint8_t* e = pbuf_chunk(&buf);
    memcpy(rec->dst_addr, e + 0, 6);
    memcpy(rec->src_addr, e + 6, 6);
    uint16_t et = be16(e + 12);
    rec->ethertype = et;
    pbuf_advance(&buf, 14);                           /* payload :63-67 */

    /* VLAN walk, vlan/generated.rs:32-39 (chunk_len >= 4), payload :65-69 */
    while ((et == 0x8100 || et == 0x88a8) && rec->n_vlan < RPKT_MAX_VLAN) {
        if (buf.chunk_len < 4) { rec->status = RPKT_S_VLAN_SHORT; return; }
        const uint8_t* v = pbuf_chunk(&buf);
        rec->vlan_tci[rec->n_vlan] = be16(v);
        et = be16(v + 2);
        rec->vlan_ethertype[rec->n_vlan] = et;
        rec->n_vlan++;
        pbuf_advance(&buf, 4);
    }
    if (et == 0x86dd && (flags & RPKT_F_IPV6)) { parse_pbuf_ip6(&buf, flags, rec); return; }
    if (et != 0x0800) { rec->status = RPKT_S_NOT_IPV4; return; }

    /* Ipv4::parse, ipv4/generated.rs:35-51 */
    rec->l3_off = (uint16_t)pbuf_cursor(&buf);
    uint64_t chunk_len = buf.chunk_len;
    if (chunk_len < 20) { rec->status = RPKT_S_IP_SHORT; return; }
    uint8_t ip[60];                                   /* the header lies inside the chunk */
    memcpy(ip, pbuf_chunk(&buf), 20);
    uint64_t header_len = (uint64_t)(ip[0] & 0xf) * 4;
    uint64_t packet_len = be16(ip + 2);
    if (header_len < 20) { rec->status = RPKT_S_IP_BAD_IHL; return; }
    if (header_len > chunk_len) { rec->status = RPKT_S_IP_IHL_GT_LEN; return; }
    if (packet_len < header_len) { rec->status = RPKT_S_IP_TOT_LT_IHL; return; }
    if (packet_len > pbuf_remaining(&buf)) { rec->status = RPKT_S_IP_TOT_GT_LEN; return; }
    memcpy(ip, pbuf_chunk(&buf), header_len);
    rec->ip_vhl = ip[0];
    rec->ip_tos = ip[1];
    rec->ip_packet_len = (uint16_t)packet_len;
    rec->ip_ident = be16(ip + 4);
    rec->ip_frag = be16(ip + 6);
    rec->ip_ttl = ip[8];
    rec->ip_protocol = ip[9];
    rec->ip_checksum = be16(ip + 10);
    rec->ip_src = be32(ip + 12);
    rec->ip_dst = be32(ip + 16);
    if (flags & RPKT_F_IP_SUM) rec->ip_sum = oracle_from_slice(ip, header_len);

    /* Ipv4::payload, ipv4/generated.rs:115-127 */
    uint64_t trim_size = pbuf_remaining(&buf) - packet_len;
    if (trim_size > 0) pbuf_trim_off(&buf, trim_size);
    pbuf_advance(&buf, header_len);
    rec->l4_off = (uint16_t)pbuf_cursor(&buf);
    rec->payload_off = rec->l4_off;
    rec->payload_len = (uint16_t)pbuf_remaining(&buf);

    parse_pbuf_l4(&buf, ip[9], ip + 12, ip + 16, 0, flags, rec);
}

/* Load chain `first .. last-1` of the caller's segment list into `m`, clamping
 * each segment to the arena exactly as the device does (include/rpkt_gpu.h). */
static void chain_load(mchain_t* m, const uint8_t* buf, uint64_t buf_bytes, const uint32_t* segs,
                       uint32_t first, uint32_t last) {
    m->base = buf;
    m->nb_segs = last - first;
    m->pkt_len = 0;
    for (uint32_t k = 0; k < m->nb_segs; k++) {
        uint64_t o = segs[2 * (first + k)], l = segs[2 * (first + k) + 1];
        if (o > buf_bytes) o = buf_bytes;
        if (o + l > buf_bytes) l = buf_bytes - o;
        m->off[k] = o;
        m->len[k] = l;
        m->pkt_len += l;
    }
}

/* Batch driver with the arguments of rpkt_gpu_parse_chains: chain p is segments
 * [a, b) with a = min(first[p], n_segs), b = min(max(first[p+1], a), n_segs). */
void oracle_parse_chains(const uint8_t* buf, uint64_t buf_bytes, const uint32_t* segs,
                         uint32_t n_segs, const uint32_t* chain_first, uint32_t n_chains,
                         uint32_t flags, uint32_t n_buckets, rpkt_rec_t* recs,
                         uint64_t* flow_ev) {
    uint32_t cap = 0;
    uint64_t *off = NULL, *len = NULL;
    for (uint32_t p = 0; p < n_chains; p++) {
        uint32_t a = chain_first[p] < n_segs ? chain_first[p] : n_segs;
        uint32_t b = chain_first[p + 1] > a ? chain_first[p + 1] : a;
        if (b > n_segs) b = n_segs;
        if (b - a > cap) {
            cap = b - a;
            off = realloc(off, cap * sizeof(uint64_t));
            len = realloc(len, cap * sizeof(uint64_t));
            if (!off || !len) die("out of memory");
        }
        mchain_t m = {buf, off, len, 0, 0};
        chain_load(&m, buf, buf_bytes, segs, a, b);
        parse_pbuf(&m, flags, &recs[p]);
        if (flow_ev) flow_ev[p] = oracle_flow_event(&recs[p], n_buckets);
    }
    free(off);
    free(len);
}

/* Replay a script of Pbuf operations over a chain of segment lengths (no data),
 * for the assertions of rpkt-dpdk/tests/pbuf.rs.  ops[2i] = 0 new, 1 advance,
 * 2 trim_off; ops[2i+1] = count.  After each op, out[6i..6i+5] = cursor,
 * chunk().len(), remaining(), chunk_headroom(), num_segs(), pkt_len(). */
void oracle_pbuf_script(const uint32_t* seg_lens, uint32_t n, const uint64_t* ops,
                        uint32_t n_ops, uint64_t* out) {
    uint64_t* off = calloc(n ? n : 1, sizeof(uint64_t));
    uint64_t* len = calloc(n ? n : 1, sizeof(uint64_t));
    mchain_t m = {NULL, off, len, 0, 0};
    pbuf_t p;
    for (uint32_t i = 0; i < n_ops; i++) {
        if (ops[2 * i] == 0) {
            m.nb_segs = n;
            m.pkt_len = 0;
            uint64_t o = 0;
            for (uint32_t k = 0; k < n; k++) {
                off[k] = o;
                len[k] = seg_lens[k];
                o += 4096;
                m.pkt_len += seg_lens[k];
            }
            pbuf_new(&p, &m);
        } else if (ops[2 * i] == 1) {
            pbuf_advance(&p, ops[2 * i + 1]);
        } else {
            pbuf_trim_off(&p, ops[2 * i + 1]);
        }
        out[6 * i + 0] = pbuf_cursor(&p);
        out[6 * i + 1] = p.chunk_len;
        out[6 * i + 2] = pbuf_remaining(&p);
        out[6 * i + 3] = pbuf_headroom(&p);
        out[6 * i + 4] = m.nb_segs;
        out[6 * i + 5] = m.pkt_len;
    }
    free(off);
    free(len);
}
