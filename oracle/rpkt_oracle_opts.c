/*
 * rpkt_oracle_opts.c — CPU restatement of rpkt's option iterators, TEST
 * INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).
 *
 * TcpOptionsIter::next (rpkt/src/tcp/generated.rs:1387-1484) and Ipv4OptionsIter::next
 * (rpkt/src/ipv4/generated.rs:1625-1722): dispatch on the first byte; the option's own
 * parse decides (Some, advance by its header_len) or Err (None); an unknown type is
 * None; an empty slice is None.  Per-type parse rules restated from the generated
 * views (fixed length: chunk >= L and header_len == L; variable: chunk >= L and
 * L <= header_len <= chunk):
 *   TCP  Eol/Nop 1 B; Mss (2) ==4 :522-533; WindowScale (3) ==3 :664-675;
 *        SackPermitted (4) ==2; Sack (5) var >=2 :942-953; Timestamp (8) ==10
 *        :1086-1097; FastOpen (34) var >=2 :1236-1247.
 *   IPv4 Eol/Nop 1 B; Timestamp (68) var >=4; RecordRoute (7) var >=3;
 *        CommercialSecurity (134) var >=6; RouteAlert (148) ==4;
 *        Loose/StrictSourceRoute (131/137) ==7.
 */
#include <stdint.h>
#include <string.h>

#include "../include/rpkt_gpu.h"

int oracle_rec_ip4_parsed(const rpkt_rec_t* r);   /* rpkt_oracle.c */

static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* returns the option length consumed (>0), 0 = malformed, -1 = unknown type;
 * *kind = kind index */
static int tcp_opt(const uint8_t* b, uint32_t n, int* kind) {
    uint32_t t = b[0], hl = n >= 2 ? b[1] : 0;
    switch (t) {
        case 0: *kind = 0; return 1;
        case 1: *kind = 1; return 1;
        case 2: *kind = 2; return (n >= 4 && hl == 4) ? 4 : 0;
        case 3: *kind = 3; return (n >= 3 && hl == 3) ? 3 : 0;
        case 4: *kind = 4; return (n >= 2 && hl == 2) ? 2 : 0;
        case 5: *kind = 5; return (n >= 2 && hl >= 2 && hl <= n) ? (int)hl : 0;
        case 8: *kind = 6; return (n >= 10 && hl == 10) ? 10 : 0;
        case 34: *kind = 7; return (n >= 2 && hl >= 2 && hl <= n) ? (int)hl : 0;
        default: return -1;
    }
}

static int ip_opt(const uint8_t* b, uint32_t n, int* kind) {
    uint32_t t = b[0], hl = n >= 2 ? b[1] : 0;
    switch (t) {
        case 0: *kind = 0; return 1;
        case 1: *kind = 1; return 1;
        case 68: *kind = 2; return (n >= 4 && hl >= 4 && hl <= n) ? (int)hl : 0;
        case 7: *kind = 3; return (n >= 3 && hl >= 3 && hl <= n) ? (int)hl : 0;
        case 148: *kind = 4; return (n >= 4 && hl == 4) ? 4 : 0;
        case 134: *kind = 5; return (n >= 6 && hl >= 6 && hl <= n) ? (int)hl : 0;
        case 137: *kind = 6; return (n >= 7 && hl == 7) ? 7 : 0;
        case 131: *kind = 7; return (n >= 7 && hl == 7) ? 7 : 0;
        default: return -1;
    }
}

int oracle_rec_is_ip6(const rpkt_rec_t* r);       /* rpkt_oracle.c */

/* Ipv6OptionsIter::next (rpkt/src/ipv6/generated.rs:1568-1615): the first byte picks the
 * option; Pad0 (0) is one byte (:1446-1453); PadN (1, :1302-1313) and Generic (2..4,
 * 6..255, :1017-1028): chunk >= 2 and 2 <= header_len = b1 + 2 <= chunk; RouterAlert
 * (5, :1160-1171): chunk >= 4 and header_len == 4.  Every type is some option, so the
 * walk stops only at the slice's end or at a failed parse.  Returns the bytes the
 * option takes, 0 = malformed; *kind = 0 Pad0, 1 PadN, 2 RouterAlert, 3 Generic. */
static int ip6_opt(const uint8_t* b, uint32_t n, int* kind) {
    uint32_t t = b[0];
    if (t == 0) { *kind = 0; return 1; }
    *kind = t == 1 ? 1 : (t == 5 ? 2 : 3);
    if (t == 5) return (n >= 4 && b[1] + 2u == 4) ? 4 : 0;
    if (n < 2) return 0;
    uint32_t hl = b[1] + 2u;                          /* header_len :1328-1330, :1043-1045 */
    return hl <= n ? (int)hl : 0;
}

/* The IPv6 half of rpkt_opts_t (include/rpkt_gpu.h): Ipv6OptionsIter over the
 * var_header_slice() (bytes [2, header_len)) of every HopByHopOption / DestOptions header
 * of the chain the parse walked (frame bytes [l3 + 40, l4_off)), in order, as a receive
 * loop walks them (ipv6_test.rs:47-69, 154-175); a malformed option ends the walking. */
static void ip6_options(const uint8_t* f, const rpkt_rec_t* r, rpkt_opts_t* o) {
    if (r->status == RPKT_S_IP6_SHORT || r->status == RPKT_S_IP6_BAD_LEN) return;
    uint32_t c = r->l3_off + 40u, l4 = r->l4_off;
    uint32_t nh = f[r->l3_off + 6];
    uint8_t* ip = (uint8_t*)o + 27;                   /* bytes 27..47: the IPv6 view */
    uint32_t count = 0;                               /* stored as u8 (ip_count) */
    for (int k = 0; k < RPKT_MAX_IP6_EXT && c < l4; k++) {
        const uint8_t* h = f + c;
        uint32_t hl = nh == 44 ? 8u : (nh == 51 ? h[1] * 4u + 8u : h[1] * 8u + 8u);
        if (nh == 0 || nh == 60) {
            if (ip[9] == 0) ip[10] = (uint8_t)nh;     /* ip6_first_hdr (byte 37) */
            ip[9]++;                                  /* ip6_opt_hdrs  (byte 36) */
            const uint8_t* b = h + 2;                 /* var_header_slice :258-261, :401-404 */
            uint32_t n = hl - 2, pos = 0;
            o->ip_stop = RPKT_OPT_END;
            while (pos < n) {
                int kind = 0, used = ip6_opt(b + pos, n - pos, &kind);
                if (used == 0) { o->ip_stop = RPKT_OPT_MALFORMED; break; }
                const uint8_t* p = b + pos;
                if (kind == 2) o->ip_route_alert = be16(p + 2);          /* :1181-1183 */
                if (kind == 3) {                                          /* :1039-1045 */
                    uint32_t dl = p[1], v = 0;
                    for (uint32_t q = 0; q < 4; q++) v = (v << 8) | (q < dl ? p[2 + q] : 0u);
                    ip[7] = p[0];                     /* ip6_generic_type (byte 34) */
                    ip[8] = p[1];                     /* ip6_generic_len  (byte 35) */
                    o->ip_sr_dest = v;                /* ip6_generic_data (bytes 40..43) */
                }
                o->ip_kinds |= (uint16_t)(1u << kind);
                if (count < 16) o->ip_trace |= (uint64_t)(kind + 1) << (4 * count);
                count++;
                pos += (uint32_t)used;
            }
            o->ip_count = (uint8_t)count;
            o->ip_end = (uint8_t)pos;
            if (o->ip_stop == RPKT_OPT_MALFORMED) break;
        }
        nh = h[0];
        c += hl;
    }
}

void oracle_options_one(const uint8_t* f, uint32_t len, const rpkt_rec_t* r, rpkt_opts_t* o) {
    memset(o, 0, sizeof(*o));
    (void)len;
    /* Ipv4OptionsIter runs over IPv4 headers only; TcpOptionsIter over any TCP header,
     * behind IPv4 or IPv6 (rpkt_oracle.c) */
    if (oracle_rec_ip4_parsed(r)) {
        const uint8_t* b = f + r->l3_off + 20;            /* var_header_slice :41-44 */
        uint32_t n = (uint32_t)(r->l4_off - r->l3_off - 20), pos = 0;
        o->ip_stop = RPKT_OPT_END;
        while (pos < n) {
            int kind = 0, used = ip_opt(b + pos, n - pos, &kind);
            if (used < 0) { o->ip_stop = RPKT_OPT_UNKNOWN; break; }
            if (used == 0) { o->ip_stop = RPKT_OPT_MALFORMED; break; }
            const uint8_t* p = b + pos;
            if (kind == 2) { o->ip_ts_len = p[1]; o->ip_ts_pointer = p[2]; o->ip_ts_oflw_flg = p[3]; }
            if (kind == 3) { o->ip_rr_len = p[1]; o->ip_rr_pointer = p[2]; }
            if (kind == 4) o->ip_route_alert = be16(p + 2);
            if (kind == 5) o->ip_cs_doi = be32(p + 2);
            if (kind == 6 || kind == 7) { o->ip_sr_pointer = p[2]; o->ip_sr_dest = be32(p + 3); }
            o->ip_kinds |= (uint16_t)(1u << kind);
            if (o->ip_count < 16) o->ip_trace |= (uint64_t)(kind + 1) << (4 * o->ip_count);
            o->ip_count++;
            pos += (uint32_t)used;
        }
        o->ip_end = (uint8_t)pos;
    }
    if (oracle_rec_is_ip6(r)) ip6_options(f, r, o);
    if (r->status == RPKT_S_OK && r->ip_protocol == 6) {
        uint32_t doff4 = (uint32_t)(r->l4_word6 >> 12) * 4;
        const uint8_t* b = f + r->l4_off + 20;
        uint32_t n = doff4 - 20, pos = 0;
        o->tcp_stop = RPKT_OPT_END;
        while (pos < n) {
            int kind = 0, used = tcp_opt(b + pos, n - pos, &kind);
            if (used < 0) { o->tcp_stop = RPKT_OPT_UNKNOWN; break; }
            if (used == 0) { o->tcp_stop = RPKT_OPT_MALFORMED; break; }
            const uint8_t* p = b + pos;
            if (kind == 2) o->tcp_mss = be16(p + 2);
            if (kind == 3) o->tcp_wscale = p[2];
            if (kind == 5) {
                o->tcp_sack_blocks = (uint8_t)((p[1] - 2) / 8);
                o->tcp_sack_left = p[1] >= 6 ? be32(p + 2) : 0;
                o->tcp_sack_right = p[1] >= 10 ? be32(p + 6) : 0;
            }
            if (kind == 6) { o->tcp_ts = be32(p + 2); o->tcp_ts_echo = be32(p + 6); }
            if (kind == 7) o->tcp_fo_len = p[1];
            o->tcp_kinds |= (uint16_t)(1u << kind);
            if (o->tcp_count < 16) o->tcp_trace |= (uint64_t)(kind + 1) << (4 * o->tcp_count);
            o->tcp_count++;
            pos += (uint32_t)used;
        }
        o->tcp_end = (uint8_t)pos;
    }
}

void oracle_options_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                          uint32_t stride, uint32_t frame_len, uint32_t n, const rpkt_rec_t* recs,
                          rpkt_opts_t* opts) {
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
        oracle_options_one(frames + off, (uint32_t)len, &recs[i], &opts[i]);
    }
}
