/*
 * rpkt_oracle_tunnel.c — CPU restatement of rpkt_gpu_parse_tunnel_batch, TEST
 * INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).
 *
 * The outer frame is oracle_parse_one's record; the tunnel is the chain of views a
 * receive loop builds on the outer view's payload (include/rpkt_gpu.h documents the
 * dispatch), each step restated from rpkt's generated parse / getters / payload() with
 * the lines cited; the inner frame is oracle_parse_one (VXLAN, GRE transparent bridging)
 * or oracle_parse_at_ip (GTP-U T-PDU, GRE over IP) on the tunnel's payload, its offsets
 * moved to the outer frame (rpkt's Cursor::cursor() counts from the original buffer,
 * rpkt/src/cursors.rs:56-59).  The cursor over a flat frame has chunk() == remaining().
 */
#include <stdint.h>
#include <string.h>

#include "../include/rpkt_gpu.h"

void oracle_parse_one(const uint8_t* frame, uint32_t frame_len, uint32_t flags, rpkt_rec_t* rec);
uint64_t oracle_flow_event(const rpkt_rec_t* r, uint32_t n_buckets);
void oracle_parse_at_ip(const uint8_t* frame, uint32_t frame_len, uint32_t flags, uint16_t et,
                        rpkt_rec_t* rec);
int oracle_rec_is_ip6(const rpkt_rec_t* r);

static uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* A view over frame bytes [s, e): rpkt's Cursor after payload()'s trim and advance. */
typedef struct { const uint8_t* f; uint32_t s, e; } view_t;
static uint32_t rem(const view_t* v) { return v->e - v->s; }
static const uint8_t* chunk(const view_t* v) { return v->f + v->s; }

/* The result the device writes: the rpkt_tun_t, and where the inner frame is. */
typedef struct { rpkt_tun_t t; uint32_t is, ie; int start; /* -1 none, 0 Ether, else et */ } tun_out_t;

static void set(tun_out_t* o, int kind, int status, uint32_t ts) {
    o->t.kind = (uint8_t)kind;
    o->t.status = (uint8_t)status;
    o->t.tun_off = (uint16_t)ts;
}

/* the inner packet by type (GRE protocol_type, or the T-PDU's version nibble as 0x0800 /
 * 0x86DD / 0): Ethernet (0x6558, RFC 1701 transparent bridging), IPv4, IPv6 (with
 * RPKT_F_IPV6); anything else leaves it undecoded */
static void inner_by_type(tun_out_t* o, uint32_t type, uint32_t is, uint32_t ie, uint32_t flags) {
    o->t.inner_off = (uint16_t)is;
    o->t.inner_type = (uint16_t)type;
    o->is = is;
    o->ie = ie;
    if (type == 0x6558) o->start = 0;
    else if (type == 0x0800 || (type == 0x86dd && (flags & RPKT_F_IPV6))) o->start = (int)type;
    else { o->t.status = RPKT_T_INNER_UNKNOWN; return; }
    o->t.status = RPKT_T_OK;
}

/* Vxlan::parse (rpkt/src/vxlan/generated.rs:32-39): chunk_len >= 8.  Getters :44-87:
 * byte 0 (gbp_extention, reserved_0, vni_present), byte 1 (dont_learn, policy_applied),
 * group_id be16[2..4], vni be24[4..7].  payload() :91-96: advance(8).  Then
 * EtherFrame::parse(vxlan.payload()) (rpkt/tests/vlan_mpls_tests.rs:250). */
static void vxlan(const view_t* v, uint32_t flags, tun_out_t* o) {
    const uint8_t* p = chunk(v);
    if (rem(v) < 8) return;                                  /* Err: T_BAD */
    o->t.hdr0 = p[0];
    o->t.hdr1 = p[1];
    o->t.aux = (uint16_t)be16(p + 2);
    o->t.id = ((uint32_t)p[4] << 16) | ((uint32_t)p[5] << 8) | p[6];
    inner_by_type(o, 0x6558, v->s + 8, v->e, flags);
}

/* One GTP-U extension header at view x, of the type the previous header named
 * (Gtpv1NextExtention, rpkt/src/gtpv1/mod.rs).  Returns its header_len, or 0 when its
 * parse returns Err or the type is not one the crate parses; *next = its
 * next_extention_header (the header's last byte). */
static uint32_t gtp_ext(const view_t* x, uint32_t type, uint32_t* next) {
    const uint32_t cl = rem(x);
    const uint8_t* p = chunk(x);
    uint32_t hl;
    switch (type) {
        case 0x40:   /* ExtUdpPort::parse gtpv1/generated.rs:336-341 (chunk >= 4), next [3] :357 */
        case 0xc0:   /* ExtPduNumber::parse :461-466, next [3] :482 */
        case 0x20:   /* ExtServiceClassIndicator::parse :747-752, next [3] :772 */
            if (cl < 4) return 0;
            hl = 4;
            break;
        case 0x03:   /* ExtLongPduNumber::parse :587-592 (chunk >= 8), next [7] :624 */
        case 0x82:
            if (cl < 8) return 0;
            hl = 8;
            break;
        case 0x81:   /* RAN / XW-RAN container: ExtContainer::parse :880-892, header_len */
        case 0x83:   /*   = byte 0 * 4 (:902-904), next = its last byte (:1001-1003) */
            if (cl < 1) return 0;
            hl = (uint32_t)p[0] * 4;
            if (hl < 1 || hl > cl) return 0;
            break;
        case 0x84: { /* NR RAN container: NrUp::group_parse :2308-2320 (byte 1 >> 4) */
            if (cl < 2) return 0;
            uint32_t min;
            switch (p[1] >> 4) {
                case 0: min = 6; break;   /* DlUserData::parse :1545-1555 */
                case 1: min = 7; break;   /* DlDataDeliveryStatus::parse :1821-1831 */
                case 2: min = 3; break;   /* AssistanceInformationData::parse :2095-2105 */
                default: return 0;
            }
            if (cl < min) return 0;
            hl = (uint32_t)p[0] * 4;    /* header_len :1613, :1889, :2143 */
            if (hl < min || hl > cl) return 0;
            break;
        }
        case 0x85:   /* PDU session container: PduSessionUp::group_parse :1507-1518 */
            if (cl < 2) return 0;
            if ((p[1] >> 4) > 1) return 0;
            if (cl < 3) return 0;        /* Dl/UlPduSessionInfo::parse :1048-1058, :1287-1297 */
            hl = (uint32_t)p[0] * 4;     /* header_len :1100, :1339 */
            if (hl < 3 || hl > cl) return 0;
            break;
        default:
            return 0;
    }
    *next = p[hl - 1];
    return hl;
}

/* Gtpv1::parse (gtpv1/generated.rs:33-49): chunk_len >= 8; header_len (:239-250: 8, or
 * 12 when any of extention_header_present / sequence_present / npdu_present);
 * packet_len = be16[2..4] + 8 (:81-84); header_len <= chunk_len, packet_len in
 * [header_len, remaining].  Getters :57-84, sequence :254-258 (12-B header).  payload()
 * :98-108: trim to packet_len, advance header_len.  A G-PDU (message_type 255,
 * gtpv1/mod.rs) of GTP version 1 carries an IP packet after its extension headers
 * (gtpv1_test.rs:199-231, 284-320, 468-505). */
static void gtpu(const view_t* v, uint32_t flags, tun_out_t* o) {
    const uint8_t* p = chunk(v);
    const uint32_t cl = rem(v);
    if (cl < 8) return;
    const uint32_t hl = (p[0] & 0x7) == 0 ? 8 : 12;
    const uint32_t plen = be16(p + 2) + 8;
    if (hl > cl || plen < hl || plen > cl) return;
    o->t.hdr0 = p[0];
    o->t.hdr1 = p[1];
    o->t.id = be32(p + 4);
    o->t.aux = hl == 12 ? (uint16_t)be16(p + 8) : 0;
    view_t x = {v->f, v->s, v->s + plen};                    /* payload(): trim ... */
    x.s += hl;                                               /* ... advance */
    if ((p[0] >> 5) != 1 || p[1] != 255) {
        o->t.status = RPKT_T_NOT_TPDU;
        o->t.inner_off = (uint16_t)x.s;
        return;
    }
    uint32_t next = (p[0] & 0x4) ? p[11] : 0;                /* next_extention_header :275 */
    for (int k = 0; next != 0; k++) {
        uint32_t nn = 0, ehl = k < RPKT_MAX_GTP_EXT ? gtp_ext(&x, next, &nn) : 0;
        if (ehl == 0) {
            o->t.status = RPKT_T_EXT_BAD;
            o->t.inner_off = (uint16_t)x.s;
            return;
        }
        x.s += ehl;                                          /* payload(): advance */
        next = nn;
    }
    uint32_t ver = rem(&x) ? chunk(&x)[0] >> 4 : 0;
    inner_by_type(o, ver == 4 ? 0x0800 : (ver == 6 ? 0x86dd : 0), x.s, x.e, flags);
}

/* GreGroup::group_parse (gre/generated.rs:800-820): chunk >= 4, then by (checksum_present,
 * routing_present, key_present, version, protocol_type): (0, 0, 1, 1, 0x880B) ->
 * GreForPPTP::parse (:371-386: chunk >= 8, header_len gre/mod.rs:87-101 <= chunk,
 * payload_len + header_len <= remaining); version 0 -> Gre::parse (:33-44: header_len
 * gre/mod.rs:68-85 in [4, chunk]); else Err.  Gre getters: checksum :236-241 (C or R),
 * key :260-267 (K; after the checksum word when C or R), protocol_type :77-81;
 * payload() :85-92: advance(header_len).  gre_test.rs:20-99. */
static void gre(const view_t* v, uint32_t flags, tun_out_t* o) {
    const uint8_t* p = chunk(v);
    const uint32_t cl = rem(v);
    if (cl < 4) return;
    const uint32_t c = p[0] >> 7, r = (p[0] >> 6) & 1, k = (p[0] >> 5) & 1, ver = p[1] & 7;
    const uint32_t pt = be16(p + 2);
    if (c == 0 && r == 0 && k == 1 && ver == 1 && pt == 0x880b) {
        if (cl < 8) return;
        const uint32_t ind = be16(p);
        const uint32_t hl = 8 + ((ind & 0x1000) ? 4 : 0) + ((ind & 0x0080) ? 4 : 0);
        if (hl > cl || be16(p + 4) + hl > cl) return;
        o->t.hdr0 = p[0];
        o->t.hdr1 = p[1];
        o->t.id = be32(p + 4);                               /* payload_len, call_id */
        o->t.status = RPKT_T_INNER_UNKNOWN;                  /* PPP, not an IP packet */
        o->t.inner_off = (uint16_t)(v->s + hl);
        o->t.inner_type = (uint16_t)pt;
        return;
    }
    if (ver != 0) return;
    const uint32_t hl = 4 + ((c | r) ? 4 : 0) + (k ? 4 : 0) + (((p[0] >> 4) & 1) ? 4 : 0);
    if (hl > cl) return;
    o->t.hdr0 = p[0];
    o->t.hdr1 = p[1];
    o->t.aux = (c | r) ? (uint16_t)be16(p + 4) : 0;
    o->t.id = k ? be32(p + ((c | r) ? 8 : 4)) : 0;
    inner_by_type(o, pt, v->s + hl, v->e, flags);
}

void oracle_tunnel_one(const uint8_t* f, uint32_t len, uint32_t flags, rpkt_rec_t* outer,
                       rpkt_tun_t* tun, rpkt_rec_t* inner) {
    oracle_parse_one(f, len, flags, outer);
    tun_out_t o;
    memset(&o, 0, sizeof(o));
    o.start = -1;
    o.t.status = RPKT_T_NONE;
    const uint32_t proto = outer->ip_protocol;                /* byte 33, IPv4 and IPv6 */
    if (outer->status == RPKT_S_OK && proto == 17) {
        /* Udp::payload() view: [payload_off, + payload_len) (udp/generated.rs:66-76) */
        uint32_t dp = outer->dst_port, sp = outer->src_port;
        uint32_t port = (dp == 4789 || dp == 2152) ? dp : ((sp == 4789 || sp == 2152) ? sp : 0);
        if (port) {
            view_t v = {f, outer->payload_off, (uint32_t)outer->payload_off + outer->payload_len};
            set(&o, port == 4789 ? RPKT_TUN_VXLAN : RPKT_TUN_GTPU, RPKT_T_BAD, v.s);
            if (port == 4789) vxlan(&v, flags, &o);
            else gtpu(&v, flags, &o);
        }
    } else if (outer->status == RPKT_S_L4_OTHER && proto == 47 &&
               (oracle_rec_is_ip6(outer) || (outer->ip_frag & 0x1fff) == 0)) {
        /* Ipv4::payload() / the IPv6 chain's cursor: [l4_off, + payload_len) */
        view_t v = {f, outer->l4_off, (uint32_t)outer->l4_off + outer->payload_len};
        set(&o, RPKT_TUN_GRE, RPKT_T_BAD, v.s);
        gre(&v, flags, &o);
    }
    *tun = o.t;
    memset(inner, 0, sizeof(*inner));
    if (o.t.status != RPKT_T_OK) {
        inner->status = RPKT_S_NO_INNER;
        return;
    }
    const uint32_t n = o.ie - o.is;
    if (o.start == 0) oracle_parse_one(f + o.is, n, flags, inner);
    else oracle_parse_at_ip(f + o.is, n, flags, (uint16_t)o.start, inner);
    /* offsets in the outer frame: the fields this record reached (0 otherwise) */
    const int st = inner->status;
    const int v6 = oracle_rec_is_ip6(inner);
    const int l3_set = !(st == RPKT_S_ETH_SHORT || st == RPKT_S_VLAN_SHORT || st == RPKT_S_NOT_IPV4);
    const int l4_set = l3_set && (v6 ? !(st == RPKT_S_IP6_SHORT || st == RPKT_S_IP6_BAD_LEN)
                                     : !(st >= RPKT_S_IP_SHORT && st <= RPKT_S_IP_TOT_GT_LEN));
    if (l3_set) inner->l3_off = (uint16_t)(inner->l3_off + o.is);
    if (l4_set) {
        inner->l4_off = (uint16_t)(inner->l4_off + o.is);
        inner->payload_off = (uint16_t)(inner->payload_off + o.is);
        if (v6) {
            uint8_t* blk = (uint8_t*)inner + 24;             /* ip6_pdst_off, bytes 34..35 */
            uint16_t pd;
            memcpy(&pd, blk + 10, 2);
            pd = (uint16_t)(pd + o.is);
            memcpy(blk + 10, &pd, 2);
        }
    }
}

void oracle_tunnel_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                         uint32_t stride, uint32_t frame_len, uint32_t n, uint32_t flags,
                         rpkt_rec_t* outer, rpkt_tun_t* tun, rpkt_rec_t* inner) {
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
        oracle_tunnel_one(frames + off, (uint32_t)len, flags, &outer[i], &tun[i], &inner[i]);
    }
}

/* The flow event rpkt_gpu_parse_tunnel_batch writes with RPKT_F_FLOW_EV: the inner
 * record's when the tunnel decoded, else the outer record's (include/rpkt_gpu.h). */
void oracle_tunnel_flow_events(const rpkt_rec_t* outer, const rpkt_tun_t* tun,
                               const rpkt_rec_t* inner, uint32_t n, uint32_t n_buckets,
                               uint64_t* ev) {
    for (uint32_t i = 0; i < n; i++)
        ev[i] = oracle_flow_event(tun[i].status == RPKT_T_OK ? &inner[i] : &outer[i], n_buckets);
}
