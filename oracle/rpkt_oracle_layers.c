/*
 * rpkt_oracle_layers.c — CPU restatement of the protocol layer walk, TEST
 * INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).
 *
 * Every protocol's parse / group_parse / payload is restated BY HAND from rpkt's
 * generated views (rpkt/src/<proto>/generated.rs, lines cited per function), not
 * from the pktfmt-derived table the kernel interprets (rpkt_amd/csrc/
 * rpkt_proto_table.h, tools/pktfmt_table.py): the two derivations check each other.
 * The cursor is rpkt's contiguous Cursor ([start, end) of one frame; chunk() ==
 * remaining(), rpkt/src/cursors.rs:34-99).  The dispatch between layers is the one
 * include/rpkt_gpu.h documents (the reference leaves it to the receive loop).
 */
#include <stdint.h>
#include <string.h>

#include "../include/rpkt_gpu.h"

typedef struct { const uint8_t* f; size_t s, e; } cur_t;

static uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* One parsed layer: its header length and the packet end after payload()'s trim. */
typedef struct { int proto; size_t hl; size_t end; } lay_t;

static size_t rem(const cur_t* c) { return c->e - c->s; }
static const uint8_t* ch(const cur_t* c) { return c->f + c->s; }

/* fixed-size header, no length fields: chunk_len >= H */
static int fixed(const cur_t* c, size_t H, int proto, lay_t* L) {
    if (rem(c) < H) return 0;
    L->proto = proto; L->hl = H; L->end = c->e;
    return 1;
}

/* header_len checked against chunk; optional packet_len (>= header_len, <= remaining)
 * and payload_len (+ header_len <= remaining) as the generated parses write them */
static int var(const cur_t* c, size_t H, size_t hl, int has_pkt, size_t pkt, int has_pay,
               size_t pay, int proto, lay_t* L) {
    size_t r = rem(c);
    if (r < H) return 0;
    if (hl < H || hl > r) return 0;
    if (has_pkt && (pkt < hl || pkt > r)) return 0;
    if (has_pay && pay + hl > r) return 0;
    L->proto = proto; L->hl = hl;
    L->end = has_pkt ? c->s + pkt : (has_pay ? c->s + hl + pay : c->e);   /* payload() trim */
    return 1;
}

/* ether/generated.rs:292-302 EtherGroup::group_parse; EtherFrame::parse :34-41;
 * EtherDot3Frame::parse :162-173 (payload_len + 14 <= remaining) */
static int g_ether(const cur_t* c, lay_t* L) {
    if (rem(c) < 14) return 0;
    uint32_t et = be16(ch(c) + 12);
    if (et >= 1536) return fixed(c, 14, RPKT_P_ETHER_ETHERFRAME, L);
    if (et <= 1500) return var(c, 14, 14, 0, 0, 1, et, RPKT_P_ETHER_ETHERDOT3FRAME, L);
    return 0;
}
/* vlan/generated.rs:312-322 VlanGroup; VlanFrame::parse :32-39; VlanDot3Frame :170-181 */
static int g_vlan(const cur_t* c, lay_t* L) {
    if (rem(c) < 4) return 0;
    uint32_t et = be16(ch(c) + 2);
    if (et >= 1536) return fixed(c, 4, RPKT_P_VLAN_VLANFRAME, L);
    if (et <= 1500) return var(c, 4, 4, 0, 0, 1, et, RPKT_P_VLAN_VLANDOT3FRAME, L);
    return 0;
}
/* ipv4/generated.rs:35-51 */
static int g_ipv4(const cur_t* c, lay_t* L) {
    if (rem(c) < 20) return 0;
    const uint8_t* p = ch(c);
    return var(c, 20, (size_t)(p[0] & 0xf) * 4, 1, be16(p + 2), 0, 0, RPKT_P_IPV4_IPV4, L);
}
/* ipv6/generated.rs:40-51 (payload_len + 40 <= remaining) */
static int g_ipv6(const cur_t* c, lay_t* L) {
    if (rem(c) < 40) return 0;
    return var(c, 40, 40, 0, 0, 1, be16(ch(c) + 4), RPKT_P_IPV6_IPV6, L);
}
/* ipv6/generated.rs:384-396 HopByHopOption, :241-253 DestOptions (8*len + 8),
 * :528-540 RoutingHeader (8*len + 8), :696-703 FragmentHeader (8 B),
 * :850-862 AuthenticationHeader (4*len + 8) */
static int g_hbh(const cur_t* c, lay_t* L) {
    if (rem(c) < 2) return 0;
    return var(c, 2, 8 * (size_t)ch(c)[1] + 8, 0, 0, 0, 0, RPKT_P_IPV6_HOPBYHOPOPTION, L);
}
static int g_dest(const cur_t* c, lay_t* L) {
    if (rem(c) < 2) return 0;
    return var(c, 2, 8 * (size_t)ch(c)[1] + 8, 0, 0, 0, 0, RPKT_P_IPV6_DESTOPTIONS, L);
}
static int g_routing(const cur_t* c, lay_t* L) {
    if (rem(c) < 8) return 0;
    return var(c, 8, 8 * (size_t)ch(c)[1] + 8, 0, 0, 0, 0, RPKT_P_IPV6_ROUTINGHEADER, L);
}
static int g_frag(const cur_t* c, lay_t* L) { return fixed(c, 8, RPKT_P_IPV6_FRAGMENTHEADER, L); }
static int g_auth(const cur_t* c, lay_t* L) {
    if (rem(c) < 12) return 0;
    return var(c, 12, 4 * (size_t)ch(c)[1] + 8, 0, 0, 0, 0, RPKT_P_IPV6_AUTHENTICATIONHEADER, L);
}
/* udp/generated.rs:31-42 */
static int g_udp(const cur_t* c, lay_t* L) {
    if (rem(c) < 8) return 0;
    return var(c, 8, 8, 1, be16(ch(c) + 4), 0, 0, RPKT_P_UDP_UDP, L);
}
/* tcp/generated.rs:34-45 */
static int g_tcp(const cur_t* c, lay_t* L) {
    if (rem(c) < 20) return 0;
    return var(c, 20, (size_t)(ch(c)[12] >> 4) * 4, 0, 0, 0, 0, RPKT_P_TCP_TCP, L);
}
/* icmpv4/generated.rs:2551-2575 Icmpv4::group_parse; members' parse: chunk >= their
 * fixed length (8; TimestampRequest/Reply 20; AddressMaskRequest/Reply 12) */
static int g_icmpv4(const cur_t* c, lay_t* L) {
    if (rem(c) < 1) return 0;
    switch (ch(c)[0]) {
        case 0: return fixed(c, 8, RPKT_P_ICMPV4_ECHOREPLY, L);
        case 3: return fixed(c, 8, RPKT_P_ICMPV4_DESTUNREACHABLE, L);
        case 4: return fixed(c, 8, RPKT_P_ICMPV4_SOURCEQUENCH, L);
        case 5: return fixed(c, 8, RPKT_P_ICMPV4_REDIRECT, L);
        case 8: return fixed(c, 8, RPKT_P_ICMPV4_ECHOREQUEST, L);
        case 9: return fixed(c, 8, RPKT_P_ICMPV4_ROUTERADVERTISEMENT, L);
        case 10: return fixed(c, 8, RPKT_P_ICMPV4_ROUTERSOLICITATION, L);
        case 11: return fixed(c, 8, RPKT_P_ICMPV4_TIMEEXCEEDED, L);
        case 12: return fixed(c, 8, RPKT_P_ICMPV4_PARAMETERPROBLEM, L);
        case 13: return fixed(c, 20, RPKT_P_ICMPV4_TIMESTAMPREQUEST, L);
        case 14: return fixed(c, 20, RPKT_P_ICMPV4_TIMESTAMPREPLY, L);
        case 15: return fixed(c, 8, RPKT_P_ICMPV4_INFORMATIONREQUEST, L);
        case 16: return fixed(c, 8, RPKT_P_ICMPV4_INFORMATIONREPLY, L);
        case 17: return fixed(c, 12, RPKT_P_ICMPV4_ADDRESSMASKREQUEST, L);
        case 18: return fixed(c, 12, RPKT_P_ICMPV4_ADDRESSMASKREPLY, L);
        case 42: return fixed(c, 8, RPKT_P_ICMPV4_EXTENDEDECHOREQUEST, L);
        case 43: return fixed(c, 8, RPKT_P_ICMPV4_EXTENDEDECHOREPLY, L);
        default: return 0;
    }
}
/* gre/mod.rs:68-101 gre_header_len / gre_pptp_header_len */
static size_t gre_hl(uint32_t ind) {
    return 4 + ((ind & 0xc000) ? 4 : 0) + ((ind & 0x2000) ? 4 : 0) + ((ind & 0x1000) ? 4 : 0);
}
static size_t gre_pptp_hl(uint32_t ind) {
    return 8 + ((ind & 0x1000) ? 4 : 0) + ((ind & 0x0080) ? 4 : 0);
}
/* gre/generated.rs:800-820 GreGroup::group_parse; Gre::parse :33-44;
 * GreForPPTP::parse :371-386 */
static int g_gre(const cur_t* c, lay_t* L) {
    if (rem(c) < 4) return 0;
    const uint8_t* p = ch(c);
    uint32_t ind = be16(p), ver = p[1] & 7;
    if ((p[0] >> 7) == 0 && ((p[0] >> 6) & 1) == 0 && ((p[0] >> 5) & 1) == 1 && ver == 1 &&
        be16(p + 2) == 0x880b) {
        if (rem(c) < 8) return 0;
        return var(c, 8, gre_pptp_hl(ind), 0, 0, 1, be16(p + 4), RPKT_P_GRE_GREFORPPTP, L);
    }
    if (ver == 0) return var(c, 4, gre_hl(ind), 0, 0, 0, 0, RPKT_P_GRE_GRE, L);
    return 0;
}
/* vxlan/generated.rs:32-39 */
static int g_vxlan(const cur_t* c, lay_t* L) { return fixed(c, 8, RPKT_P_VXLAN_VXLAN, L); }
/* gtpv1/generated.rs:33-49; header_len gtpv1.pktfmt (8, or 12 if any of E/S/PN) */
static int g_gtpv1(const cur_t* c, lay_t* L) {
    if (rem(c) < 8) return 0;
    const uint8_t* p = ch(c);
    size_t hl = (p[0] & 7) == 0 ? 8 : 12;
    return var(c, 8, hl, 1, 8 + (size_t)be16(p + 2), 0, 0, RPKT_P_GTPV1_GTPV1, L);
}
/* gtpv2/generated.rs:31-47; header_len 12 if teid_present (:66-68) else 8 */
static int g_gtpv2(const cur_t* c, lay_t* L) {
    if (rem(c) < 4) return 0;
    const uint8_t* p = ch(c);
    size_t hl = (p[0] & 0x8) ? 12 : 8;
    return var(c, 4, hl, 1, (size_t)be16(p + 2) + 4, 0, 0, RPKT_P_GTPV2_GTPV2, L);
}
/* mpls/generated.rs:32-39, arp/generated.rs:37-44, llc/generated.rs:31-38 */
static int g_mpls(const cur_t* c, lay_t* L) { return fixed(c, 4, RPKT_P_MPLS_MPLS, L); }
static int g_arp(const cur_t* c, lay_t* L) { return fixed(c, 28, RPKT_P_ARP_ARP, L); }
static int g_llc(const cur_t* c, lay_t* L) { return fixed(c, 3, RPKT_P_LLC_LLC, L); }
/* pppoe/generated.rs:358-368 PppoeGroup; PppoeSession::parse :33-44 (len + 6);
 * PppoeDiscovery::parse :209-220 */
static int g_pppoe(const cur_t* c, lay_t* L) {
    if (rem(c) < 2) return 0;
    const uint8_t* p = ch(c);
    if (p[1] == 0) {
        if (rem(c) < 8) return 0;
        return var(c, 8, 8, 1, (size_t)be16(p + 4) + 6, 0, 0, RPKT_P_PPPOE_PPPOESESSION, L);
    }
    if (rem(c) < 6) return 0;
    return var(c, 6, 6, 1, (size_t)be16(p + 4) + 6, 0, 0, RPKT_P_PPPOE_PPPOEDISCOVERY, L);
}
/* stp/generated.rs:1467-1480 StpGroup; StpTcnBpdu :34-41 (4), StpConfBpdu :167 (35),
 * RstpConfBpdu :471 (36), MstpConfBpdu :787-798 (version3_len + 38, :1065) */
static int g_stp(const cur_t* c, lay_t* L) {
    if (rem(c) < 4) return 0;
    const uint8_t* p = ch(c);
    uint32_t v = p[2], t = p[3];
    if (v == 0 && t == 128) return fixed(c, 4, RPKT_P_STP_STPTCNBPDU, L);
    if (v == 0 && t == 0) return fixed(c, 35, RPKT_P_STP_STPCONFBPDU, L);
    if (v == 2 && t == 2) return fixed(c, 36, RPKT_P_STP_RSTPCONFBPDU, L);
    if (v == 3 && t == 2) {
        if (rem(c) < 102) return 0;
        return var(c, 102, (size_t)be16(p + 36) + 38, 0, 0, 0, 0, RPKT_P_STP_MSTPCONFBPDU, L);
    }
    return 0;
}

typedef int (*group_fn)(const cur_t*, lay_t*);
static const group_fn GROUP_FNS[RPKT_N_GROUPS_HOST] = {
    g_ether, g_vlan, g_ipv4, g_ipv6, g_hbh, g_dest, g_routing, g_frag, g_auth, g_udp, g_tcp,
    g_icmpv4, g_gre, g_vxlan, g_gtpv1, g_gtpv2, g_mpls, g_arp, g_llc, g_pppoe, g_stp};

#define NEXT_END (-1)
#define NEXT_UNKNOWN (-2)

static int by_ethertype(uint32_t et) {
    switch (et) {
        case 0x0800: return RPKT_GROUP_IPV4;
        case 0x86dd: return RPKT_GROUP_IPV6;
        case 0x8100: case 0x88a8: return RPKT_GROUP_VLAN;
        case 0x0806: return RPKT_GROUP_ARP;
        case 0x8847: case 0x8848: return RPKT_GROUP_MPLS;
        case 0x8863: case 0x8864: return RPKT_GROUP_PPPOE;
        default: return NEXT_UNKNOWN;
    }
}
static int by_ip_proto(uint32_t p) {
    switch (p) {
        case 0: return RPKT_GROUP_IPV6_HOPBYHOP;
        case 1: return RPKT_GROUP_ICMPV4;
        case 4: return RPKT_GROUP_IPV4;
        case 6: return RPKT_GROUP_TCP;
        case 17: return RPKT_GROUP_UDP;
        case 41: return RPKT_GROUP_IPV6;
        case 43: return RPKT_GROUP_IPV6_ROUTING;
        case 44: return RPKT_GROUP_IPV6_FRAGMENT;
        case 47: return RPKT_GROUP_GRE;
        case 51: return RPKT_GROUP_IPV6_AUTH;
        case 59: return NEXT_END;                              /* no next header */
        case 60: return RPKT_GROUP_IPV6_DESTOPTS;
        default: return NEXT_UNKNOWN;
    }
}
/* by the first nibble of the payload (MPLS bottom of stack, GTP-U T-PDU) */
static int by_ip_version(const cur_t* c, uint32_t* key) {
    if (rem(c) < 1) return NEXT_END;
    *key = ch(c)[0] >> 4;
    return *key == 4 ? RPKT_GROUP_IPV4 : (*key == 6 ? RPKT_GROUP_IPV6 : NEXT_UNKNOWN);
}

/* The next group after layer `L` whose header starts at `h` (cursor c now at its
 * payload); *key = the value looked up. */
static int next_group(int proto, const uint8_t* h, const cur_t* c, uint32_t* key) {
    switch (proto) {
        case RPKT_P_ETHER_ETHERFRAME: *key = be16(h + 12); return by_ethertype(*key);
        case RPKT_P_VLAN_VLANFRAME: *key = be16(h + 2); return by_ethertype(*key);
        case RPKT_P_ETHER_ETHERDOT3FRAME: case RPKT_P_VLAN_VLANDOT3FRAME: return RPKT_GROUP_LLC;
        case RPKT_P_IPV4_IPV4:
            if ((be16(h + 6) & 0x1fff) != 0) return NEXT_END;    /* non-first fragment */
            *key = h[9]; return by_ip_proto(*key);
        case RPKT_P_IPV6_IPV6: *key = h[6]; return by_ip_proto(*key);
        case RPKT_P_IPV6_FRAGMENTHEADER:
            if ((be16(h + 2) >> 3) != 0) return NEXT_END;        /* non-first fragment */
            *key = h[0]; return by_ip_proto(*key);
        case RPKT_P_IPV6_HOPBYHOPOPTION: case RPKT_P_IPV6_DESTOPTIONS:
        case RPKT_P_IPV6_ROUTINGHEADER: case RPKT_P_IPV6_AUTHENTICATIONHEADER:
            *key = h[0]; return by_ip_proto(*key);
        case RPKT_P_UDP_UDP: {
            uint32_t dp = be16(h + 2), sp = be16(h);
            uint32_t port = (dp == 4789 || dp == 2152 || dp == 2123) ? dp
                          : ((sp == 4789 || sp == 2152 || sp == 2123) ? sp : 0);
            if (port == 0) return NEXT_END;
            *key = port;
            if (port == 4789) return RPKT_GROUP_VXLAN;
            if (rem(c) < 1) return NEXT_END;
            *key = ch(c)[0] >> 5;                              /* GTP version */
            return *key == 1 ? RPKT_GROUP_GTPV1 : (*key == 2 ? RPKT_GROUP_GTPV2 : NEXT_UNKNOWN);
        }
        case RPKT_P_GRE_GRE:
            *key = be16(h + 2);
            if (*key == 0x6558) return RPKT_GROUP_ETHER;        /* transparent bridging */
            return by_ethertype(*key);
        case RPKT_P_VXLAN_VXLAN: return RPKT_GROUP_ETHER;
        case RPKT_P_GTPV1_GTPV1:
            if ((h[0] & 0x4) || h[1] != 255) return NEXT_END;    /* ext headers / not T-PDU */
            return by_ip_version(c, key);
        case RPKT_P_MPLS_MPLS:
            if ((h[2] & 1) == 0) return RPKT_GROUP_MPLS;          /* not bottom of stack */
            return by_ip_version(c, key);
        case RPKT_P_PPPOE_PPPOESESSION:
            *key = be16(h + 6);
            return *key == 0x0021 ? RPKT_GROUP_IPV4 : (*key == 0x0057 ? RPKT_GROUP_IPV6 : NEXT_UNKNOWN);
        case RPKT_P_LLC_LLC: return (h[0] == 0x42 && h[1] == 0x42) ? RPKT_GROUP_STP : NEXT_END;
        default: return NEXT_END;   /* TCP, ICMPv4, ARP, STP, GTPv2, GRE for PPTP, PPPoE disc. */
    }
}

void oracle_layers_one(const uint8_t* f, uint32_t len, rpkt_layers_t* o) {
    memset(o, 0, sizeof(*o));
    cur_t c = {f, 0, len};
    int g = RPKT_GROUP_ETHER;
    for (;;) {
        if (o->n == RPKT_MAX_LAYERS) { o->stop = RPKT_L_MAX; break; }
        lay_t L;
        if (!GROUP_FNS[g](&c, &L)) { o->stop = RPKT_L_ERR; o->err_group = (uint8_t)g; break; }
        const uint8_t* h = f + c.s;
        o->proto[o->n] = (uint8_t)L.proto;
        o->off[o->n] = (uint16_t)c.s;
        o->n++;
        c.e = L.end;                                          /* payload(): trim ... */
        c.s += L.hl;                                          /* ... then advance */
        uint32_t key = 0;
        int nx = next_group(L.proto, h, &c, &key);
        if (nx == NEXT_END) { o->stop = RPKT_L_END; break; }
        if (nx == NEXT_UNKNOWN) {
            o->stop = RPKT_L_UNKNOWN; o->next_key = key; o->key_proto = (uint8_t)L.proto; break;
        }
        g = nx;
    }
    o->payload_off = (uint16_t)c.s;
    o->payload_len = (uint32_t)(c.e - c.s);
}

void oracle_layers_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                         uint32_t stride, uint32_t frame_len, uint32_t n, rpkt_layers_t* out) {
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
        oracle_layers_one(frames + off, (uint32_t)len, &out[i]);
    }
}
