// rpkt_gen.cpp — seeded synthetic frame generator (host C++), the loopback/
// synthetic ingress that replaces rpkt-dpdk's NIC rx for the benchmark.
//
// Frames are built the way rpkt's build side does it — headers prepended onto a
// payload with setters, checksums stamped last (benches/rpkt/rpkt_build.rs:9-28,
// rpkt-dpdk/examples/loopback_tx.rs:70-99 for the UDP template, :52-68 for the
// gen_ip_addrs flow spread) — with seeded fault injection on top (bad checksums,
// truncation, bad IHL / data offset / lengths) so every parse status occurs.
//
// Every frame i is a pure function of (config, seed, i, len_i): generation is
// parallel and reproducible.  The checksum arithmetic here is the product's own
// build-side RFC 1071 code, independent of oracle/.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#define RPKT_GEN_MAX_EXT 10

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {  // splitmix64
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
    bool chance(uint32_t per_10000) { return below(10000) < per_10000; }
};

inline void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
inline void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

// RFC 1071 one's-complement sum (big-endian words, odd tail << 8), folded.
uint32_t ones_sum(const uint8_t* d, size_t n, uint32_t acc = 0) {
    uint64_t a = acc;
    size_t i = 0;
    for (; i + 1 < n; i += 2) a += ((uint32_t)d[i] << 8) | d[i + 1];
    if (i < n) a += (uint32_t)d[i] << 8;
    while (a >> 16) a = (a & 0xffff) + (a >> 16);
    return (uint32_t)a;
}

const uint8_t kDmac[6] = {0xac, 0xdc, 0xca, 0x79, 0xe5, 0xc6};  // loopback_tx.rs:38
const uint8_t kSmac[6] = {0xac, 0xdc, 0xca, 0x79, 0xca, 0x86};  // loopback_tx.rs:39
const uint32_t kDip = (192u << 24) | (168u << 16) | (23u << 8) | 2u;  // loopback_tx.rs:40

// gen_ip_addrs(fst, snd, size)[k], loopback_tx.rs:52-68
uint32_t gen_ip(uint32_t fst, uint32_t snd, uint32_t size, uint32_t k) {
    k %= size;
    uint32_t third, fourth;
    if (k < (size / 250) * 250) { third = 2 + k / 250; fourth = 2 + k % 250; }
    else { third = 2 + size / 250; fourth = 2 + (k - (size / 250) * 250); }
    return (fst << 24) | (snd << 16) | (third << 8) | fourth;
}

struct Spec {
    int nvlan = 0;
    uint32_t tpid0 = 0x8100;
    int ihl = 5;
    bool tcp = false;
    int doff = 5;
    uint32_t src = 0, dst = kDip;
    uint32_t sport = 60376, dport = 161;  // loopback_tx.rs:41-42
    uint32_t ttl = 64, ident = 0;
    int pad = 0;             // Ethernet padding bytes past IPv4 packet_len
    bool bad_ip = false, bad_l4 = false, udp_zero = false;
    bool rand_payload = false;
    uint8_t payload_byte = 0xae;  // loopback_tx.rs:45
    int fault = 0;           // 0 none; 1 truncate; 2 bad ihl; 3 tot>len; 4 bad udp len/doff; 5 tot<ihl; 6 not ipv4; 7 other proto; 8 short L4
    // IPv6 (configs 10-12): extension header chain (next-header values 0 HopByHop,
    // 60 DestOptions, 43 Routing, 44 Fragment, 51 AH), the upper-layer protocol when it is
    // neither TCP nor UDP (0 = by `tcp`), and IPv6 faults: 1 payload_len > remaining,
    // 2 an extension header_len past the payload, 3 a non-atomic fragment, 4 AH header_len
    // 8, 5 a payload_len that cuts the first extension header short
    bool v6 = false;
    int n_ext = 0;
    uint8_t ext[RPKT_GEN_MAX_EXT] = {};
    uint32_t v6_proto = 0;
    int v6_fault = 0;
};

// Option bytes for an IPv4 header of `bytes` option space (NOP / RecordRoute / EOL).
void ipv4_options(uint8_t* o, int bytes, Rng& r) {
    int i = 0;
    while (i < bytes) {
        int left = bytes - i;
        uint32_t pick = r.below(3);
        if (pick == 1 && left >= 7) {            // Record Route (type 7): len, ptr, slots
            int slots = std::min((left - 3) / 4, 9);
            int len = 3 + 4 * slots;
            o[i] = 7; o[i + 1] = (uint8_t)len; o[i + 2] = 4;
            for (int k = 3; k < len; k++) o[i + k] = (uint8_t)r.next();
            i += len;
        } else if (pick == 2) {                 // EOL, then zero fill
            for (; i < bytes; i++) o[i] = 0;
        } else {
            o[i++] = 1;                          // NOP
        }
    }
}

// TCP options (NOP / MSS / WS / SACK-perm / TS) filling `bytes`.
void tcp_options(uint8_t* o, int bytes, Rng& r) {
    int i = 0;
    while (i < bytes) {
        int left = bytes - i;
        uint32_t pick = r.below(5);
        if (pick == 1 && left >= 4) { o[i] = 2; o[i + 1] = 4; put16(o + i + 2, 1460); i += 4; }
        else if (pick == 2 && left >= 3) { o[i] = 3; o[i + 1] = 3; o[i + 2] = 7; i += 3; }
        else if (pick == 3 && left >= 2) { o[i] = 4; o[i + 1] = 2; i += 2; }
        else if (pick == 4 && left >= 10) {
            o[i] = 8; o[i + 1] = 10; put32(o + i + 2, (uint32_t)r.next()); put32(o + i + 6, (uint32_t)r.next());
            i += 10;
        } else { o[i++] = 1; }
    }
}

// Build one frame of exactly `len` bytes from spec into out.
void build(const Spec& s, uint32_t len, uint8_t* out, Rng& r) {
    static thread_local uint8_t scratch[(1u << 16) + 1024];
    const uint32_t cap = std::min<uint32_t>(std::max<uint32_t>(len, 256) + 256, sizeof(scratch));
    memset(scratch, 0, cap);
    uint8_t* f = scratch;
    memcpy(f, kDmac, 6);
    memcpy(f + 6, kSmac, 6);
    uint32_t off = 12;
    if (s.nvlan >= 1) {
        put16(f + off, s.tpid0); off += 2;
        put16(f + off, (r.below(8) << 13) | (r.below(2) << 12) | r.below(4096)); off += 2;
    }
    if (s.nvlan >= 2) {
        put16(f + off, 0x8100); off += 2;
        put16(f + off, (r.below(8) << 13) | (r.below(2) << 12) | r.below(4096)); off += 2;
    }
    put16(f + off, s.fault == 6 ? 0x86dd : 0x0800); off += 2;
    const uint32_t l3 = off;
    const uint32_t ihl4 = (uint32_t)s.ihl * 4;
    const uint32_t l4h = s.tcp ? (uint32_t)s.doff * 4 : 8;
    // IPv4 packet_len fills the frame minus padding (never below the headers).
    int64_t tot = (int64_t)len - l3 - s.pad;
    if (tot < (int64_t)(ihl4 + l4h)) tot = ihl4 + l4h;
    const uint32_t l4 = l3 + ihl4;
    const uint32_t l4len = (uint32_t)tot - ihl4;
    // payload
    uint8_t* pl = f + l4 + l4h;
    int64_t pln = (int64_t)l4len - l4h;
    for (int64_t k = 0; k < pln; k++) pl[k] = s.rand_payload ? (uint8_t)r.next() : s.payload_byte;
    // L4 header (rpkt_build.rs:13-16 / loopback_tx.rs:73-77 for UDP)
    uint8_t* h4 = f + l4;
    put16(h4, s.sport);
    put16(h4 + 2, s.dport);
    if (s.tcp) {
        put32(h4 + 4, (uint32_t)r.next());
        put32(h4 + 8, (uint32_t)r.next());
        uint32_t flags = 0x10 | (r.below(2) << 3);
        put16(h4 + 12, ((uint32_t)s.doff << 12) | flags);
        put16(h4 + 14, 1024 + r.below(60000));
        put16(h4 + 16, 0);
        put16(h4 + 18, 0);
        tcp_options(h4 + 20, (int)l4h - 20, r);
    } else {
        put16(h4 + 4, l4len);
        put16(h4 + 6, 0);
    }
    // IPv4 header (rpkt_build.rs:18-22)
    uint8_t* ip = f + l3;
    ip[0] = (uint8_t)(0x40 | s.ihl);
    ip[1] = 0;
    put16(ip + 2, (uint32_t)tot);
    put16(ip + 4, s.ident);
    put16(ip + 6, 0x4000);
    ip[8] = (uint8_t)s.ttl;
    ip[9] = s.tcp ? 6 : 17;
    put16(ip + 10, 0);
    put32(ip + 12, s.src);
    put32(ip + 16, s.dst);
    ipv4_options(ip + 20, (int)ihl4 - 20, r);
    // checksums: L4 over pseudo header + segment, then IPv4 header
    uint32_t ps = (s.src >> 16) + (s.src & 0xffff) + (s.dst >> 16) + (s.dst & 0xffff) +
                  (s.tcp ? 6u : 17u) + l4len;
    uint32_t ck = (~ones_sum(h4, l4len, ps)) & 0xffff;
    if (!s.tcp && ck == 0) ck = 0xffff;                     // RFC 768
    if (s.bad_l4) { ck ^= 0x5a5a; if (ck == 0) ck = 1; }
    if (!s.tcp && s.udp_zero) ck = 0;
    put16(h4 + (s.tcp ? 16 : 6), ck);
    uint32_t ick = (~ones_sum(ip, ihl4)) & 0xffff;
    if (s.bad_ip) ick ^= 0x00ff;
    put16(ip + 10, ick);
    // structural faults (after checksums: the frame is then malformed on purpose)
    switch (s.fault) {
        case 2: ip[0] = (uint8_t)(0x40 | r.below(5)); break;                 // ihl < 5
        case 3: put16(ip + 2, (uint32_t)tot + 1 + r.below(64)); break;       // tot > remaining
        case 4:
            if (s.tcp) h4[12] = (uint8_t)((r.below(5)) << 4);                // doff < 5
            else put16(h4 + 4, r.chance(5000) ? r.below(8) : l4len + 1 + r.below(16));
            break;
        case 5: put16(ip + 2, r.below(ihl4)); break;                          // tot < ihl
        case 7: {                                                             // other protocol
            uint32_t p = r.below(256);
            ip[9] = (uint8_t)((p == 6 || p == 17) ? 47 : p);
            if (r.below(8) == 0) { ip[9] = 1; put16(ip + 2, ihl4); }          // empty ICMP
            break;
        }
        case 8: put16(ip + 2, ihl4 + r.below(s.tcp ? 20 : 8)); break;          // L4 too short
        default: break;
    }
    memcpy(out, f, len);
}

// IPv6 options (Pad1 / PadN / RouterAlert / a generic type) filling `bytes` of a
// HopByHop or DestOptions header (ipv6/generated.rs:1540-1552 types).
void ipv6_options(uint8_t* o, int bytes, Rng& r) {
    int i = 0;
    while (i < bytes) {
        int left = bytes - i;
        uint32_t pick = r.below(4);
        if (pick == 1 && left >= 4) { o[i] = 5; o[i + 1] = 2; put16(o + i + 2, r.below(3)); i += 4; }
        else if (pick == 2 && left >= 3) {
            int dl = std::min(left - 2, 1 + (int)r.below(6));
            o[i] = (uint8_t)(r.below(2) ? 11 : 0xc2); o[i + 1] = (uint8_t)dl;
            for (int k = 0; k < dl; k++) o[i + 2 + k] = (uint8_t)r.next();
            i += 2 + dl;
        } else if (left >= 2 && pick != 3) {
            o[i] = 1; o[i + 1] = (uint8_t)(left - 2);             // PadN to the end
            for (int k = 2; k < left; k++) o[i + k] = 0;
            i = bytes;
        } else { o[i++] = 0; }                                    // Pad1
    }
}

// Byte length of extension header kind `t` in s (drawn once per frame by the caller).
struct Ext6 { uint8_t type; uint32_t len; uint32_t rt_type, rt_n, rt_left; };

// One IPv6 frame of exactly `len` bytes: Ether [+ tags] + IPv6 + the extension chain of
// s.ext + UDP/TCP (or s.v6_proto), checksums with the IPv6 pseudo header over the
// routing header's final address when segments are left (RFC 8200 section 8.1; the
// product's own arithmetic, independent of oracle/).
void build6(const Spec& s, uint32_t len, uint8_t* out, Rng& r) {
    static thread_local uint8_t scratch[(1u << 16) + 2048];
    const uint32_t cap = std::min<uint32_t>(std::max<uint32_t>(len, 512) + 512, sizeof(scratch));
    memset(scratch, 0, cap);
    uint8_t* f = scratch;
    memcpy(f, kDmac, 6);
    memcpy(f + 6, kSmac, 6);
    uint32_t off = 12;
    if (s.nvlan >= 1) {
        put16(f + off, s.tpid0); off += 2;
        put16(f + off, (r.below(8) << 13) | (r.below(2) << 12) | r.below(4096)); off += 2;
    }
    if (s.nvlan >= 2) {
        put16(f + off, 0x8100); off += 2;
        put16(f + off, (r.below(8) << 13) | (r.below(2) << 12) | r.below(4096)); off += 2;
    }
    put16(f + off, 0x86dd); off += 2;
    const uint32_t l3 = off;
    // extension header sizes
    Ext6 e[RPKT_GEN_MAX_EXT];
    uint32_t ext_total = 0;
    for (int k = 0; k < s.n_ext; k++) {
        Ext6& x = e[k];
        x.type = s.ext[k];
        x.rt_type = x.rt_n = x.rt_left = 0;
        switch (x.type) {
            case 0: case 60: x.len = 8 * (1 + r.below(3)); break;
            case 43: {
                uint32_t pick = r.below(3);
                x.rt_type = pick == 0 ? 0 : (pick == 1 ? 4 : 2);
                x.rt_n = x.rt_type == 2 ? 1 : 1 + r.below(3);
                x.rt_left = r.below(x.rt_n + 1);
                x.len = 8 + 16 * x.rt_n;
                break;
            }
            case 44: x.len = 8; break;
            default: x.len = 12 + 4 * r.below(4); break;           // 51 AH
        }
        ext_total += x.len;
    }
    const uint32_t up = s.v6_proto ? s.v6_proto : (s.tcp ? 6u : 17u);
    const uint32_t l4h = up == 6 ? (uint32_t)s.doff * 4 : (up == 17 ? 8u : 8u);
    int64_t plen = (int64_t)len - l3 - 40 - s.pad;
    if (plen < (int64_t)(ext_total + l4h)) plen = ext_total + l4h;
    if (plen > 65535) plen = 65535;
    const uint32_t l4 = l3 + 40 + ext_total;
    const uint32_t l4len = (uint32_t)plen - ext_total;
    // payload
    uint8_t* pl = f + l4 + l4h;
    for (int64_t k = 0; k < (int64_t)l4len - l4h; k++)
        pl[k] = s.rand_payload ? (uint8_t)r.next() : s.payload_byte;
    // IPv6 header (ipv6/generated.rs:16-20 template, setters :107-135)
    uint8_t* ip = f + l3;
    put32(ip, (6u << 28) | (r.below(256) << 20) | r.below(1u << 20));
    put16(ip + 4, (uint32_t)plen);
    ip[6] = (uint8_t)(s.n_ext ? s.ext[0] : up);
    ip[7] = (uint8_t)(1 + r.below(255));
    put32(ip + 8, 0x20010db8u); put32(ip + 12, 0); put32(ip + 16, (uint32_t)r.next());
    put32(ip + 20, s.src);
    put32(ip + 24, 0x20010db8u); put32(ip + 28, 0xffff0000u); put32(ip + 32, 0);
    put32(ip + 36, s.dst);
    const uint8_t* pdst = ip + 24;
    // extension headers
    uint32_t c = l3 + 40;
    for (int k = 0; k < s.n_ext; k++) {
        uint8_t* h = f + c;
        const Ext6& x = e[k];
        h[0] = (uint8_t)(k + 1 < s.n_ext ? s.ext[k + 1] : up);
        switch (x.type) {
            case 0: case 60:
                h[1] = (uint8_t)(x.len / 8 - 1);
                ipv6_options(h + 2, (int)x.len - 2, r);
                break;
            case 43:
                h[1] = (uint8_t)(x.len / 8 - 1);
                h[2] = (uint8_t)x.rt_type;
                h[3] = (uint8_t)x.rt_left;
                put32(h + 4, x.rt_type == 4 ? ((x.rt_n - 1) << 24) : 0);
                for (uint32_t a = 0; a < x.rt_n; a++) {
                    put32(h + 8 + 16 * a, 0x20010db8u); put32(h + 12 + 16 * a, 0xeeee0000u + a);
                    put32(h + 16 + 16 * a, (uint32_t)r.next()); put32(h + 20 + 16 * a, (uint32_t)r.next());
                }
                if (x.rt_left > 0)
                    pdst = h + 8 + (x.rt_type == 4 ? 0 : 16 * (x.rt_n - 1));
                break;
            case 44:
                h[1] = 0;
                put16(h + 2, s.v6_fault == 3 ? ((1 + r.below(8000)) << 3) | r.below(2) : 0);
                put32(h + 4, (uint32_t)r.next());
                break;
            default:
                h[1] = (uint8_t)(x.len / 4 - 2);
                put32(h + 4, (uint32_t)r.next());
                put32(h + 8, (uint32_t)r.next());
                for (uint32_t k2 = 12; k2 < x.len; k2++) h[k2] = (uint8_t)r.next();
                break;
        }
        c += x.len;
    }
    // L4 header and its checksum over the IPv6 pseudo header (src, final dst, u32 length,
    // next header)
    uint8_t* h4 = f + l4;
    put16(h4, s.sport);
    put16(h4 + 2, s.dport);
    if (up == 6) {
        put32(h4 + 4, (uint32_t)r.next());
        put32(h4 + 8, (uint32_t)r.next());
        put16(h4 + 12, ((uint32_t)s.doff << 12) | 0x10 | (r.below(2) << 3));
        put16(h4 + 14, 1024 + r.below(60000));
        put16(h4 + 16, 0);
        put16(h4 + 18, 0);
        tcp_options(h4 + 20, (int)l4h - 20, r);
    } else if (up == 17) {
        put16(h4 + 4, l4len);
        put16(h4 + 6, 0);
    } else {
        for (uint32_t k = 4; k < 8; k++) h4[k] = (uint8_t)r.next();
    }
    if (up == 6 || up == 17) {
        uint32_t ps = ones_sum(ip + 8, 16, 0);
        ps = ones_sum(pdst, 16, ps);
        ps += (l4len >> 16) + (l4len & 0xffff) + up;
        uint32_t ck = (~ones_sum(h4, l4len, ps)) & 0xffff;
        if (up == 17 && ck == 0) ck = 0xffff;                    // RFC 768 / 8200
        if (s.bad_l4) { ck ^= 0x5a5a; if (ck == 0) ck = 1; }
        if (up == 17 && s.udp_zero) ck = 0;
        put16(h4 + (up == 6 ? 16 : 6), ck);
    }
    // structural faults (after the checksums)
    switch (s.v6_fault) {
        case 1: put16(ip + 4, (uint32_t)plen + 1 + r.below(64)); break;   // payload_len > remaining
        case 2:
            if (s.n_ext) f[l3 + 40 + 1] = (uint8_t)(200 + r.below(56));    // header_len past the payload
            break;
        case 5:                                                           // first extension header cut short
            if (s.n_ext) put16(ip + 4, r.below(2));
            break;
        case 4: {                                                         // AH with header_len 8
            uint32_t cc = l3 + 40;
            for (int k = 0; k < s.n_ext; k++) {
                if (e[k].type == 51) { f[cc + 1] = 0; break; }
                cc += e[k].len;
            }
            break;
        }
        default: break;
    }
    switch (s.fault) {
        case 4:
            if (up == 6) h4[12] = (uint8_t)((r.below(5)) << 4);
            else if (up == 17) put16(h4 + 4, r.chance(5000) ? r.below(8) : l4len + 1 + r.below(16));
            break;
        case 8: put16(ip + 4, ext_total + r.below(up == 6 ? 20 : 8)); break;   // L4 too short
        default: break;
    }
    memcpy(out, f, len);
}

// ---- tunnels (configs 13, 14): VXLAN, GTP-U with extension headers, GRE ----
// The inner frame is built by build() / build6() (an inner IP packet: that frame without
// its 14 Ethernet bytes), the tunnel and outer headers are prepended and the outer sums
// stamped last (RFC 7348 VXLAN over UDP 4789, 3GPP TS 29.281 GTP-U over UDP 2152, RFC
// 2784/2890 GRE), as rpkt's build side would (vlan_mpls_tests.rs:254-300,
// gtpv1_test.rs:236-282, gre_test.rs:213-278).  fuzz: random tunnel-header faults.
uint32_t put_ext(uint8_t* h, uint32_t type, uint32_t next, Rng& r) {
    // one GTP-U extension header of `type`, its next type last; returns its length
    uint32_t n;
    switch (type) {
        case 0x03: case 0x82: n = 8; break;                     // long PDU number
        case 0x81: case 0x83: case 0x84: case 0x85: n = 4 * (1 + r.below(3)); break;
        default: n = 4; break;                                  // 0x40 / 0xc0 / 0x20
    }
    h[0] = (uint8_t)(n / 4);
    for (uint32_t k = 1; k + 1 < n; k++) h[k] = (uint8_t)r.next();
    if (type == 0x84) h[1] = (uint8_t)((r.below(3) << 4) | (h[1] & 0xf));   // NrUp member
    if (type == 0x85) h[1] = (uint8_t)((r.below(2) << 4) | (h[1] & 0xf));   // Dl / Ul
    if (type == 0x84 && n < 8) { n = 8; h[0] = 2; for (uint32_t k = 2; k < 7; k++) h[k] = (uint8_t)r.next(); }
    h[n - 1] = (uint8_t)next;
    return n;
}

void build_tunnel(int config, uint32_t i, uint32_t len, uint8_t* out, Rng& r) {
    static thread_local uint8_t f[(1u << 16) + 2048];
    static const uint32_t kExtTypes[10] = {0xc0, 0x40, 0x20, 0x03, 0x82, 0x81, 0x83, 0x84, 0x85, 0xc0};
    const bool fuzz = config == 14;
    memset(f, 0, std::min<uint32_t>(len + 512, sizeof(f)));
    const uint32_t kind = r.below(10) < 4 ? 1u : (r.below(6) < 4 ? 2u : 3u);   // VXLAN, GTP-U, GRE
    // tunnel header bytes
    uint8_t th[64];
    uint32_t thl = 0, inner_eth = 0, gre_c = 0;
    uint32_t gtp_len_at = 0;
    if (kind == 1) {                                            // VXLAN: I flag, vni
        th[0] = 0x08 | (r.below(2) ? 0x80 : 0); th[1] = (uint8_t)(r.below(2) ? 0x48 : 0);
        put16(th + 2, r.below(65536)); put32(th + 4, (r.below(1u << 24)) << 8);
        thl = 8; inner_eth = 1;
    } else if (kind == 2) {                                     // GTP-U G-PDU, 0-3 extensions
        const uint32_t n_ext = r.below(4);
        const bool seq = r.below(2) == 1;
        th[0] = (uint8_t)(0x30 | (n_ext ? 0x04 : 0) | (seq ? 0x02 : 0));
        th[1] = 255;
        put32(th + 4, (uint32_t)r.next());
        thl = 8;
        if (n_ext || seq) {
            put16(th + 8, seq ? r.below(65536) : 0); th[10] = 0;
            uint32_t types[4];
            for (uint32_t k = 0; k < n_ext; k++) types[k] = kExtTypes[r.below(10)];
            th[11] = (uint8_t)(n_ext ? types[0] : 0);
            thl = 12;
            for (uint32_t k = 0; k < n_ext; k++)
                thl += put_ext(th + thl, types[k], k + 1 < n_ext ? types[k + 1] : 0, r);
        }
        gtp_len_at = 2;
    } else {                                                    // GRE v0: C / K / S bits
        const bool c = r.below(2) == 1, k = r.below(2) == 1, sq = r.below(4) == 0;
        inner_eth = r.below(5) == 0;
        th[0] = (uint8_t)((c ? 0x80 : 0) | (k ? 0x20 : 0) | (sq ? 0x10 : 0)); th[1] = 0;
        put16(th + 2, inner_eth ? 0x6558 : 0x0800);
        thl = 4;
        if (c) { put32(th + thl, 0); gre_c = thl; thl += 4; }
        if (k) { put32(th + thl, (uint32_t)r.next()); thl += 4; }
        if (sq) { put32(th + thl, (uint32_t)r.next()); thl += 4; }
    }
    const uint32_t outer_l4 = 14 + 20;
    const uint32_t tstart = outer_l4 + (kind == 3 ? 0 : 8);
    const uint32_t istart = tstart + thl;
    const uint32_t ilen = len > istart + 64 ? len - istart : 64;
    // the inner frame: config 11's mix (IPv4 / IPv6 + extension headers, TCP / UDP)
    {
        static const uint8_t kExt6[5] = {0, 60, 43, 44, 51};
        Spec si;
        si.v6 = r.below(4) == 0;
        si.tcp = r.below(2) == 1;
        si.src = gen_ip(10, 1, 8192, r.below(8192)); si.dst = gen_ip(10, 2, 4096, i);
        si.sport = 1024 + r.below(60000); si.dport = si.tcp ? 443 : 53;
        si.rand_payload = true;
        si.bad_ip = r.chance(100); si.bad_l4 = r.chance(100);
        si.ident = i & 0xffff;
        if (si.v6) { si.n_ext = (int)r.below(3); for (int k = 0; k < si.n_ext; k++) si.ext[k] = kExt6[r.below(5)]; }
        if (fuzz) {
            si.ihl = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            si.doff = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            si.fault = r.below(4) == 0 ? 2 + (int)r.below(7) : 0;
        }
        std::vector<uint8_t> tmp(ilen + 14 + 64);
        if (si.v6) build6(si, inner_eth ? ilen : ilen + 14, tmp.data(), r);
        else build(si, inner_eth ? ilen : ilen + 14, tmp.data(), r);
        memcpy(f + istart, tmp.data() + (inner_eth ? 0 : 14), ilen);
        if (!inner_eth && kind == 3 && si.v6) put16(th + 2, 0x86dd);
    }
    memcpy(f + tstart, th, thl);
    const uint32_t total = istart + ilen;                       // == len unless len < istart + 64
    // outer Ether + IPv4 (+ UDP)
    memcpy(f, kDmac, 6); memcpy(f + 6, kSmac, 6); put16(f + 12, 0x0800);
    uint8_t* ip = f + 14;
    ip[0] = 0x45; ip[1] = 0; put16(ip + 2, total - 14); put16(ip + 4, i & 0xffff);
    put16(ip + 6, 0x4000); ip[8] = 64; ip[9] = (uint8_t)(kind == 3 ? 47 : 17);
    put32(ip + 12, gen_ip(172, 74, 8192, r.below(8192))); put32(ip + 16, kDip);
    if (kind != 3) {
        uint8_t* u = f + outer_l4;
        put16(u, 1024 + r.below(60000)); put16(u + 2, kind == 1 ? 4789 : 2152);
        put16(u + 4, total - outer_l4);
        if (gtp_len_at) put16(f + tstart + 2, total - tstart - 8);   // GTP length
        const bool zero = kind == 1 && r.below(2) == 0;         // VXLAN: RFC 7348 allows 0
        uint32_t ps = ones_sum(ip + 12, 8, 0) + 17 + (total - outer_l4);
        uint32_t ck = zero ? 0 : ((~ones_sum(u, total - outer_l4, ps)) & 0xffff);
        if (!zero && ck == 0) ck = 0xffff;
        if (!zero && r.chance(100)) { ck ^= 0x5a5a; if (ck == 0) ck = 1; }
        put16(u + 6, ck);
    } else if (th[0] & 0x80) {                                  // the GRE checksum
        uint32_t ck = (~ones_sum(f + tstart, total - tstart, 0)) & 0xffff;
        if (r.chance(100)) ck ^= 0x0101;
        put16(f + tstart + gre_c, ck);
    }
    uint32_t ick = (~ones_sum(ip, 20)) & 0xffff;
    if (r.chance(100)) ick ^= 0x00ff;
    put16(ip + 10, ick);
    if (fuzz) {                                                 // tunnel-header faults
        switch (r.below(8)) {
            case 0: f[tstart + r.below(thl)] = (uint8_t)r.next(); break;     // any header byte
            case 1: if (kind == 2) put16(f + tstart + 2, r.below(65536)); break;   // GTP length
            case 2: if (kind == 2 && thl > 12) f[tstart + 12 + r.below(thl - 12)] = (uint8_t)r.next(); break;
            case 3: if (kind == 2) f[tstart + 1] = (uint8_t)r.below(256); break;  // message type
            case 4: if (kind == 3) f[tstart + 1] = (uint8_t)r.below(8); break;    // GRE version
            default: break;
        }
    }
    memcpy(out, f, len);
}

// config: 1 bench_rpkt (1k x 64B UDP, rpkt_build.rs header values), 2 64B UDP,
// 3 1500B TCP, 4 IMIX mixed, 5 VLAN/QinQ + options TCP, 6 fuzz (all statuses),
// 10 / 11 dual stack 64 B / 1500 B, 12 dual-stack fuzz (every IPv4 and IPv6 status).
Spec spec_for(int config, uint64_t seed, uint32_t i, uint32_t len, Rng& r) {
    Spec s;
    switch (config) {
        case 1:  // benches/rpkt/rpkt_build.rs:13-27
            s.src = (192u << 24) | (168u << 16) | (29u << 8) | 58u;
            s.dst = (192u << 24) | (168u << 16) | (29u << 8) | 160u;
            s.ttl = 128; s.ident = 0x5c65;
            break;
        case 2:
            s.src = gen_ip(172, 74, 8192, i);
            s.bad_ip = r.chance(100);
            s.ttl = 64; s.ident = i & 0xffff;
            break;
        case 3:
            s.tcp = true; s.src = gen_ip(172, 74, 8192, i); s.rand_payload = true;
            s.sport = 1024 + r.below(60000); s.dport = 80;
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            s.ident = i & 0xffff;
            break;
        case 4:
            s.tcp = r.below(2) == 1; s.src = gen_ip(172, 74, 8192, r.below(8192));
            s.sport = 1024 + r.below(4096); s.dport = s.tcp ? 80 : 53;
            s.rand_payload = true;
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            s.ident = i & 0xffff;
            break;
        case 5:
            s.nvlan = r.below(2) ? 2 : 1;
            s.tpid0 = s.nvlan == 2 ? 0x88a8 : 0x8100;
            s.ihl = 5 + (int)r.below(11);
            s.tcp = true; s.doff = 5 + (int)r.below(11);
            s.src = gen_ip(172, 74, 8192, r.below(8192)); s.sport = 1024 + r.below(60000);
            s.dport = 443; s.rand_payload = true;
            s.pad = r.chance(1000) ? (int)r.below(9) : 0;
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            break;
        case 10:  // dual stack, 64 B: IPv4/UDP (config 2's flows) or IPv6/UDP, 50/50
            s.v6 = r.below(2) == 1;
            s.src = gen_ip(172, 74, 8192, i);
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            s.ttl = 64; s.ident = i & 0xffff;
            break;
        case 11: {  // dual stack, 1500 B: IPv4 or IPv6 (0-3 extension headers), TCP or UDP
            static const uint8_t kExt[5] = {0, 60, 43, 44, 51};
            s.v6 = r.below(2) == 1;
            s.nvlan = r.below(4) == 0 ? 1 : 0;
            s.tcp = r.below(2) == 1; s.src = gen_ip(172, 74, 8192, r.below(8192));
            s.sport = 1024 + r.below(60000); s.dport = s.tcp ? 443 : 4433;
            s.rand_payload = true;
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            s.ident = i & 0xffff;
            if (s.v6) {
                s.n_ext = (int)r.below(4);
                for (int k = 0; k < s.n_ext; k++) s.ext[k] = kExt[r.below(5)];
            }
            break;
        }
        case 12: {  // dual-stack fuzz: every IPv4 and IPv6 status (configs 6's IPv4 faults)
            static const uint8_t kExt[5] = {0, 60, 43, 44, 51};
            static const uint8_t kOther[6] = {58, 50, 59, 89, 47, 1};
            s.v6 = r.below(3) != 0;
            s.nvlan = (int)r.below(4) == 0 ? (int)r.below(3) : 0;
            s.tpid0 = r.below(2) ? 0x88a8 : 0x8100;
            s.ihl = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            s.tcp = r.below(2) == 1;
            s.doff = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            s.src = (uint32_t)r.next(); s.dst = (uint32_t)r.next();
            s.sport = r.below(65536); s.dport = r.below(65536);
            s.rand_payload = true;
            s.pad = r.below(8) == 0 ? (int)r.below(12) : 0;
            s.bad_ip = r.chance(1000); s.bad_l4 = r.chance(1000);
            s.udp_zero = r.chance(500);
            if (s.v6) {
                s.n_ext = r.below(16) == 0 ? 7 + (int)r.below(3) : (int)r.below(4);
                for (int k = 0; k < s.n_ext; k++) s.ext[k] = kExt[r.below(5)];
                if (r.below(8) == 0) s.v6_proto = kOther[r.below(6)];
                const uint32_t f6 = r.below(12);
                s.v6_fault = f6 < 5 ? (int)f6 + 1 : 0;
                s.fault = r.below(6) == 0 ? (r.below(3) == 0 ? 4 : (r.below(2) ? 8 : 1)) : 0;
            } else {
                s.fault = r.below(4) == 0 ? 1 + (int)r.below(8) : 0;
            }
            break;
        }
        case 7:  // jumbo frames (rpkt-dpdk/examples/jumboframe_tx.rs:45, PACKET_LEN 8000)
            s.tcp = r.below(2) == 1; s.src = gen_ip(172, 74, 8192, r.below(8192));
            s.sport = 1024 + r.below(4096); s.dport = s.tcp ? 80 : 161;
            s.rand_payload = true;
            s.bad_ip = r.chance(100); s.bad_l4 = r.chance(100);
            s.ident = i & 0xffff;
            break;
        default: {  // 6 (and 8, chained): fuzz — every status, odd alignments, tiny frames
            s.nvlan = (int)r.below(4) == 0 ? (int)r.below(3) : 0;
            s.tpid0 = r.below(2) ? 0x88a8 : 0x8100;
            s.ihl = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            s.tcp = r.below(2) == 1;
            s.doff = r.below(4) == 0 ? 5 + (int)r.below(11) : 5;
            s.src = (uint32_t)r.next(); s.dst = (uint32_t)r.next();
            s.sport = r.below(65536); s.dport = r.below(65536);
            s.rand_payload = true;
            s.pad = r.below(8) == 0 ? (int)r.below(12) : 0;
            s.bad_ip = r.chance(1000); s.bad_l4 = r.chance(1000);
            s.udp_zero = r.chance(500);
            s.fault = r.below(4) == 0 ? 1 + (int)r.below(8) : 0;
            break;
        }
    }
    (void)seed; (void)len;
    return s;
}

void fill_range(int config, uint64_t seed, uint64_t first, const uint32_t* offsets,
                const uint32_t* lens, uint32_t stride, uint32_t lo, uint32_t hi, uint8_t* frames) {
    for (uint32_t i = lo; i < hi; i++) {
        const uint64_t gi = first + i;                    // global frame index
        Rng r(seed * 0x100000001b3ull ^ (0x9e3779b97f4a7c15ull * (gi + 1)));
        uint32_t len = lens[i];
        uint64_t off = offsets ? offsets[i] : (uint64_t)i * stride;
        Spec s = spec_for(config, seed, (uint32_t)gi, len, r);
        if (config == 13 || config == 14) {
            if (config == 14 && r.below(8) == 0) {          // truncated tunnel frames
                std::vector<uint8_t> tmp(len + 200);
                build_tunnel(config, (uint32_t)gi, len + 200, tmp.data(), r);
                memcpy(frames + off, tmp.data(), len);
            } else {
                build_tunnel(config, (uint32_t)gi, len, frames + off, r);
            }
            continue;
        }
        if ((config == 6 || config == 8 || config == 12) && s.fault == 1) {
            // truncation: build a full frame then cut it at a random length
            uint32_t full = len + 64;
            std::vector<uint8_t> tmp(full);
            Spec s2 = s;
            s2.fault = 0;
            if (s2.v6) build6(s2, full, tmp.data(), r);
            else build(s2, full, tmp.data(), r);
            memcpy(frames + off, tmp.data(), len);
        } else if (s.v6) {
            build6(s, len, frames + off, r);
        } else {
            build(s, len, frames + off, r);
        }
    }
}

}  // namespace

extern "C" {

// Frame lengths for a config (IMIX 64/570/1500 at 7:4:1; config 5 U[64,1518];
// fuzz U[0,300] with a 1500-B tail).  Deterministic in (config, seed, i).
void rpkt_gen_lengths(int config, uint64_t seed, uint64_t first, uint32_t n, uint32_t* lens) {
    for (uint32_t i = 0; i < n; i++) {
        Rng r(seed * 0x2545f4914f6cdd1dull ^ (0xd1b54a32d192ed03ull * (first + i + 1)));
        uint32_t L;
        switch (config) {
            case 1: case 2: case 10: L = 64; break;
            case 3: case 11: case 13: L = 1500; break;
            case 14: L = r.below(8) == 0 ? 40 + r.below(80) : 100 + r.below(1419); break;
            case 4: { uint32_t k = r.below(12); L = k < 7 ? 64 : (k < 11 ? 570 : 1500); break; }
            case 5: L = 64 + r.below(1518 - 64 + 1); break;
            case 7: L = 8000; break;
            case 8: {
                uint32_t k = r.below(4);
                L = k == 0 ? r.below(301) : (k == 1 ? 1000 + r.below(600) : 1600 + r.below(7401));
                break;
            }
            default: L = r.below(8) == 0 ? 1000 + r.below(600) : r.below(301); break;
        }
        lens[i] = L;
    }
}

// Fill frames [first, first + n) of the global sequence.  Packed layout: offsets
// (n+1 entries, relative to `frames`) given; strided: offsets NULL.
int rpkt_gen_fill(int config, uint64_t seed, uint64_t first, uint32_t n, const uint32_t* lens,
                  const uint32_t* offsets, uint32_t stride, uint8_t* frames, int threads) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n / 1024 + 1) threads = (int)(n / 1024 + 1);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        uint32_t lo = (uint32_t)((uint64_t)n * t / threads);
        uint32_t hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
        th.emplace_back(fill_range, config, seed, first, offsets, lens, stride, lo, hi, frames);
    }
    for (auto& x : th) x.join();
    return 0;
}

// Scatter packed frame bytes into mbuf-style segments: segment k copies lens[k]
// bytes from src + src_off[k] to dst + dst_off[k] (the chain layouts of gen.py).
int rpkt_gen_scatter(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off,
                     const uint32_t* lens, uint32_t n_segs, uint8_t* dst, int threads) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n_segs / 1024 + 1) threads = (int)(n_segs / 1024 + 1);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        uint32_t lo = (uint32_t)((uint64_t)n_segs * t / threads);
        uint32_t hi = (uint32_t)((uint64_t)n_segs * (t + 1) / threads);
        th.emplace_back([=] {
            for (uint32_t k = lo; k < hi; k++) memcpy(dst + dst_off[k], src + src_off[k], lens[k]);
        });
    }
    for (auto& x : th) x.join();
    return 0;
}

}  // extern "C"
