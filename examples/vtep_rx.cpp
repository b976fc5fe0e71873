// vtep_rx.cpp — a VXLAN tunnel endpoint's receive loop through the C ABI only
// (include/rpkt_gpu.h): bursts of VXLAN frames from many tenants (VNIs) parsed as one
// ring (rpkt_gpu_parse_tunnel_ring), the inner flows counted per bucket
// (rpkt_gpu_flow_count), everything checked against the host's own view of the frames.
// The per-frame chain it replaces is the reference's tunnel test walk,
// Udp::payload -> Vxlan::parse -> EtherFrame::parse -> Ipv4 -> Udp (rpkt/tests/
// vlan_mpls_tests.rs:224-251), run in the rx loop of rpkt-dpdk/examples/loopback_rx.rs:96-121.
//   usage: vtep_rx [n_buckets]
//   hipcc -O2 -Iinclude examples/vtep_rx.cpp -Lrpkt_amd/_build -lrpkt_gpu \
//         -Wl,-rpath,$PWD/rpkt_amd/_build -o examples/vtep_rx && ./examples/vtep_rx
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rpkt_gpu.h"

#define HIP_OK(x)                                                          \
    do {                                                                   \
        if ((x) != hipSuccess) {                                           \
            fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);       \
            return 2;                                                      \
        }                                                                  \
    } while (0)

static void put16(uint8_t* p, unsigned v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t* p, uint32_t v) { put16(p, v >> 16); put16(p + 2, v & 0xffff); }

// RFC 1071 sum of big-endian 16-bit words (odd tail byte as the high byte), unfolded
static uint32_t sum16(const uint8_t* p, size_t n, uint32_t acc = 0) {
    for (size_t k = 0; k + 1 < n; k += 2) acc += (uint32_t)p[k] << 8 | p[k + 1];
    if (n & 1) acc += (uint32_t)p[n - 1] << 8;
    return acc;
}
static uint16_t fold_not(uint32_t acc) {
    while (acc >> 16) acc = (acc & 0xffff) + (acc >> 16);
    return (uint16_t)~acc;
}

struct Burst {
    uint32_t n, payload;
    std::vector<uint8_t> bytes;
};

// frame i of a burst: outer Ether / IPv4 / UDP 4789 / VXLAN (VNI of tenant i % 16) /
// inner Ether / IPv4 / UDP / payload; every 97th inner UDP checksum is corrupted
static uint32_t vni_of(uint32_t i) { return 5000 + (i % 16); }
static uint32_t inner_src(uint32_t b, uint32_t i) { return 10u << 24 | (b + 1) << 16 | (i & 0xffff); }
static uint32_t inner_dst(uint32_t i) { return 10u << 24 | 200u << 16 | (i % 16); }
static uint16_t inner_sport(uint32_t i) { return (uint16_t)(1000 + i % 7); }

static void make_frame(uint8_t* f, uint32_t b, uint32_t i, uint32_t payload) {
    const uint32_t len = 92 + payload;
    memset(f, 0, len);
    const uint8_t mac_a[6] = {0x02, 0, 0, 0, 0, 0x01}, mac_b[6] = {0x02, 0, 0, 0, 0, 0x02};
    memcpy(f, mac_a, 6); memcpy(f + 6, mac_b, 6); put16(f + 12, 0x0800);
    uint8_t* ip = f + 14;                                         // outer IPv4
    ip[0] = 0x45; put16(ip + 2, len - 14); ip[8] = 64; ip[9] = 17;
    put32(ip + 12, 0xc0a80101u); put32(ip + 16, 0xc0a80102u);
    put16(ip + 10, fold_not(sum16(ip, 20)));
    uint8_t* udp = ip + 20;                                       // outer UDP, checksum 0
    put16(udp, 49152 + i % 1024); put16(udp + 2, 4789); put16(udp + 4, len - 34);
    uint8_t* vx = udp + 8;                                        // VXLAN, I bit + VNI
    vx[0] = 0x08; vx[4] = (uint8_t)(vni_of(i) >> 16); vx[5] = (uint8_t)(vni_of(i) >> 8);
    vx[6] = (uint8_t)vni_of(i);
    uint8_t* ie = vx + 8;                                         // inner Ether
    memcpy(ie, mac_b, 6); memcpy(ie + 6, mac_a, 6); put16(ie + 12, 0x0800);
    uint8_t* iip = ie + 14;                                       // inner IPv4
    iip[0] = 0x45; put16(iip + 2, 28 + payload); iip[8] = 63; iip[9] = 17;
    put32(iip + 12, inner_src(b, i)); put32(iip + 16, inner_dst(i));
    put16(iip + 10, fold_not(sum16(iip, 20)));
    uint8_t* iu = iip + 20;                                       // inner UDP + payload
    put16(iu, inner_sport(i)); put16(iu + 2, 53); put16(iu + 4, 8 + payload);
    for (uint32_t k = 0; k < payload; ++k) iu[8 + k] = (uint8_t)(i * 7 + k);
    uint32_t acc = sum16(iip + 12, 8) + 17 + 8 + payload;         // pseudo header
    uint16_t c = fold_not(sum16(iu, 8 + payload, acc));
    if (c == 0) c = 0xffff;
    if (i % 97 == 96) c ^= 0x5a5a;
    put16(iu + 6, c);
}

int main(int argc, char** argv) {
    const uint32_t nb = argc > 1 ? (uint32_t)atoi(argv[1]) : 1024;
    Burst bursts[4] = {{32, 18, {}}, {64, 100, {}}, {1000, 600, {}}, {5000, 1400, {}}};
    const int S = 4;
    uint32_t total = 0;
    std::vector<uint64_t> expect((size_t)(nb + 1) * 4, 0);
    for (int b = 0; b < S; ++b) {
        Burst& B = bursts[b];
        const uint32_t len = 92 + B.payload;
        B.bytes.resize((size_t)B.n * len);
        for (uint32_t i = 0; i < B.n; ++i) {
            make_frame(&B.bytes[(size_t)i * len], b, i, B.payload);
            uint64_t* row = &expect[(size_t)(rpkt_flow_hash(inner_src(b, i), inner_dst(i),
                                                            inner_sport(i), 53, 17) % nb) * 4];
            row[0] += 1;
            row[1] += 42 + B.payload;                             // the inner frame's length
            row[3] += i % 97 == 96;
        }
        total += B.n;
    }

    // device buffers: one frame buffer and four record arrays per burst
    std::vector<rpkt_tun_ring_slot_t> slots(S);
    std::vector<uint8_t*> frames(S);
    std::vector<rpkt_rec_t*> outer(S), inner(S);
    std::vector<rpkt_tun_t*> tun(S);
    std::vector<rpkt_flow_ev_t*> ev(S);
    uint32_t nmax = 0;
    for (int b = 0; b < S; ++b) {
        const Burst& B = bursts[b];
        HIP_OK(hipMalloc(&frames[b], B.bytes.size()));
        HIP_OK(hipMalloc(&outer[b], (size_t)B.n * sizeof(rpkt_rec_t)));
        HIP_OK(hipMalloc(&inner[b], (size_t)B.n * sizeof(rpkt_rec_t)));
        HIP_OK(hipMalloc(&tun[b], (size_t)B.n * sizeof(rpkt_tun_t)));
        HIP_OK(hipMalloc(&ev[b], (size_t)B.n * sizeof(rpkt_flow_ev_t)));
        HIP_OK(hipMemcpy(frames[b], B.bytes.data(), B.bytes.size(), hipMemcpyHostToDevice));
        const uint32_t len = 92 + B.payload;
        slots[b].batch = rpkt_batch_t{frames[b], B.bytes.size(), nullptr, len, len, B.n, 0};
        slots[b].outer_dev = outer[b];
        slots[b].tun_dev = tun[b];
        slots[b].inner_dev = inner[b];
        slots[b].flow_ev_dev = ev[b];
        nmax = B.n > nmax ? B.n : nmax;
    }
    uint64_t* ctr = nullptr;
    void* ws = nullptr;
    const size_t ncnt = (size_t)(nb + 1) * 4;
    HIP_OK(hipMalloc(&ctr, ncnt * 8));
    HIP_OK(hipMalloc(&ws, rpkt_gpu_flow_workspace_bytes(nmax, nb) + 16));
    HIP_OK(hipMemset(ctr, 0, ncnt * 8));

    // the receive pass: one ring launch, then the counters of every burst's inner flows
    const uint32_t flags = RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_FLOW_EV;
    int rc = rpkt_gpu_parse_tunnel_ring(slots.data(), S, flags, nb, nullptr);
    for (int b = 0; b < S && rc == RPKT_OK; ++b)
        rc = rpkt_gpu_flow_count(ev[b], bursts[b].n, nb, ctr, ws, nullptr);
    if (rc != RPKT_OK || hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "ring/count failed rc=%d (%s) hip=%d\n", rc, rpkt_gpu_status_name(rc),
                rpkt_gpu_last_hip_error());
        return 1;
    }

    // what a VTEP reads back: the tunnel records (VNI) and the inner verdicts
    uint32_t tun_ok = 0, vni_ok = 0, inner_ok = 0, l4_bad = 0, l4_bad_expected = 0;
    for (int b = 0; b < S; ++b) {
        const uint32_t n = bursts[b].n;
        std::vector<rpkt_tun_t> t(n);
        std::vector<rpkt_rec_t> r(n);
        HIP_OK(hipMemcpy(t.data(), tun[b], n * sizeof(rpkt_tun_t), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(r.data(), inner[b], n * sizeof(rpkt_rec_t), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) {
            tun_ok += t[i].kind == RPKT_TUN_VXLAN && t[i].status == RPKT_T_OK;
            vni_ok += t[i].id == vni_of(i);
            const bool ok = r[i].status == RPKT_S_OK && r[i].ip_sum == 0xffff;
            inner_ok += ok && r[i].l4_sum == 0xffff;
            l4_bad += ok && r[i].l4_sum != 0xffff;
            l4_bad_expected += i % 97 == 96;
        }
    }
    std::vector<uint64_t> got(ncnt);
    HIP_OK(hipMemcpy(got.data(), ctr, ncnt * 8, hipMemcpyDeviceToHost));
    uint32_t rows_diff = 0;
    for (size_t k = 0; k < ncnt; k += 4)
        rows_diff += memcmp(&got[k], &expect[k], 32) != 0;
    printf("vtep_rx: %u frames in %d bursts, one ring launch: VXLAN tunnels decoded %u, VNI "
           "right %u, inner sums valid %u, inner UDP sums bad %u (corrupted %u); counter rows "
           "differing from the host count: %u\n",
           total, S, tun_ok, vni_ok, inner_ok, l4_bad, l4_bad_expected, rows_diff);
    const bool pass = tun_ok == total && vni_ok == total && l4_bad == l4_bad_expected &&
                      inner_ok + l4_bad == total && rows_diff == 0;
    return pass ? 0 : 1;
}
