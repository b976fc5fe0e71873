// flow_reduce.cpp — config 4's multi-GPU shape through the C ABI only, the way a
// Rust or C++ receive host drives it: one shard of frames per visible GPU, parse
// with flow events, accumulate the per-flow counters on each GPU, then one RCCL
// all-reduce of the counters (rpkt_gpu_flow_reduce) over a communicator made by
// ncclCommInitAll.  Checks every counter row against the host's own count, using
// rpkt_flow_hash (the exported host copy of the device hash).
//   usage: flow_reduce [frames_per_gpu] [n_buckets] [n_gpus (0 = all visible)]
// Replaces the per-queue counters of rpkt-dpdk/examples/loopback_tx.rs:176-181 and
// the thread-per-queue split of rss_rx.rs:54-113.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rpkt_gpu.h"

static void put16(uint8_t* p, unsigned v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t* p, uint32_t v) { put16(p, v >> 16); put16(p + 2, v & 0xffff); }

// RFC 1071 sum of big-endian words (no complement), odd tail byte << 8
static uint32_t sum16(const uint8_t* p, size_t n, uint32_t acc = 0) {
    for (size_t i = 0; i + 1 < n; i += 2) acc += (uint32_t)(p[i] << 8 | p[i + 1]);
    if (n & 1) acc += (uint32_t)p[n - 1] << 8;
    return acc;
}
static uint16_t fold(uint32_t s) {
    while (s >> 16) s = (s & 0xffff) + (s >> 16);
    return (uint16_t)s;
}

struct Shard {
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> offs;
};

// Frame k of shard g: UDP or TCP over IPv4, one of 97 flows, 64..1500 B; every
// 13th frame has a bad IPv4 checksum, every 17th a bad L4 checksum, every 29th is
// ARP (does not parse to L4).
static void make_shard(Shard& s, uint32_t n, uint32_t g) {
    s.offs.assign(n + 1, 0);
    s.bytes.clear();
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t key = (k * 2654435761u + g * 40503u) % 97u;
        const bool tcp = key & 1, arp = (k % 29) == 28;
        const uint32_t len = 64 + (k * 37u + g * 11u) % 1437u;
        size_t o = s.bytes.size();
        s.offs[k] = (uint32_t)o;
        s.bytes.resize(o + len, 0);
        uint8_t* f = &s.bytes[o];
        for (uint32_t i = 0; i < len; i++) f[i] = (uint8_t)(i * 7 + k);
        const uint8_t mac[6] = {0x02, 0, 0, 0, 0, (uint8_t)g};
        memcpy(f, mac, 6);
        memcpy(f + 6, mac, 6);
        put16(f + 12, arp ? 0x0806 : 0x0800);
        if (arp) continue;
        uint8_t* ip = f + 14;
        const uint32_t tot = len - 14, l4 = tot - 20;
        ip[0] = 0x45; ip[1] = 0; put16(ip + 2, tot); put16(ip + 4, k & 0xffff); put16(ip + 6, 0x4000);
        ip[8] = 64; ip[9] = tcp ? 6 : 17; put16(ip + 10, 0);
        put32(ip + 12, 0x0a000000u | key); put32(ip + 16, 0xc0a81702u);
        uint8_t* t = ip + 20;
        put16(t, 1024 + key); put16(t + 2, tcp ? 443 : 53);
        if (tcp) {
            put32(t + 4, k); put32(t + 8, 0); t[12] = 5 << 4; t[13] = 0x18; put16(t + 14, 512);
            put16(t + 16, 0); put16(t + 18, 0);
        } else {
            put16(t + 4, l4); put16(t + 6, 0);
        }
        put16(ip + 10, (uint16_t)~fold(sum16(ip, 20)) ^ ((k % 13) == 12 ? 0x1111 : 0));
        uint32_t ps = sum16(ip + 12, 8) + (tcp ? 6u : 17u) + l4;
        uint16_t c = (uint16_t)~fold(sum16(t, l4, ps));
        if (!tcp && c == 0) c = 0xffff;
        if ((k % 17) == 16) {                   // wrong, and never the UDP "no checksum" 0
            c ^= 0x0101;
            if (!tcp && c == 0) c = 0x0202;
        }
        put16(t + (tcp ? 16 : 6), c);
    }
    s.offs[n] = (uint32_t)s.bytes.size();
}

#define HIP_OK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 2; } } while (0)

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 200000;
    const uint32_t nb = argc > 2 ? (uint32_t)atoi(argv[2]) : 8192;
    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    if (argc > 3 && atoi(argv[3]) > 0 && atoi(argv[3]) < ndev) ndev = atoi(argv[3]);
    if (ndev < 1) return 2;
    std::vector<int> devs(ndev);
    for (int g = 0; g < ndev; g++) devs[g] = g;
    std::vector<ncclComm_t> comms(ndev);
    if (ncclCommInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) {
        fprintf(stderr, "ncclCommInitAll failed\n");
        return 2;
    }
    const size_t ncnt = ((size_t)nb + 1) * 4;
    std::vector<uint64_t> expect(ncnt, 0);
    std::vector<Shard> shards(ndev);
    std::vector<uint8_t*> frames(ndev);
    std::vector<uint32_t*> offs(ndev);
    std::vector<rpkt_rec_t*> recs(ndev);
    std::vector<rpkt_flow_ev_t*> ev(ndev);
    std::vector<uint64_t*> ctr(ndev);
    std::vector<void*> ws(ndev);
    std::vector<hipStream_t> st(ndev);
    for (int g = 0; g < ndev; g++) {
        Shard& s = shards[g];
        make_shard(s, n, (uint32_t)g);
        for (uint32_t k = 0; k < n; k++) {          // the host's own count of this shard
            const uint8_t* f = &s.bytes[s.offs[k]];
            const uint32_t len = s.offs[k + 1] - s.offs[k];
            uint64_t* row = &expect[(size_t)nb * 4];
            if (f[12] == 0x08 && f[13] == 0x00) {
                const uint8_t* ip = f + 14;
                const uint8_t* t = ip + 20;
                const uint32_t src = (uint32_t)ip[12] << 24 | ip[13] << 16 | ip[14] << 8 | ip[15];
                const uint32_t dst = (uint32_t)ip[16] << 24 | ip[17] << 16 | ip[18] << 8 | ip[19];
                row = &expect[(size_t)(rpkt_flow_hash(src, dst, (uint16_t)(t[0] << 8 | t[1]),
                                                      (uint16_t)(t[2] << 8 | t[3]), ip[9]) % nb) * 4];
                row[2] += (k % 13) == 12;
                row[3] += (k % 17) == 16;
            }
            row[0] += 1;
            row[1] += len;
        }
        HIP_OK(hipSetDevice(g));
        HIP_OK(hipStreamCreate(&st[g]));
        HIP_OK(hipMalloc(&frames[g], s.bytes.size()));
        HIP_OK(hipMalloc(&offs[g], s.offs.size() * 4));
        HIP_OK(hipMalloc(&recs[g], (size_t)n * sizeof(rpkt_rec_t)));
        HIP_OK(hipMalloc(&ev[g], (size_t)n * sizeof(rpkt_flow_ev_t)));
        HIP_OK(hipMalloc(&ctr[g], ncnt * 8));
        HIP_OK(hipMalloc(&ws[g], rpkt_gpu_flow_workspace_bytes(n, nb) + 16));
        HIP_OK(hipMemcpy(frames[g], s.bytes.data(), s.bytes.size(), hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(offs[g], s.offs.data(), s.offs.size() * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemsetAsync(ctr[g], 0, ncnt * 8, st[g]));
    }
    int rc = RPKT_OK;
    for (int g = 0; g < ndev && rc == RPKT_OK; g++) {    // each GPU: parse + count its shard
        HIP_OK(hipSetDevice(g));
        rpkt_batch_t b = {frames[g], shards[g].bytes.size(), offs[g], 0, 0, n, 0};
        rc = rpkt_gpu_parse_batch(&b, RPKT_F_IP_SUM | RPKT_F_L4_SUM | RPKT_F_FLOW_EV, recs[g],
                                  ev[g], nb, st[g]);
        if (rc == RPKT_OK) rc = rpkt_gpu_flow_count(ev[g], n, nb, ctr[g], ws[g], st[g]);
    }
    if (rc != RPKT_OK) {
        fprintf(stderr, "parse/count failed rc=%d hip=%d\n", rc, rpkt_gpu_last_hip_error());
        return 1;
    }
    if (ncclGroupStart() != ncclSuccess) return 2;         // one process drives every GPU
    for (int g = 0; g < ndev && rc == RPKT_OK; g++) {
        HIP_OK(hipSetDevice(g));
        rc = rpkt_gpu_flow_reduce(ctr[g], nb, -1, comms[g], st[g]);
    }
    if (ncclGroupEnd() != ncclSuccess || rc != RPKT_OK) {
        fprintf(stderr, "flow_reduce failed rc=%d nccl=%d\n", rc, rpkt_gpu_last_coll_error());
        return 1;
    }
    int bad = 0;
    std::vector<uint64_t> got(ncnt);
    for (int g = 0; g < ndev; g++) {
        HIP_OK(hipSetDevice(g));
        HIP_OK(hipStreamSynchronize(st[g]));
        HIP_OK(hipMemcpy(got.data(), ctr[g], ncnt * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < ncnt; i++) bad += got[i] != expect[i];
    }
    uint64_t pkts = 0, bytes = 0, ipb = 0, l4b = 0;
    for (size_t r = 0; r <= nb; r++) {
        pkts += got[r * 4]; bytes += got[r * 4 + 1]; ipb += got[r * 4 + 2]; l4b += got[r * 4 + 3];
    }
    printf("%s; rccl %d\n", rpkt_gpu_build_info(), rpkt_gpu_coll_version());
    printf("%d GPU(s) x %u frames, %u buckets: pkts=%llu bytes=%llu ip_bad=%llu l4_bad=%llu "
           "unparsed=%llu; counter words differing from the host count on any GPU: %d\n",
           ndev, n, nb, (unsigned long long)pkts, (unsigned long long)bytes,
           (unsigned long long)ipb, (unsigned long long)l4b,
           (unsigned long long)got[(size_t)nb * 4], bad);
    for (int g = 0; g < ndev; g++) {
        (void)hipSetDevice(g);
        (void)hipFree(frames[g]); (void)hipFree(offs[g]); (void)hipFree(recs[g]);
        (void)hipFree(ev[g]); (void)hipFree(ctr[g]); (void)hipFree(ws[g]);
        (void)hipStreamDestroy(st[g]);
        ncclCommDestroy(comms[g]);
    }
    return (bad == 0 && pkts == (uint64_t)n * ndev) ? 0 : 1;
}
