// parse_batch.cpp — a non-Python host calling the engine through its C ABI only
// (include/rpkt_gpu.h): the shape of the call a Rust (cgo/FFI) or C++ caller makes.
// Builds one Ether/IPv4/UDP frame the way benches/rpkt/rpkt_build.rs:9-28 does,
// replicates it n times into a device batch, parses it and prints the getters of
// record 0 like benches/rpkt/rpkt_parse.rs:62-80 asserts them.
//   hipcc -O2 -Iinclude examples/parse_batch.cpp -Lrpkt_amd/_build -lrpkt_gpu \
//         -Wl,-rpath,$PWD/rpkt_amd/_build -o examples/parse_batch && ./examples/parse_batch
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "rpkt_gpu.h"

static void put16(uint8_t* p, unsigned v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000, stride = 64;
    uint8_t f[64] = {0};
    const uint8_t dst[6] = {0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0};
    const uint8_t src[6] = {0x00, 0x50, 0x56, 0xae, 0x76, 0xf5};
    memcpy(f, dst, 6); memcpy(f + 6, src, 6); put16(f + 12, 0x0800);
    uint8_t* ip = f + 14;
    ip[0] = 0x45; put16(ip + 2, 50); put16(ip + 4, 0x5c65); ip[8] = 128; ip[9] = 17;
    const uint8_t sa[4] = {192, 168, 29, 58}, da[4] = {192, 168, 29, 160};
    memcpy(ip + 12, sa, 4); memcpy(ip + 16, da, 4);
    uint8_t* udp = ip + 20;
    put16(udp, 60376); put16(udp + 2, 161); put16(udp + 4, 30); put16(udp + 6, 0xbc86);
    std::vector<uint8_t> host((size_t)n * stride);
    for (uint32_t i = 0; i < n; i++) memcpy(&host[(size_t)i * stride], f, stride);

    uint8_t* frames = nullptr;
    rpkt_rec_t* recs = nullptr;
    if (hipMalloc(&frames, host.size()) != hipSuccess ||
        hipMalloc(&recs, (size_t)n * sizeof(rpkt_rec_t)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    if (hipMemcpy(frames, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) return 2;
    rpkt_batch_t b = {frames, host.size(), nullptr, stride, 0, n, 0};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int rc = rpkt_gpu_parse_batch(&b, RPKT_F_IP_SUM | RPKT_F_L4_SUM, recs, nullptr, 0, nullptr);
    (void)hipEventRecord(e0, nullptr);
    for (int k = 0; k < 20 && rc == RPKT_OK; k++)
        rc = rpkt_gpu_parse_batch(&b, RPKT_F_IP_SUM | RPKT_F_L4_SUM, recs, nullptr, 0, nullptr);
    (void)hipEventRecord(e1, nullptr);
    if (rc != RPKT_OK || hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "parse failed rc=%d hip=%d\n", rc, rpkt_gpu_last_hip_error());
        return 1;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    rpkt_rec_t r;
    if (hipMemcpy(&r, recs, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("%s\n", rpkt_gpu_build_info());
    printf("status=%s ethertype=0x%04x proto=%u src=%u.%u.%u.%u ident=0x%04x sport=%u dport=%u "
           "udp_len=%u ck=0x%04x ip_sum=0x%04x l4_sum=0x%04x\n",
           rpkt_gpu_status_name(r.status), r.ethertype, r.ip_protocol, r.ip_src >> 24,
           (r.ip_src >> 16) & 255, (r.ip_src >> 8) & 255, r.ip_src & 255, r.ip_ident, r.src_port,
           r.dst_port, r.l4_word6, r.l4_checksum, r.ip_sum, r.l4_sum);
    printf("%u frames: %.2f us per batch, %.0f Mpps\n", n, ms * 1e3 / 20, n / (ms * 1e3 / 20));
    int ok = r.status == RPKT_S_OK && r.src_port == 60376 && r.dst_port == 161 &&
             r.ip_ident == 0x5c65 && r.l4_word6 == 30;
    (void)hipFree(frames);
    (void)hipFree(recs);
    return ok ? 0 : 1;
}
