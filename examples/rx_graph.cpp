// rx_graph.cpp — a receive loop of small batches, captured once as a HIP graph.
//
// A DPDK receive loop takes bursts of 32-64 frames per call (rpkt-dpdk/examples/
// loopback_rx.rs:17, 96-121) and keeps per-queue counters (loopback_tx.rs:176-181).  On
// the GPU a batch of tens of thousands of 64-B frames parses in a few microseconds, about
// what a dependent kernel launch costs, so a loop over many small batches is
// launch-bound.  One pass of this loop over a ring of `slots` batches is: per slot,
// rpkt_gpu_parse_batch with flow events into the pass's event buffer; then one
// rpkt_gpu_flow_count over the whole pass's events into the loop's counters.  The slots'
// parses are independent: with `streams` > 1 they are forked over that many HIP streams
// (events order the fork and the join before the counters), so their kernels can overlap.
// The pass runs eagerly (the ABI called per batch) and captured with
// hipStreamBeginCapture and replayed as one graph; both must give byte-identical records
// and counters.  The ring's device buffers are baked into the graph; a NIC (or a copy
// engine) refills the same slots between passes.
//   hipcc -O2 -Iinclude examples/rx_graph.cpp -Lrpkt_amd/_build -lrpkt_gpu \
//         -Wl,-rpath,$PWD/rpkt_amd/_build -o examples/rx_graph
//   ./examples/rx_graph [frames per slot] [slots] [timed passes] [streams]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "rpkt_gpu.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)
#define RC(x) do { int r_ = (x); if (r_ != RPKT_OK) { \
    fprintf(stderr, "%s:%d rc %d hip %d\n", __FILE__, __LINE__, r_, rpkt_gpu_last_hip_error()); \
    return 1; } } while (0)

static void put16(uint8_t* p, unsigned v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

// one Ether/IPv4/UDP frame of the rpkt_build.rs shape, source address and ports varied
static void make_frame(uint8_t* f, uint32_t k) {
    memset(f, 0, 64);
    const uint8_t dst[6] = {0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0};
    const uint8_t src[6] = {0x00, 0x50, 0x56, 0xae, 0x76, 0xf5};
    memcpy(f, dst, 6); memcpy(f + 6, src, 6); put16(f + 12, 0x0800);
    uint8_t* ip = f + 14;
    ip[0] = 0x45; put16(ip + 2, 50); put16(ip + 4, 0x5c65); ip[8] = 128; ip[9] = 17;
    ip[12] = 172; ip[13] = 74; ip[14] = (uint8_t)(k >> 8); ip[15] = (uint8_t)k;
    ip[16] = 192; ip[17] = 168; ip[18] = 23; ip[19] = 2;
    uint32_t s = 0;                                          // a valid IPv4 header checksum
    for (int i = 0; i < 20; i += 2) s += (uint32_t)(ip[i] << 8 | ip[i + 1]);
    while (s >> 16) s = (s & 0xffff) + (s >> 16);
    put16(ip + 10, ~s & 0xffff);
    uint8_t* udp = ip + 20;
    put16(udp, 1024 + (k % 4096)); put16(udp + 2, 161); put16(udp + 4, 30);
    memset(udp + 8, 0xae, 22);
}

struct Slot {
    uint8_t* frames;
    rpkt_rec_t* recs;
    rpkt_flow_ev_t* ev;          // the slot's part of the pass's event buffer
    rpkt_batch_t b;
};

struct Fork {                    // side streams and their fork / join events
    std::vector<hipStream_t> side;
    hipEvent_t fork;
    std::vector<hipEvent_t> join;
};

// one pass of the loop on stream st: the slots' parses (one rpkt_gpu_parse_ring call when
// `rs` is given, else one rpkt_gpu_parse_batch per slot, over the side streams when there
// are any), then the pass's flow counters
static int pass(std::vector<Slot>& ring, rpkt_flow_ev_t* ev_all, uint32_t n_ev, uint64_t* counters,
                void* ws, uint32_t nb, hipStream_t st, Fork& F,
                const std::vector<rpkt_ring_slot_t>* rs) {
    if (rs) {
        const int rc = rpkt_gpu_parse_ring(rs->data(), (uint32_t)rs->size(),
                                           RPKT_F_IP_SUM | RPKT_F_FLOW_EV, nb, st);
        return rc ? rc : rpkt_gpu_flow_count(ev_all, n_ev, nb, counters, ws, st);
    }
    const size_t S = F.side.size();
    if (S) {
        if (hipEventRecord(F.fork, st) != hipSuccess) return RPKT_E_HIP;
        for (hipStream_t x : F.side)
            if (hipStreamWaitEvent(x, F.fork, 0) != hipSuccess) return RPKT_E_HIP;
    }
    for (size_t q = 0; q < ring.size(); q++) {
        Slot& s = ring[q];
        const int rc = rpkt_gpu_parse_batch(&s.b, RPKT_F_IP_SUM | RPKT_F_FLOW_EV, s.recs, s.ev, nb,
                                            S ? F.side[q % S] : st);
        if (rc) return rc;
    }
    for (size_t k = 0; k < S; k++)
        if (hipEventRecord(F.join[k], F.side[k]) != hipSuccess ||
            hipStreamWaitEvent(st, F.join[k], 0) != hipSuccess)
            return RPKT_E_HIP;
    return rpkt_gpu_flow_count(ev_all, n_ev, nb, counters, ws, st);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 32768;      // frames per batch
    const uint32_t slots = argc > 2 ? (uint32_t)atoi(argv[2]) : 32;     // batches per pass
    const int reps = argc > 3 ? atoi(argv[3]) : 50;                     // timed passes
    const uint32_t streams = argc > 4 ? (uint32_t)atoi(argv[4]) : 4;    // parse streams
    const uint32_t nb = 1024, stride = 64, n_ev = n * slots;
    std::vector<uint8_t> host((size_t)n * stride);
    std::vector<Slot> ring(slots);
    rpkt_flow_ev_t* ev_all = nullptr;
    CK(hipMalloc(&ev_all, (size_t)n_ev * sizeof(rpkt_flow_ev_t)));
    for (uint32_t q = 0; q < slots; q++) {
        for (uint32_t i = 0; i < n; i++) make_frame(&host[(size_t)i * stride], q * 7919u + i);
        Slot& s = ring[q];
        CK(hipMalloc(&s.frames, host.size()));
        CK(hipMalloc(&s.recs, (size_t)n * sizeof(rpkt_rec_t)));
        CK(hipMemcpy(s.frames, host.data(), host.size(), hipMemcpyHostToDevice));
        s.ev = ev_all + (size_t)q * n;
        s.b = rpkt_batch_t{s.frames, host.size(), nullptr, stride, 0, n, 0};
    }
    const size_t cbytes = ((size_t)nb + 1) * 4 * sizeof(uint64_t);
    void* ws = nullptr;
    CK(hipMalloc(&ws, rpkt_gpu_flow_workspace_bytes(n_ev, nb)));
    uint64_t* counters = nullptr;
    CK(hipMalloc(&counters, cbytes));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    Fork one, many;                                   // no side streams / `streams` of them
    CK(hipEventCreateWithFlags(&many.fork, hipEventDisableTiming));
    for (uint32_t k = 0; k < (streams > 1 ? streams : 0); k++) {
        hipStream_t x;
        hipEvent_t e;
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        many.side.push_back(x);
        many.join.push_back(e);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("%s\n", rpkt_gpu_build_info());
    printf("ring: %u slots x %u frames x 64 B; per pass %u parses + one flow count of %u events\n",
           slots, n, slots, n_ev);

    std::vector<rpkt_ring_slot_t> rs(slots);
    for (uint32_t q = 0; q < slots; q++) rs[q] = rpkt_ring_slot_t{ring[q].b, ring[q].recs, ring[q].ev};

    std::vector<uint64_t> c_ref, c_got((size_t)(nb + 1) * 4);
    std::vector<rpkt_rec_t> r_ref, r_got((size_t)n);
    bool same = true;
    const double frames = (double)n_ev * reps;
    // eager / graph x {one stream, `streams` streams, the ring call}
    for (int mode = 0; mode < 6; mode++) {
        const bool graph = mode & 1;
        const int how = mode >> 1;                    // 0: one stream, 1: forked, 2: ring
        Fork& F = how == 1 ? many : one;
        if (how == 1 && F.side.empty()) continue;
        const std::vector<rpkt_ring_slot_t>* R = how == 2 ? &rs : nullptr;
        CK(hipMemset(counters, 0, cbytes));
        CK(hipMemset(ring[slots - 1].recs, 0, (size_t)n * sizeof(rpkt_rec_t)));
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        size_t nodes = 0;
        if (graph) {
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            const int rc_cap = pass(ring, ev_all, n_ev, counters, ws, nb, st, F, R);
            CK(hipStreamEndCapture(st, &g));
            RC(rc_cap);
            CK(hipGraphGetNodes(g, nullptr, &nodes));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        }
        auto run = [&]() -> int {
            if (graph) return hipGraphLaunch(ge, st) == hipSuccess ? RPKT_OK : RPKT_E_HIP;
            return pass(ring, ev_all, n_ev, counters, ws, nb, st, F, R);
        };
        RC(run());                                     // the warm pass
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) RC(run());
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(c_got.data(), counters, cbytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r_got.data(), ring[slots - 1].recs, (size_t)n * sizeof(rpkt_rec_t),
                     hipMemcpyDeviceToHost));
        uint64_t pkts = 0;
        for (uint32_t k = 0; k <= nb; k++) pkts += c_got[(size_t)k * 4];
        if (c_ref.empty()) {
            c_ref = c_got;
            r_ref = r_got;
        }
        const bool ok = pkts == (uint64_t)n_ev * (reps + 1) && c_got == c_ref &&
                        memcmp(r_got.data(), r_ref.data(), (size_t)n * sizeof(rpkt_rec_t)) == 0;
        same = same && ok;
        const std::string what = how == 2 ? std::string("ring call") :
            std::to_string(F.side.empty() ? 1u : (uint32_t)F.side.size()) + " stream(s)";
        printf("%-5s %-11s: %8.1f us per pass, %6.0f Mpps%s%s\n", graph ? "graph" : "eager",
               what.c_str(), ms * 1e3 / reps, frames / (ms * 1e3),
               graph ? (", " + std::to_string(nodes) + " nodes").c_str() : "",
               ok ? "" : "  MISMATCH");
        if (graph) {
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        }
    }
    printf("counters and records identical in every mode: %s\n", same ? "yes" : "NO");
    for (Slot& s : ring) {
        (void)hipFree(s.frames);
        (void)hipFree(s.recs);
    }
    (void)hipFree(ev_all);
    (void)hipFree(ws);
    (void)hipFree(counters);
    return same ? 0 : 1;
}
