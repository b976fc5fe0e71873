// slotbw.hip — development microbenchmark (not part of the engine): does a mixed
// read/write stream move faster when its reads and writes are separated in time across
// the whole chip?  A mixed stream (the parse's frames in, records out) reaches about
// 5.7 TB/s on MI355X while a pure read stream reaches 6.1 and a pure write stream 6.3
// (tools/copybw.hip).  Here every wave reads its input slice and owes output in
// proportion, as wave_mix does, but it issues writes only inside the write window of a
// time slot taken from the chip-wide 100-MHz real-time counter, and reads only outside
// it, holding at most KMAX owed 1-KiB units.  Bytes read + written are counted.
//   hipcc --offload-arch=gfx950 -O3 -o tools/slotbw tools/slotbw.hip && ./tools/slotbw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)0x7fffffff, 0x00020000);
}

// the reference: writes in proportion as the wave reads (bench.py's wave_mix), nt both ways
__global__ __launch_bounds__(256) void mix_ref(const u32x4* __restrict__ in, uint32_t in16,
                                               u32x4* __restrict__ out, uint32_t out16) {
    const uint32_t lane = threadIdx.x & 63, gw = blockIdx.x * 4 + threadIdx.x / 64, nw = gridDim.x * 4;
    const uint32_t in_u = in16 / 64, out_u = out16 / 64;
    const uint32_t i0 = (uint32_t)((uint64_t)in_u * gw / nw), i1 = (uint32_t)((uint64_t)in_u * (gw + 1) / nw);
    const uint32_t o0 = (uint32_t)((uint64_t)out_u * gw / nw), o1 = (uint32_t)((uint64_t)out_u * (gw + 1) / nw);
    const __amdgpu_buffer_rsrc_t ri = rsrc(in), ro = rsrc(out);
    u32x4 acc = {0, 0, 0, 0};
    uint32_t o = o0;
    for (uint32_t i = i0; i < i1; i += 4) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)(i + u < i1 ? ((i + u) * 64u + lane) * 16u : 0x7fffff00u), 0, 2);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= x[u];
        const uint32_t done = i + 4 < i1 ? i + 4 - i0 : i1 - i0;
        const uint32_t due = o0 + (uint32_t)((uint64_t)(o1 - o0) * done / (i1 - i0));
        for (; o < due; ++o) __builtin_amdgcn_raw_buffer_store_b128(acc + o, ro, (int)((o * 64u + lane) * 16u), 0, 2);
    }
    for (; o < o1; ++o) __builtin_amdgcn_raw_buffer_store_b128(acc + o, ro, (int)((o * 64u + lane) * 16u), 0, 2);
}

// time-slotted: reads outside the write window, owed writes inside it (period and window
// in 10-ns ticks of the real-time counter, the same clock on every CU)
template <uint32_t KMAX>
__global__ __launch_bounds__(256) void slot_mix(const u32x4* __restrict__ in, uint32_t in16,
                                                u32x4* __restrict__ out, uint32_t out16,
                                                uint32_t period, uint32_t wopen) {
    const uint32_t lane = threadIdx.x & 63, gw = blockIdx.x * 4 + threadIdx.x / 64, nw = gridDim.x * 4;
    const uint32_t in_u = in16 / 64, out_u = out16 / 64;
    const uint32_t i0 = (uint32_t)((uint64_t)in_u * gw / nw), i1 = (uint32_t)((uint64_t)in_u * (gw + 1) / nw);
    const uint32_t o0 = (uint32_t)((uint64_t)out_u * gw / nw), o1 = (uint32_t)((uint64_t)out_u * (gw + 1) / nw);
    const __amdgpu_buffer_rsrc_t ri = rsrc(in), ro = rsrc(out);
    u32x4 acc = {0, 0, 0, 0};
    uint32_t i = i0, o = o0;
    while (o < o1) {                                        // every branch is wave-uniform
        const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
        const bool wph = (t % period) < wopen;
        const uint32_t due = i >= i1 ? o1 : o0 + (uint32_t)((uint64_t)(o1 - o0) * (i - i0) / (i1 - i0));
        if ((wph || i >= i1) && o < due) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (o + u < due)
                    __builtin_amdgcn_raw_buffer_store_b128(acc + (o + u), ro, (int)(((o + u) * 64u + lane) * 16u), 0, 2);
            o = o + 4 < due ? o + 4 : due;
        } else if (!wph && i < i1 && due - o < KMAX) {
            u32x4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                x[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)(i + u < i1 ? ((i + u) * 64u + lane) * 16u : 0x7fffff00u), 0, 2);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= x[u];
            i = i + 4 < i1 ? i + 4 : i1;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    u32x4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0x5a, bytes));
    CK(hipMemset(b, 0, bytes));
    const int reps = 10;
    char nm[128];
    auto rep = [&](const char* name, float ms, double moved) {
        printf("%-52s %8.1f us  %6.3f TB/s\n", name, ms * 1e3, moved / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    // config 2's 64 : 80 mix (512 MiB in, 640 MiB out) and config 3's 1500 : 80
    struct Mix { const char* name; uint32_t in16, out16; } mixes[] = {
        {"64:80", (uint32_t)((512u << 20) / 16), (uint32_t)((640u << 20) / 16)},
        {"1500:80", (uint32_t)((960u << 20) / 16), (uint32_t)((51u << 20) / 16)},
    };
    for (int warm = 0; warm < 20; ++warm)
        hipLaunchKernelGGL(mix_ref, dim3(4096), dim3(256), 0, 0, a, mixes[0].in16, b, mixes[0].out16);
    CK(hipDeviceSynchronize());
    for (const Mix& m : mixes) {
        const double moved = 16.0 * ((double)m.in16 + m.out16);
        const double wf = (double)m.out16 / ((double)m.in16 + m.out16);
        for (int g : {4096, 1024}) {
            snprintf(nm, sizeof nm, "mix %s reference %dx256", m.name, g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(mix_ref, dim3(g), dim3(256), 0, 0, a, m.in16, b, m.out16); }, reps), moved);
            // windows of at least 5 ticks: with a 1-tick window a wave whose poll loop
            // aliases with the period can miss every window (the round-3 log's last
            // entries, 1500:80 at P=20, w=1, never finished)
            for (uint32_t P : {100u, 200u, 500u, 1000u, 2000u}) {
                for (double f : {wf * 0.9, wf, wf * 1.1}) {
                    const uint32_t w = (uint32_t)(P * f + 0.5) > 5u ? (uint32_t)(P * f + 0.5) : 5u;
                    snprintf(nm, sizeof nm, "mix %s slot P=%u w=%u K=64 %dx256", m.name, P, w, g);
                    rep(nm, timeit([&] { hipLaunchKernelGGL((slot_mix<64>), dim3(g), dim3(256), 0, 0, a, m.in16, b, m.out16, P, w); }, reps), moved);
                }
                const uint32_t w = (uint32_t)(P * wf + 0.5) > 5u ? (uint32_t)(P * wf + 0.5) : 5u;
                snprintf(nm, sizeof nm, "mix %s slot P=%u w=%u K=8 %dx256", m.name, P, w, g);
                rep(nm, timeit([&] { hipLaunchKernelGGL((slot_mix<8>), dim3(g), dim3(256), 0, 0, a, m.in16, b, m.out16, P, w); }, reps), moved);
            }
        }
    }
    return 0;
}
