// copybw.hip — development microbenchmark (not part of the engine): the HBM copy ceiling
// by access shape, to anchor the roofline the parse is compared with.  Counts read +
// written bytes.  Buffers are 1 GiB each (4x the Infinity Cache), so every launch
// streams from HBM.
//   hipcc --offload-arch=gfx950 -O3 -o tools/copybw tools/copybw.hip && ./tools/copybw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// grid-stride float4 copy, U loads in flight per thread; NTL / NTS: non-temporal
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void gs_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                               uint32_t n16) {
    const uint32_t T = gridDim.x * blockDim.x, t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t i = t;
    for (; i + (U - 1) * T < n16; i += U * T) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = NTL ? __builtin_nontemporal_load(&in[i + u * T]) : in[i + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NTS) __builtin_nontemporal_store(x[u], &out[i + u * T]);
            else out[i + u * T] = x[u];
        }
    }
    for (; i < n16; i += T) out[i] = in[i];
}

// one contiguous slice per block (256 threads x 16 B = 4 KiB per step), U steps in flight
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void blk_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                uint32_t n16) {
    const uint32_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint32_t s = blockIdx.x * per, e = s + per < n16 ? s + per : n16;
    for (uint32_t i = s + threadIdx.x; i < e; i += 256 * U) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = i + u * 256;
            x[u] = j < e ? (NTL ? __builtin_nontemporal_load(&in[j]) : in[j]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = i + u * 256;
            if (j < e) {
                if (NTS) __builtin_nontemporal_store(x[u], &out[j]);
                else out[j] = x[u];
            }
        }
    }
}

// write-only and read-only streams (each direction's own ceiling)
__global__ __launch_bounds__(256) void gs_fill(u32x4* __restrict__ out, uint32_t n16) {
    const uint32_t T = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += T)
        __builtin_nontemporal_store(u32x4{i, i, i, i}, &out[i]);
}
__global__ __launch_bounds__(256) void gs_read(const u32x4* __restrict__ in, uint32_t n16, uint32_t* sink) {
    const uint32_t T = gridDim.x * blockDim.x, t = blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    uint32_t i = t;
    for (; i + 7 * T < n16; i += 8 * T) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(&in[i + u * T]);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[t] = 1;
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
    const uint32_t n16 = (uint32_t)(bytes / 16);
    u32x4 *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 1 << 24));
    CK(hipMemset(a, 0x5a, bytes));
    CK(hipMemset(b, 0, bytes));
    for (int i = 0; i < 100; ++i)                       // clocks up
        hipLaunchKernelGGL((gs_copy<4, false, false>), dim3(4096), dim3(256), 0, 0, a, b, n16);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    auto rep = [&](const char* name, float ms, double moved) {
        printf("%-44s %8.1f us  %6.3f TB/s\n", name, ms * 1e3, moved / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    char nm[96];
    rep("hipMemcpyAsync D2D", timeit([&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); }, reps), 2.0 * bytes);
    rep("read only (nt, U8, 8192x256)", timeit([&] {
        hipLaunchKernelGGL(gs_read, dim3(8192), dim3(256), 0, 0, a, n16, sink); }, reps), bytes);
    rep("write only (nt, 8192x256)", timeit([&] {
        hipLaunchKernelGGL(gs_fill, dim3(8192), dim3(256), 0, 0, b, n16); }, reps), bytes);
    for (int g : {1024, 2048, 4096, 8192, 16384, 65536}) {
        snprintf(nm, sizeof nm, "gs_copy U1 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<1, false, false>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
        snprintf(nm, sizeof nm, "gs_copy U4 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<4, false, false>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
    }
    for (int g : {2048, 8192}) {
        snprintf(nm, sizeof nm, "gs_copy U4 ntl %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<4, true, false>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
        snprintf(nm, sizeof nm, "gs_copy U4 nts %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<4, false, true>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
        snprintf(nm, sizeof nm, "gs_copy U4 ntl+nts %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<4, true, true>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
        snprintf(nm, sizeof nm, "gs_copy U8 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_copy<8, false, false>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
    }
    for (int g : {1024, 2048, 4096, 8192}) {
        snprintf(nm, sizeof nm, "blk_copy U4 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((blk_copy<4, false, false>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
        snprintf(nm, sizeof nm, "blk_copy U4 ntl+nts %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((blk_copy<4, true, true>), dim3(g), dim3(256), 0, 0, a, b, n16); }, reps), 2.0 * bytes);
    }
    return 0;
}
