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
// write-only by policy (AUX bits of buffer_store: 0 default, 1 glc/sc0, 2 slc/nt, 3 both)
// and by stores per thread per iteration
template <int AUX, int U>
__global__ __launch_bounds__(256) void gs_store(u32x4* __restrict__ out, uint32_t n16) {
    const uint32_t T = gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)0x7fffffff, 0x00020000);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * T < n16; i += U * T) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{i, i, i, i}, r, (int)((i + u * T) * 16u), 0, AUX);
    }
}
// one contiguous slice per wave (1 KiB per store instruction), U stores in flight
template <int AUX, int U>
__global__ __launch_bounds__(256) void wave_store(u32x4* __restrict__ out, uint32_t n16) {
    const uint32_t lane = threadIdx.x & 63, gw = blockIdx.x * 4 + threadIdx.x / 64, nw = gridDim.x * 4;
    const uint32_t units = n16 / 64, u0 = (uint32_t)((uint64_t)units * gw / nw), u1 = (uint32_t)((uint64_t)units * (gw + 1) / nw);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)0x7fffffff, 0x00020000);
    for (uint32_t u = u0; u < u1; u += U) {
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (u + k < u1)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{u, u, u, u}, r, (int)(((u + k) * 64u + lane) * 16u), 0, AUX);
    }
}

// wave-contiguous mixed stream (bench.py's wave_mix): each wave owns a slice of the input
// and one of the output in 1-KiB units and writes its output in proportion as it reads
template <int AUXL, int AUXS, bool COPY>
__global__ __launch_bounds__(256) void wave_mix(const u32x4* __restrict__ in, uint32_t in16,
                                                u32x4* __restrict__ out, uint32_t out16) {
    const uint32_t lane = threadIdx.x & 63, gw = blockIdx.x * 4 + threadIdx.x / 64, nw = gridDim.x * 4;
    const uint32_t in_u = in16 / 64, out_u = out16 / 64;
    const uint32_t i0 = (uint32_t)((uint64_t)in_u * gw / nw), i1 = (uint32_t)((uint64_t)in_u * (gw + 1) / nw);
    const uint32_t o0 = (uint32_t)((uint64_t)out_u * gw / nw), o1 = (uint32_t)((uint64_t)out_u * (gw + 1) / nw);
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)0x7fffffff, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    uint32_t o = o0;
    for (uint32_t i = i0; i < i1; i += 4) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)(i + u < i1 ? ((i + u) * 64u + lane) * 16u : 0x7fffff00u), 0, AUXL);
        if (COPY) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < i1) __builtin_amdgcn_raw_buffer_store_b128(x[u], ro, (int)(((i + u) * 64u + lane) * 16u), 0, AUXS);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= x[u];
            const uint32_t done = i + 4 < i1 ? i + 4 - i0 : i1 - i0;
            const uint32_t due = o0 + (uint32_t)((uint64_t)(o1 - o0) * done / (i1 - i0));
            for (; o < due; ++o) __builtin_amdgcn_raw_buffer_store_b128(acc + o, ro, (int)((o * 64u + lane) * 16u), 0, AUXS);
        }
    }
    if (!COPY)
        for (; o < o1; ++o) __builtin_amdgcn_raw_buffer_store_b128(acc + o, ro, (int)((o * 64u + lane) * 16u), 0, AUXS);
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
    const uint32_t w16 = (uint32_t)(((size_t)1 << 29) / 16);   // 512 MiB writes (the descriptor's range is int)
    for (int g : {1024, 4096, 16384}) {
        snprintf(nm, sizeof nm, "store aux0 U1 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_store<0, 1>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "store aux1 U1 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_store<1, 1>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "store aux2 U1 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_store<2, 1>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "store aux3 U1 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_store<3, 1>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "store aux2 U4 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((gs_store<2, 4>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "wave_store aux0 U4 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_store<0, 4>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
        snprintf(nm, sizeof nm, "wave_store aux2 U4 %dx256", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_store<2, 4>), dim3(g), dim3(256), 0, 0, b, w16); }, reps), (double)w16 * 16);
    }
    {
        const uint32_t h16 = (uint32_t)(((size_t)1 << 29) / 16);    // 512 MiB each way
        const uint32_t m_in = (uint32_t)((512u << 20) / 16), m_out = (uint32_t)((640u << 20) / 16);
        for (int g : {1024, 2048, 4096, 8192}) {
            snprintf(nm, sizeof nm, "wave_mix copy 1:1 def/def %dx256", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL((wave_mix<0, 0, true>), dim3(g), dim3(256), 0, 0, a, h16, b, h16); }, reps), 2.0 * h16 * 16);
            snprintf(nm, sizeof nm, "wave_mix copy 1:1 nt/nt %dx256", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL((wave_mix<2, 2, true>), dim3(g), dim3(256), 0, 0, a, h16, b, h16); }, reps), 2.0 * h16 * 16);
            snprintf(nm, sizeof nm, "wave_mix copy 1:1 nt/def %dx256", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL((wave_mix<2, 0, true>), dim3(g), dim3(256), 0, 0, a, h16, b, h16); }, reps), 2.0 * h16 * 16);
            snprintf(nm, sizeof nm, "wave_mix 64:80 nt/nt %dx256", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL((wave_mix<2, 2, false>), dim3(g), dim3(256), 0, 0, a, m_in, b, m_out); }, reps), 16.0 * (m_in + m_out));
            snprintf(nm, sizeof nm, "wave_mix 64:80 nt/def %dx256", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL((wave_mix<2, 0, false>), dim3(g), dim3(256), 0, 0, a, m_in, b, m_out); }, reps), 16.0 * (m_in + m_out));
        }
    }
    rep("hipMemsetAsync 512 MiB", timeit([&] { CK(hipMemsetAsync(b, 0, (size_t)w16 * 16, 0)); }, reps), (double)w16 * 16);
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
