// readbw.hip — development microbenchmark (not part of the engine): what HBM gives a
// pure 16-B/lane read stream over a config-3-sized buffer (1.573 GB), by access shape.
// Answers: is the parse at 1500 B bound by the read stream, or by how it reads?
//   hipcc --offload-arch=gfx950 -O3 -o tools/readbw tools/readbw.hip
//   ./tools/readbw [bytes]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, uint32_t off, int aux) {
    if (aux == 2) return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2);
    if (aux == 1) return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 1);
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
}

// A: grid-stride (what tools/ablate.py v14 measured)
template <int U>
__global__ __launch_bounds__(256) void grid_stride(const u32x4* __restrict__ in, uint32_t n16,
                                                   uint32_t* out) {
    const uint32_t T = gridDim.x * blockDim.x, t = blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    uint32_t i = t;
    for (; i + (U - 1) * T < n16; i += U * T) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = in[i + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
    }
    for (; i < n16; i += T) acc ^= in[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[t] = 1;
}

// B: one wave per contiguous segment of SEG bytes (the parse's 64-frame tile shape),
// U 16-B loads per lane in flight; AUX cache policy.  WPB waves per block.
template <int U, int AUX, int WPB>
__global__ __launch_bounds__(64 * WPB) void wave_seg(const uint8_t* in, uint32_t bytes, uint32_t seg,
                                                     uint32_t* out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t w = blockIdx.x * WPB + wid;
    const uint32_t s = w * seg;
    if (s >= bytes) return;
    const uint32_t e = s + seg < bytes ? s + seg : bytes;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)bytes, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t a = s + lane * 16; a < e; a += 1024 * U) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(r, a + u * 1024, AUX);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1;
}

// C: persistent waves walking segments with a grid stride (nseg segments, G waves)
template <int U, int AUX>
__global__ __launch_bounds__(256) void persist_seg(const uint8_t* in, uint32_t bytes, uint32_t seg,
                                                   uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t w0 = blockIdx.x * 4 + (threadIdx.x >> 6), G = gridDim.x * 4;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)bytes, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    const uint32_t nseg = (bytes + seg - 1) / seg;
    for (uint32_t w = w0; w < nseg; w += G) {
        const uint32_t s = w * seg, e = s + seg < bytes ? s + seg : bytes;
        for (uint32_t a = s + lane * 16; a < e; a += 1024 * U) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = ld(r, a + u * 1024, AUX);
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= x[u];
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1;
}

// D: copy reference: read stream + a 1/18.75 write stream (records at 1500 B: 80/1500)
template <int U, int ST>
__global__ __launch_bounds__(256) void seg_rw(const uint8_t* in, uint32_t bytes, uint32_t seg,
                                              u32x4* rec, uint32_t rec_per_seg) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t s = w * seg;
    if (s >= bytes) return;
    const uint32_t e = s + seg < bytes ? s + seg : bytes;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)bytes, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t a = s + lane * 16; a < e; a += 1024 * U) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(r, a + u * 1024, 2);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
    }
    for (uint32_t k = lane; k < rec_per_seg; k += 64) {
        u32x4* dst = &rec[(size_t)w * rec_per_seg + k];
        if constexpr (ST == 0) *dst = acc + k;
        else if constexpr (ST == 1) __builtin_nontemporal_store(acc + k, dst);
        else __builtin_amdgcn_raw_buffer_store_b128(acc + k, __builtin_amdgcn_make_buffer_rsrc((void*)rec, (short)0, (int)0x7fffffff, 0x00020000), (int)(((size_t)w * rec_per_seg + k) * 16), 0, ST == 2 ? 1 : 3);
    }
}

// E: read stream + records, the records of all 4 waves of a block written together at
// the end of the block (20 KB contiguous per block) after a barrier
__global__ __launch_bounds__(256) void seg_rw_block(const uint8_t* in, uint32_t bytes, uint32_t seg,
                                                    u32x4* rec, uint32_t rec_per_seg) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t s = w * seg;
    const uint32_t e = s + seg < bytes ? s + seg : bytes;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)bytes, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t a = s + lane * 16; a < e; a += 1024 * 8) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = ld(r, a + u * 1024, 2);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u];
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < 4 * rec_per_seg; k += 256)
        __builtin_nontemporal_store(acc + k, &rec[(size_t)blockIdx.x * 4 * rec_per_seg + k]);
}
// F: pure write stream
__global__ __launch_bounds__(256) void wr_only(u32x4* out, uint32_t n16) {
    const uint32_t T = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += T)
        __builtin_nontemporal_store(u32x4{i, i, i, i}, &out[i]);
}
// G: records written at the START of each wave's segment (then the read)
__global__ __launch_bounds__(256) void seg_wr_first(const uint8_t* in, uint32_t bytes, uint32_t seg,
                                                    u32x4* rec, uint32_t rec_per_seg, uint32_t* o) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t s = w * seg;
    if (s >= bytes) return;
    const uint32_t e = s + seg < bytes ? s + seg : bytes;
    for (uint32_t k = lane; k < rec_per_seg; k += 64)
        __builtin_nontemporal_store(u32x4{k, w, 0, 0}, &rec[(size_t)w * rec_per_seg + k]);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)bytes, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t a = s + lane * 16; a < e; a += 1024 * 8) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = ld(r, a + u * 1024, 2);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= x[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) o[threadIdx.x] = 1;
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        tot += ms;
        if (ms < best) best = ms;
    }
    return tot / 5;
}

int main(int argc, char** argv) {
    uint32_t bytes = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 1048576u * 1500u;
    uint8_t* buf;
    uint32_t* out;
    u32x4* rec;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMalloc(&rec, (size_t)1048576 * 80));
    CK(hipMemset(buf, 0x5a, bytes));
    // warm the clocks
    for (int i = 0; i < 200; ++i)
        hipLaunchKernelGGL((grid_stride<8>), dim3(4096), dim3(256), 0, 0, (const u32x4*)buf, bytes / 16, out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    auto rep = [&](const char* name, float ms) {
        printf("%-44s %8.1f us  %6.3f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    const uint32_t n16 = bytes / 16;
    rep("grid_stride U8 4096x256", timeit([&] {
        hipLaunchKernelGGL((grid_stride<8>), dim3(4096), dim3(256), 0, 0, (const u32x4*)buf, n16, out); }, reps));
    rep("grid_stride U8 2048x256", timeit([&] {
        hipLaunchKernelGGL((grid_stride<8>), dim3(2048), dim3(256), 0, 0, (const u32x4*)buf, n16, out); }, reps));
    rep("grid_stride U4 16384x256", timeit([&] {
        hipLaunchKernelGGL((grid_stride<4>), dim3(16384), dim3(256), 0, 0, (const u32x4*)buf, n16, out); }, reps));
    const uint32_t segs[] = {96000u};
    for (uint32_t seg : segs) {
        const uint32_t nw = (bytes + seg - 1) / seg;
        char nm[96];
        snprintf(nm, sizeof nm, "wave_seg %u U8 def 4w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<8, 0, 4>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, seg, out); }, reps));
        snprintf(nm, sizeof nm, "wave_seg %u U8 nt 4w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<8, 2, 4>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, seg, out); }, reps));
        snprintf(nm, sizeof nm, "wave_seg %u U4 nt 4w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<4, 2, 4>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, seg, out); }, reps));
        snprintf(nm, sizeof nm, "wave_seg %u U16 nt 4w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<16, 2, 4>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, seg, out); }, reps));
        snprintf(nm, sizeof nm, "wave_seg %u U8 nt 1w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<8, 2, 1>), dim3(nw), dim3(64), 0, 0, buf, bytes, seg, out); }, reps));
        snprintf(nm, sizeof nm, "wave_seg %u U8 slc1 4w", seg);
        rep(nm, timeit([&] { hipLaunchKernelGGL((wave_seg<8, 1, 4>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, seg, out); }, reps));
    }
    for (int g : {256}) {
        char nm[96];
        snprintf(nm, sizeof nm, "persist_seg 96000 U8 nt grid %d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((persist_seg<8, 2>), dim3(g), dim3(256), 0, 0, buf, bytes, 96000u, out); }, reps));
        snprintf(nm, sizeof nm, "persist_seg 96000 U8 def grid %d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL((persist_seg<8, 0>), dim3(g), dim3(256), 0, 0, buf, bytes, 96000u, out); }, reps));
    }
    {
        const uint32_t nw = (bytes + 95999) / 96000;
        rep("seg_rw 96000 U8 nt + 5120 B recs plain", timeit([&] {
            hipLaunchKernelGGL((seg_rw<8, 0>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u); }, reps));
        rep("seg_rw 96000 U8 nt + 5120 B recs nt", timeit([&] {
            hipLaunchKernelGGL((seg_rw<8, 1>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u); }, reps));
        rep("seg_rw 96000 U8 nt + 5120 B recs aux1", timeit([&] {
            hipLaunchKernelGGL((seg_rw<8, 2>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u); }, reps));
        rep("seg_rw 96000 U8 nt + 5120 B recs aux3", timeit([&] {
            hipLaunchKernelGGL((seg_rw<8, 3>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u); }, reps));
        rep("seg_rw_block 96000 nt + 20 KB recs/block", timeit([&] {
            hipLaunchKernelGGL(seg_rw_block, dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u); }, reps));
        rep("seg_wr_first 96000 nt, recs first", timeit([&] {
            hipLaunchKernelGGL(seg_wr_first, dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 320u, out); }, reps));
        float ms = timeit([&] { hipLaunchKernelGGL(wr_only, dim3(8192), dim3(256), 0, 0, rec, 1048576u * 5u); }, reps);
        printf("%-44s %8.1f us  %6.3f TB/s (of 84 MB)\n", "wr_only 84 MB nt", ms * 1e3, 83886080.0 / (ms * 1e-3) / 1e12);
        rep("seg_rw 96000 U8 nt + 0 recs", timeit([&] {
            hipLaunchKernelGGL((seg_rw<8, 1>), dim3((nw + 3) / 4), dim3(256), 0, 0, buf, bytes, 96000u, rec, 0u); }, reps));
    }
    CK(hipFree(buf));
    return 0;
}
