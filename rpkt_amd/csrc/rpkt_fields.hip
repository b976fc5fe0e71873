// rpkt_fields.hip — header-field getters over the protocol-layer walk.
//
// The getters rpkt generates for each protocol's header view (pktfmt/src/codegen/
// field.rs:115-250: `read_repr` / `read_multi_bytes` read bytes [start, end] big-endian,
// shift right by 7 - end bit, mask to the field width) evaluated for a list of
// (protocol, occurrence, bit offset, width) requests over every frame of a batch,
// on the layer offsets rpkt_gpu_layers_batch found.
//
// One lane per frame (its 64-B layer record read once, the requests sixteen at a time),
// values staged through LDS and stored as contiguous rows.  A field is three aligned
// dword loads and a funnel shift; the gather touches one or two lines per layer a request
// names, so the kernel is latency-bound on those loads, not HBM-bound.
#include "rpkt_common.h"

namespace {

constexpr int kFieldBlock = 128;            // LDS stage <= 128 * 65 * 4 = 33 KB

struct FieldReqs {
    rpkt_field_req_t r[RPKT_MAX_FIELD_REQS];
};

struct LayerView {
    uint32_t n;
    uint32_t proto[4];   // proto[16], four per dword
    uint32_t off[8];     // off[16], two per dword
};

__device__ __forceinline__ LayerView load_layers(const rpkt_layers_t* layers, uint32_t i) {
    const u32x4* p = reinterpret_cast<const u32x4*>(layers + i);
    const u32x4 a = p[0], b = p[1], c = p[2], d = p[3];
    LayerView v;
    v.n = a[0] & 0xffu;
    v.proto[0] = b[0]; v.proto[1] = b[1]; v.proto[2] = b[2]; v.proto[3] = b[3];
    v.off[0] = c[0]; v.off[1] = c[1]; v.off[2] = c[2]; v.off[3] = c[3];
    v.off[4] = d[0]; v.off[5] = d[1]; v.off[6] = d[2]; v.off[7] = d[3];
    return v;
}

// Offset of the nth layer whose protocol is `proto`; false when the stack has fewer
// such layers.  Branch-free: a per-byte equality mask of the 16 protocol bytes (exact
// zero-byte test on proto ^ layer bytes), cut to the n layers, then the nth set bit by
// a 4-step popcount select, and the offset picked from the 8 offset dwords.
__device__ __forceinline__ bool find_layer(const LayerView& L, uint32_t proto, uint32_t nth,
                                           uint32_t& loff) {
    const uint32_t rep = proto * 0x01010101u;
    uint32_t m = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) {
        const uint32_t x = L.proto[w] ^ rep;
        const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
        m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u))
             << (4 * w);
    }
    m &= 0xffffu >> (16u - min(L.n, (uint32_t)RPKT_MAX_LAYERS));
    uint32_t pos = 0, r = nth, mm = m;
#pragma unroll
    for (uint32_t s = 8; s > 0; s >>= 1) {
        const uint32_t c = __builtin_popcount(mm & ((1u << s) - 1u));
        const bool skip = r >= c;
        r = skip ? r - c : r;
        mm = skip ? mm >> s : mm;
        pos = skip ? pos + s : pos;
    }
    // the offset dword by a mux tree on the index bits: a chain of (index == q) selects
    // over the array is turned by the compiler into an indexed load from a private copy
    // of the 52-B record in scratch (written per lane and re-read, through L2 and HBM)
    const uint32_t q = pos >> 1;
    const bool q0 = q & 1u, q1 = q & 2u, q2 = q & 4u;
    const uint32_t a0 = q0 ? L.off[1] : L.off[0], a1 = q0 ? L.off[3] : L.off[2];
    const uint32_t a2 = q0 ? L.off[5] : L.off[4], a3 = q0 ? L.off[7] : L.off[6];
    const uint32_t b0 = q1 ? a1 : a0, b1 = q1 ? a3 : a2;
    const uint32_t dw = q2 ? b1 : b0;
    loff = (dw >> (16 * (pos & 1))) & 0xffffu;
    return (uint32_t)__builtin_popcount(m) > nth;
}

// Bytes [a, a+9) of the batch, as (big-endian first 8, ninth), from the three aligned
// dwords d[0..2] at a & ~3: a funnel shift and a byte swap.  Bytes past the field are
// the frame's (or the next frame's) and are shifted out by the caller.
__device__ __forceinline__ void take9(const uint32_t (&d)[3], uint32_t a, uint64_t& hi,
                                      uint32_t& ninth) {
    const uint32_t sh = 8u * (a & 3u);
    uint64_t q = ((uint64_t)d[1] << 32) | d[0];
    q = sh ? (q >> sh) | ((uint64_t)d[2] << (64u - sh)) : q;
    hi = __builtin_bswap64(q);
    ninth = (d[2] >> sh) & 0xffu;
}

// The same bytes by byte loads (bytes at or past `limit` read 0): for the rare field
// in the last, partial dword of the buffer, which a dword load drops whole.
// (returned by value: out-parameters of a call that is not inlined live in scratch)
struct Bytes9 {
    uint64_t hi;
    uint32_t ninth;
};
__device__ __noinline__ Bytes9 load9_bytes(__amdgpu_buffer_rsrc_t rs, uint32_t a, uint32_t limit) {
    uint64_t h = 0;
    for (uint32_t j = 0; j < 8; ++j) h = (h << 8) | (a + j < limit ? gbyte(rs, a + j) : 0u);
    return Bytes9{h, a + 8 < limit ? gbyte(rs, a + 8) : 0u};
}

// Requests whose loads are in flight together (the ablation macro: 16 is fastest, 8 at
// 74 VGPRs 65.0 vs 63.9 us, 4 at 60 VGPRs 177 us; profiles/r02_ab_fgroup).
#ifndef RPKT_FIELDS_GROUP
#define RPKT_FIELDS_GROUP 16
#endif
constexpr uint32_t kReqGroup = RPKT_FIELDS_GROUP;
#ifndef RPKT_FIELDS_SAMELAYER
#define RPKT_FIELDS_SAMELAYER 1  // requests on the layer of the one before skip the search
#endif

// One lane per frame: its layer record once, then the requests in groups of sixteen whose
// 48 dword loads are issued before any is used (the request list is wave-uniform,
// read from the kernel arguments by scalar loads; the host pads it to a multiple of
// sixteen with requests no layer matches; their loads read offset 0, which is cheaper
// than a wave-uniform branch around them: 99 vs 90 us).  A group's values are staged in
// LDS (frame stride 2k+1 dwords: conflict-free) and stored as rows of up to 16 u64 per
// frame, non-temporal (written once, never re-read here); the row index is a shift, not
// a division by the run-time request count (70.7 -> 63.0 us same-process, profiles/r02_ab_fgroup).
__global__ __launch_bounds__(kFieldBlock) void fields_kernel(
    const uint8_t* __restrict__ frames, uint32_t frames_bytes,
    const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len, uint32_t n,
    const rpkt_layers_t* __restrict__ layers, FieldReqs reqs, uint32_t n_req, uint32_t same_prev,
    uint64_t* __restrict__ values, uint32_t* __restrict__ present) {
    extern __shared__ uint32_t stage[];                  // kFieldBlock * (2 kReqGroup + 1)
    const uint32_t base = blockIdx.x * kFieldBlock, t = threadIdx.x, i = base + t;
    const uint32_t nf = min(n - base, (uint32_t)kFieldBlock);
    constexpr uint32_t fs = 2 * kReqGroup + 1;
    const uint32_t full_dwords = frames_bytes & ~3u;
    const bool live = i < n;
    const Frame fr = live ? frame_span(offsets, stride, frame_len, frames_bytes, i) : Frame{0u, 0u};
    const LayerView L = live ? load_layers(layers, i) : LayerView{};
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, frames_bytes);
    uint64_t* const out = values + (uint64_t)base * n_req;
    uint32_t mask = 0;
    // the layer of the last request searched: a request naming the same (protocol, nth)
    // as the one before it (bit r of same_prev, wave-uniform) reuses it
    uint32_t cur_loff = 0;
    bool cur_found = false;
    // a group of requests at a time: loads, values into the LDS stage, then the group's
    // values of the block's frames stored as rows of g consecutive u64 per frame (the
    // stage holds one group, so the block's LDS does not limit the waves per CU)
    for (uint32_t r0 = 0; r0 < n_req; r0 += kReqGroup) {
        if (live) {
            uint32_t d[kReqGroup][3], a[kReqGroup], ok[kReqGroup];
#pragma unroll
            for (uint32_t j = 0; j < kReqGroup; ++j) {
                const rpkt_field_req_t q = reqs.r[r0 + j];
                const uint32_t eb = ((uint32_t)q.bit_off + q.bits - 1) >> 3;
#if RPKT_FIELDS_SAMELAYER
                if (!((same_prev >> (r0 + j)) & 1u)) cur_found = find_layer(L, q.proto, q.nth, cur_loff);
#else
                cur_found = find_layer(L, q.proto, q.nth, cur_loff);
#endif
                ok[j] = cur_found & (cur_loff + eb < fr.len);
                a[j] = ok[j] ? fr.off + cur_loff + (q.bit_off >> 3) : 0u;
                const uint32_t a4 = a[j] & ~3u;
                d[j][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)a4, 0, 0);
                d[j][1] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a4 + 4u), 0, 0);
                d[j][2] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a4 + 8u), 0, 0);
            }
#pragma unroll
            for (uint32_t j = 0; j < kReqGroup; ++j) {
                const rpkt_field_req_t q = reqs.r[r0 + j];
                const uint32_t bits = q.bits, s = q.bit_off & 7u;
                uint64_t hi;
                uint32_t ninth;
                take9(d[j], a[j], hi, ninth);
                if (ok[j] && a[j] + 9u > full_dwords) {
                    const Bytes9 b9 = load9_bytes(rs, a[j], frames_bytes);
                    hi = b9.hi;
                    ninth = b9.ninth;
                }
                // the 64 bits from the field's first bit on, then its top `bits`
                const uint64_t w = s ? (hi << s) | (uint64_t)(ninth >> (8 - s)) : hi;
                const uint64_t v = ok[j] ? w >> ((64u - bits) & 63u) : 0ull;
                mask |= ok[j] << (r0 + j);
                stage[t * fs + 2 * j] = (uint32_t)v;
                stage[t * fs + 2 * j + 1] = (uint32_t)(v >> 32);
            }
        }
        __syncthreads();
        const uint32_t g = min(kReqGroup, n_req - r0);
        for (uint32_t e = t; e < nf * g; e += kFieldBlock) {
            const uint32_t f = g == kReqGroup ? e / kReqGroup : e / g, r = e - f * g;
            __builtin_nontemporal_store(
                ((uint64_t)stage[f * fs + 2 * r + 1] << 32) | stage[f * fs + 2 * r],
                out + (uint64_t)f * n_req + r0 + r);
        }
        __syncthreads();
    }
    if (live && present) __builtin_nontemporal_store(mask, present + i);
}

}  // namespace

extern "C" {

int rpkt_gpu_fields_batch(const rpkt_batch_t* b, const rpkt_layers_t* layers_dev,
                          const rpkt_field_req_t* reqs, uint32_t n_req, uint64_t* values_dev,
                          uint32_t* present_dev, void* stream) {
    if (!b || !layers_dev || !reqs || !values_dev) return RPKT_E_INVAL;
    if (n_req == 0 || n_req > RPKT_MAX_FIELD_REQS) return RPKT_E_INVAL;
    FieldReqs rq = {};
    uint32_t same_prev = 0;                                 // bit r: request r names the
                                                            // layer request r - 1 names
    for (uint32_t k = 0; k < RPKT_MAX_FIELD_REQS; ++k)      // padding: matches no layer
        rq.r[k] = rpkt_field_req_t{0xff, 0, 8, 0, 0, 0};
    for (uint32_t k = 0; k < n_req; ++k) {
        const rpkt_field_req_t& t = reqs[k];
        if (t.bits == 0 || t.bits > 64 || t.proto >= RPKT_N_PROTOCOLS) return RPKT_E_INVAL;
        if ((uint32_t)t.bit_off + t.bits > 65535u * 8u) return RPKT_E_INVAL;
        rq.r[k] = t;
        if (k && t.proto == reqs[k - 1].proto && t.nth == reqs[k - 1].nth) same_prev |= 1u << k;
    }
    for (uint32_t k = n_req + 1; k < RPKT_MAX_FIELD_REQS; ++k) same_prev |= 1u << k;   // padding
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)layers_dev & 15u) != 0 || ((uintptr_t)values_dev & 7u) != 0 ||
        ((uintptr_t)present_dev & 3u) != 0)
        return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint32_t grid = (b->n + kFieldBlock - 1) / kFieldBlock;
    const size_t lds = (size_t)kFieldBlock * (2 * kReqGroup + 1) * 4;
    return launch(fields_kernel, dim3(grid), dim3(kFieldBlock), lds, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  layers_dev, rq, n_req, same_prev, values_dev, present_dev);
}

}  // extern "C"
