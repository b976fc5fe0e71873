// rpkt_fields.hip — header-field getters over the protocol-layer walk.
//
// The getters rpkt generates for each protocol's header view (pktfmt/src/codegen/
// field.rs:115-250: `read_repr` / `read_multi_bytes` read bytes [start, end] big-endian,
// shift right by 7 - end bit, mask to the field width) evaluated for a list of
// (protocol, occurrence, bit offset, width) requests over every frame of a batch,
// on the layer offsets rpkt_gpu_layers_batch found.
//
// One lane per (frame, request) output element, so the values are stored as one
// contiguous 8-B-per-lane row per wave; the n_req lanes of a frame read the same
// 64-B layer record and header bytes, which L1/L2 serve after the first lane.  The
// gather is a handful of byte loads per lane: latency-bound, not HBM-bound.
#include "rpkt_common.h"

namespace {

constexpr int kFieldBlock = 256;

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

// Offset of the nth layer whose protocol is `proto` (unrolled selects, no scratch
// indexing); returns false when the stack has fewer such layers.
__device__ __forceinline__ bool find_layer(const LayerView& L, uint32_t proto, uint32_t nth,
                                           uint32_t& loff) {
    uint32_t seen = 0, found = 0, off = 0;
#pragma unroll
    for (uint32_t k = 0; k < RPKT_MAX_LAYERS; ++k) {
        const uint32_t p = (L.proto[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint32_t o = (L.off[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        const uint32_t hit = (k < L.n) & (p == proto);
        const uint32_t take = hit & (seen == nth) & (found ^ 1u);
        off = take ? o : off;
        found |= take;
        seen += hit;
    }
    loff = off;
    return found != 0;
}

__global__ __launch_bounds__(kFieldBlock) void fields_kernel(
    const uint8_t* __restrict__ frames, uint32_t frames_bytes,
    const uint32_t* __restrict__ offsets, uint32_t stride, uint32_t frame_len, uint32_t n,
    const rpkt_layers_t* __restrict__ layers, FieldReqs reqs, uint32_t n_req,
    uint64_t* __restrict__ values, uint32_t* __restrict__ present) {
    const uint64_t e = (uint64_t)blockIdx.x * kFieldBlock + threadIdx.x;
    if (e >= (uint64_t)n * n_req) return;
    const uint32_t i = (uint32_t)(e / n_req), r = (uint32_t)(e - (uint64_t)i * n_req);
    const Frame fr = frame_span(offsets, stride, frame_len, frames_bytes, i);
    const LayerView L = load_layers(layers, i);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(frames, frames_bytes);

    const rpkt_field_req_t q = reqs.r[r];
    const uint32_t bit_off = q.bit_off, bits = q.bits;
    const uint32_t sb = bit_off >> 3, eb = (bit_off + bits - 1) >> 3;
    uint32_t loff;
    const bool ok = find_layer(L, q.proto, q.nth, loff) && loff + eb < fr.len;
    uint64_t v = 0;
    if (ok) {
        const uint32_t a = fr.off + loff + sb, nb = eb - sb + 1;   // 1..9 bytes
        uint64_t hi = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
            if (j < nb) hi |= (uint64_t)gbyte(rs, a + j) << (56 - 8 * j);
        const uint32_t s = bit_off & 7u;
        const uint32_t lo = nb == 9 ? gbyte(rs, a + 8) : 0u;
        // the 64 bits from the field's first bit on, then the field's top `bits`
        const uint64_t w = s ? (hi << s) | (uint64_t)(lo >> (8 - s)) : hi;
        v = w >> (64 - bits);
    }
    values[e] = v;

    if (present && r == 0) {
        uint32_t mask = 0;
        for (uint32_t k = 0; k < n_req; ++k) {
            const rpkt_field_req_t t = reqs.r[k];
            uint32_t o;
            const uint32_t end = ((uint32_t)t.bit_off + t.bits - 1) >> 3;
            if (find_layer(L, t.proto, t.nth, o) && o + end < fr.len) mask |= 1u << k;
        }
        present[i] = mask;
    }
}

}  // namespace

extern "C" {

int rpkt_gpu_fields_batch(const rpkt_batch_t* b, const rpkt_layers_t* layers_dev,
                          const rpkt_field_req_t* reqs, uint32_t n_req, uint64_t* values_dev,
                          uint32_t* present_dev, void* stream) {
    if (!b || !layers_dev || !reqs || !values_dev) return RPKT_E_INVAL;
    if (n_req == 0 || n_req > RPKT_MAX_FIELD_REQS) return RPKT_E_INVAL;
    FieldReqs rq = {};
    for (uint32_t k = 0; k < n_req; ++k) {
        const rpkt_field_req_t& t = reqs[k];
        if (t.bits == 0 || t.bits > 64 || t.proto >= RPKT_N_PROTOCOLS) return RPKT_E_INVAL;
        if ((uint32_t)t.bit_off + t.bits > 65535u * 8u) return RPKT_E_INVAL;
        rq.r[k] = t;
    }
    if (b->n == 0) return RPKT_OK;
    if (!b->frames_dev) return RPKT_E_INVAL;
    if (b->frames_bytes > kMaxFrameBytes) return RPKT_E_TOO_LARGE;
    if (!b->offsets_dev && b->stride == 0) return RPKT_E_INVAL;
    if (((uintptr_t)layers_dev & 15u) != 0 || ((uintptr_t)values_dev & 7u) != 0 ||
        ((uintptr_t)present_dev & 3u) != 0)
        return RPKT_E_ALIGN;
    const uint32_t flen = b->offsets_dev ? 0 : (b->frame_len ? b->frame_len : b->stride);
    const uint64_t total = (uint64_t)b->n * n_req;
    const uint64_t grid = (total + kFieldBlock - 1) / kFieldBlock;
    if (grid > 0x7fffffffull) return RPKT_E_TOO_LARGE;
    return launch(fields_kernel, dim3((uint32_t)grid), dim3(kFieldBlock), 0, (hipStream_t)stream,
                  b->frames_dev, (uint32_t)b->frames_bytes, b->offsets_dev, b->stride, flen, b->n,
                  layers_dev, rq, n_req, values_dev, present_dev);
}

}  // extern "C"
