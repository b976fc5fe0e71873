/*
 * rpkt_oracle_fields.c — CPU restatement of the header-field getters over the layer
 * walk, TEST INFRASTRUCTURE ONLY (the checker for rpkt_gpu_fields_batch; never linked
 * into or called by the product path).
 *
 * rpkt's header views read every field with code pktfmt generates
 * (pktfmt/src/codegen/field.rs:115-250):
 *   - read_multi_bytes (:115-160): the big-endian integer of bytes
 *     [start.byte_pos, end.byte_pos], `>> (7 - end.bit_pos)` when the field does not
 *     end on a byte boundary, `& ones_mask(bit)` when it does not start on one;
 *   - read_repr (:162-250): single-byte fields the same way on one byte; ByteSlice
 *     fields (byte-aligned, e.g. MAC and IP addresses) are the slice itself.
 * This restatement walks the field bit by bit (MSB first) instead, so it shares no
 * arithmetic with the kernel's shift-and-mask form.  The layer each request reads is
 * the nth layer of rpkt_layers_t with that protocol (oracle_layers_batch).
 *
 * Parity is pinned by the getter values the reference's own tests assert on its
 * fixtures (tests/test_oracle_fields.py cites them).
 */
#include <stdint.h>
#include <string.h>

#include "../include/rpkt_gpu.h"

static int find_layer(const rpkt_layers_t* L, uint32_t proto, uint32_t nth, uint32_t* off) {
    uint32_t seen = 0;
    for (uint32_t k = 0; k < L->n && k < RPKT_MAX_LAYERS; k++) {
        if (L->proto[k] != proto) continue;
        if (seen++ == nth) { *off = L->off[k]; return 1; }
    }
    return 0;
}

static int one_field(const uint8_t* fr, uint32_t flen, const rpkt_layers_t* L,
                     const rpkt_field_req_t* q, uint64_t* out) {
    uint32_t loff;
    *out = 0;
    if (!find_layer(L, q->proto, q->nth, &loff)) return 0;
    uint32_t last_byte = (q->bit_off + q->bits - 1u) / 8u;
    if ((uint64_t)loff + last_byte >= flen) return 0;
    const uint8_t* h = fr + loff;
    uint64_t v = 0;
    for (uint32_t b = q->bit_off; b < (uint32_t)q->bit_off + q->bits; b++)
        v = (v << 1) | ((h[b / 8u] >> (7u - b % 8u)) & 1u);
    *out = v;
    return 1;
}

void oracle_fields_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                         uint32_t stride, uint32_t frame_len, uint32_t n,
                         const rpkt_layers_t* layers, const rpkt_field_req_t* reqs,
                         uint32_t n_req, uint64_t* values, uint32_t* present) {
    for (uint32_t i = 0; i < n; i++) {
        uint64_t off, len;
        if (offsets) {
            off = offsets[i];
            len = offsets[i + 1] >= offsets[i] ? offsets[i + 1] - offsets[i] : 0;
        } else {
            off = (uint64_t)i * stride;
            len = frame_len ? frame_len : stride;
        }
        if (off > frames_bytes) off = frames_bytes;
        if (off + len > frames_bytes) len = frames_bytes - off;
        uint32_t mask = 0;
        for (uint32_t r = 0; r < n_req; r++)
            if (one_field(frames + off, (uint32_t)len, &layers[i], &reqs[r],
                          &values[(uint64_t)i * n_req + r]))
                mask |= 1u << r;
        if (present) present[i] = mask;
    }
}
