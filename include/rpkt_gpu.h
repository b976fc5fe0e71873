/*
 * rpkt_gpu.h — C ABI of the MI355X packet-batch parse + checksum engine.
 *
 * This is the drop-in boundary for rpkt's Ether -> (802.1Q/802.1ad)* -> IPv4 ->
 * {TCP, UDP} decode-and-verify path.  rpkt itself has no FFI for this path: its
 * "operator API" is the generic header views over `T: Buf`
 *   EtherFrame::parse      rpkt/src/ether/generated.rs:34-41
 *   VlanFrame::parse       rpkt/src/vlan/generated.rs:32-39
 *   Ipv4::parse            rpkt/src/ipv4/generated.rs:35-51
 *   Udp::parse             rpkt/src/udp/generated.rs:31-42
 *   Tcp::parse             rpkt/src/tcp/generated.rs:34-45
 *   checksum::from_slice   rpkt/src/checksum.rs:33-62
 *   checksum::combine      rpkt/src/checksum.rs:68-74
 * which a caller drives one frame at a time (benches/rpkt/rpkt_parse.rs:62-80,
 * rpkt-dpdk/examples/loopback_rx.rs:96-121).  The entry points below replace that
 * per-frame loop with one call over a device-resident batch of frames, and return
 * one fixed-size record per frame holding every getter value the chain above
 * exposes, the parse outcome and the raw RFC 1071 sums.
 *
 * Conventions (no HIP/torch types cross this header):
 *   - every pointer named *_dev is device memory owned by the caller;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream);
 *   - calls are asynchronous on `stream` and never allocate or synchronise;
 *   - API-level failures are negative return codes; per-frame parse failures are
 *     never errors, they are reported in rpkt_rec_t.status.
 */
#ifndef RPKT_GPU_H
#define RPKT_GPU_H

#include <stddef.h>

#include "rpkt_protocols.h"
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPKT_ABI_VERSION 1u

/* ---- per-frame status: which rpkt `parse` would return Err (first one) ----
 * The chain is EtherFrame::parse -> while ethertype in {VLAN, QINQ}:
 * VlanFrame::parse -> (ethertype == IPV4) -> Ipv4::parse -> protocol dispatch ->
 * Udp::parse | Tcp::parse.  At most RPKT_MAX_VLAN tags are walked; a further
 * tag leaves the dispatch ethertype at 0x8100/0x88a8 -> RPKT_S_NOT_IPV4. */
enum rpkt_status {
    RPKT_S_OK = 0,              /* Udp::parse or Tcp::parse returned Ok           */
    RPKT_S_ETH_SHORT = 1,       /* chunk_len < 14     ether/generated.rs:36        */
    RPKT_S_VLAN_SHORT = 2,      /* chunk_len < 4      vlan/generated.rs:34         */
    RPKT_S_NOT_IPV4 = 3,        /* ethertype != 0x0800 (caller check, rpkt_parse.rs:66) */
    RPKT_S_IP_SHORT = 4,        /* chunk_len < 20     ipv4/generated.rs:37         */
    RPKT_S_IP_BAD_IHL = 5,      /* header_len < 20    ipv4/generated.rs:43         */
    RPKT_S_IP_IHL_GT_LEN = 6,   /* header_len > chunk_len   ipv4/generated.rs:44   */
    RPKT_S_IP_TOT_LT_IHL = 7,   /* packet_len < header_len  ipv4/generated.rs:45   */
    RPKT_S_IP_TOT_GT_LEN = 8,   /* packet_len > remaining   ipv4/generated.rs:46   */
    RPKT_S_L4_OTHER = 9,        /* IPv4 ok, protocol not TCP(6)/UDP(17)            */
    RPKT_S_UDP_SHORT = 10,      /* chunk_len < 8      udp/generated.rs:33          */
    RPKT_S_UDP_BAD_LEN = 11,    /* len < 8 || len > remaining  udp/generated.rs:38 */
    RPKT_S_TCP_SHORT = 12,      /* chunk_len < 20     tcp/generated.rs:36          */
    RPKT_S_TCP_BAD_DOFF = 13,   /* hlen < 20 || hlen > chunk_len  tcp/generated.rs:41 */
    /* IPv6 (RPKT_F_IPV6 only): ethertype 0x86DD -> Ipv6::parse -> extension headers */
    RPKT_S_IP6_SHORT = 14,      /* chunk_len < 40     ipv6/generated.rs:42         */
    RPKT_S_IP6_BAD_LEN = 15,    /* payload_len + 40 > remaining  ipv6/generated.rs:47 */
    RPKT_S_IP6_EXT_SHORT = 16,  /* extension header: chunk_len < its fixed size
                                   (2 HopByHop/DestOptions, 8 Routing/Fragment, 12 AH;
                                   ipv6/generated.rs:243,386,530,698,852)          */
    RPKT_S_IP6_EXT_BAD_LEN = 17,/* extension header: header_len < min or > chunk_len
                                   (ipv6/generated.rs:248,391,535,857)             */
    RPKT_S_IP6_FRAGMENT = 18,   /* a Fragment header with offset != 0 or M set: the
                                   upper-layer header needs reassembly, not parsed */
    RPKT_S_ICMP_EMPTY = 19,     /* IPv4 parsed, protocol 1 (ICMP), empty payload: the
                                   reference's calculate_icmp_checksum panics on it
                                   (icmp_data.len() - 1 underflows,
                                   icmpv4/generated.rs:2684); otherwise as L4_OTHER */
    RPKT_S_NO_INNER = 20        /* rpkt_gpu_parse_tunnel_batch's inner record of a frame
                                   whose tunnel was not decoded (rpkt_tun_t.status != OK):
                                   every other field 0 */
};

#define RPKT_MAX_VLAN 2
/* Extension headers walked after the IPv6 header: HopByHop (0), Routing (43),
 * Fragment (44), DestOptions (60), AH (51).  A chain longer than this leaves the next
 * header at an extension type -> RPKT_S_L4_OTHER (as a third VLAN tag -> NOT_IPV4). */
#define RPKT_MAX_IP6_EXT 8

/* ---- API return codes ---- */
enum rpkt_err {
    RPKT_OK = 0,
    RPKT_E_INVAL = -1,       /* NULL pointer / zero stride / bad flags            */
    RPKT_E_HIP = -2,         /* a HIP runtime call failed (see rpkt_gpu_last_hip_error) */
    RPKT_E_TOO_LARGE = -3,   /* frames_bytes >= 4 GiB: split the batch             */
    RPKT_E_ALIGN = -4,       /* out/flow buffer not 16-byte aligned               */
    RPKT_E_COLL = -5         /* an RCCL call failed (see rpkt_gpu_last_coll_error) */
};

/* ---- flags for rpkt_gpu_parse_batch ---- */
enum rpkt_flags {
    RPKT_F_IP_SUM = 1u,      /* compute ip_sum = from_slice(ipv4 header[0..ihl4])  */
    RPKT_F_L4_SUM = 2u,      /* compute l4_sum = combine(pseudo, from_slice(l4))    */
    RPKT_F_FLOW_EV = 4u,     /* also write one rpkt_flow_ev_t per frame             */
    RPKT_F_IPV6 = 8u         /* also decode and verify IPv6 (ethertype 0x86DD); without
                                it such frames stop at RPKT_S_NOT_IPV4 as before      */
};

/* Record layout: 80 bytes, 16-byte aligned, little-endian host order.
 * Field  <-> rpkt getter (all getters of the path are recoverable exactly):
 *   ethertype          EtherFrame::ethertype          ether/generated.rs:55-59
 *   dst_addr/src_addr  EtherFrame::{dst,src}_addr     ether/generated.rs:47-54
 *   vlan_tci[i]        be16[0..2] of tag i: priority = tci>>13, dei = tci&0x1000,
 *                      vlan_id = tci&0xfff            vlan/generated.rs:45-56
 *   vlan_ethertype[i]  VlanFrame::ethertype           vlan/generated.rs:57-61
 *   ip_vhl             byte 0: version = >>4, header_len = (&0xf)*4
 *   ip_tos             byte 1: dscp = >>2, ecn = &3
 *   ip_frag            be16[6..8]: flag_reserved = >>15, dont_frag = &0x4000,
 *                      more_frag = &0x2000, frag_offset = &0x1fff
 *                      (Ipv4 getters ipv4/generated.rs:61-112, 269-288)
 *   l4_word6           TCP: be16[12..14] (header_len = (>>12)*4, reserved =
 *                      (>>8)&0xf, flags = &0xff); UDP: packet_len be16[4..6]
 *   l4_checksum        TCP be16[16..18] / UDP be16[6..8]
 *   tcp_*              Tcp getters tcp/generated.rs:55-122
 *   l3_off             frame offset of the IPv4 header (EtherFrame/VlanFrame::payload)
 *   l4_off             frame offset of Ipv4::payload() (trimmed to packet_len)
 *   payload_off/_len   Udp::payload() / Tcp::payload() when status == OK,
 *                      otherwise Ipv4::payload() when IPv4 parsed
 *   ip_sum             checksum::from_slice(ipv4[0..header_len]); 0xffff <=> valid
 *   l4_sum             checksum::combine(&[pseudo(src,dst,proto,l4_len),
 *                      from_slice(l4[0..l4_len])]); 0xffff <=> valid
 *                      Status L4_OTHER (RPKT_F_L4_SUM), no pseudo header:
 *                      - IPv4 protocol 1 (ICMP): from_slice over the whole IPv4 payload
 *                        [l4_off, l3_off + packet_len); the reference's
 *                        calculate_icmp_checksum (icmpv4/generated.rs:2678-2701) over the
 *                        same bytes is !l4_sum, so 0xffff <=> it returns 0 (a valid
 *                        message, icmpv4_test.rs:82-96); an empty payload is
 *                        RPKT_S_ICMP_EMPTY, not summed;
 *                      - protocol / next header 47 (GRE) with the checksum-present bit
 *                        (byte 0 & 0x80, gre/generated.rs:55) and >= 4 payload bytes:
 *                        from_slice over the GRE header and its payload (RFC 2784 section
 *                        2.5; Gre::checksum, gre/generated.rs:239): 0xffff <=> valid.
 *                      (These are the sums of the outer layer only: a frame whose l4_sum
 *                      is one of them keeps status L4_OTHER, so the compact verdict bit 1
 *                      and the flow event's bit 49 do not cover them.)
 * Fields of layers that were not reached are zero.  Sums not requested by the
 * flags, or whose layer did not parse, are zero.
 *
 * IPv6 frames (RPKT_F_IPV6, dispatch ethertype 0x86DD: `ethertype`, or
 * vlan_ethertype[n_vlan-1] when tagged) use bytes 24..43 as the IPv6 block below
 * instead of the IPv4 fields; everything else keeps its meaning.  Chain:
 * Ipv6::parse (ipv6/generated.rs:40-51) -> Ipv6::payload (trim to payload_len,
 * advance 40, :83-92) -> up to RPKT_MAX_IP6_EXT extension headers, each its parse and
 * payload() (DestOptions :241-279, HopByHopOption :384-421, RoutingHeader :528-577,
 * FragmentHeader :696-739, AuthenticationHeader :850-899) -> Udp|Tcp::parse.
 *   24 u32 ip6_vtcfl     be32 of bytes 0..3: version = >>28, traffic_class =
 *                        (>>20)&0xff, flow_label = &0xfffff     (:57-67)
 *   28 u16 ip6_payload_len                                      (:77-79)
 *   30 u8  ip6_next_header   the IPv6 header's next_header       (:69-71)
 *   31 u8  ip6_hop_limit                                         (:73-75)
 *   32 u8  ip6_n_ext     extension headers walked
 *   33 u8  ip_protocol   the upper-layer protocol: the next_header where the walk
 *                        stopped (the extension type that failed for IP6_EXT_*,
 *                        the Fragment header's next_header for IP6_FRAGMENT)
 *   34 u16 ip6_pdst_off  frame offset of the 16-B address the L4 pseudo header uses
 *                        as destination: dst_addr (l3 + 24), or, after a Routing
 *                        header with segments_left > 0 (RFC 8200 section 8.1), its
 *                        final address -- the last of the list for types 0 and 2, the
 *                        first (Segment List[0]) for type 4; other types keep dst_addr
 *   36 u32 ip6_src_fold  src_addr as four be32 words XORed (the flow key)
 *   40 u32 ip6_dst_fold  dst_addr likewise (src_addr/dst_addr themselves: frame bytes
 *                        l3_off + 8 and l3_off + 24, or rpkt_gpu_fields_batch)
 * l4_off = the cursor after the extension headers (the header where the walk stopped);
 * payload_off/_len = Udp/Tcp::payload() when status == OK, otherwise [l4_off, end of
 * the trimmed IPv6 payload).  ip_sum = 0 (IPv6 has no header checksum).  l4_sum =
 * combine(&[pseudo_v6(src, pdst, u32 l4_len, next header), from_slice(l4)]); a UDP
 * checksum of 0 is NOT "not computed" over IPv6 (RFC 8200 section 8.1). */
typedef struct rpkt_rec {
    uint8_t  status;            /*  0 enum rpkt_status                          */
    uint8_t  n_vlan;            /*  1 tags walked, 0..RPKT_MAX_VLAN             */
    uint16_t ethertype;         /*  2                                           */
    uint8_t  dst_addr[6];       /*  4                                           */
    uint8_t  src_addr[6];       /* 10                                           */
    uint16_t vlan_tci[2];       /* 16                                           */
    uint16_t vlan_ethertype[2]; /* 20                                           */
    uint8_t  ip_vhl;            /* 24                                           */
    uint8_t  ip_tos;            /* 25                                           */
    uint16_t ip_packet_len;     /* 26                                           */
    uint16_t ip_ident;          /* 28                                           */
    uint16_t ip_frag;           /* 30                                           */
    uint8_t  ip_ttl;            /* 32                                           */
    uint8_t  ip_protocol;       /* 33                                           */
    uint16_t ip_checksum;       /* 34                                           */
    uint32_t ip_src;            /* 36 a.b.c.d -> (a<<24)|(b<<16)|(c<<8)|d        */
    uint32_t ip_dst;            /* 40                                           */
    uint16_t src_port;          /* 44                                           */
    uint16_t dst_port;          /* 46                                           */
    uint32_t tcp_seq;           /* 48                                           */
    uint32_t tcp_ack;           /* 52                                           */
    uint16_t l4_word6;          /* 56                                           */
    uint16_t tcp_window;        /* 58                                           */
    uint16_t l4_checksum;       /* 60                                           */
    uint16_t tcp_urgent;        /* 62                                           */
    uint16_t l3_off;            /* 64                                           */
    uint16_t l4_off;            /* 66                                           */
    uint16_t payload_off;       /* 68                                           */
    uint16_t payload_len;       /* 70                                           */
    uint16_t ip_sum;            /* 72                                           */
    uint16_t l4_sum;            /* 74                                           */
    uint32_t frame_len;         /* 76 Cursor::remaining() of the whole frame    */
} rpkt_rec_t;

#define RPKT_REC_BYTES 80u

/* Per-frame flow event (RPKT_F_FLOW_EV), 8 bytes:
 *   bits  0..31  frame_len
 *   bits 32..47  flow bucket = rpkt_flow_hash(5-tuple) % n_buckets (status OK),
 *                n_buckets for frames that did not parse to L4
 *   bit  48      ip header sum != 0xffff (IPv4 header parsed; never for IPv6)
 *   bit  49      l4 sum != 0xffff (an IPv4 UDP checksum field of 0 counts as valid)
 * IPv6 frames hash ip6_src_fold / ip6_dst_fold in place of the IPv4 addresses.
 * Counters (rpkt_gpu_flow_count) are u64[(n_buckets + 1) * 4]:
 *   row b = {pkts, bytes, ip_bad, l4_bad}; row n_buckets = unparsed frames. */
typedef uint64_t rpkt_flow_ev_t;
#define RPKT_FLOW_MAX_BUCKETS 65535u

/* Frame batch descriptor.  Frame i is [off_i, off_i + len_i) of `frames_dev`:
 *   packed  (offsets_dev != NULL): off_i = offsets[i], len_i = offsets[i+1] - offsets[i]
 *                                  (n + 1 entries, non-decreasing);
 *   strided (offsets_dev == NULL): off_i = i * stride, len_i = frame_len (0 -> stride).
 * Loads are bounds-checked in hardware against frames_bytes, so a malformed
 * descriptor yields wrong records, never a fault.  frames_bytes < 4 GiB. */
typedef struct rpkt_batch {
    const uint8_t*  frames_dev;
    uint64_t        frames_bytes;
    const uint32_t* offsets_dev;
    uint32_t        stride;
    uint32_t        frame_len;
    uint32_t        n;
    uint32_t        reserved;
} rpkt_batch_t;

/* ABI version and build information (host-only, no device calls). */
uint32_t rpkt_gpu_abi_version(void);
const char* rpkt_gpu_build_info(void);
const char* rpkt_gpu_status_name(int status);
/* Last HIP error code seen by this thread (hipError_t as int), 0 if none. */
int rpkt_gpu_last_hip_error(void);
/* Human-readable runtime/device description into buf (diagnostics). */
int rpkt_gpu_device_info(char* buf, size_t len);

/* Parse + verify a batch.  Replaces, per frame i, the reference sequence
 *   EtherFrame::parse -> [VlanFrame::parse]* -> Ipv4::parse -> Udp|Tcp::parse
 * plus the checksum composition selected by `flags`, writing recs_dev[i]
 * (n * 80 bytes, 16-byte aligned).  flow_ev_dev (n * 8 bytes) is written when
 * RPKT_F_FLOW_EV is set, using n_buckets (1..RPKT_FLOW_MAX_BUCKETS). */
int rpkt_gpu_parse_batch(const rpkt_batch_t* batch, uint32_t flags,
                         rpkt_rec_t* recs_dev, rpkt_flow_ev_t* flow_ev_dev,
                         uint32_t n_buckets, void* stream);

/* Compact record: 16 bytes, the projection of rpkt_rec_t a caller needs to locate the
 * layers and read the verdicts, for receive loops that read getters from the frame
 * itself (rpkt's views hold only the buffer and read fields lazily,
 * ipv4/generated.rs:17-20).  Fields equal the rpkt_rec_t fields of the same name;
 * verdict bit 0 = RPKT_F_IP_SUM requested and ip_sum == 0xffff (IPv6: requested and
 * the IPv6 header parsed -- it carries no checksum), bit 1 = RPKT_F_L4_SUM requested,
 * status OK and (l4_sum == 0xffff or, IPv4 only, a UDP checksum field of 0: "not
 * computed"), bit 2 = the frame was dispatched to Ipv6::parse (RPKT_F_IPV6). */
typedef struct rpkt_rec16 {
    uint8_t  status;            /*  0 enum rpkt_status                          */
    uint8_t  n_vlan;            /*  1                                           */
    uint8_t  ip_protocol;       /*  2                                           */
    uint8_t  verdict;           /*  3 bit 0 IPv4 header sum ok, bit 1 L4 sum ok */
    uint16_t l3_off;            /*  4                                           */
    uint16_t l4_off;            /*  6                                           */
    uint16_t payload_off;       /*  8                                           */
    uint16_t payload_len;       /* 10                                           */
    uint16_t ip_sum;            /* 12                                           */
    uint16_t l4_sum;            /* 14                                           */
} rpkt_rec16_t;

#define RPKT_REC16_BYTES 16u

/* rpkt_gpu_parse_batch writing rpkt_rec16_t records (recs_dev n * 16 B, 16-byte
 * aligned): the same parse, sums and flow events, one fifth of the record bytes. */
int rpkt_gpu_parse_batch_compact(const rpkt_batch_t* batch, uint32_t flags,
                                 rpkt_rec16_t* recs_dev, rpkt_flow_ev_t* flow_ev_dev,
                                 uint32_t n_buckets, void* stream);

/* A receive ring's slots (a NIC ring's bursts, rpkt-dpdk/examples/loopback_rx.rs:96-121)
 * parsed in one launch per RPKT_RING_MAX_SLOTS slots: results equal one
 * rpkt_gpu_parse_batch call per slot (records into each slot's recs_dev, flow events into
 * its flow_ev_dev when RPKT_F_FLOW_EV is set), but small batches no longer pay a
 * dependent kernel launch each.  Slots with n == 0 are skipped; every slot is checked
 * before anything is launched.  Layouts may differ from slot to slot.  recs_dev points to
 * rpkt_rec_t records for rpkt_gpu_parse_ring and to rpkt_rec16_t records for
 * rpkt_gpu_parse_ring_compact (equal to rpkt_gpu_parse_batch_compact per slot). */
typedef struct rpkt_ring_slot {
    rpkt_batch_t    batch;
    void*           recs_dev;
    rpkt_flow_ev_t* flow_ev_dev;
} rpkt_ring_slot_t;
#define RPKT_RING_MAX_SLOTS 32u
int rpkt_gpu_parse_ring(const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags,
                        uint32_t n_buckets, void* stream);
int rpkt_gpu_parse_ring_compact(const rpkt_ring_slot_t* slots, uint32_t n_slots, uint32_t flags,
                                uint32_t n_buckets, void* stream);

/* Accumulate flow events into counters_dev (u64[(n_buckets+1)*4], caller
 * zeroes it once; calls add).  workspace_dev must hold
 * rpkt_gpu_flow_workspace_bytes(n, n_buckets) bytes.  Calls that add into the
 * same counters (or share a workspace) must be ordered, e.g. on one stream: up
 * to 8192 buckets each bucket is added by one thread without atomics, so the
 * counters are bitwise reproducible. */
size_t rpkt_gpu_flow_workspace_bytes(uint32_t n, uint32_t n_buckets);
int rpkt_gpu_flow_count(const rpkt_flow_ev_t* flow_ev_dev, uint32_t n,
                        uint32_t n_buckets, uint64_t* counters_dev,
                        void* workspace_dev, void* stream);

/* Sum the flow counters of every rank (the path's only collective):
 * one RCCL ncclAllReduce (root == -1) or ncclReduce to rank `root` of
 * u64[(n_buckets+1)*4] in place, ncclUint64 / ncclSum, on `nccl_comm` (an
 * ncclComm_t passed as void*) and `stream`.  Asynchronous like every call here.
 * Replaces the per-queue counters a DPDK receive thread keeps and the final sum
 * over threads (rpkt-dpdk/examples/loopback_tx.rs:176-181, rss_rx.rs:54-113).
 * counters_dev 8-byte aligned.  RPKT_E_COLL: rpkt_gpu_last_coll_error() holds the
 * ncclResult_t. */
int rpkt_gpu_flow_reduce(uint64_t* counters_dev, uint32_t n_buckets, int root, void* nccl_comm,
                         void* stream);
/* Last ncclResult_t seen by this thread (0 if none); RCCL version (ncclGetVersion). */
int rpkt_gpu_last_coll_error(void);
int rpkt_gpu_coll_version(void);

/* A communicator the library makes itself, so a host need not take one from another
 * runtime (torch's ProcessGroupNCCL) for rpkt_gpu_flow_reduce: rank 0 calls
 * rpkt_gpu_coll_unique_id (ncclGetUniqueId) and hands the RPKT_COLL_ID_BYTES bytes to
 * every rank by any channel (the reference's receive threads share memory; ranks of
 * one host here use the torch group, an MPI broadcast or a file), then every rank
 * calls rpkt_gpu_comm_init (ncclCommInitRank on its current HIP device; collective:
 * it returns when all `world` ranks have joined) and, when done,
 * rpkt_gpu_comm_destroy.  *comm_out is an ncclComm_t as void*. */
#define RPKT_COLL_ID_BYTES 128
int rpkt_gpu_coll_unique_id(uint8_t* id_out);
int rpkt_gpu_comm_init(void** comm_out, int world, const uint8_t* id, int rank);
int rpkt_gpu_comm_destroy(void* comm);
/* rpkt_gpu_comm_init with a deadline (timeout_ms <= 0: blocking, as rpkt_gpu_comm_init):
 * a non-blocking ncclCommInitRankConfig polled with ncclCommGetAsyncError.  When not
 * every rank joins within timeout_ms (a peer failed before its init) or the init fails,
 * the half-made communicator is aborted and RPKT_E_COLL returned
 * (rpkt_gpu_last_coll_error() = 7, ncclInProgress, on a timeout), so no rank is left
 * blocked and the group can agree on a fallback.  rpkt_gpu_comm_abort (ncclCommAbort)
 * releases a communicator without waiting for its peers. */
int rpkt_gpu_comm_init_timeout(void** comm_out, int world, const uint8_t* id, int rank,
                               int timeout_ms);
int rpkt_gpu_comm_abort(void* comm);

/* Batched checksum::from_slice over byte ranges of a device buffer:
 * out_dev[i] = from_slice(buf[start_i .. start_i + len_i]) for
 * ranges_dev[i] = {start_i, len_i}.  Drop-in for rpkt/src/checksum.rs:33-62. */
int rpkt_gpu_checksum_ranges(const uint8_t* buf_dev, uint64_t buf_bytes,
                             const uint32_t* ranges_dev, uint32_t n,
                             uint16_t* out_dev, void* stream);

/* Batched checksum::from_buf over multi-segment buffers (mbuf chains, rpkt-dpdk's
 * Pbuf): chain p is segments chain_first_dev[p] .. chain_first_dev[p+1]-1 (n_chains+1
 * entries), segment i = buf[segs_dev[2i] .. segs_dev[2i] + segs_dev[2i+1]).
 * out_dev[p] = from_buf over the chain's bytes in order, pairing a segment's odd tail
 * byte with the next segment's first byte.  Drop-in for rpkt/src/checksum.rs:8-27
 * (with from_slice_with_tail_byte :77-111).  workspace_dev holds
 * rpkt_gpu_checksum_chains_workspace_bytes(n_segs) bytes. */
size_t rpkt_gpu_checksum_chains_workspace_bytes(uint32_t n_segs);
int rpkt_gpu_checksum_chains(const uint8_t* buf_dev, uint64_t buf_bytes, const uint32_t* segs_dev,
                             uint32_t n_segs, const uint32_t* chain_first_dev, uint32_t n_chains,
                             uint16_t* out_dev, void* workspace_dev, void* stream);

/* Mbuf-chain batch (rpkt-dpdk's Mbuf segments read through a Pbuf,
 * rpkt-dpdk/src/pbuf.rs).  Segment k = buf_dev[segs_dev[2k] .. segs_dev[2k] +
 * segs_dev[2k+1]) (data offset, data_len; clamped to buf_bytes like frames; segs_dev
 * 8-byte aligned).  Chain p = segments [a, b) with a = min(chain_first_dev[p], n_segs),
 * b = min(max(chain_first_dev[p+1], a), n_segs) (n_chains + 1 entries); its pkt_len is
 * the sum of its segments' lengths.  buf_bytes < 4 GiB, n_segs < 2^31. */
typedef struct rpkt_chains {
    const uint8_t*  buf_dev;
    uint64_t        buf_bytes;
    const uint32_t* segs_dev;
    const uint32_t* chain_first_dev;
    uint32_t        n_segs;
    uint32_t        n_chains;
} rpkt_chains_t;

/* Parse + verify mbuf chains: rpkt_gpu_parse_batch's chain and record per chain, with
 * each view's tests taken as they are over a Pbuf: header sizes against chunk() (the
 * rest of the segment holding the header's first byte; Pbuf::new starts at segment 0
 * even when it is empty), totals against remaining(), the packet end cut by the
 * IPv4/IPv6/UDP trim_off.  With RPKT_F_IPV6 the IPv6 chain too: the 40-byte header and
 * each extension header tested against its own chunk.  Record offsets are logical
 * positions in the chain's bytes,
 * frame_len = pkt_len, l4_sum = from_buf over the segments (rpkt/src/checksum.rs:8-27).
 * The caller's segments are never modified (the reference's trim_off truncates the
 * mbuf chain, mbuf.rs:346-382).  recs_dev n_chains * 80 B, 16-byte aligned. */
int rpkt_gpu_parse_chains(const rpkt_chains_t* chains, uint32_t flags, rpkt_rec_t* recs_dev,
                          rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream);

/* ---- Tunnels: the inner frame of VXLAN, GTP-U and GRE ------------------------- */

/* rpkt_gpu_parse_tunnel_batch decodes one tunnel level after the outer parse, as the
 * reference's receive loops chain the views (the dispatch is the caller's in rpkt):
 *   VXLAN   Udp::payload -> Vxlan::parse (vxlan/generated.rs:32-39) -> payload() (advance 8)
 *           -> EtherFrame::parse ... (rpkt/tests/vlan_mpls_tests.rs:224-251);
 *   GTP-U   Udp::payload -> Gtpv1::parse (gtpv1/generated.rs:33-49) -> payload() (trim to
 *           packet_len, advance header_len, :98-108) -> the extension headers named by
 *           next_extention_header (ExtPduNumber, ExtUdpPort, ExtLongPduNumber,
 *           ExtServiceClassIndicator, ExtContainer, NrUp / PduSessionUp::group_parse, each
 *           its parse and payload()) -> Ipv4|Ipv6::parse (gtpv1_test.rs:199-231, 284-320,
 *           468-505);
 *   GRE     Ipv4|Ipv6::payload -> GreGroup::group_parse (gre/generated.rs:800-820) ->
 *           Gre::payload() (advance header_len) -> Ipv4|Ipv6|EtherFrame::parse
 *           (gre_test.rs:20-99).
 * Dispatch: an outer frame that parsed OK as UDP with destination port 4789 (VXLAN) or
 * 2152 (GTP-U), else with that source port; or an outer IPv4 (first fragment) / IPv6
 * frame whose upper-layer protocol is 47 (status L4_OTHER).  GTP-U carries an inner
 * packet only as a GTPv1 (version 1) G-PDU (message type 255), by the version nibble of
 * its first byte (4 / 6).  GRE's protocol type selects 0x0800 IPv4, 0x86DD IPv6,
 * 0x6558 Ethernet (transparent bridging).  IPv6 inner packets need RPKT_F_IPV6. */
enum rpkt_tun_kind {
    RPKT_TUN_NONE = 0,
    RPKT_TUN_VXLAN = 1,
    RPKT_TUN_GTPU = 2,
    RPKT_TUN_GRE = 3
};
enum rpkt_tun_status {
    RPKT_T_OK = 0,            /* tunnel decoded: the inner record holds the inner frame     */
    RPKT_T_NONE = 1,          /* no tunnel dispatch on this frame (kind NONE)               */
    RPKT_T_BAD = 2,           /* Vxlan::parse / Gtpv1::parse / GreGroup::group_parse Err     */
    RPKT_T_NOT_TPDU = 3,      /* GTP: not a GTPv1 G-PDU (version != 1 or message != 255)    */
    RPKT_T_EXT_BAD = 4,       /* GTP: an extension header's parse Err, an unknown next
                                 extension type, or more than RPKT_MAX_GTP_EXT of them      */
    RPKT_T_INNER_UNKNOWN = 5  /* the inner protocol is none of Ether / IPv4 / IPv6 (an
                                 IPv6 one without RPKT_F_IPV6, an empty T-PDU, GRE for
                                 PPTP's PPP payload): inner_type says what it is, or 0     */
};
#define RPKT_MAX_GTP_EXT 8

/* One frame's tunnel, 16 bytes. */
typedef struct rpkt_tun {
    uint8_t  kind;       /*  0 enum rpkt_tun_kind                                     */
    uint8_t  status;     /*  1 enum rpkt_tun_status                                   */
    uint16_t tun_off;    /*  2 frame offset of the VXLAN / GTPv1 / GRE header           */
    uint16_t inner_off;  /*  4 frame offset of the inner frame: the tunnel's payload()  */
    uint16_t inner_type; /*  6 0x6558 (an Ethernet frame), 0x0800, 0x86DD; GRE: its
                             protocol_type (0x880B for PPTP); GTP: 0 when the T-PDU's
                             version nibble is not 4 / 6                                 */
    uint32_t id;         /*  8 Vxlan::vni, Gtpv1::teid, Gre::key (0 without the K bit)  */
    uint8_t  hdr0;       /* 12 header byte 0: VXLAN flags (gbp_extention, vni_present),
                             GTPv1 version / protocol_type / E / S / PN, GRE C / R / K / S
                             / recursion_control                                         */
    uint8_t  hdr1;       /* 13 header byte 1: VXLAN dont_learn / policy_applied, GTPv1
                             message_type, GRE flags / version                           */
    uint16_t aux;        /* 14 Vxlan::group_id; Gtpv1::sequence (a 12-B header, else 0);
                             Gre::checksum (C or R bit, else 0)                          */
} rpkt_tun_t;

#define RPKT_TUN_BYTES 16u

/* Parse + verify a batch and decode one tunnel level per frame:
 *   outer_dev[i]  the record rpkt_gpu_parse_batch writes for frame i with the same flags;
 *   tun_dev[i]    its tunnel (kind NONE / status NONE when there is none);
 *   inner_dev[i]  the record of the inner frame [inner_off, the tunnel payload's end):
 *                 rpkt_gpu_parse_batch's record of those bytes (an inner IPv4 / IPv6
 *                 packet is parsed from its IP header: ethertype = inner_type, n_vlan 0,
 *                 MACs 0), with l3_off / l4_off / payload_off / ip6_pdst_off as offsets in
 *                 the OUTER frame (rpkt's Cursor::cursor() of the inner views) and
 *                 frame_len = the inner frame's length; status RPKT_S_NO_INNER (all else
 *                 0) when tun_dev[i].status != RPKT_T_OK.
 * flags: RPKT_F_IP_SUM, RPKT_F_L4_SUM, RPKT_F_IPV6, applied to both levels, and
 * RPKT_F_FLOW_EV: flow_ev_dev[i] (n * 8 B, 8-byte aligned; n_buckets 1..
 * RPKT_FLOW_MAX_BUCKETS) is the flow event of the INNER record when the tunnel decoded
 * (tun_dev[i].status == RPKT_T_OK: the inner 5-tuple, the inner frame's length, the inner
 * sums' bad bits -- per-subscriber / per-tenant accounting of the overlay through
 * rpkt_gpu_flow_count and rpkt_gpu_flow_reduce), else of the outer record, exactly as
 * rpkt_gpu_parse_batch forms it from a record.  Each byte is read from HBM about once:
 * the outer L4 sum (UDP, or GRE with its checksum) reuses the inner L4 sum's stream over
 * the bytes the two share.  outer_dev / inner_dev n * 80 B, tun_dev n * 16 B, all
 * 16-byte aligned. */
int rpkt_gpu_parse_tunnel_batch(const rpkt_batch_t* batch, uint32_t flags, rpkt_rec_t* outer_dev,
                                rpkt_tun_t* tun_dev, rpkt_rec_t* inner_dev,
                                rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream);

/* A receive ring of tunnelled bursts (a VTEP's / UPF's rx queue: the loopback_rx.rs:96-121
 * loop with the tunnel views of vlan_mpls_tests.rs:237-251 / gtpv1_test.rs:199-231 on
 * each frame) in one launch per RPKT_RING_MAX_SLOTS slots: results equal one
 * rpkt_gpu_parse_tunnel_batch call per slot, into that slot's outer_dev / tun_dev /
 * inner_dev (and flow_ev_dev when RPKT_F_FLOW_EV is set).  Slots with n == 0 are skipped;
 * every slot is checked before anything is launched; layouts may differ from slot to
 * slot. */
typedef struct rpkt_tun_ring_slot {
    rpkt_batch_t    batch;
    rpkt_rec_t*     outer_dev;
    rpkt_tun_t*     tun_dev;
    rpkt_rec_t*     inner_dev;
    rpkt_flow_ev_t* flow_ev_dev;
} rpkt_tun_ring_slot_t;
int rpkt_gpu_parse_tunnel_ring(const rpkt_tun_ring_slot_t* slots, uint32_t n_slots,
                               uint32_t flags, uint32_t n_buckets, void* stream);

/* ---- TX side ---------------------------------------------------------------- */

/* Build flags: fill a checksum the way the NIC TX offload requested by the
 * reference computes it (rpkt-dpdk/examples/loopback_rx.rs:133): field zeroed, the
 * complement of the RFC 1071 sum; a UDP result of 0 is sent as 0xffff.  Without the
 * flag the checksum field is the record's (a set_checksum setter value). */
#define RPKT_BUILD_IP_CSUM 1u
#define RPKT_BUILD_L4_CSUM 2u

/* Batched header build (benches/rpkt/rpkt_build.rs:9-28): for each frame i of
 * `batch` (payload already in place), write the headers the record recs_dev[i] asks
 * for, as Udp|Tcp::prepend_header + setters, Ipv4::prepend_header + setters,
 * VlanFrame::prepend_header + setters (n_vlan tags), EtherFrame::prepend_header +
 * setters would: l3 = 14 + 4 n_vlan, l4 = l3 + IHL*4, UDP (protocol 17, 8 B) or TCP
 * (6, the 20 fixed bytes; doff from l4_word6) or no L4 header.  Length fields are
 * set from the frame span (prepend_header's remaining()): IPv4 packet_len =
 * len - l3, UDP length = len - l4.  Option bytes are left as the buffer holds them.
 * A frame too short for its headers (where prepend_header asserts) is left
 * untouched; built_dev[i] (optional, n bytes) = 1 if written, else 0.  Records use
 * the rpkt_rec_t getter layout, so building from parse records reproduces frames.
 * frames_dev and recs_dev 16-byte aligned. */
int rpkt_gpu_build_batch(const rpkt_batch_t* batch, const rpkt_rec_t* recs_dev, uint32_t flags,
                         uint8_t* built_dev, void* stream);

/* Encapsulation build: rpkt_gpu_build_batch plus, for each frame whose tun_dev[i].kind is
 * not RPKT_TUN_NONE, the tunnel header written first, inside-out as the reference builds
 * these frames (the inner frame, and a GTP-U frame's extension headers, are payload already
 * in place):
 *   VXLAN  Vxlan::prepend_header + set_gbp_extention / set_vni_present / set_dont_learn /
 *          set_policy_applied (hdr0, hdr1) + set_group_id (aux) + set_vni (id), at the
 *          outer UDP payload (l4 + 8; the record's protocol must be 17), byte 7 0
 *          (vxlan/generated.rs:99-150; vlan_mpls_tests.rs:254-300);
 *   GTP-U  Gtpv1::prepend_header(header of hdr0, hdr1) (length = remaining - 8) + set_teid
 *          (id), and for a 12-B header (any of E/S/PN in hdr0) set_sequence (aux); bytes
 *          10-11 (npdu, next_extention_header) are left as the buffer holds them, as the
 *          extension headers after them (gtpv1/generated.rs:110-170, 254-310;
 *          gtpv1_test.rs:236-282);
 *   GRE    Gre::prepend_header(hdr0, hdr1) + set_protocol_type (inner_type), with a
 *          checksum word (C or R) = aux, or with RPKT_BUILD_L4_CSUM and the C bit the RFC
 *          2784 checksum over the GRE header and payload; a key word (K) = id; offset and
 *          sequence words left as the buffer holds them; at l4 (protocol 47)
 *          (gre/generated.rs:95-267; gre_test.rs:213-278).
 * The outer UDP checksum fill then covers the tunnel header.  status, tun_off and inner_off
 * are not read.  A frame whose tunnel header does not end within the frame and within
 * its first RPKT_TUN_BUILD_MAX_END bytes (the header window at any 16-B phase: every IPv4
 * outer frame and IPv6 ones with short extension chains), or does not match the record's
 * protocol, is left untouched (built 0).  tun_dev n * 16 B, 16-byte aligned. */
#define RPKT_TUN_BUILD_MAX_END 113u
int rpkt_gpu_build_tunnel_batch(const rpkt_batch_t* batch, const rpkt_rec_t* recs_dev,
                                const rpkt_tun_t* tun_dev, uint32_t flags, uint8_t* built_dev,
                                void* stream);

/* Firewall forward (rpkt-dpdk/examples/loopback_rx.rs:96-140), one fused pass per
 * frame: the parse chain of rpkt_gpu_parse_batch with both sums, then frame i is
 * forwarded when it is an untagged IPv4/UDP frame that parsed OK with a valid IPv4
 * sum and a valid UDP sum (or UDP checksum 0) -- the RX offload verdicts of the
 * reference -- and its source address is not in forbid_dev (n_forbid u32
 * addresses, sorted ascending).  A forwarded frame is rewritten in place: ports and
 * addresses swapped, TTL - 1 (wrapping), dst/src MAC = dmac/smac, IPv4 and UDP
 * checksums recomputed (the reference's TX offload).  keep_dev[i] = 1 if forwarded;
 * other frames are not written.  frames_dev 16-byte aligned.
 * With fwd->flags = RPKT_F_IPV6 the parse also decodes IPv6 and an untagged IPv6/UDP
 * frame is forwarded the same way: parsed OK with a valid L4 sum (a zero UDP checksum is
 * invalid over IPv6), never matched against the (IPv4) forbidden list; addresses (16 B)
 * and ports swapped, hop_limit - 1 (wrapping), MACs set, the UDP checksum updated over
 * the IPv6 pseudo header (its destination stays a routing header's final address).
 * IPv6 records are built by rpkt_gpu_build_batch as Ipv6::prepend_header + setters
 * (ipv6/generated.rs:94-135): bytes 0..7 of the header from the record (ip6_vtcfl,
 * payload_len = remaining, next_header, hop_limit), the addresses and the extension
 * headers up to l4_off left as the buffer holds them (the record keeps the addresses
 * folded), the L4 checksum over the IPv6 pseudo header (src, the address at
 * ip6_pdst_off -- dst_addr when that offset does not lie in [l3 + 24, l4_off - 16] --,
 * u32 length, next header), a UDP result of 0 sent as 0xffff. */
typedef struct rpkt_fwd {
    uint8_t         dmac[6];
    uint8_t         smac[6];
    const uint32_t* forbid_dev;
    uint32_t        n_forbid;
    uint32_t        flags;      /* 0, or RPKT_F_IPV6 (was `reserved`, always 0) */
} rpkt_fwd_t;
int rpkt_gpu_forward_batch(const rpkt_batch_t* batch, const rpkt_fwd_t* fwd, uint8_t* keep_dev,
                           void* stream);

/* ---- Option iterators ----------------------------------------------------------- */

/* Why an option walk stopped (the iterator's next() returned None). */
enum rpkt_opt_stop {
    RPKT_OPT_NONE = 0,       /* no option slice: that header was not parsed */
    RPKT_OPT_END = 1,        /* the slice was consumed (buf.len() < 1) */
    RPKT_OPT_UNKNOWN = 2,    /* a type outside the option group */
    RPKT_OPT_MALFORMED = 3   /* the type's parse returned Err (short or bad length) */
};

/* Option kind indices (bits of *_kinds, 4-bit codes index + 1 in *_trace).
 * TCP (tcp/generated.rs:1357-1366): 0 Eol, 1 Nop, 2 Mss, 3 WindowScale,
 *   4 SackPermitted, 5 Sack, 6 Timestamp, 7 FastOpen.
 * IPv4 (ipv4/generated.rs:1595-1604): 0 Eol, 1 Nop, 2 Timestamp (68),
 *   3 RecordRoute (7), 4 RouteAlert (148), 5 CommercialSecurity (134),
 *   6 StrictSourceRoute (137), 7 LooseSourceRoute (131). */

/* One frame's option walks, 64 bytes: TcpOptionsIter over tcp.var_header_slice()
 * and Ipv4OptionsIter over ipv4.var_header_slice(), with the getters of the options
 * they yield (the last one of each kind). */
typedef struct rpkt_opts {
    uint8_t  tcp_count;         /*  0 options yielded                         */
    uint8_t  tcp_stop;          /*  1 rpkt_opt_stop                           */
    uint8_t  tcp_wscale;        /*  2 WindowScale::shift_count                */
    uint8_t  tcp_sack_blocks;   /*  3 (Sack::header_len - 2) / 8              */
    uint16_t tcp_kinds;         /*  4 bit k: kind index k yielded             */
    uint16_t tcp_mss;           /*  6 Mss::mss                                */
    uint32_t tcp_ts;            /*  8 Timestamp::ts                           */
    uint32_t tcp_ts_echo;       /* 12 Timestamp::ts_echo                      */
    uint32_t tcp_sack_left;     /* 16 first SACK block (Sack var_header_slice) */
    uint32_t tcp_sack_right;    /* 20                                         */
    uint16_t tcp_fo_len;        /* 24 FastOpen::header_len                    */
    uint8_t  tcp_end;           /* 26 slice bytes consumed when the walk stopped */
    uint8_t  ip_end;            /* 27                                         */
    uint8_t  ip_count;          /* 28                                         */
    uint8_t  ip_stop;           /* 29                                         */
    uint16_t ip_kinds;          /* 30                                         */
    uint16_t ip_route_alert;    /* 32 RouteAlert::data                        */
    uint8_t  ip_rr_len;         /* 34 RecordRoute::header_len                 */
    uint8_t  ip_rr_pointer;     /* 35 RecordRoute::pointer                    */
    uint8_t  ip_ts_len;         /* 36 Timestamp::header_len                   */
    uint8_t  ip_ts_pointer;     /* 37 Timestamp::pointer                      */
    uint8_t  ip_ts_oflw_flg;    /* 38 oflw << 4 | flg                         */
    uint8_t  ip_sr_pointer;     /* 39 Strict/LooseSourceRoute::pointer        */
    uint32_t ip_sr_dest;        /* 40 Strict/LooseSourceRoute::dest_addr      */
    uint32_t ip_cs_doi;         /* 44 CommercialSecurity::doi                 */
    uint64_t tcp_trace;         /* 48 kinds of the first 16 options, 4 bits each (index + 1) */
    uint64_t ip_trace;          /* 56                                         */
} rpkt_opts_t;

#define RPKT_OPTS_BYTES 64u

/* IPv6 frames (records of an RPKT_F_IPV6 parse): TcpOptionsIter as for IPv4, and in
 * place of the IPv4 walk, Ipv6OptionsIter (ipv6/generated.rs:1556-1615) over the
 * var_header_slice() of every HopByHopOption / DestOptions header of the extension chain
 * the parse walked ([l3 + 40, l4)), in order (ipv6_test.rs:47-69, 154-175); a malformed
 * option ends the walking.  Kinds (bits of ip_kinds, codes index + 1 in ip_trace):
 * 0 Pad0, 1 PadN, 2 RouterAlert, 3 Generic (every other type).  The IPv6 view of bytes
 * 27..47:
 *   27 ip_end          bytes consumed in the last header walked
 *   28 ip_count        options yielded over every header walked
 *   29 ip_stop         NONE (no options header), END, or MALFORMED
 *   30 ip_kinds
 *   32 ip_route_alert  RouterAlert::router_alert (the last one)
 *   34 u8 generic type / 35 u8 generic data length: Generic::type_ and header_len - 2
 *   36 u8 option headers walked / 37 u8 the first one's type (0 HopByHop, 60 DestOptions)
 *   40 u32 generic data: the first <= 4 bytes of that Generic's var_header_slice(),
 *          big-endian, zero-filled (ipv6_test.rs:54)
 * other bytes of the half are 0. */

/* Walk the IPv4 and TCP options of every frame of a parsed batch: recs_dev from
 * rpkt_gpu_parse_batch on the same batch locates the slices (ip: [l3 + 20, l4),
 * tcp: [l4 + 20, payload_off) for status OK / TCP).  opts_dev n * 64 B, 16-B aligned.
 * For an IPv6 record the first header of the extension chain is the record's
 * ip6_next_header (byte 30), which the parse copied from frame byte l3 + 6: the records
 * must come from a parse of these same frames (the compact entry below, whose record has
 * no such field, reads frame byte l3 + 6 itself; both agree whenever that holds). */
int rpkt_gpu_options_batch(const rpkt_batch_t* batch, const rpkt_rec_t* recs_dev,
                           rpkt_opts_t* opts_dev, void* stream);

/* The same walks located by compact records (rpkt_gpu_parse_batch_compact on the same
 * batch): status, ip_protocol, l3_off, l4_off and payload_off (the TCP slice's end)
 * are all the walks read, so the 16-B record serves as well as the 80-B one and the
 * results are identical.  recs_dev n * 16 B, opts_dev n * 64 B, both 16-byte aligned. */
int rpkt_gpu_options_batch_compact(const rpkt_batch_t* batch, const rpkt_rec16_t* recs_dev,
                                   rpkt_opts_t* opts_dev, void* stream);

/* Parse + verify and the option walks in one pass: rpkt_gpu_parse_batch's records (and
 * flow events) plus, per frame, the rpkt_opts_t that rpkt_gpu_options_batch would
 * produce from those records -- the walks run on the header bytes the parse has just
 * read, as rpkt's iterators walk the var_header_slice() of the views the parse returned
 * (ipv4/generated.rs:57-60, 1625-1722; tcp/generated.rs:1387-1484), so the option bytes
 * are not fetched a second time.  Outputs are byte-identical to the two separate calls.
 * opts_dev n * 64 B, 16-byte aligned. */
int rpkt_gpu_parse_options_batch(const rpkt_batch_t* batch, uint32_t flags,
                                 rpkt_rec_t* recs_dev, rpkt_opts_t* opts_dev,
                                 rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets, void* stream);
/* The same with compact records (rpkt_gpu_parse_batch_compact's rpkt_rec16_t). */
int rpkt_gpu_parse_options_batch_compact(const rpkt_batch_t* batch, uint32_t flags,
                                         rpkt_rec16_t* recs_dev, rpkt_opts_t* opts_dev,
                                         rpkt_flow_ev_t* flow_ev_dev, uint32_t n_buckets,
                                         void* stream);

/* ---- Protocol layer walk ---------------------------------------------------------- */

/* The protocol stack of each frame, walked with the header views of every protocol
 * rpkt generates from its pktfmt specs (include/rpkt_protocols.h): each layer is the
 * protocol's group_parse / parse (the pktfmt codegen rules: header_len, payload_len /
 * packet_len checks against chunk() and remaining()) and payload() (trim, advance).
 * Which group follows a layer is the dispatch a receive loop writes by hand in the
 * reference (ethertype, IP protocol / next header, UDP ports 4789 VXLAN and
 * 2152 / 2123 GTP, GRE protocol type, MPLS bottom of stack, PPPoE data type,
 * LLC 0x42 STP); DESIGN.md lists it. */
enum rpkt_layer_stop {
    RPKT_L_END = 1,        /* a terminal protocol (TCP, UDP payload, ICMP, ARP, STP, ...) */
    RPKT_L_UNKNOWN = 2,    /* the next protocol is outside the graph: next_key holds it */
    RPKT_L_ERR = 3,        /* the next group's parse returned Err: err_group names it */
    RPKT_L_MAX = 4         /* RPKT_MAX_LAYERS layers walked */
};
#define RPKT_MAX_LAYERS 16

typedef struct rpkt_layers {
    uint8_t  n;                       /*  0 layers parsed                           */
    uint8_t  stop;                    /*  1 rpkt_layer_stop                         */
    uint8_t  err_group;               /*  2 RPKT_GROUP_* the walk failed in (ERR)   */
    uint8_t  key_proto;               /*  3 UNKNOWN: protocol whose next key it is  */
    uint16_t payload_off;             /*  4 cursor after the last layer's payload() */
    uint16_t reserved;                /*  6                                         */
    uint32_t payload_len;             /*  8 remaining() of that payload             */
    uint32_t next_key;                /* 12 UNKNOWN: the unrecognised value         */
    uint8_t  proto[RPKT_MAX_LAYERS];  /* 16 RPKT_P_* of layer k                     */
    uint16_t off[RPKT_MAX_LAYERS];    /* 32 offset of layer k in the frame          */
} rpkt_layers_t;

#define RPKT_LAYERS_BYTES 64u

/* layers_dev n * 64 B, 16-byte aligned. */
int rpkt_gpu_layers_batch(const rpkt_batch_t* batch, rpkt_layers_t* layers_dev, void* stream);

/* ---- Field getters over the layer walk ---------------------------------------------- */

/* The header-field getters rpkt generates for every protocol of the walk
 * (pktfmt/src/codegen/field.rs:115-250, `read_repr` / `read_multi_bytes`): a field of
 * `bits` bits at bit `bit_off` of the protocol's header is the big-endian integer of
 * bytes [bit_off/8, (bit_off+bits-1)/8], shifted right by 7 - (end bit in its byte)
 * and masked to `bits` bits.  Byte-slice fields (MAC, IPv6 addresses) are
 * byte-aligned: a request of up to 64 bits of one returns those bytes as a big-endian
 * integer (ask for a 128-bit address as two 64-bit halves).  Offsets and widths per
 * field come from the same specs (rpkt_amd/proto_fields.json).
 *
 * Request r of frame i reads the `nth` (0 = outermost) layer k of rpkt_layers_t i
 * whose proto[k] == proto.  values_dev[i * n_req + r] is the field, or 0 when the
 * frame has no such layer or the field's bytes pass the frame's end; bit r of
 * present_dev[i] (optional, may be NULL) says which.  Replaces, per frame, the
 * getter calls a receive loop makes on the header views it parsed, e.g.
 * Ipv6::src_addr (ipv6/generated.rs), Arp::operation, Vxlan::vni, Gtpv1::teid. */
typedef struct rpkt_field_req {
    uint8_t  proto;      /* RPKT_P_*                                             */
    uint8_t  nth;        /* occurrence of proto in the stack, 0 = outermost      */
    uint8_t  bits;       /* 1..64                                                */
    uint8_t  reserved;   /* 0                                                    */
    uint16_t bit_off;    /* from the start of the protocol's header              */
    uint16_t reserved2;  /* 0                                                    */
} rpkt_field_req_t;

#define RPKT_MAX_FIELD_REQS 32

/* reqs: host memory, n_req in 1..RPKT_MAX_FIELD_REQS; layers_dev from
 * rpkt_gpu_layers_batch on the same batch; values_dev n * n_req * 8 B, 8-B aligned;
 * present_dev n * 4 B or NULL. */
int rpkt_gpu_fields_batch(const rpkt_batch_t* batch, const rpkt_layers_t* layers_dev,
                          const rpkt_field_req_t* reqs, uint32_t n_req, uint64_t* values_dev,
                          uint32_t* present_dev, void* stream);

/* 5-tuple hash used for flow buckets (host copy of the device function). */
uint32_t rpkt_flow_hash(uint32_t ip_src, uint32_t ip_dst, uint16_t src_port,
                        uint16_t dst_port, uint8_t protocol);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RPKT_GPU_H */
