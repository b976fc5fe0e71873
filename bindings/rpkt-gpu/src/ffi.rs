//! Raw bindings of `include/rpkt_gpu.h` (the C ABI of `librpkt_gpu.so`).
//!
//! Every declaration here mirrors the header one for one: `tests/test_rust_binding.py`
//! checks the function names and arities against the header and every `#[repr(C)]`
//! struct's field order and widths against the C layout (`offsetof` from a compiled
//! probe), so the two cannot drift apart silently.
#![allow(non_camel_case_types)]

use core::ffi::{c_char, c_int, c_void};

pub const RPKT_ABI_VERSION: u32 = 1;
pub const RPKT_MAX_VLAN: usize = 2;
pub const RPKT_REC_BYTES: usize = 80;
pub const RPKT_REC16_BYTES: usize = 16;
pub const RPKT_OPTS_BYTES: usize = 64;
pub const RPKT_LAYERS_BYTES: usize = 64;
pub const RPKT_TUN_BYTES: usize = 16;
pub const RPKT_MAX_GTP_EXT: usize = 8;
// enum rpkt_tun_kind / rpkt_tun_status
pub const RPKT_TUN_NONE: u8 = 0;
pub const RPKT_TUN_VXLAN: u8 = 1;
pub const RPKT_TUN_GTPU: u8 = 2;
pub const RPKT_TUN_GRE: u8 = 3;
pub const RPKT_T_OK: u8 = 0;
pub const RPKT_T_NONE: u8 = 1;
pub const RPKT_T_BAD: u8 = 2;
pub const RPKT_T_NOT_TPDU: u8 = 3;
pub const RPKT_T_EXT_BAD: u8 = 4;
pub const RPKT_T_INNER_UNKNOWN: u8 = 5;
pub const RPKT_MAX_LAYERS: usize = 16;
pub const RPKT_MAX_FIELD_REQS: u32 = 32;
pub const RPKT_FLOW_MAX_BUCKETS: u32 = 65535;
pub const RPKT_COLL_ID_BYTES: usize = 128;

// enum rpkt_status: which rpkt `parse` returned Err first
pub const RPKT_S_OK: u8 = 0;
pub const RPKT_S_ETH_SHORT: u8 = 1;
pub const RPKT_S_VLAN_SHORT: u8 = 2;
pub const RPKT_S_NOT_IPV4: u8 = 3;
pub const RPKT_S_IP_SHORT: u8 = 4;
pub const RPKT_S_IP_BAD_IHL: u8 = 5;
pub const RPKT_S_IP_IHL_GT_LEN: u8 = 6;
pub const RPKT_S_IP_TOT_LT_IHL: u8 = 7;
pub const RPKT_S_IP_TOT_GT_LEN: u8 = 8;
pub const RPKT_S_L4_OTHER: u8 = 9;
pub const RPKT_S_UDP_SHORT: u8 = 10;
pub const RPKT_S_UDP_BAD_LEN: u8 = 11;
pub const RPKT_S_TCP_SHORT: u8 = 12;
pub const RPKT_S_TCP_BAD_DOFF: u8 = 13;
pub const RPKT_S_IP6_SHORT: u8 = 14;
pub const RPKT_S_IP6_BAD_LEN: u8 = 15;
pub const RPKT_S_IP6_EXT_SHORT: u8 = 16;
pub const RPKT_S_IP6_EXT_BAD_LEN: u8 = 17;
pub const RPKT_S_IP6_FRAGMENT: u8 = 18;
pub const RPKT_S_ICMP_EMPTY: u8 = 19;
pub const RPKT_S_NO_INNER: u8 = 20;
pub const RPKT_MAX_IP6_EXT: usize = 8;

// enum rpkt_err
pub const RPKT_OK: c_int = 0;
pub const RPKT_E_INVAL: c_int = -1;
pub const RPKT_E_HIP: c_int = -2;
pub const RPKT_E_TOO_LARGE: c_int = -3;
pub const RPKT_E_ALIGN: c_int = -4;
pub const RPKT_E_COLL: c_int = -5;

// enum rpkt_flags / build flags
pub const RPKT_F_IP_SUM: u32 = 1;
pub const RPKT_F_L4_SUM: u32 = 2;
pub const RPKT_F_FLOW_EV: u32 = 4;
pub const RPKT_F_IPV6: u32 = 8;
pub const RPKT_BUILD_IP_CSUM: u32 = 1;
pub const RPKT_BUILD_L4_CSUM: u32 = 2;

// enum rpkt_opt_stop / rpkt_layer_stop
pub const RPKT_OPT_NONE: u8 = 0;
pub const RPKT_OPT_END: u8 = 1;
pub const RPKT_OPT_UNKNOWN: u8 = 2;
pub const RPKT_OPT_MALFORMED: u8 = 3;
pub const RPKT_L_END: u8 = 1;
pub const RPKT_L_UNKNOWN: u8 = 2;
pub const RPKT_L_ERR: u8 = 3;
pub const RPKT_L_MAX: u8 = 4;

/// One parsed frame: every getter of the Ether / VLAN / IPv4 / UDP|TCP chain, the
/// payload cursors and the two RFC 1071 sums (include/rpkt_gpu.h, 80 bytes).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_rec_t {
    pub status: u8,
    pub n_vlan: u8,
    pub ethertype: u16,
    pub dst_addr: [u8; 6],
    pub src_addr: [u8; 6],
    pub vlan_tci: [u16; 2],
    pub vlan_ethertype: [u16; 2],
    pub ip_vhl: u8,
    pub ip_tos: u8,
    pub ip_packet_len: u16,
    pub ip_ident: u16,
    pub ip_frag: u16,
    pub ip_ttl: u8,
    pub ip_protocol: u8,
    pub ip_checksum: u16,
    pub ip_src: u32,
    pub ip_dst: u32,
    pub src_port: u16,
    pub dst_port: u16,
    pub tcp_seq: u32,
    pub tcp_ack: u32,
    pub l4_word6: u16,
    pub tcp_window: u16,
    pub l4_checksum: u16,
    pub tcp_urgent: u16,
    pub l3_off: u16,
    pub l4_off: u16,
    pub payload_off: u16,
    pub payload_len: u16,
    pub ip_sum: u16,
    pub l4_sum: u16,
    pub frame_len: u32,
}
const _: () = assert!(core::mem::size_of::<rpkt_rec_t>() == RPKT_REC_BYTES);

/// Compact record: the cursors and verdicts (16 bytes).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_rec16_t {
    pub status: u8,
    pub n_vlan: u8,
    pub ip_protocol: u8,
    pub verdict: u8,
    pub l3_off: u16,
    pub l4_off: u16,
    pub payload_off: u16,
    pub payload_len: u16,
    pub ip_sum: u16,
    pub l4_sum: u16,
}
const _: () = assert!(core::mem::size_of::<rpkt_rec16_t>() == RPKT_REC16_BYTES);

pub type rpkt_flow_ev_t = u64;

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rpkt_batch_t {
    pub frames_dev: *const u8,
    pub frames_bytes: u64,
    pub offsets_dev: *const u32,
    pub stride: u32,
    pub frame_len: u32,
    pub n: u32,
    pub reserved: u32,
}

/// One slot of a receive ring (rpkt_gpu_parse_ring): a batch, its records and (with
/// RPKT_F_FLOW_EV) its flow events.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rpkt_ring_slot_t {
    pub batch: rpkt_batch_t,
    /// `*mut rpkt_rec_t` for rpkt_gpu_parse_ring, `*mut rpkt_rec16_t` for the compact call
    pub recs_dev: *mut c_void,
    pub flow_ev_dev: *mut rpkt_flow_ev_t,
}
pub const RPKT_RING_MAX_SLOTS: u32 = 32;

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rpkt_chains_t {
    pub buf_dev: *const u8,
    pub buf_bytes: u64,
    pub segs_dev: *const u32,
    pub chain_first_dev: *const u32,
    pub n_segs: u32,
    pub n_chains: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rpkt_fwd_t {
    pub dmac: [u8; 6],
    pub smac: [u8; 6],
    pub forbid_dev: *const u32,
    pub n_forbid: u32,
    /// 0, or RPKT_F_IPV6: also forward untagged IPv6/UDP frames
    pub flags: u32,
}

/// One frame's option walks (TcpOptionsIter / Ipv4OptionsIter), 64 bytes.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_opts_t {
    pub tcp_count: u8,
    pub tcp_stop: u8,
    pub tcp_wscale: u8,
    pub tcp_sack_blocks: u8,
    pub tcp_kinds: u16,
    pub tcp_mss: u16,
    pub tcp_ts: u32,
    pub tcp_ts_echo: u32,
    pub tcp_sack_left: u32,
    pub tcp_sack_right: u32,
    pub tcp_fo_len: u16,
    pub tcp_end: u8,
    pub ip_end: u8,
    pub ip_count: u8,
    pub ip_stop: u8,
    pub ip_kinds: u16,
    pub ip_route_alert: u16,
    pub ip_rr_len: u8,
    pub ip_rr_pointer: u8,
    pub ip_ts_len: u8,
    pub ip_ts_pointer: u8,
    pub ip_ts_oflw_flg: u8,
    pub ip_sr_pointer: u8,
    pub ip_sr_dest: u32,
    pub ip_cs_doi: u32,
    pub tcp_trace: u64,
    pub ip_trace: u64,
}
const _: () = assert!(core::mem::size_of::<rpkt_opts_t>() == RPKT_OPTS_BYTES);

/// One frame's tunnel (rpkt_gpu_parse_tunnel_batch), 16 bytes.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_tun_t {
    pub kind: u8,
    pub status: u8,
    pub tun_off: u16,
    pub inner_off: u16,
    pub inner_type: u16,
    pub id: u32,
    pub hdr0: u8,
    pub hdr1: u8,
    pub aux: u16,
}
const _: () = assert!(core::mem::size_of::<rpkt_tun_t>() == RPKT_TUN_BYTES);

/// One slot of a ring of tunnelled bursts (rpkt_gpu_parse_tunnel_ring): a batch, its outer,
/// tunnel and inner records and (with RPKT_F_FLOW_EV) its flow events.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rpkt_tun_ring_slot_t {
    pub batch: rpkt_batch_t,
    pub outer_dev: *mut rpkt_rec_t,
    pub tun_dev: *mut rpkt_tun_t,
    pub inner_dev: *mut rpkt_rec_t,
    pub flow_ev_dev: *mut rpkt_flow_ev_t,
}

/// One frame's protocol stack from the pktfmt-derived walk, 64 bytes.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_layers_t {
    pub n: u8,
    pub stop: u8,
    pub err_group: u8,
    pub key_proto: u8,
    pub payload_off: u16,
    pub reserved: u16,
    pub payload_len: u32,
    pub next_key: u32,
    pub proto: [u8; RPKT_MAX_LAYERS],
    pub off: [u16; RPKT_MAX_LAYERS],
}
const _: () = assert!(core::mem::size_of::<rpkt_layers_t>() == RPKT_LAYERS_BYTES);

#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct rpkt_field_req_t {
    pub proto: u8,
    pub nth: u8,
    pub bits: u8,
    pub reserved: u8,
    pub bit_off: u16,
    pub reserved2: u16,
}
const _: () = assert!(core::mem::size_of::<rpkt_field_req_t>() == 8);

extern "C" {
    pub fn rpkt_gpu_abi_version() -> u32;
    pub fn rpkt_gpu_build_info() -> *const c_char;
    pub fn rpkt_gpu_status_name(status: c_int) -> *const c_char;
    pub fn rpkt_gpu_last_hip_error() -> c_int;
    pub fn rpkt_gpu_device_info(buf: *mut c_char, len: usize) -> c_int;

    pub fn rpkt_gpu_parse_batch(batch: *const rpkt_batch_t, flags: u32, recs_dev: *mut rpkt_rec_t,
                                flow_ev_dev: *mut rpkt_flow_ev_t, n_buckets: u32,
                                stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_parse_batch_compact(batch: *const rpkt_batch_t, flags: u32,
                                        recs_dev: *mut rpkt_rec16_t,
                                        flow_ev_dev: *mut rpkt_flow_ev_t, n_buckets: u32,
                                        stream: *mut c_void) -> c_int;

    /// Every slot parsed as by rpkt_gpu_parse_batch (or _compact), RPKT_RING_MAX_SLOTS
    /// slots per launch.
    pub fn rpkt_gpu_parse_ring(slots: *const rpkt_ring_slot_t, n_slots: u32, flags: u32,
                               n_buckets: u32, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_parse_ring_compact(slots: *const rpkt_ring_slot_t, n_slots: u32, flags: u32,
                                       n_buckets: u32, stream: *mut c_void) -> c_int;

    pub fn rpkt_gpu_flow_workspace_bytes(n: u32, n_buckets: u32) -> usize;
    pub fn rpkt_gpu_flow_count(flow_ev_dev: *const rpkt_flow_ev_t, n: u32, n_buckets: u32,
                               counters_dev: *mut u64, workspace_dev: *mut c_void,
                               stream: *mut c_void) -> c_int;
    /// One RCCL all-reduce (root = -1) or reduce-to-root of u64[(n_buckets+1)*4] on the
    /// caller's communicator (an `ncclComm_t`, e.g. from ncclCommInitRank).
    pub fn rpkt_gpu_flow_reduce(counters_dev: *mut u64, n_buckets: u32, root: c_int,
                                nccl_comm: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_last_coll_error() -> c_int;
    pub fn rpkt_gpu_coll_version() -> c_int;
    /// ncclGetUniqueId into `id_out` (RPKT_COLL_ID_BYTES bytes), on rank 0.
    pub fn rpkt_gpu_coll_unique_id(id_out: *mut u8) -> c_int;
    /// ncclCommInitRank on the current device; collective over `world` ranks.
    pub fn rpkt_gpu_comm_init(comm_out: *mut *mut c_void, world: c_int, id: *const u8,
                              rank: c_int) -> c_int;
    pub fn rpkt_gpu_comm_destroy(comm: *mut c_void) -> c_int;
    /// rpkt_gpu_comm_init with a deadline: non-blocking init polled for `timeout_ms`,
    /// aborted (RPKT_E_COLL, last_coll_error 7) when not every rank joins in time.
    pub fn rpkt_gpu_comm_init_timeout(comm_out: *mut *mut c_void, world: c_int, id: *const u8,
                                      rank: c_int, timeout_ms: c_int) -> c_int;
    /// ncclCommAbort: release a communicator without waiting for its peers.
    pub fn rpkt_gpu_comm_abort(comm: *mut c_void) -> c_int;

    pub fn rpkt_gpu_checksum_ranges(buf_dev: *const u8, buf_bytes: u64, ranges_dev: *const u32,
                                    n: u32, out_dev: *mut u16, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_checksum_chains_workspace_bytes(n_segs: u32) -> usize;
    pub fn rpkt_gpu_checksum_chains(buf_dev: *const u8, buf_bytes: u64, segs_dev: *const u32,
                                    n_segs: u32, chain_first_dev: *const u32, n_chains: u32,
                                    out_dev: *mut u16, workspace_dev: *mut c_void,
                                    stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_parse_chains(chains: *const rpkt_chains_t, flags: u32,
                                 recs_dev: *mut rpkt_rec_t, flow_ev_dev: *mut rpkt_flow_ev_t,
                                 n_buckets: u32, stream: *mut c_void) -> c_int;

    pub fn rpkt_gpu_build_batch(batch: *const rpkt_batch_t, recs_dev: *const rpkt_rec_t,
                                flags: u32, built_dev: *mut u8, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_forward_batch(batch: *const rpkt_batch_t, fwd: *const rpkt_fwd_t,
                                  keep_dev: *mut u8, stream: *mut c_void) -> c_int;

    pub fn rpkt_gpu_options_batch(batch: *const rpkt_batch_t, recs_dev: *const rpkt_rec_t,
                                  opts_dev: *mut rpkt_opts_t, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_options_batch_compact(batch: *const rpkt_batch_t,
                                          recs_dev: *const rpkt_rec16_t,
                                          opts_dev: *mut rpkt_opts_t, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_parse_options_batch(batch: *const rpkt_batch_t, flags: u32,
                                        recs_dev: *mut rpkt_rec_t, opts_dev: *mut rpkt_opts_t,
                                        flow_ev_dev: *mut rpkt_flow_ev_t, n_buckets: u32,
                                        stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_parse_options_batch_compact(batch: *const rpkt_batch_t, flags: u32,
                                                recs_dev: *mut rpkt_rec16_t,
                                                opts_dev: *mut rpkt_opts_t,
                                                flow_ev_dev: *mut rpkt_flow_ev_t, n_buckets: u32,
                                                stream: *mut c_void) -> c_int;

    pub fn rpkt_gpu_parse_tunnel_batch(batch: *const rpkt_batch_t, flags: u32,
                                       outer_dev: *mut rpkt_rec_t, tun_dev: *mut rpkt_tun_t,
                                       inner_dev: *mut rpkt_rec_t,
                                       flow_ev_dev: *mut rpkt_flow_ev_t, n_buckets: u32,
                                       stream: *mut c_void) -> c_int;
    /// Every slot parsed as by rpkt_gpu_parse_tunnel_batch, RPKT_RING_MAX_SLOTS slots per
    /// launch.
    pub fn rpkt_gpu_parse_tunnel_ring(slots: *const rpkt_tun_ring_slot_t, n_slots: u32,
                                      flags: u32, n_buckets: u32, stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_build_tunnel_batch(batch: *const rpkt_batch_t, recs_dev: *const rpkt_rec_t,
                                       tun_dev: *const rpkt_tun_t, flags: u32, built_dev: *mut u8,
                                       stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_layers_batch(batch: *const rpkt_batch_t, layers_dev: *mut rpkt_layers_t,
                                 stream: *mut c_void) -> c_int;
    pub fn rpkt_gpu_fields_batch(batch: *const rpkt_batch_t, layers_dev: *const rpkt_layers_t,
                                 reqs: *const rpkt_field_req_t, n_req: u32, values_dev: *mut u64,
                                 present_dev: *mut u32, stream: *mut c_void) -> c_int;

    pub fn rpkt_flow_hash(ip_src: u32, ip_dst: u32, src_port: u16, dst_port: u16,
                          protocol: u8) -> u32;
}
