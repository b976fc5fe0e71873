"""Record layout of include/rpkt_gpu.h (rpkt_rec_t, 80 bytes) as a numpy dtype,
status names and the flow-event bit layout.  Pure host code, no device calls."""
import numpy as np

REC_BYTES = 80

REC_DTYPE = np.dtype([
    ("status", "u1"), ("n_vlan", "u1"), ("ethertype", "<u2"),
    ("dst_addr", "u1", (6,)), ("src_addr", "u1", (6,)),
    ("vlan_tci", "<u2", (2,)), ("vlan_ethertype", "<u2", (2,)),
    ("ip_vhl", "u1"), ("ip_tos", "u1"), ("ip_packet_len", "<u2"), ("ip_ident", "<u2"),
    ("ip_frag", "<u2"), ("ip_ttl", "u1"), ("ip_protocol", "u1"), ("ip_checksum", "<u2"),
    ("ip_src", "<u4"), ("ip_dst", "<u4"),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("tcp_seq", "<u4"), ("tcp_ack", "<u4"),
    ("l4_word6", "<u2"), ("tcp_window", "<u2"), ("l4_checksum", "<u2"), ("tcp_urgent", "<u2"),
    ("l3_off", "<u2"), ("l4_off", "<u2"), ("payload_off", "<u2"), ("payload_len", "<u2"),
    ("ip_sum", "<u2"), ("l4_sum", "<u2"), ("frame_len", "<u4"),
])
assert REC_DTYPE.itemsize == REC_BYTES

REC16_BYTES = 16
REC16_DTYPE = np.dtype([          # rpkt_rec16_t (include/rpkt_gpu.h), 16 B
    ("status", "u1"), ("n_vlan", "u1"), ("ip_protocol", "u1"), ("verdict", "u1"),
    ("l3_off", "<u2"), ("l4_off", "<u2"), ("payload_off", "<u2"), ("payload_len", "<u2"),
    ("ip_sum", "<u2"), ("l4_sum", "<u2"),
])
assert REC16_DTYPE.itemsize == REC16_BYTES


def project16(recs, flags):
    """The compact records rpkt_gpu_parse_batch_compact writes, from full records
    (the projection include/rpkt_gpu.h defines; used to check the GPU against the
    oracle's full records)."""
    out = np.zeros(recs.shape[0], dtype=REC16_DTYPE)
    for k in ("status", "n_vlan", "ip_protocol", "l3_off", "l4_off", "payload_off",
              "payload_len", "ip_sum", "l4_sum"):
        out[k] = recs[k]
    v6 = is_ip6(recs)
    ip6_parsed = v6 & ~np.isin(recs["status"], [STATUS["IP6_SHORT"], STATUS["IP6_BAD_LEN"]])
    ip_ok = np.where(v6, ip6_parsed, recs["ip_sum"] == 0xffff) & bool(flags & F_IP_SUM)
    l4_ok = bool(flags & F_L4_SUM) & (recs["status"] == 0) & (
        (recs["l4_sum"] == 0xffff) |
        (~v6 & (recs["ip_protocol"] == 17) & (recs["l4_checksum"] == 0)))
    out["verdict"] = (ip_ok.astype(np.uint8) | (l4_ok.astype(np.uint8) << 1) |
                      (v6.astype(np.uint8) << 2))
    return out


def dispatch_ethertype(recs):
    """The ethertype the IP parse was chosen on: ethertype, or the last VLAN tag's."""
    nv = recs["n_vlan"].astype(np.int64)
    last = recs["vlan_ethertype"][np.arange(recs.shape[0]), np.clip(nv - 1, 0, 1)]
    return np.where(nv > 0, last, recs["ethertype"])


def is_ip6(recs):
    """Records that hold the IPv6 block (include/rpkt_gpu.h): dispatched to Ipv6::parse."""
    pre = np.isin(recs["status"], [STATUS["ETH_SHORT"], STATUS["VLAN_SHORT"], STATUS["NOT_IPV4"]])
    return ~pre & (dispatch_ethertype(recs) == 0x86DD)


def ip6_block(recs):
    """The IPv6 view of record bytes 24..43 (include/rpkt_gpu.h) as a structured array."""
    raw = np.ascontiguousarray(recs).view(np.uint8).reshape(-1, REC_BYTES)[:, 24:44]
    return np.ascontiguousarray(raw).view(IP6_BLOCK_DTYPE).reshape(-1)


def as_records16(raw):
    """View a uint8 buffer of n*16 bytes as compact records."""
    a = np.asarray(raw)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a.reshape(-1).view(REC16_DTYPE)


# enum rpkt_status (include/rpkt_gpu.h)
STATUS = {
    "OK": 0, "ETH_SHORT": 1, "VLAN_SHORT": 2, "NOT_IPV4": 3, "IP_SHORT": 4,
    "IP_BAD_IHL": 5, "IP_IHL_GT_LEN": 6, "IP_TOT_LT_IHL": 7, "IP_TOT_GT_LEN": 8,
    "L4_OTHER": 9, "UDP_SHORT": 10, "UDP_BAD_LEN": 11, "TCP_SHORT": 12, "TCP_BAD_DOFF": 13,
    "IP6_SHORT": 14, "IP6_BAD_LEN": 15, "IP6_EXT_SHORT": 16, "IP6_EXT_BAD_LEN": 17,
    "IP6_FRAGMENT": 18, "ICMP_EMPTY": 19, "NO_INNER": 20,
}
STATUS_NAME = {v: k for k, v in STATUS.items()}

# enum rpkt_flags
F_IP_SUM = 1
F_L4_SUM = 2
F_FLOW_EV = 4
F_IPV6 = 8

MAX_VLAN = 2
MAX_IP6_EXT = 8

IP6_BLOCK_DTYPE = np.dtype([      # rpkt_rec_t bytes 24..43 of an IPv6 record
    ("ip6_vtcfl", "<u4"), ("ip6_payload_len", "<u2"), ("ip6_next_header", "u1"),
    ("ip6_hop_limit", "u1"), ("ip6_n_ext", "u1"), ("ip_protocol", "u1"), ("ip6_pdst_off", "<u2"),
    ("ip6_src_fold", "<u4"), ("ip6_dst_fold", "<u4"),
])
assert IP6_BLOCK_DTYPE.itemsize == 20
FLOW_MAX_BUCKETS = 65535


OPTS_BYTES = 64
OPTS_DTYPE = np.dtype([          # rpkt_opts_t (include/rpkt_gpu.h), 64 B
    ("tcp_count", "u1"), ("tcp_stop", "u1"), ("tcp_wscale", "u1"), ("tcp_sack_blocks", "u1"),
    ("tcp_kinds", "<u2"), ("tcp_mss", "<u2"), ("tcp_ts", "<u4"), ("tcp_ts_echo", "<u4"),
    ("tcp_sack_left", "<u4"), ("tcp_sack_right", "<u4"), ("tcp_fo_len", "<u2"),
    ("tcp_end", "u1"), ("ip_end", "u1"), ("ip_count", "u1"), ("ip_stop", "u1"),
    ("ip_kinds", "<u2"), ("ip_route_alert", "<u2"), ("ip_rr_len", "u1"), ("ip_rr_pointer", "u1"),
    ("ip_ts_len", "u1"), ("ip_ts_pointer", "u1"), ("ip_ts_oflw_flg", "u1"),
    ("ip_sr_pointer", "u1"), ("ip_sr_dest", "<u4"), ("ip_cs_doi", "<u4"),
    ("tcp_trace", "<u8"), ("ip_trace", "<u8"),
])
assert OPTS_DTYPE.itemsize == OPTS_BYTES
OPT_STOP = {"NONE": 0, "END": 1, "UNKNOWN": 2, "MALFORMED": 3}
IP6_OPT_KINDS = ("Pad0", "Padn", "RouterAlert", "Generic")
IP6_OPTS_DTYPE = np.dtype([      # rpkt_opts_t bytes 27..47 of an IPv6 frame (include/rpkt_gpu.h)
    ("end", "u1"), ("count", "u1"), ("stop", "u1"), ("kinds", "<u2"), ("router_alert", "<u2"), ("generic_type", "u1"), ("generic_len", "u1"), ("n_hdrs", "u1"),
    ("first_hdr", "u1"), ("pad1", "u1", (2,)), ("generic_data", "<u4"), ("pad2", "u1", (4,)),
])
assert IP6_OPTS_DTYPE.itemsize == 21


def ip6_opts_view(opts):
    """The IPv6 option-walk view of rpkt_opts_t records (bytes 27..47; trace: ip_trace)."""
    raw = np.ascontiguousarray(opts).view(np.uint8).reshape(-1, OPTS_BYTES)[:, 27:48]
    return np.ascontiguousarray(raw).view(IP6_OPTS_DTYPE).reshape(-1)
TCP_KINDS = ("Eol", "Nop", "Mss", "WindowScale", "SackPermitted", "Sack", "Timestamp", "FastOpen")
IP_KINDS = ("Eol", "Nop", "Timestamp", "RecordRoute", "RouteAlert", "CommercialSecurity",
            "StrictSourceRoute", "LooseSourceRoute")


LAYERS_BYTES = 64
LAYERS_DTYPE = np.dtype([        # rpkt_layers_t (include/rpkt_gpu.h), 64 B
    ("n", "u1"), ("stop", "u1"), ("err_group", "u1"), ("key_proto", "u1"),
    ("payload_off", "<u2"), ("reserved", "<u2"), ("payload_len", "<u4"), ("next_key", "<u4"),
    ("proto", "u1", (16,)), ("off", "<u2", (16,)),
])
assert LAYERS_DTYPE.itemsize == LAYERS_BYTES
LAYER_STOP = {"END": 1, "UNKNOWN": 2, "ERR": 3, "MAX": 4}

FIELD_REQ_DTYPE = np.dtype([      # rpkt_field_req_t (include/rpkt_gpu.h), 8 B
    ("proto", "u1"), ("nth", "u1"), ("bits", "u1"), ("reserved", "u1"),
    ("bit_off", "<u2"), ("reserved2", "<u2"),
])
assert FIELD_REQ_DTYPE.itemsize == 8
MAX_FIELD_REQS = 32


def protocol_names():
    """Protocol id -> name, from include/rpkt_protocols.h."""
    import os
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                       "rpkt_protocols.h")
    out = {}
    for m in re.finditer(r"#define RPKT_P_(\w+) (\d+)", open(hdr).read()):
        out[int(m.group(2))] = m.group(1)
    return out


def trace_kinds(trace, count, names):
    """The first min(count, 16) option kinds of a *_trace field, by name."""
    return [names[((int(trace) >> (4 * k)) & 15) - 1] for k in range(min(int(count), 16))]


def as_opts(raw):
    """View a uint8 buffer of n * 64 bytes as rpkt_opts_t records."""
    a = np.ascontiguousarray(raw).view(np.uint8)
    return a.view(OPTS_DTYPE)


def as_records(raw):
    """View a uint8 buffer of n*80 bytes (numpy or CPU torch) as a record array."""
    a = np.asarray(raw)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a.reshape(-1).view(REC_DTYPE)


def flow_ev_fields(ev):
    """Split rpkt_flow_ev_t values into (frame_len, bucket, ip_bad, l4_bad)."""
    ev = np.asarray(ev, dtype=np.uint64)
    return (ev & np.uint64(0xffffffff), (ev >> np.uint64(32)) & np.uint64(0xffff),
            (ev >> np.uint64(48)) & np.uint64(1), (ev >> np.uint64(49)) & np.uint64(1))


TUN_BYTES = 16
TUN_DTYPE = np.dtype([           # rpkt_tun_t (include/rpkt_gpu.h), 16 B
    ("kind", "u1"), ("status", "u1"), ("tun_off", "<u2"), ("inner_off", "<u2"),
    ("inner_type", "<u2"), ("id", "<u4"), ("hdr0", "u1"), ("hdr1", "u1"), ("aux", "<u2"),
])
assert TUN_DTYPE.itemsize == TUN_BYTES
TUN_KIND = {"NONE": 0, "VXLAN": 1, "GTPU": 2, "GRE": 3}
TUN_STATUS = {"OK": 0, "NONE": 1, "BAD": 2, "NOT_TPDU": 3, "EXT_BAD": 4, "INNER_UNKNOWN": 5}
MAX_GTP_EXT = 8


def as_tunnels(raw):
    """View a uint8 buffer of n*16 bytes as rpkt_tun_t records."""
    a = np.asarray(raw)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a.reshape(-1).view(TUN_DTYPE)

