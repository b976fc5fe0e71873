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

# enum rpkt_status (include/rpkt_gpu.h)
STATUS = {
    "OK": 0, "ETH_SHORT": 1, "VLAN_SHORT": 2, "NOT_IPV4": 3, "IP_SHORT": 4,
    "IP_BAD_IHL": 5, "IP_IHL_GT_LEN": 6, "IP_TOT_LT_IHL": 7, "IP_TOT_GT_LEN": 8,
    "L4_OTHER": 9, "UDP_SHORT": 10, "UDP_BAD_LEN": 11, "TCP_SHORT": 12, "TCP_BAD_DOFF": 13,
}
STATUS_NAME = {v: k for k, v in STATUS.items()}

# enum rpkt_flags
F_IP_SUM = 1
F_L4_SUM = 2
F_FLOW_EV = 4

MAX_VLAN = 2
FLOW_MAX_BUCKETS = 65535


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
