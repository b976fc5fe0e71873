"""Build the golden fixtures under tests/golden/ from the reference's own test data.

Run once in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

What it writes (all DATA, no reference source):
  packets/*.dat        verbatim copies of rpkt/tests/packet_examples/*.dat (hex
                       text, one frame each; loader rpkt/tests/common/mod.rs:3-29)
  packets/bench_frame.dat
                       the 110-byte FRAME_BYTES array of
                       benches/rpkt/rpkt_parse.rs:9-17, written as hex text
  expected.json        getter values the reference's tests assert on those
                       frames (transcribed below with file:line), plus the
                       checksum validity known from the captures themselves

Checksum pinning: the fixtures are real captures whose stored IPv4/TCP/UDP
checksums were computed by the sending network stack.  For a frame whose
stored checksum is correct, RFC 1071 requires ip_sum == 0xffff and
l4_sum == 0xffff, independent of any implementation here.  Frames captured
with TX checksum offload (stored value not final) are marked "invalid"; their
exact sums are the SURVEY.md Appendix A values (computed there by a scratch
re-implementation, so they pin consistency, not the reference).
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
SRC = os.path.join(REF, "rpkt", "tests", "packet_examples")

# benches/rpkt/rpkt_parse.rs:9-17
BENCH_FRAME = [
    0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0, 0x00, 0x50, 0x56, 0xae, 0x76, 0xf5, 0x08, 0x00, 0x45, 0x00,
    0x00, 0x5e, 0x5c, 0x65, 0x00, 0x00, 0x80, 0x11, 0x00, 0x00, 0xc0, 0xa8, 0x1d, 0x3a, 0xc0, 0xa8,
    0x1d, 0xa0, 0xeb, 0xd8, 0x00, 0xa1, 0x00, 0x4a, 0xbc, 0x86, 0x30, 0x40, 0x02, 0x01, 0x03, 0x30,
    0x0f, 0x02, 0x03, 0x00, 0x91, 0xc8, 0x02, 0x02, 0x05, 0xdc, 0x04, 0x01, 0x04, 0x02, 0x01, 0x03,
    0x04, 0x15, 0x30, 0x13, 0x04, 0x00, 0x02, 0x01, 0x00, 0x02, 0x01, 0x00, 0x04, 0x05, 0x61, 0x64,
    0x6d, 0x69, 0x6e, 0x04, 0x00, 0x04, 0x00, 0x30, 0x13, 0x04, 0x00, 0x04, 0x00, 0xa0, 0x0d, 0x02,
    0x03, 0x00, 0x91, 0xc8, 0x02, 0x01, 0x00, 0x02, 0x01, 0x00, 0x30, 0x00, 0x00, 0x00,
]


def ip(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


# Getter KATs.  Keys are record-field names (include/rpkt_gpu.h); "cite" is the
# reference assert block they come from.
EXPECTED = {
    "bench_frame.dat": {
        "cite": "benches/rpkt/rpkt_parse.rs:62-80",
        "status": "OK", "ethertype": 0x0800, "ip_protocol": 17,
        "ip_src": ip("192.168.29.58"), "ip_dst": ip("192.168.29.160"),
        "ip_checksum": 0x0000, "ip_ident": 0x5c65,
        "src_port": 60376, "dst_port": 161, "l4_word6": 74, "l4_checksum": 0xbc86,
        "payload_off": 42, "payload_len": 66,          # rpkt_parse.rs:101-105
        "dst_addr": [0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0],  # rpkt_parse.rs:22-33
        "src_addr": [0x00, 0x50, 0x56, 0xae, 0x76, 0xf5],  # rpkt_parse.rs:34-45
        "sums": "invalid",
    },
    "IPv4Option1.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:17-36",
        "status": "L4_OTHER", "ethertype": 0x0800, "ip_header_len": 44, "ip_dscp": 0,
        "ip_ecn": 0, "ip_ident": 30775, "ip_packet_len": 108, "ip_dont_frag": 0,
        "ip_more_frag": 0, "ip_ttl": 64, "ip_protocol": 1, "ip_checksum": 0x752d,
        "ip_src": ip("127.0.0.1"), "ip_dst": ip("127.0.0.1"), "l4_off": 14 + 44,
        "sums": "valid",                     # ICMP: calculate_icmp_checksum == 0
    },
    "IPv4Option2.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:165-185",
        "status": "L4_OTHER", "ip_header_len": 60, "ip_packet_len": 124, "ip_ident": 33505,
        "ip_dont_frag": 1, "ip_more_frag": 0, "ip_ttl": 64, "ip_protocol": 1,
        "ip_checksum": 0x0d44, "ip_src": ip("10.0.0.6"), "ip_dst": ip("10.0.0.138"),
        "sums": "valid",                     # ICMP: calculate_icmp_checksum == 0
    },
    "IPv4Option3.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:311-331",
        "status": "L4_OTHER", "ip_header_len": 24, "ip_packet_len": 36, "ip_ident": 0,
        "ip_dont_frag": 1, "ip_ttl": 1, "ip_protocol": 2, "ip_checksum": 0xfa48,
        "ip_src": ip("10.0.0.138"), "ip_dst": ip("224.0.0.1"),
        "sums": "ip_valid",
    },
    "IPv4Option4.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:434-454",
        "status": "OK", "ip_header_len": 60, "ip_packet_len": 80, "ip_ident": 0,
        "ip_dont_frag": 1, "ip_ttl": 64, "ip_protocol": 6, "ip_checksum": 0xead8,
        "ip_src": ip("10.0.0.138"), "ip_dst": ip("10.0.0.6"),
        "sums": "valid",
    },
    "IPv4Option6.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:625-645",
        "status": "L4_OTHER", "ip_header_len": 28, "ip_packet_len": 36, "ip_ident": 13132,
        "ip_dont_frag": 0, "ip_ttl": 64, "ip_protocol": 1, "ip_checksum": 0x2871,
        "ip_src": ip("10.0.0.6"), "ip_dst": ip("10.0.0.138"),
        "sums": "valid",                     # ICMP: calculate_icmp_checksum == 0
    },
    "IPv4Option7.dat": {
        "cite": "rpkt/tests/ipv4_test.rs:756-776",
        "status": "L4_OTHER", "ip_header_len": 28, "ip_packet_len": 36, "ip_ident": 18339,
        "ip_dont_frag": 0, "ip_ttl": 64, "ip_protocol": 1, "ip_checksum": 0x1420,
        "ip_src": ip("10.0.0.6"), "ip_dst": ip("10.0.0.138"),
        "sums": "valid",                     # ICMP: calculate_icmp_checksum == 0
    },
    "TcpPacketWithOptions.dat": {
        "cite": "rpkt/tests/tcp_test.rs:17-43",
        "status": "OK", "ip_protocol": 6, "src_port": 44147, "dst_port": 80,
        "tcp_seq": 777047406, "tcp_ack": 3761117865, "tcp_header_len": 32,
        "tcp_flags": 0x18, "tcp_window": 913, "l4_checksum": 0xac20, "tcp_urgent": 0,
        "sums": "ip_valid_l4_invalid", "l4_sum": 0x4ca9,
    },
    "TcpPacketWithOptions2.dat": {
        "cite": "rpkt/tests/tcp_test.rs:183-209",
        "status": "OK", "ip_protocol": 6, "src_port": 80, "dst_port": 44160,
        "tcp_seq": 3089746840, "tcp_ack": 3916895622, "tcp_header_len": 36,
        "tcp_flags": 0x18, "tcp_window": 20178, "l4_checksum": 0xdea1, "tcp_urgent": 0,
        "sums": "valid",
    },
    "TcpPacketWithMssSackperm.dat": {
        "cite": "rpkt/tests/tcp_test.rs:376-402",
        "status": "OK", "ip_protocol": 6, "src_port": 2000, "dst_port": 6712,
        "tcp_seq": 191135221, "tcp_ack": 4211666100, "tcp_header_len": 28,
        "tcp_flags": 0x12, "tcp_window": 64240, "l4_checksum": 0xe310, "tcp_urgent": 0,
        "sums": "valid",
    },
    "TcpPacketWithSack.dat": {
        "cite": "rpkt/tests/tcp_test.rs:551-576",
        "status": "OK", "ip_protocol": 6, "src_port": 54436, "dst_port": 80,
        "tcp_seq": 3714426508, "tcp_ack": 2530491013, "tcp_header_len": 32,
        "tcp_flags": 0x10, "tcp_window": 4380, "l4_checksum": 0x8497, "tcp_urgent": 0,
        "sums": "valid",
    },
    "QinQ_802.1_AD.dat": {
        "cite": "rpkt/tests/vlan_mpls_tests.rs:96-130",
        "status": "L4_OTHER", "ethertype": 0x88a8, "n_vlan": 2,
        "vlan0_id": 30, "vlan0_ethertype": 0x8100,
        "vlan1_priority": 0, "vlan1_dei": 0, "vlan1_id": 100, "vlan1_ethertype": 0x0800,
        "ip_version": 4, "ip_header_len": 20, "ip_dscp": 0, "ip_packet_len": 1474,
        "ip_ident": 0x54b0, "ip_flag_reserved": 0, "ip_dont_frag": 0, "ip_more_frag": 0,
        "ip_frag_offset": 0, "ip_ttl": 255, "ip_protocol": 253, "ip_checksum": 0xddbf,
        "ip_src": ip("192.85.1.22"), "ip_dst": ip("192.85.1.14"),
        "payload_len": 1454,                            # vlan_mpls_tests.rs:129
        "sums": "ip_valid",
    },
    "gtp-c1.dat": {"cite": "rpkt/tests/gtpv1_test.rs:22-34", "status": "OK",
                   "ip_protocol": 17, "src_port": 2123, "dst_port": 2123,
                   "l4_checksum": 0xa9d9, "sums": "valid"},
    "gtp-u-1ext.dat": {"cite": "rpkt/tests/gtpv1_test.rs:200-212", "status": "OK",
                       "ip_protocol": 17, "src_port": 2152, "dst_port": 2152,
                       "l4_checksum": 0xb58d, "sums": "valid"},
    "gtp-u-2ext.dat": {"cite": "rpkt/tests/gtpv1_test.rs:285-297", "status": "OK",
                       "ip_protocol": 17, "src_port": 2152, "dst_port": 2152,
                       "l4_checksum": 0x983c, "sums": "valid"},
    "gtp_nr_container.dat": {"cite": "rpkt/tests/gtpv1_test.rs:377-389", "status": "OK",
                             "ip_protocol": 17, "src_port": 2152, "dst_port": 2152,
                             "l4_checksum": 0x9fd9, "sums": "valid"},
    "gtp_pdu_session_container.dat": {
        "cite": "rpkt/tests/gtpv1_test.rs:468-480", "status": "OK", "ip_protocol": 17,
        "src_port": 2152, "dst_port": 2152, "l4_checksum": 0x1714,
        "sums": "ip_valid_l4_invalid", "l4_sum": 0x9d0c},
    "gtpv2-with-teid.dat": {"cite": "rpkt/tests/gtpv2_test.rs:16-27", "status": "OK",
                            "ip_protocol": 17, "src_port": 2123, "l4_checksum": 0x0000,
                            "sums": "ip_valid_udp_zero", "l4_sum": 0x992d},
    "gtpv2-with-piggyback.dat": {"status": "OK", "ip_protocol": 17, "sums": "valid"},
    "Vxlan1.dat": {"status": "OK", "ip_protocol": 17, "sums": "valid"},
    "Vxlan2.dat": {"status": "OK", "ip_protocol": 17, "sums": "valid"},
    # non-IPv4 frames: the chain stops at the ethertype dispatch
    "ArpRequestPacket.dat": {"status": "NOT_IPV4", "ethertype": 0x0806},
    "ArpResponsePacket.dat": {"status": "NOT_IPV4", "ethertype": 0x0806},
    "ArpRequestWithVlan.dat": {
        "cite": "rpkt/tests/vlan_mpls_tests.rs:16-32",
        "status": "NOT_IPV4", "ethertype": 0x8100, "n_vlan": 2,
        "vlan0_priority": 5, "vlan0_dei": 1, "vlan0_id": 666, "vlan0_ethertype": 0x8100,
        "vlan1_priority": 2, "vlan1_dei": 0, "vlan1_id": 200, "vlan1_ethertype": 0x0806},
    "EthDot3.dat": {"status": "NOT_IPV4"},
}
for g in ("GREv0_1.dat", "GREv0_2.dat", "GREv0_3.dat", "GREv0_4.dat", "GREv1_1.dat",
          "GREv1_3.dat"):
    EXPECTED[g] = {"status": "L4_OTHER", "ip_protocol": 47, "sums": "ip_valid"}
# GRE with checksum_present: the RFC 2784 sum over the GRE header + payload is valid
# (gre_test.rs:35-41 asserts GREv0_1's stored checksum 30719)
for g in ("GREv0_1.dat", "GREv0_3.dat"):
    EXPECTED[g]["sums"] = "valid"


def main():
    out = os.path.join(HERE, "packets")
    os.makedirs(out, exist_ok=True)
    if not os.path.isdir(SRC):
        sys.exit("reference fixtures not found at %s" % SRC)
    n = 0
    for f in sorted(os.listdir(SRC)):
        if f.endswith(".dat"):
            shutil.copyfile(os.path.join(SRC, f), os.path.join(out, f))
            n += 1
    with open(os.path.join(out, "bench_frame.dat"), "w") as fh:
        fh.write("".join("%02x" % b for b in BENCH_FRAME) + "\n")
    with open(os.path.join(HERE, "expected.json"), "w") as fh:
        json.dump(EXPECTED, fh, indent=1, sort_keys=True)
    print("copied %d fixtures, wrote expected.json with %d entries" % (n, len(EXPECTED)))


if __name__ == "__main__":
    main()
