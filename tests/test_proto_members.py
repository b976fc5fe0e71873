"""The layer walk's compiled group-member tests (rpkt_proto_table.h kMembers / kGroups,
tools/pktfmt_table.py member_tests) against the pktfmt conditions they compile
(tests/golden/proto_table.json): for every member, `(key & mask) - lo <= span` on the
big-endian dword at its group's key byte must equal "every condition field lies in
one of its ranges", for boundary and random header bytes."""
import json
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TABLE = json.load(open(os.path.join(HERE, "golden", "proto_table.json")))
HDR = open(os.path.join(ROOT, "rpkt_amd", "csrc", "rpkt_proto_table.h")).read()


def c_array(name):
    body = HDR[HDR.index(name):]
    body = body[body.index("{") + 1:body.index("};")]
    return [[int(x, 0) for x in re.findall(r"0x[0-9a-f]+|\d+", row.split("//")[0])]
            for row in body.strip().split("\n") if row.strip().startswith("{")]


MEMBERS = c_array("kMembers[RPKT_N_PROTOS]")
GROUPS = c_array("kGroups[RPKT_N_GROUPS]")


def field(hdr, off, bits):
    """pktfmt bit order: big-endian, bit 0 = MSB of byte 0."""
    v = int.from_bytes(bytes(hdr[off // 8:(off + bits + 7) // 8 + 1]), "big")
    total = 8 * (len(hdr[off // 8:(off + bits + 7) // 8 + 1]))
    return (v >> (total - (off % 8) - bits)) & ((1 << bits) - 1)


def test_tables_line_up():
    assert len(MEMBERS) == len(TABLE["packets"])
    assert len(GROUPS) == len(TABLE["groups"])
    for g, row in zip(TABLE["groups"], GROUPS):
        assert row[0] == g["members"][0] and row[1] == len(g["members"])


def test_member_tests_match_conditions():
    rng = np.random.default_rng(11)
    for g, grow in zip(TABLE["groups"], GROUPS):
        key = grow[4]
        for pid in g["members"]:
            p = TABLE["packets"][pid]
            mask, lo, span = MEMBERS[pid]
            samples = [rng.integers(0, 256, 20, dtype=np.uint8) for _ in range(3000)]
            # boundary values of every condition field, planted in random headers
            for c in p["cond"]:
                for lo_, hi_ in c["ranges"]:
                    for v in {lo_, hi_, max(lo_ - 1, 0), min(hi_ + 1, (1 << c["bits"]) - 1)}:
                        h = rng.integers(0, 256, 20, dtype=np.uint8)
                        val = int.from_bytes(bytes(h[c["off"] // 8:c["off"] // 8 + 4]), "big")
                        sh = 32 - c["off"] % 8 - c["bits"]
                        val = (val & ~(((1 << c["bits"]) - 1) << sh)) | (v << sh)
                        h[c["off"] // 8:c["off"] // 8 + 4] = np.frombuffer(
                            (val & 0xffffffff).to_bytes(4, "big"), dtype=np.uint8)
                        samples.append(h)
            for h in samples:
                want = all(any(a <= field(h, c["off"], c["bits"]) <= b for a, b in c["ranges"])
                           for c in p["cond"])
                K = int.from_bytes(bytes(h[key:key + 4]), "big")
                got = ((K & mask) - lo) % (1 << 32) <= span
                assert got == want, (p["name"], h.tobytes().hex())
