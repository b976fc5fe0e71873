"""Field requests for rpkt_gpu_fields_batch, by protocol and field name.

The offsets and widths are the header layouts of the reference's pktfmt specs
(`pktfmt/protocols/*.pktfmt`, `header = [ name = Field {bit = ..} ... ]`), emitted by
tools/pktfmt_table.py into proto_fields.json.  The getter of a field named `x` in
protocol `P` is rpkt's `P::x()` (the generated `<proto>/generated.rs`): the
big-endian bits, masked (pktfmt/src/codegen/field.rs:115-250).  Fields wider than
64 bits (IPv6 addresses, 128) are byte slices in rpkt; request them as two 64-bit
halves (`part="hi"` / `"lo"`) and join with `join128`.
"""
import json
import os

import numpy as np

from .records import FIELD_REQ_DTYPE, MAX_FIELD_REQS

_TABLE = None


def table():
    """{"IPV6_IPV6": {"id": 5, "hdr": 40, "fields": {"src_addr": [64, 128], ...}}, ...}"""
    global _TABLE
    if _TABLE is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                               "proto_fields.json")) as fh:
            _TABLE = json.load(fh)
    return _TABLE


def field(proto, name, nth=0, part=None):
    """One request tuple (proto id, nth, bits, bit_off) for field `name` of `proto`
    (a key of table(), e.g. "IPV4_IPV4", "VXLAN_VXLAN", "ARP_ARP")."""
    p = table()[proto]
    off, bits = p["fields"][name]
    if bits > 64:
        if part not in ("hi", "lo") or bits != 128:
            raise ValueError("%s.%s is %d bits: request part='hi' or 'lo' of a 128-bit field"
                             % (proto, name, bits))
        off, bits = (off, 64) if part == "hi" else (off + 64, 64)
    elif part is not None:
        raise ValueError("%s.%s is %d bits: no parts" % (proto, name, bits))
    return (p["id"], nth, bits, off)


def requests(items):
    """FIELD_REQ_DTYPE array from a list of request tuples / (proto, name[, nth[, part]])."""
    out = np.zeros(len(items), dtype=FIELD_REQ_DTYPE)
    if not 1 <= len(items) <= MAX_FIELD_REQS:
        raise ValueError("1..%d field requests per call" % MAX_FIELD_REQS)
    for k, it in enumerate(items):
        if isinstance(it[0], str):
            it = field(*it)
        pid, nth, bits, off = it
        out[k] = (pid, nth, bits, 0, off, 0)
    return out


def join128(hi, lo):
    """The 16 bytes of a 128-bit field (rpkt's byte slice) from its two halves."""
    return int(hi).to_bytes(8, "big") + int(lo).to_bytes(8, "big")
