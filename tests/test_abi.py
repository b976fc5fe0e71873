"""The C-ABI library builds, loads and exports exactly what include/rpkt_gpu.h
declares.  CPU only: no call here reaches a kernel launch."""
import ctypes
import os
import re

import pytest

from rpkt_amd import engine, records
from rpkt_amd.build import build_gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "rpkt_gpu.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rpkt_\w+)\s*\(", src)) - {"rpkt_rec", "rpkt_batch"})


@pytest.fixture(scope="module")
def L():
    build_gpu()
    return engine.lib()


def test_every_declared_symbol_is_exported(L):
    names = declared_functions()
    assert len(names) >= 9
    for name in names:
        assert hasattr(L, name), name
    assert sorted(engine.EXPORTS) == names


def dynamic_exports(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if ln.split()[-1].startswith("rpkt_")})


def test_product_library_exports_exactly_the_header(L):
    """The product library's rpkt_* exports are the header's declarations, no more: the
    kernel ablation variants and streaming references live in librpkt_gpu_ablate.so."""
    from rpkt_amd.build import ABLATE_LIB, GPU_LIB
    assert dynamic_exports(GPU_LIB) == declared_functions()
    dev = dynamic_exports(ABLATE_LIB)
    assert set(declared_functions()) < set(dev)
    assert {"rpkt_gpu_debug_variant", "rpkt_gpu_debug_forward_variant",
            "rpkt_gpu_debug_layers_variant"} <= set(dev)


def test_library_loads_without_rccl(L):
    """RCCL is resolved when the collective is first used (rpkt_coll.hip), so a parse-only
    host needs no librccl to load the engine."""
    import subprocess
    from rpkt_amd.build import GPU_LIB
    out = subprocess.run(["readelf", "-d", GPU_LIB], capture_output=True, text=True,
                         check=True).stdout
    assert "rccl" not in out
    assert isinstance(L.rpkt_gpu_coll_version(), int)


def test_collective_binds_torchs_rccl(L):
    """Under PyTorch the engine's RCCL calls bind the copy torch already loaded (whose
    ProcessGroupNCCL owns the communicator handed to rpkt_gpu_flow_reduce): same version,
    and no second librccl mapped into the process."""
    import subprocess
    import sys
    code = (
        "import torch, ctypes\n"
        "from rpkt_amd import engine\n"
        "v = engine.lib().rpkt_gpu_coll_version()\n"
        "a, b, c = torch.cuda.nccl.version()\n"
        "maps = {l.split()[-1] for l in open('/proc/self/maps').read().splitlines() if 'rccl' in l}\n"
        "print(v, a * 10000 + b * 100 + c, len(maps))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                         timeout=600, check=True).stdout.split()
    v, tv, copies = (int(x) for x in out[-3:])
    assert v == tv and copies == 1


def test_abi_version_and_info(L):
    assert L.rpkt_gpu_abi_version() == 1
    assert b"gfx950" in L.rpkt_gpu_build_info()


def test_status_names_match_records(L):
    for name, code in records.STATUS.items():
        assert L.rpkt_gpu_status_name(code).decode() == name
    assert L.rpkt_gpu_status_name(99) == b"?"


def struct_offsets(src, name):
    """Offsets in the `/* NN` comments of one typedef struct of the header."""
    body = src[src.index("typedef struct %s {" % name):]
    body = body[:body.index("}")]
    return [int(m) for m in re.findall(r";\s*/\*\s*(\d+) ", body)]


def test_record_layout_matches_header():
    src = open(HDR).read()
    offs = struct_offsets(src, "rpkt_rec")
    assert offs == [records.REC_DTYPE.fields[n][1] for n in records.REC_DTYPE.names]
    assert records.REC_BYTES == 80


def test_rec16_layout_matches_header():
    src = open(HDR).read()
    offs = struct_offsets(src, "rpkt_rec16")
    assert offs == [records.REC16_DTYPE.fields[n][1] for n in records.REC16_DTYPE.names]
    assert records.REC16_BYTES == 16


def test_projection_of_oracle_records():
    """project16 keeps the record fields and derives the verdict bits as documented."""
    from oracle import oracle
    from rpkt_amd import gen
    import numpy as np
    hb = gen.make_batch(6, 4000, seed=3)
    for flags in (0, 1, 2, 3):
        r = oracle.parse_batch(hb.frames, hb.n, flags=flags, offsets=hb.offsets, stride=hb.stride)
        c = records.project16(r, flags)
        assert np.array_equal(c["l4_off"], r["l4_off"]) and np.array_equal(c["status"], r["status"])
        assert not (c["verdict"] & 1).any() if not flags & 1 else (c["verdict"] & 1).any()
        assert not (c["verdict"] & 2).any() if not flags & 2 else (c["verdict"] & 2).any()
        assert ((c["verdict"] & 2) == 0)[r["status"] != 0].all()


def test_opts_layout_matches_header():
    src = open(HDR).read()
    offs = struct_offsets(src, "rpkt_opts")
    assert offs == [records.OPTS_DTYPE.fields[n][1] for n in records.OPTS_DTYPE.names]
    assert records.OPTS_BYTES == 64


def test_flow_hash_matches_oracle(L):
    from oracle import oracle
    import numpy as np
    rng = np.random.default_rng(3)
    for _ in range(500):
        a, b = (int(x) for x in rng.integers(0, 2**32, 2))
        sp, dp = (int(x) for x in rng.integers(0, 2**16, 2))
        pr = int(rng.integers(0, 256))
        assert L.rpkt_flow_hash(a, b, sp, dp, pr) == oracle.flow_hash(a, b, sp, dp, pr)


def test_argument_validation_without_launch(L):
    d = engine.Batch(None, 0, None, 64, 0, 0, 0)
    assert L.rpkt_gpu_parse_batch(None, 3, None, None, 0, None) == -1      # NULL batch
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 3, 16, None, 0, None) == 0   # n == 0
    d.n = 10
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 3, 16, None, 0, None) == -1  # NULL frames
    d.frames_dev = 4096
    d.frames_bytes = 1 << 32
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 3, 16, None, 0, None) == -3  # > 4 GiB
    d.frames_bytes = 640
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 3, 8, None, 0, None) == -4   # misaligned
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 0x80, 16, None, 0, None) == -1  # bad flag
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 7, 16, None, 0, None) == -1  # FLOW_EV, NULL
    d.stride = 0
    assert L.rpkt_gpu_parse_batch(ctypes.byref(d), 3, 16, None, 0, None) == -1  # no layout
    assert L.rpkt_gpu_flow_count(None, 10, 0, None, None, None) == -1
    assert L.rpkt_gpu_checksum_ranges(None, 0, None, 0, None, None) == 0
    assert L.rpkt_gpu_flow_workspace_bytes(1 << 20, 8192) > 0


def test_ring_argument_validation_without_launch(L):
    """rpkt_gpu_parse_ring checks every slot before it launches anything; a ring of
    empty slots launches nothing."""
    S = (engine.RingSlot * 3)()
    P = ctypes.cast(S, ctypes.POINTER(engine.RingSlot))
    assert L.rpkt_gpu_parse_ring(None, 1, 3, 0, None) == -1                   # NULL slots
    assert L.rpkt_gpu_parse_ring(None, 0, 3, 0, None) == 0                    # nothing to do
    assert L.rpkt_gpu_parse_ring(P, 3, 3, 0, None) == 0                       # all n == 0
    assert L.rpkt_gpu_parse_ring(P, 3, 0x80, 0, None) == -1                   # bad flag
    # FLOW_EV with 0 buckets: nothing to do for empty slots (as parse_batch with n == 0)
    assert L.rpkt_gpu_parse_ring(P, 3, 7, 0, None) == 0
    S[1].batch = engine.Batch(4096, 640, None, 64, 0, 10, 0)
    S[1].recs_dev = 16
    S[1].flow_ev_dev = 64
    assert L.rpkt_gpu_parse_ring(P, 3, 7, 0, None) == -1                      # FLOW_EV, 0 buckets
    S[1].flow_ev_dev = None
    S[2].batch = engine.Batch(4096, 1 << 32, None, 64, 0, 10, 0)
    S[2].recs_dev = 16
    assert L.rpkt_gpu_parse_ring(P, 3, 3, 0, None) == -3                      # slot 2 > 4 GiB
    S[2].batch.frames_bytes = 640
    S[2].recs_dev = 24
    assert L.rpkt_gpu_parse_ring(P, 3, 3, 0, None) == -4                      # slot 2 misaligned
    S[2].recs_dev = 32
    assert L.rpkt_gpu_parse_ring(P, 3, 7, 64, None) == -1                     # no flow events
    S[1].flow_ev_dev, S[2].flow_ev_dev = 64, 68
    assert L.rpkt_gpu_parse_ring(P, 3, 7, 64, None) == -4                     # events misaligned
    S[2].batch.stride = 0
    assert L.rpkt_gpu_parse_ring(P, 3, 3, 0, None) == -1                      # no layout
    assert L.rpkt_gpu_parse_ring_compact(P, 3, 3, 0, None) == -1              # the same checks


def test_engine_refuses_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(engine.RpktError):
        engine.alloc_records(4)


def test_cpp_example_builds_against_header():
    from rpkt_amd.build import build_example
    assert all(os.path.exists(p) for p in build_example())


def test_flow_reduce_validation_without_launch(L):
    """rpkt_gpu_flow_reduce's argument checks (no communicator is ever touched)."""
    assert L.rpkt_gpu_flow_reduce(None, 8192, -1, 4096, None) == -1          # NULL counters
    assert L.rpkt_gpu_flow_reduce(4096, 8192, -1, None, None) == -1          # NULL comm
    assert L.rpkt_gpu_flow_reduce(4096, 0, -1, 4096, None) == -1             # no buckets
    assert L.rpkt_gpu_flow_reduce(4096, 65536, -1, 4096, None) == -1         # too many
    assert L.rpkt_gpu_flow_reduce(4096, 8192, -2, 4096, None) == -1          # bad root
    assert L.rpkt_gpu_flow_reduce(4100, 8192, -1, 4096, None) == -4          # misaligned
    assert L.rpkt_gpu_last_coll_error() == 0
    assert L.rpkt_gpu_coll_version() >= 21000                                # RCCL 2.x


def test_layers_layout_matches_header():
    src = open(HDR).read()
    body = src[src.index("typedef struct rpkt_layers {"):]
    body = body[:body.index("}")]
    offs = [int(m) for m in re.findall(r";\s*/\*\s*(\d+) ", body)]
    assert offs == [records.LAYERS_DTYPE.fields[n][1] for n in records.LAYERS_DTYPE.names]


def test_protocol_ids_match_table():
    import json
    t = json.load(open(os.path.join(os.path.dirname(HDR), "..", "tests", "golden",
                                    "proto_table.json")))
    names = records.protocol_names()
    assert len(names) == len(t["packets"])
    for p in t["packets"]:
        assert names[p["id"]] == ("%s_%s" % (p["spec"], p["name"])).upper()


def test_field_req_layout_matches_header(tmp_path):
    """offsetof() of rpkt_field_req_t, compiled from the header, against FIELD_REQ_DTYPE."""
    import subprocess
    names = records.FIELD_REQ_DTYPE.names
    prog = ['#include <stdio.h>', '#include <stddef.h>', '#include "rpkt_gpu.h"',
            'int main(void) { printf("%zu %d", sizeof(rpkt_field_req_t), RPKT_MAX_FIELD_REQS);']
    prog += ['printf(" %%zu", offsetof(rpkt_field_req_t, %s));' % n for n in names]
    prog += ['return 0; }']
    src = tmp_path / "offs.c"
    src.write_text("\n".join(prog))
    exe = tmp_path / "offs"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HDR), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got[0] == records.FIELD_REQ_DTYPE.itemsize == 8
    assert got[1] == records.MAX_FIELD_REQS
    assert got[2:] == [records.FIELD_REQ_DTYPE.fields[n][1] for n in names]


def test_fields_batch_argument_checks(L):
    """Host-side validation of rpkt_gpu_fields_batch (returns before any device call)."""
    import ctypes
    import numpy as np
    from rpkt_amd import fields
    reqs = fields.requests([("IPV4_IPV4", "ttl")])
    b = engine.Batch(frames_dev=16, frames_bytes=64, offsets_dev=None, stride=64,
                     frame_len=64, n=0, reserved=0)
    rp = reqs.ctypes.data_as(ctypes.c_void_p)
    assert L.rpkt_gpu_fields_batch(None, 16, rp, 1, 16, None, None) == -1
    assert L.rpkt_gpu_fields_batch(ctypes.byref(b), 16, rp, 0, 16, None, None) == -1
    assert L.rpkt_gpu_fields_batch(ctypes.byref(b), 16, rp, 33, 16, None, None) == -1
    assert L.rpkt_gpu_fields_batch(ctypes.byref(b), 16, rp, 1, 16, None, None) == 0   # n == 0
    for key, val in (("bits", 0), ("bits", 65), ("proto", 200)):
        bad = reqs.copy()
        bad[key] = val
        assert L.rpkt_gpu_fields_batch(ctypes.byref(b), 16, bad.ctypes.data_as(ctypes.c_void_p),
                                       1, 16, None, None) == -1, (key, val)
    b.n = 4
    assert L.rpkt_gpu_fields_batch(ctypes.byref(b), 8, rp, 1, 16, None, None) == -4  # align
    assert np.asarray(reqs).size == 1


def test_unit_hash_headers_match_the_includes():
    """A unit's hash (rpkt_gpu_build_info: parse=… tx=… walks=… fields=…, which ties the
    committed profiles to kernel sources) covers exactly the csrc headers it includes,
    directly or through another header."""
    import re
    from rpkt_amd import build
    csrc = os.path.join(os.path.dirname(build.__file__), "csrc")

    def includes(name, seen):
        with open(os.path.join(csrc, name)) as fh:
            for h in re.findall(r'#include "([^"/]+)"', fh.read()):
                if h not in seen:
                    seen.add(h)
                    includes(h, seen)
        return seen

    for src in build.GPU_SRC:
        u = os.path.basename(src)
        assert set(build.UNIT_HEADERS[u]) == includes(u, set()), u
    assert set(build.UNIT_HEADERS) == {os.path.basename(f) for f in build.GPU_SRC}


def test_forward_refuses_unknown_flags_without_launch(L):
    """rpkt_fwd_t.flags (was `reserved`): any bit but RPKT_F_IPV6 is refused before anything
    is launched (a caller that left the old field uninitialised gets RPKT_E_INVAL, not
    IPv6 forwarding), in the 128-B and the 64-B-window (strided short frames) entry."""
    fwd = engine.Fwd()
    keep = 4096
    for stride in (64, 1500):                        # the w64 and the 128-B compile
        d = engine.Batch(4096, stride * 10, None, stride, 0, 10, 0)
        for bad in (1, 4, 16, 0x80000000, 8 | 2):
            fwd.flags = bad
            assert L.rpkt_gpu_forward_batch(ctypes.byref(d), ctypes.byref(fwd), keep, None) == -1
    d = engine.Batch(None, 0, None, 64, 0, 0, 0)
    fwd.flags = 8
    assert L.rpkt_gpu_forward_batch(ctypes.byref(d), ctypes.byref(fwd), keep, None) == 0   # n == 0
    fwd.flags = 16
    assert L.rpkt_gpu_forward_batch(ctypes.byref(d), ctypes.byref(fwd), keep, None) == -1
