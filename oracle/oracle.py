"""ctypes wrapper of the CPU oracle (oracle/_build/librpkt_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  Nothing in rpkt_amd/ imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "librpkt_oracle.so")
NATIVE_LIB_PATH = os.path.join(HERE, "_build", "librpkt_oracle_native.so")
ASAN_LIB_PATH = os.path.join(HERE, "_build", "librpkt_oracle_asan.so")

_lib = None
# RPKT_ORACLE_BUILD=asan: the sanitizer build (tests/test_oracle_asan.py sets it in a child)
_lib_path = ASAN_LIB_PATH if os.environ.get("RPKT_ORACLE_BUILD") == "asan" else LIB_PATH


def build():
    """Compile the oracle with its Makefile (gcc, seconds)."""
    subprocess.check_call(["make", "-s", "-C", HERE])


def use_native_build():
    """Switch this process to an -O3 -march=native build of the oracle compiled on
    the host it runs on (the CPU-baseline build SURVEY.md §8d names).  Must be
    called before the first oracle call.  Returns the compiler flags used, or None
    (and keeps the shipped x86-64-v3 build) when gcc fails here."""
    global _lib_path
    if _lib is not None:
        raise RuntimeError("oracle already loaded from %s" % _lib_path)
    try:
        subprocess.check_call(["make", "-s", "-C", HERE, "native"], stdout=subprocess.DEVNULL)
    except (OSError, subprocess.CalledProcessError):
        return None
    _lib_path = NATIVE_LIB_PATH
    return "-O3 -march=native"


def use_asan_build():
    """Load the ASan/UBSan build instead (host sanitizer runs of the CPU tests; the
    process must have libasan preloaded, see tests/test_oracle_asan.py)."""
    global _lib_path
    if _lib is not None:
        raise RuntimeError("oracle already loaded from %s" % _lib_path)
    subprocess.check_call(["make", "-s", "-C", HERE, "asan"], stdout=subprocess.DEVNULL)
    _lib_path = ASAN_LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if _lib_path == LIB_PATH and not os.path.exists(LIB_PATH):
            build()
        if _lib_path == ASAN_LIB_PATH and not os.path.exists(ASAN_LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", HERE, "asan"])
        L = ctypes.CDLL(_lib_path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_from_slice.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_from_slice.restype = ctypes.c_uint16
        L.oracle_icmp_checksum.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_icmp_checksum.restype = ctypes.c_int
        L.oracle_combine.argtypes = [ctypes.POINTER(ctypes.c_uint16), ctypes.c_size_t]
        L.oracle_combine.restype = ctypes.c_uint16
        L.oracle_from_buf.argtypes = [ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.c_size_t, ctypes.c_size_t]
        L.oracle_from_buf.restype = ctypes.c_uint16
        L.oracle_parse_one.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_void_p]
        L.oracle_parse_one.restype = None
        L.oracle_parse_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_void_p]
        L.oracle_parse_batch.restype = None
        L.oracle_parse_batch_mt.argtypes = L.oracle_parse_batch.argtypes + [ctypes.c_int]
        L.oracle_parse_batch_mt.restype = ctypes.c_int
        L.oracle_flow_hash.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16,
                                       ctypes.c_uint16, ctypes.c_uint8]
        L.oracle_flow_hash.restype = ctypes.c_uint32
        L.oracle_flow_count.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p]
        L.oracle_flow_count.restype = None
        L.oracle_packet_l4.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint16,
                                       ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16,
                                       ctypes.c_uint16]
        L.oracle_packet_l4.restype = ctypes.c_int
        L.oracle_packet_l4_loop.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint16,
                                            ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16,
                                            ctypes.c_uint16]
        L.oracle_packet_l4_loop.restype = ctypes.c_uint64
        L.oracle_packet_l4_loop_mt.argtypes = (L.oracle_packet_l4_loop.argtypes[:5] + [ctypes.c_int]
                                               + L.oracle_packet_l4_loop.argtypes[5:])
        L.oracle_packet_l4_loop_mt.restype = ctypes.c_uint64
        L.oracle_parse_chains_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int]
        L.oracle_parse_chains_mt.restype = ctypes.c_int
        L.oracle_parse_chains.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p]
        L.oracle_parse_chains.restype = None
        L.oracle_pbuf_script.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_pbuf_script.restype = None
        L.oracle_build_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_build_batch.restype = None
        L.oracle_build_tunnel_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_void_p]
        L.oracle_build_tunnel_batch.restype = None
        L.oracle_forward_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint32]
        L.oracle_forward_batch.restype = None
        L.oracle_options_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_options_batch.restype = None
        L.oracle_tunnel_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]
        L.oracle_tunnel_batch.restype = None
        L.oracle_tunnel_flow_events.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_tunnel_flow_events.restype = None
        L.oracle_layers_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]
        L.oracle_layers_batch.restype = None
        L.oracle_fields_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_fields_batch.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def from_slice(data):
    b = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return int(lib().oracle_from_slice(b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), b.size))


def icmp_checksum(data):
    """rpkt/src/icmpv4/generated.rs:2678-2701 calculate_icmp_checksum restated; None for
    the empty slice (where the reference panics)."""
    b = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
    r = int(lib().oracle_icmp_checksum(b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), b.size))
    return None if r < 0 else r


def combine(words):
    a = (ctypes.c_uint16 * len(words))(*words)
    return int(lib().oracle_combine(a, len(words)))


def from_buf(segments, length=None):
    segs = [np.ascontiguousarray(np.frombuffer(bytes(s), dtype=np.uint8)) for s in segments]
    total = sum(s.size for s in segs)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    ptrs = (u8p * len(segs))(*[s.ctypes.data_as(u8p) for s in segs])
    lens = (ctypes.c_size_t * len(segs))(*[s.size for s in segs])
    return int(lib().oracle_from_buf(ptrs, lens, len(segs), total if length is None else length))


def parse_one(frame, flags=3):
    from rpkt_amd.records import REC_DTYPE
    b = np.ascontiguousarray(np.frombuffer(bytes(frame), dtype=np.uint8))
    rec = np.zeros(1, dtype=REC_DTYPE)
    lib().oracle_parse_one(_ptr(b), b.size, flags, _ptr(rec))
    return rec[0]


def _out_buffer(out, n, dtype, what):
    """A caller's preallocated result array (checked), or a fresh zeroed one."""
    if out is None:
        return np.zeros(n, dtype=dtype)
    if out.dtype != dtype or out.shape != (n,) or not out.flags.c_contiguous:
        raise ValueError("%s: expected a contiguous (%d,) %s array" % (what, n, dtype))
    return out


def parse_batch(frames, n, flags=3, offsets=None, stride=0, frame_len=0, n_buckets=0,
                threads=1, flow_ev=False, out=None, ev_out=None):
    """Oracle records (and optionally flow events) for a host batch.  out / ev_out: arrays
    the records / events are written into (every record is written whole, so a reused
    buffer needs no zeroing): a timed loop then allocates nothing per call."""
    from rpkt_amd.records import REC_DTYPE
    frames = frames if (isinstance(frames, np.ndarray) and frames.dtype == np.uint8
                        and frames.flags.c_contiguous) else np.ascontiguousarray(frames, dtype=np.uint8)
    recs = _out_buffer(out, n, REC_DTYPE, "out")
    ev = _out_buffer(ev_out, n, np.uint64, "ev_out") if (flow_ev or ev_out is not None) else None
    flow_ev = ev is not None
    offs = offsets if (offsets is None or (isinstance(offsets, np.ndarray) and offsets.dtype == np.uint32
                                           and offsets.flags.c_contiguous)) \
        else np.ascontiguousarray(offsets, dtype=np.uint32)
    if threads > 1:
        lib().oracle_parse_batch_mt(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n,
                                    flags, n_buckets, _ptr(recs), _ptr(ev), threads)
    else:
        lib().oracle_parse_batch(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n,
                                 flags, n_buckets, _ptr(recs), _ptr(ev))
    return (recs, ev) if flow_ev else recs


def parse_chains(buf, segs, chain_first, flags=3, n_buckets=0, flow_ev=False, threads=1,
                 out=None, ev_out=None):
    """Oracle records for mbuf chains (rpkt_gpu_parse_chains arguments, host memory):
    segs = u32 (offset, length) pairs into buf, chain_first = n_chains + 1 entries.
    out / ev_out: preallocated results, as parse_batch."""
    from rpkt_amd.records import REC_DTYPE
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    segs = np.ascontiguousarray(segs, dtype=np.uint32).reshape(-1)
    cf = np.ascontiguousarray(chain_first, dtype=np.uint32)
    n = cf.size - 1
    recs = _out_buffer(out, n, REC_DTYPE, "out")
    ev = _out_buffer(ev_out, n, np.uint64, "ev_out") if (flow_ev or ev_out is not None) else None
    flow_ev = ev is not None
    if threads > 1:
        lib().oracle_parse_chains_mt(_ptr(buf), buf.size, _ptr(segs), segs.size // 2, _ptr(cf), n,
                                     flags, n_buckets, _ptr(recs), _ptr(ev), threads)
    else:
        lib().oracle_parse_chains(_ptr(buf), buf.size, _ptr(segs), segs.size // 2, _ptr(cf), n,
                                  flags, n_buckets, _ptr(recs), _ptr(ev))
    return (recs, ev) if flow_ev else recs


def packet_l4(frame, want):
    """benches/rpkt/rpkt_parse.rs:62-80 `packet_l4` on one frame: 0 when every assert
    holds.  want = (src u32, dst u32, ip checksum, ident, sport, dport, udp length,
    udp checksum)."""
    b = np.ascontiguousarray(np.frombuffer(bytes(frame), dtype=np.uint8))
    return int(lib().oracle_packet_l4(_ptr(b), b.size, *want))


def packet_l4_loop(frames, n, stride, frame_len, reps, want):
    """`reps` passes of packet_l4 over n frames at `stride` (config 1's timed loop, all in
    C); returns the number of failed frames over all passes."""
    f = np.ascontiguousarray(frames, dtype=np.uint8)
    return int(lib().oracle_packet_l4_loop(_ptr(f), n, stride, frame_len, reps, *want))


def packet_l4_loop_mt(frames, n, stride, frame_len, reps, want, threads):
    """packet_l4_loop on `threads` host threads at once, each making `reps` passes over
    the same n frames (criterion's loop run once per core); returns the failed frames
    over all threads and passes."""
    f = np.ascontiguousarray(frames, dtype=np.uint8)
    return int(lib().oracle_packet_l4_loop_mt(_ptr(f), n, stride, frame_len, reps, threads, *want))


def pbuf_script(seg_lens, ops):
    """Replay Pbuf operations [('new'|'advance'|'trim_off', count)] over segments of
    the given lengths; returns one dict of the observable state per op."""
    kinds = {"new": 0, "advance": 1, "trim_off": 2}
    sl = np.ascontiguousarray(seg_lens, dtype=np.uint32)
    o = np.array([[kinds[k], c] for k, c in ops], dtype=np.uint64).reshape(-1)
    out = np.zeros(6 * len(ops), dtype=np.uint64)
    lib().oracle_pbuf_script(_ptr(sl), sl.size, _ptr(o), len(ops), _ptr(out))
    keys = ("cursor", "chunk_len", "remaining", "headroom", "num_segs", "pkt_len")
    return [dict(zip(keys, (int(x) for x in out[6 * i:6 * i + 6]))) for i in range(len(ops))]


def build_batch(frames, n, recs, flags=3, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_build_batch on the CPU: returns (new frames buffer, built flags)."""
    out = np.array(frames, dtype=np.uint8, copy=True)
    recs = np.ascontiguousarray(recs)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    built = np.zeros(n, dtype=np.uint8)
    lib().oracle_build_batch(_ptr(out), out.size, _ptr(offs), stride, frame_len, n, _ptr(recs),
                             flags, _ptr(built))
    return out, built


def build_tunnel_batch(frames, n, recs, tun, flags=3, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_build_tunnel_batch on the CPU: returns (new frames buffer, built flags)."""
    out = np.array(frames, dtype=np.uint8, copy=True)
    recs = np.ascontiguousarray(recs)
    tun = np.ascontiguousarray(tun)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    built = np.zeros(n, dtype=np.uint8)
    lib().oracle_build_tunnel_batch(_ptr(out), out.size, _ptr(offs), stride, frame_len, n,
                                    _ptr(recs), _ptr(tun), flags, _ptr(built))
    return out, built


def forward_batch(frames, n, recs, dmac, smac, forbid=(), offsets=None, stride=0, frame_len=0,
                  flags=0):
    """rpkt_gpu_forward_batch on the CPU: returns (new frames buffer, keep flags).  flags
    (rpkt_fwd_t.flags): RPKT_F_IPV6 (8) also forwards IPv6 frames (recs from a parse with
    RPKT_F_IPV6)."""
    out = np.array(frames, dtype=np.uint8, copy=True)
    recs = np.ascontiguousarray(recs)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    fb = np.ascontiguousarray(np.sort(np.asarray(forbid, dtype=np.uint32)))
    dm = np.frombuffer(bytes(dmac), dtype=np.uint8).copy()
    sm = np.frombuffer(bytes(smac), dtype=np.uint8).copy()
    keep = np.zeros(n, dtype=np.uint8)
    lib().oracle_forward_batch(_ptr(out), out.size, _ptr(offs), stride, frame_len, n, _ptr(recs),
                               _ptr(dm), _ptr(sm), _ptr(fb) if fb.size else None, fb.size,
                               _ptr(keep), flags)
    return out, keep


def options_batch(frames, n, recs, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_options_batch on the CPU: rpkt_opts_t per frame."""
    from rpkt_amd.records import OPTS_DTYPE
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    recs = np.ascontiguousarray(recs)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    out = np.zeros(n, dtype=OPTS_DTYPE)
    lib().oracle_options_batch(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n,
                               _ptr(recs), _ptr(out))
    return out


def tunnel_batch(frames, n, flags=3, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_parse_tunnel_batch on the CPU: (outer records, rpkt_tun_t, inner records)."""
    from rpkt_amd.records import REC_DTYPE, TUN_DTYPE
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    outer = np.zeros(n, dtype=REC_DTYPE)
    tun = np.zeros(n, dtype=TUN_DTYPE)
    inner = np.zeros(n, dtype=REC_DTYPE)
    lib().oracle_tunnel_batch(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n, flags,
                              _ptr(outer), _ptr(tun), _ptr(inner))
    return outer, tun, inner


def tunnel_flow_events(outer, tun, inner, n_buckets):
    """rpkt_gpu_parse_tunnel_batch's RPKT_F_FLOW_EV events from its three record arrays:
    the inner record's event when the tunnel decoded, else the outer record's."""
    outer, tun, inner = (np.ascontiguousarray(x) for x in (outer, tun, inner))
    ev = np.zeros(outer.size, dtype=np.uint64)
    lib().oracle_tunnel_flow_events(_ptr(outer), _ptr(tun), _ptr(inner), outer.size, n_buckets,
                                    _ptr(ev))
    return ev


def tunnel_one(frame, flags=3):
    """(outer record, rpkt_tun_t, inner record) of one frame."""
    b = np.frombuffer(bytes(frame), dtype=np.uint8)
    o, t, i = tunnel_batch(b, 1, flags, offsets=np.array([0, b.size], np.uint32))
    return o[0], t[0], i[0]


def layers_batch(frames, n, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_layers_batch on the CPU: rpkt_layers_t per frame."""
    from rpkt_amd.records import LAYERS_DTYPE
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    out = np.zeros(n, dtype=LAYERS_DTYPE)
    lib().oracle_layers_batch(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n,
                              _ptr(out))
    return out


def fields_batch(frames, n, layers, reqs, offsets=None, stride=0, frame_len=0):
    """rpkt_gpu_fields_batch on the CPU: (values n x n_req uint64, present n uint32)."""
    from rpkt_amd.records import FIELD_REQ_DTYPE, LAYERS_DTYPE
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    layers = np.ascontiguousarray(layers, dtype=LAYERS_DTYPE)
    reqs = np.ascontiguousarray(reqs, dtype=FIELD_REQ_DTYPE)
    values = np.zeros((n, reqs.size), dtype=np.uint64)
    present = np.zeros(n, dtype=np.uint32)
    lib().oracle_fields_batch(_ptr(frames), frames.size, _ptr(offs), stride, frame_len, n,
                              _ptr(layers), _ptr(reqs), reqs.size, _ptr(values), _ptr(present))
    return values, present


def leg_callable(mode, frames, n, offsets=None, stride=0, frame_len=0, recs=None, tun=None,
                 layers=None, reqs=None, flags=3, dmac=b"", smac=b"", forbid=()):
    """A closure that runs one bench leg's CPU restatement over a host sample with every
    output allocated here, once, and its C arguments converted once (bench.py's per-leg
    cpu_baseline times the closure alone: no allocation per call).  mode: build / forward
    / encap (in place on a private copy of the frames, which each call rewrites again),
    opts / optsc (both: Ipv4OptionsIter + TcpOptionsIter from full records), layers,
    fields, tunnel.  The closure's `arrays` attribute holds its buffers."""
    from rpkt_amd.records import FIELD_REQ_DTYPE, LAYERS_DTYPE, OPTS_DTYPE, REC_DTYPE, TUN_DTYPE
    L = lib()
    src = np.ascontiguousarray(frames, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint32) if offsets is not None else None
    head = (src, offs, stride, frame_len, n)
    if mode in ("build", "forward", "encap"):
        buf = src.copy()
        done = np.zeros(n, dtype=np.uint8)
        r = np.ascontiguousarray(recs)
        head = (buf, offs, stride, frame_len, n)
        if mode == "build":
            fn, arrays, rest = L.oracle_build_batch, [buf, done, r], (r, flags, done)
        elif mode == "encap":
            t = np.ascontiguousarray(tun)
            fn, arrays, rest = L.oracle_build_tunnel_batch, [buf, done, r, t], (r, t, flags, done)
        else:
            fb = np.ascontiguousarray(np.sort(np.asarray(forbid, dtype=np.uint32)))
            dm = np.frombuffer(bytes(dmac), dtype=np.uint8).copy()
            sm = np.frombuffer(bytes(smac), dtype=np.uint8).copy()
            fn, arrays = L.oracle_forward_batch, [buf, done, r, fb, dm, sm]
            rest = (r, dm, sm, fb if fb.size else None, fb.size, done, flags)
    elif mode in ("opts", "optsc"):
        r = np.ascontiguousarray(recs)
        out = np.zeros(n, dtype=OPTS_DTYPE)
        fn, arrays, rest = L.oracle_options_batch, [r, out], (r, out)
    elif mode == "layers":
        out = np.zeros(n, dtype=LAYERS_DTYPE)
        fn, arrays, rest = L.oracle_layers_batch, [out], (out,)
    elif mode == "fields":
        lay = np.ascontiguousarray(layers, dtype=LAYERS_DTYPE)
        q = np.ascontiguousarray(reqs, dtype=FIELD_REQ_DTYPE)
        values = np.zeros((n, q.size), dtype=np.uint64)
        present = np.zeros(n, dtype=np.uint32)
        fn, arrays, rest = L.oracle_fields_batch, [lay, q, values, present], \
            (lay, q, q.size, values, present)
    elif mode == "tunnel":
        outer = np.zeros(n, dtype=REC_DTYPE)
        tu = np.zeros(n, dtype=TUN_DTYPE)
        inner = np.zeros(n, dtype=REC_DTYPE)
        fn, arrays, rest = L.oracle_tunnel_batch, [outer, tu, inner], (flags, outer, tu, inner)
    else:
        raise ValueError("leg_callable: unknown mode %r" % mode)
    # (frames, frames bytes, offsets, stride, frame_len, n, ...) as C arguments, once
    conv = lambda x: _ptr(x) if isinstance(x, np.ndarray) else x      # noqa: E731
    args = (conv(head[0]), head[0].size, _ptr(head[1]), head[2], head[3], head[4]) + \
        tuple(conv(x) for x in rest)

    def run():
        fn(*args)
    run.arrays = [src, offs] + arrays
    return run


def flow_count(ev, n_buckets):
    ev = np.ascontiguousarray(ev, dtype=np.uint64)
    counters = np.zeros((n_buckets + 1) * 4, dtype=np.uint64)
    lib().oracle_flow_count(_ptr(ev), ev.size, n_buckets, _ptr(counters))
    return counters


def flow_hash(src, dst, sp, dp, proto):
    return int(lib().oracle_flow_hash(src, dst, sp, dp, proto))


def load_dat(path):
    """rpkt/tests/common/mod.rs:3-29: hex text, two characters per byte."""
    with open(path) as fh:
        s = fh.read().strip()
    return bytes(int(s[i:i + 2], 16) for i in range(0, len(s), 2))
