"""Device batch API: rpkt's decode-and-verify chain over a device-resident batch.

Thin ctypes layer over the C ABI in include/rpkt_gpu.h (librpkt_gpu.so, HIP for
gfx950).  torch supplies device memory and the current HIP stream only; no torch
type crosses the ABI.  There is no CPU fallback: if the HIP library is missing
or no GPU is visible, every call raises.
"""
import ctypes
import os

import numpy as np

from .build import ABLATE_LIB, GPU_LIB
from .records import LAYERS_BYTES, OPTS_BYTES, REC_BYTES, REC16_BYTES, F_FLOW_EV

RPKT_OK = 0
ERRORS = {-1: "RPKT_E_INVAL", -2: "RPKT_E_HIP", -3: "RPKT_E_TOO_LARGE", -4: "RPKT_E_ALIGN",
          -5: "RPKT_E_COLL"}


class RpktError(RuntimeError):
    pass


class Batch(ctypes.Structure):
    """rpkt_batch_t"""
    _fields_ = [("frames_dev", ctypes.c_void_p), ("frames_bytes", ctypes.c_uint64),
                ("offsets_dev", ctypes.c_void_p), ("stride", ctypes.c_uint32),
                ("frame_len", ctypes.c_uint32), ("n", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class Chains(ctypes.Structure):
    """rpkt_chains_t"""
    _fields_ = [("buf_dev", ctypes.c_void_p), ("buf_bytes", ctypes.c_uint64),
                ("segs_dev", ctypes.c_void_p), ("chain_first_dev", ctypes.c_void_p),
                ("n_segs", ctypes.c_uint32), ("n_chains", ctypes.c_uint32)]


class RingSlot(ctypes.Structure):
    """rpkt_ring_slot_t"""
    _fields_ = [("batch", Batch), ("recs_dev", ctypes.c_void_p), ("flow_ev_dev", ctypes.c_void_p)]


class TunRingSlot(ctypes.Structure):
    """rpkt_tun_ring_slot_t"""
    _fields_ = [("batch", Batch), ("outer_dev", ctypes.c_void_p), ("tun_dev", ctypes.c_void_p),
                ("inner_dev", ctypes.c_void_p), ("flow_ev_dev", ctypes.c_void_p)]


class Fwd(ctypes.Structure):
    """rpkt_fwd_t"""
    _fields_ = [("dmac", ctypes.c_uint8 * 6), ("smac", ctypes.c_uint8 * 6),
                ("forbid_dev", ctypes.c_void_p), ("n_forbid", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


EXPORTS = ["rpkt_gpu_abi_version", "rpkt_gpu_build_info", "rpkt_gpu_status_name",
           "rpkt_gpu_last_hip_error", "rpkt_gpu_device_info", "rpkt_gpu_parse_batch", "rpkt_gpu_flow_workspace_bytes",
           "rpkt_gpu_flow_count", "rpkt_gpu_checksum_ranges", "rpkt_flow_hash",
           "rpkt_gpu_checksum_chains_workspace_bytes", "rpkt_gpu_checksum_chains",
           "rpkt_gpu_parse_chains", "rpkt_gpu_build_batch", "rpkt_gpu_forward_batch",
           "rpkt_gpu_options_batch", "rpkt_gpu_layers_batch", "rpkt_gpu_fields_batch",
           "rpkt_gpu_flow_reduce", "rpkt_gpu_last_coll_error", "rpkt_gpu_coll_version",
           "rpkt_gpu_parse_batch_compact", "rpkt_gpu_options_batch_compact",
           "rpkt_gpu_parse_options_batch", "rpkt_gpu_parse_options_batch_compact",
           "rpkt_gpu_parse_ring", "rpkt_gpu_parse_ring_compact", "rpkt_gpu_coll_unique_id",
           "rpkt_gpu_comm_init", "rpkt_gpu_comm_destroy", "rpkt_gpu_comm_init_timeout",
           "rpkt_gpu_comm_abort", "rpkt_gpu_parse_tunnel_batch", "rpkt_gpu_build_tunnel_batch",
           "rpkt_gpu_parse_tunnel_ring"]
COLL_ID_BYTES = 128

_lib = None


def lib():
    """Load librpkt_gpu.so (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is None:
        # Bind to the HIP runtime torch already carries: loading ours first would
        # pull a second runtime (/opt/rocm) into the process, and only one of the
        # two can own the device.
        import torch  # noqa: F401
        if not os.path.exists(GPU_LIB):
            raise RpktError("HIP engine not built: %s missing (run __graft_entry__.build())"
                            % GPU_LIB)
        L = ctypes.CDLL(GPU_LIB)
        L.rpkt_gpu_abi_version.restype = ctypes.c_uint32
        L.rpkt_gpu_build_info.restype = ctypes.c_char_p
        L.rpkt_gpu_status_name.argtypes = [ctypes.c_int]
        L.rpkt_gpu_status_name.restype = ctypes.c_char_p
        L.rpkt_gpu_last_hip_error.restype = ctypes.c_int
        L.rpkt_gpu_device_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.rpkt_gpu_device_info.restype = ctypes.c_int
        L.rpkt_gpu_parse_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p]
        L.rpkt_gpu_parse_batch.restype = ctypes.c_int
        L.rpkt_gpu_parse_batch_compact.argtypes = L.rpkt_gpu_parse_batch.argtypes
        L.rpkt_gpu_parse_batch_compact.restype = ctypes.c_int
        L.rpkt_gpu_parse_ring.argtypes = [ctypes.POINTER(RingSlot), ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.rpkt_gpu_parse_ring.restype = ctypes.c_int
        L.rpkt_gpu_parse_ring_compact.argtypes = L.rpkt_gpu_parse_ring.argtypes
        L.rpkt_gpu_parse_ring_compact.restype = ctypes.c_int
        L.rpkt_gpu_flow_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.rpkt_gpu_flow_workspace_bytes.restype = ctypes.c_size_t
        L.rpkt_gpu_flow_count.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_flow_count.restype = ctypes.c_int
        L.rpkt_gpu_checksum_ranges.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_checksum_ranges.restype = ctypes.c_int
        L.rpkt_gpu_checksum_chains_workspace_bytes.argtypes = [ctypes.c_uint32]
        L.rpkt_gpu_checksum_chains_workspace_bytes.restype = ctypes.c_size_t
        L.rpkt_gpu_checksum_chains.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_checksum_chains.restype = ctypes.c_int
        L.rpkt_gpu_parse_chains.argtypes = [ctypes.POINTER(Chains), ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_void_p]
        L.rpkt_gpu_parse_chains.restype = ctypes.c_int
        L.rpkt_gpu_build_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_build_batch.restype = ctypes.c_int
        L.rpkt_gpu_forward_batch.argtypes = [ctypes.POINTER(Batch), ctypes.POINTER(Fwd),
                                             ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_forward_batch.restype = ctypes.c_int
        L.rpkt_gpu_options_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_options_batch.restype = ctypes.c_int
        L.rpkt_gpu_options_batch_compact.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_options_batch_compact.restype = ctypes.c_int
        L.rpkt_gpu_parse_options_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_uint32,
                                                   ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_uint32,
                                                   ctypes.c_void_p]
        L.rpkt_gpu_parse_options_batch.restype = ctypes.c_int
        L.rpkt_gpu_parse_options_batch_compact.argtypes = L.rpkt_gpu_parse_options_batch.argtypes
        L.rpkt_gpu_parse_options_batch_compact.restype = ctypes.c_int
        L.rpkt_gpu_parse_tunnel_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_uint32,
                                                  ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_uint32, ctypes.c_void_p]
        L.rpkt_gpu_parse_tunnel_batch.restype = ctypes.c_int
        L.rpkt_gpu_parse_tunnel_ring.argtypes = [ctypes.POINTER(TunRingSlot), ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.rpkt_gpu_parse_tunnel_ring.restype = ctypes.c_int
        L.rpkt_gpu_build_tunnel_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_build_tunnel_batch.restype = ctypes.c_int
        L.rpkt_gpu_layers_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p,
                                            ctypes.c_void_p]
        L.rpkt_gpu_layers_batch.restype = ctypes.c_int
        L.rpkt_gpu_fields_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_fields_batch.restype = ctypes.c_int
        L.rpkt_gpu_flow_reduce.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.rpkt_gpu_flow_reduce.restype = ctypes.c_int
        L.rpkt_gpu_last_coll_error.restype = ctypes.c_int
        L.rpkt_gpu_coll_version.restype = ctypes.c_int
        L.rpkt_gpu_coll_unique_id.argtypes = [ctypes.c_void_p]
        L.rpkt_gpu_coll_unique_id.restype = ctypes.c_int
        L.rpkt_gpu_comm_init.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int]
        L.rpkt_gpu_comm_init.restype = ctypes.c_int
        L.rpkt_gpu_comm_destroy.argtypes = [ctypes.c_void_p]
        L.rpkt_gpu_comm_destroy.restype = ctypes.c_int
        L.rpkt_gpu_comm_init_timeout.argtypes = L.rpkt_gpu_comm_init.argtypes + [ctypes.c_int]
        L.rpkt_gpu_comm_init_timeout.restype = ctypes.c_int
        L.rpkt_gpu_comm_abort.argtypes = [ctypes.c_void_p]
        L.rpkt_gpu_comm_abort.restype = ctypes.c_int
        L.rpkt_flow_hash.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16,
                                     ctypes.c_uint16, ctypes.c_uint8]
        L.rpkt_flow_hash.restype = ctypes.c_uint32
        _lib = L
    return _lib


_ablate = None


def ablate_lib():
    """librpkt_gpu_ablate.so: the product entry points plus the development hooks
    (rpkt_gpu_debug_*: kernel ablation variants and streaming references) that tools/
    and bench.py's copy ceiling use.  Never used by the product path."""
    global _ablate
    if _ablate is None:
        lib()                                   # torch's HIP runtime first, as for lib()
        if not os.path.exists(ABLATE_LIB):
            raise RpktError("development library not built: %s missing" % ABLATE_LIB)
        _ablate = ctypes.CDLL(ABLATE_LIB)
    return _ablate


def device_info():
    buf = ctypes.create_string_buffer(512)
    lib().rpkt_gpu_device_info(buf, 512)
    return buf.value.decode()


def _check(rc, what):
    if rc != RPKT_OK:
        extra = ""
        if rc == -2:
            extra = " (hipError %d)" % lib().rpkt_gpu_last_hip_error()
        elif rc == -5:
            extra = " (ncclResult %d)" % lib().rpkt_gpu_last_coll_error()
        raise RpktError("%s failed: %s%s" % (what, ERRORS.get(rc, rc), extra))


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RpktError("no GPU visible: the rpkt_amd engine has no CPU path")
    return torch


def _stream_ptr(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class DeviceBatch:
    """A batch resident in HBM: frames (uint8) and, for packed layout, u32 offsets."""

    def __init__(self, frames, n, offsets=None, stride=0, frame_len=0):
        self.frames, self.n, self.offsets = frames, n, offsets
        self.stride, self.frame_len = stride, frame_len

    @classmethod
    def from_host(cls, hb, device="cuda"):
        torch = _torch()
        frames = torch.from_numpy(np.ascontiguousarray(hb.frames)).to(device)
        offs = None
        if hb.offsets is not None:
            offs = torch.from_numpy(hb.offsets.view(np.int32)).to(device)
        return cls(frames, hb.n, offs, hb.stride, hb.frame_len)

    def shard(self, lo, hi):
        """Frames [lo, hi) as a view (packed offsets stay absolute: no copy)."""
        if self.offsets is not None:
            return DeviceBatch(self.frames, hi - lo, self.offsets[lo:hi + 1])
        return DeviceBatch(self.frames[lo * self.stride:], hi - lo, None, self.stride,
                           self.frame_len)

    def desc(self):
        return Batch(self.frames.data_ptr(), self.frames.numel(),
                     self.offsets.data_ptr() if self.offsets is not None else None,
                     self.stride, self.frame_len, self.n, 0)


def alloc_records(n, device="cuda"):
    torch = _torch()
    return torch.empty(n * REC_BYTES, dtype=torch.uint8, device=device)


def parse_batch(batch, flags=3, recs=None, flow_ev=None, n_buckets=0, stream=None):
    """rpkt_gpu_parse_batch: returns the uint8 record tensor (n * 80 bytes)."""
    torch = _torch()
    if recs is None:
        recs = alloc_records(batch.n, batch.frames.device)
    if flags & F_FLOW_EV and flow_ev is None:
        flow_ev = torch.empty(batch.n, dtype=torch.int64, device=batch.frames.device)
    d = batch.desc()
    rc = lib().rpkt_gpu_parse_batch(ctypes.byref(d), flags, recs.data_ptr(),
                                    flow_ev.data_ptr() if flow_ev is not None else None,
                                    n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_batch")
    return (recs, flow_ev) if flags & F_FLOW_EV else recs


def parse_tunnel_batch(batch, flags=3, outer=None, tun=None, inner=None, stream=None,
                       flow_ev=None, n_buckets=0):
    """rpkt_gpu_parse_tunnel_batch: returns (outer records, rpkt_tun_t, inner records) as
    uint8 tensors (n * 80, n * 16, n * 80 bytes); with RPKT_F_FLOW_EV also the flow events
    (int64 tensor of n: the inner record's event when the tunnel decoded, else the outer's)."""
    torch = _torch()
    dev = batch.frames.device
    outer = alloc_records(batch.n, dev) if outer is None else outer
    inner = alloc_records(batch.n, dev) if inner is None else inner
    tun = torch.empty(batch.n * 16, dtype=torch.uint8, device=dev) if tun is None else tun
    if flags & F_FLOW_EV and flow_ev is None:
        flow_ev = torch.empty(batch.n, dtype=torch.int64, device=dev)
    d = batch.desc()
    rc = lib().rpkt_gpu_parse_tunnel_batch(ctypes.byref(d), flags, outer.data_ptr(),
                                           tun.data_ptr(), inner.data_ptr(),
                                           flow_ev.data_ptr() if flow_ev is not None else None,
                                           n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_tunnel_batch")
    return (outer, tun, inner, flow_ev) if flags & F_FLOW_EV else (outer, tun, inner)


def tunnel_ring_slots(batches, outers, tuns, inners, flow_evs=None):
    """The rpkt_tun_ring_slot_t array of a ring of tunnelled bursts: batch k with its outer
    record, tunnel record and inner record tensors (n * 80, n * 16, n * 80 bytes) and
    (optional) its flow-event tensor.  As ring_slots: build it once, keep the tensors alive
    and in place while it is used."""
    k = len(batches)
    if not (len(outers) == len(tuns) == len(inners) == k) or \
            (flow_evs is not None and len(flow_evs) != k):
        raise RpktError("tunnel_ring_slots: %d batches, %d/%d/%d record tensors"
                        % (k, len(outers), len(tuns), len(inners)))
    arr = (TunRingSlot * k)()
    for j, db in enumerate(batches):
        for t, per, what in ((outers[j], REC_BYTES, "outer"), (tuns[j], 16, "tunnel"),
                             (inners[j], REC_BYTES, "inner")):
            if t.numel() * t.element_size() < db.n * per:
                raise RpktError("tunnel_ring_slots: slot %d %s records too small" % (j, what))
        if flow_evs is not None and flow_evs[j].numel() * flow_evs[j].element_size() < 8 * db.n:
            raise RpktError("tunnel_ring_slots: slot %d flow-event tensor too small" % j)
        arr[j].batch = db.desc()
        arr[j].outer_dev = outers[j].data_ptr()
        arr[j].tun_dev = tuns[j].data_ptr()
        arr[j].inner_dev = inners[j].data_ptr()
        arr[j].flow_ev_dev = flow_evs[j].data_ptr() if flow_evs is not None else None
    return arr


def parse_tunnel_ring(slots, flags=3, n_buckets=0, stream=None):
    """rpkt_gpu_parse_tunnel_ring: every slot of `slots` (tunnel_ring_slots()) parsed as by
    parse_tunnel_batch, RPKT_RING_MAX_SLOTS slots per kernel launch."""
    rc = lib().rpkt_gpu_parse_tunnel_ring(slots, len(slots), flags, n_buckets,
                                          _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_tunnel_ring")


def parse_batch_compact(batch, flags=3, recs=None, flow_ev=None, n_buckets=0, stream=None):
    """rpkt_gpu_parse_batch_compact: the same parse writing 16-byte rpkt_rec16_t
    records; returns the uint8 record tensor (n * 16 bytes)."""
    torch = _torch()
    if recs is None:
        recs = torch.empty(batch.n * REC16_BYTES, dtype=torch.uint8, device=batch.frames.device)
    if flags & F_FLOW_EV and flow_ev is None:
        flow_ev = torch.empty(batch.n, dtype=torch.int64, device=batch.frames.device)
    d = batch.desc()
    rc = lib().rpkt_gpu_parse_batch_compact(ctypes.byref(d), flags, recs.data_ptr(),
                                            flow_ev.data_ptr() if flow_ev is not None else None,
                                            n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_batch_compact")
    return (recs, flow_ev) if flags & F_FLOW_EV else recs


def ring_slots(batches, recs, flow_evs=None, compact=None):
    """The rpkt_ring_slot_t array of a receive ring: batch k, its record tensor and
    (optional) its flow-event tensor.  Build it once per ring and pass it to parse_ring
    on every pass: it holds device addresses only, so the batches and tensors must stay
    alive (and in place) as long as the array is used.  Every batch needs its record
    tensor (and flow-event tensor), each large enough for its frames: 80-B records, or
    16-B ones with compact=True (compact=None: either, checked again by parse_ring)."""
    if len(recs) != len(batches) or (flow_evs is not None and len(flow_evs) != len(batches)):
        raise RpktError("ring_slots: %d batches, %d record tensors, %s flow-event tensors"
                        % (len(batches), len(recs), len(flow_evs) if flow_evs is not None
                           else "no"))
    arr = (RingSlot * len(batches))()
    small = []
    for k, (db, r) in enumerate(zip(batches, recs)):
        have = r.numel() * r.element_size()
        if have < db.n * (REC16_BYTES if compact else REC_BYTES):
            if compact is False or have < db.n * REC16_BYTES:
                raise RpktError("ring_slots: slot %d holds %d record bytes for %d frames"
                                % (k, have, db.n))
            small.append(k)
        if flow_evs is not None and flow_evs[k].numel() * flow_evs[k].element_size() < 8 * db.n:
            raise RpktError("ring_slots: slot %d flow-event tensor too small" % k)
        arr[k].batch = db.desc()
        arr[k].recs_dev = r.data_ptr()
        arr[k].flow_ev_dev = flow_evs[k].data_ptr() if flow_evs is not None else None
    # record bytes the slots can hold: 80-B parses refused by parse_ring if any is 16-B sized
    arr._rpkt_compact_only = bool(small)
    return arr


def parse_ring(slots, flags=3, n_buckets=0, stream=None, compact=False):
    """rpkt_gpu_parse_ring[_compact]: every slot of `slots` (ring_slots(), with 80-B or,
    compact, 16-B record tensors) parsed as by parse_batch[_compact],
    RPKT_RING_MAX_SLOTS slots per kernel launch."""
    if not compact and getattr(slots, "_rpkt_compact_only", False):
        raise RpktError("parse_ring: some slot's records are sized for 16-B compact records")
    fn = lib().rpkt_gpu_parse_ring_compact if compact else lib().rpkt_gpu_parse_ring
    rc = fn(slots, len(slots), flags, n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_ring%s" % ("_compact" if compact else ""))


def flow_workspace(n, n_buckets, device="cuda"):
    torch = _torch()
    nb = int(lib().rpkt_gpu_flow_workspace_bytes(n, n_buckets))
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=device)


def flow_count(flow_ev, n, n_buckets, counters=None, workspace=None, stream=None):
    """rpkt_gpu_flow_count: counters u64[(n_buckets+1)*4] (+= into `counters`)."""
    torch = _torch()
    dev = flow_ev.device
    if counters is None:
        counters = torch.zeros((n_buckets + 1) * 4, dtype=torch.int64, device=dev)
    if workspace is None:
        workspace = flow_workspace(n, n_buckets, dev)
    rc = lib().rpkt_gpu_flow_count(flow_ev.data_ptr(), n, n_buckets, counters.data_ptr(),
                                   workspace.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_flow_count")
    return counters


def flow_reduce(counters, n_buckets, comm, root=-1, stream=None):
    """rpkt_gpu_flow_reduce: sum `counters` (u64[(n_buckets+1)*4] as int64) over every
    rank of the RCCL communicator `comm` (an ncclComm_t as int, e.g. from
    nccl_comm_of()), in place; root -1 = all-reduce, else reduce to that rank."""
    if counters.numel() != (n_buckets + 1) * 4:
        raise RpktError("counters must hold (n_buckets + 1) * 4 words")
    rc = lib().rpkt_gpu_flow_reduce(counters.data_ptr(), n_buckets, root,
                                    ctypes.c_void_p(int(comm)), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_flow_reduce")
    return counters


def nccl_comm_of(group=None):
    """The ncclComm_t (as int) of torch.distributed's RCCL process group for the current
    device, or None when the group's backend is not nccl (gloo rehearsals)."""
    torch = _torch()
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    g = group if group is not None else dist.group.WORLD
    if dist.get_backend(g) != "nccl":
        return None
    ptr = int(g._get_backend(torch.device("cuda", torch.cuda.current_device()))._comm_ptr())
    return ptr or None


def coll_unique_id():
    """rpkt_gpu_coll_unique_id: a fresh RCCL unique id (bytes) for rpkt_gpu_comm_init."""
    buf = (ctypes.c_uint8 * COLL_ID_BYTES)()
    _check(lib().rpkt_gpu_coll_unique_id(buf), "rpkt_gpu_coll_unique_id")
    return bytes(buf)


def comm_init(world, uid, rank):
    """rpkt_gpu_comm_init on the current device: the library's own ncclComm_t (as int).
    Collective: returns when all `world` ranks have called it with the same id."""
    if len(uid) != COLL_ID_BYTES:
        raise RpktError("comm_init: the id must be %d bytes" % COLL_ID_BYTES)
    buf = (ctypes.c_uint8 * COLL_ID_BYTES).from_buffer_copy(uid)
    comm = ctypes.c_void_p()
    _check(lib().rpkt_gpu_comm_init(ctypes.byref(comm), world, buf, rank), "rpkt_gpu_comm_init")
    return int(comm.value)


def comm_init_timeout(world, uid, rank, timeout_ms):
    """rpkt_gpu_comm_init_timeout: the same join, aborted after `timeout_ms` when not every
    rank arrives (RpktError; last_coll_error() == 7 on a timeout)."""
    if len(uid) != COLL_ID_BYTES:
        raise RpktError("comm_init: the id must be %d bytes" % COLL_ID_BYTES)
    buf = (ctypes.c_uint8 * COLL_ID_BYTES).from_buffer_copy(uid)
    comm = ctypes.c_void_p()
    rc = lib().rpkt_gpu_comm_init_timeout(ctypes.byref(comm), world, buf, rank, int(timeout_ms))
    _check(rc, "rpkt_gpu_comm_init_timeout")
    return int(comm.value)


def last_coll_error():
    return int(lib().rpkt_gpu_last_coll_error())


def comm_destroy(comm):
    _check(lib().rpkt_gpu_comm_destroy(ctypes.c_void_p(int(comm))), "rpkt_gpu_comm_destroy")


def comm_abort(comm):
    _check(lib().rpkt_gpu_comm_abort(ctypes.c_void_p(int(comm))), "rpkt_gpu_comm_abort")


def checksum_ranges(buf, ranges, out=None, stream=None):
    """rpkt_gpu_checksum_ranges: batched checksum::from_slice over (start, len) pairs."""
    torch = _torch()
    n = ranges.numel() // 2
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=buf.device)
    rc = lib().rpkt_gpu_checksum_ranges(buf.data_ptr(), buf.numel(), ranges.data_ptr(), n,
                                        out.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_checksum_ranges")
    return out


def checksum_chains(buf, segs, chain_first, out=None, stream=None):
    """rpkt_gpu_checksum_chains: batched checksum::from_buf over segment chains.
    segs: int32 tensor of (start, len) pairs; chain_first: n_chains + 1 indices."""
    torch = _torch()
    n_segs = segs.numel() // 2
    n_chains = chain_first.numel() - 1
    if out is None:
        out = torch.empty(max(n_chains, 0), dtype=torch.int16, device=buf.device)
    ws = torch.empty(int(lib().rpkt_gpu_checksum_chains_workspace_bytes(n_segs)),
                     dtype=torch.uint8, device=buf.device)
    rc = lib().rpkt_gpu_checksum_chains(buf.data_ptr(), buf.numel(), segs.data_ptr(), n_segs,
                                        chain_first.data_ptr(), n_chains, out.data_ptr(),
                                        ws.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_checksum_chains")
    return out


class DeviceChains:
    """Mbuf chains resident in HBM: the segment arena, (offset, length) u32 pairs and
    the n + 1 chain_first indices (rpkt_chains_t)."""

    def __init__(self, buf, segs, chain_first, n):
        self.buf, self.segs, self.chain_first, self.n = buf, segs, chain_first, n

    @classmethod
    def from_host(cls, hc, device="cuda"):
        torch = _torch()
        host = np.ascontiguousarray(hc.buf)
        if not host.flags.writeable:                 # torch refuses read-only numpy memory
            host = host.copy()
        buf = torch.from_numpy(host).to(device)
        segs = torch.from_numpy(np.ascontiguousarray(hc.segs).view(np.int32).reshape(-1)).to(device)
        first = torch.from_numpy(np.ascontiguousarray(hc.chain_first).view(np.int32)).to(device)
        return cls(buf, segs, first, hc.n)

    @property
    def frames(self):
        return self.buf

    def desc(self):
        return Chains(self.buf.data_ptr(), self.buf.numel(), self.segs.data_ptr(),
                      self.chain_first.data_ptr(), self.segs.numel() // 2, self.n)


def parse_chains(chains, flags=3, recs=None, flow_ev=None, n_buckets=0, stream=None):
    """rpkt_gpu_parse_chains: returns the uint8 record tensor (n * 80 bytes)."""
    torch = _torch()
    if recs is None:
        recs = alloc_records(chains.n, chains.buf.device)
    if flags & F_FLOW_EV and flow_ev is None:
        flow_ev = torch.empty(chains.n, dtype=torch.int64, device=chains.buf.device)
    d = chains.desc()
    rc = lib().rpkt_gpu_parse_chains(ctypes.byref(d), flags, recs.data_ptr(),
                                     flow_ev.data_ptr() if flow_ev is not None else None,
                                     n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_chains")
    return (recs, flow_ev) if flags & F_FLOW_EV else recs


def build_batch(batch, recs, flags=3, built=None, stream=None):
    """rpkt_gpu_build_batch: write each frame's headers from its record, in place in
    batch.frames (payload already there).  Returns the per-frame built flags (u8)."""
    torch = _torch()
    if built is None:
        built = torch.empty(batch.n, dtype=torch.uint8, device=batch.frames.device)
    d = batch.desc()
    rc = lib().rpkt_gpu_build_batch(ctypes.byref(d), recs.data_ptr(), flags, built.data_ptr(),
                                    _stream_ptr(stream))
    _check(rc, "rpkt_gpu_build_batch")
    return built


def build_tunnel_batch(batch, recs, tun, flags=3, built=None, stream=None):
    """rpkt_gpu_build_tunnel_batch: the outer headers of recs plus each frame's tunnel
    header of tun (uint8 tensors of n * 80 / n * 16 bytes); returns the built flags."""
    torch = _torch()
    if built is None:
        built = torch.empty(batch.n, dtype=torch.uint8, device=batch.frames.device)
    d = batch.desc()
    rc = lib().rpkt_gpu_build_tunnel_batch(ctypes.byref(d), recs.data_ptr(), tun.data_ptr(),
                                           flags, built.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_build_tunnel_batch")
    return built


def forbid_list(addrs, device="cuda"):
    """Device copy of a forbidden-source list for forward_batch: IPv4 addresses as
    host-order u32 values, sorted ascending (the C ABI's binary search), int32 bits."""
    torch = _torch()
    a = np.unique(np.asarray(addrs, dtype=np.int64) & 0xFFFFFFFF).astype(np.uint32)
    return torch.from_numpy(a.view(np.int32).copy()).to(device)


def forward_batch(batch, dmac, smac, forbid=None, keep=None, stream=None, flags=0):
    """rpkt_gpu_forward_batch (loopback_rx firewall: parse, verdict, rewrite in place).
    forbid: None or a tensor from forbid_list(); flags: 0 or RPKT_F_IPV6 (8), which also
    forwards untagged IPv6/UDP frames."""
    torch = _torch()
    if keep is None:
        keep = torch.empty(batch.n, dtype=torch.uint8, device=batch.frames.device)
    f = Fwd()
    f.dmac[:] = list(bytes(dmac))
    f.smac[:] = list(bytes(smac))
    f.flags = flags
    if forbid is not None and forbid.numel():
        if forbid.dtype != torch.int32:
            raise RpktError("forbid must come from forbid_list() (sorted u32 as int32)")
        f.forbid_dev, f.n_forbid = forbid.data_ptr(), forbid.numel()
    d = batch.desc()
    rc = lib().rpkt_gpu_forward_batch(ctypes.byref(d), ctypes.byref(f), keep.data_ptr(),
                                      _stream_ptr(stream))
    _check(rc, "rpkt_gpu_forward_batch")
    return keep


def options_batch(batch, recs, opts=None, stream=None, compact=False):
    """rpkt_gpu_options_batch: IPv4 and TCP option walks of a parsed batch
    (recs from parse_batch, or from parse_batch_compact with compact=True:
    rpkt_gpu_options_batch_compact); returns the uint8 tensor of n * 64-byte rpkt_opts_t."""
    torch = _torch()
    if recs.numel() != batch.n * (REC16_BYTES if compact else REC_BYTES):
        raise RpktError("records: %d bytes for %d frames" % (recs.numel(), batch.n))
    if opts is None:
        opts = torch.empty(batch.n * OPTS_BYTES, dtype=torch.uint8, device=batch.frames.device)
    d = batch.desc()
    fn = lib().rpkt_gpu_options_batch_compact if compact else lib().rpkt_gpu_options_batch
    rc = fn(ctypes.byref(d), recs.data_ptr(), opts.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_options_batch_compact" if compact else "rpkt_gpu_options_batch")
    return opts


def parse_options_batch(batch, flags=3, recs=None, opts=None, flow_ev=None, n_buckets=0,
                        stream=None, compact=False):
    """rpkt_gpu_parse_options_batch[_compact]: the parse and both option walks in one
    pass.  Returns (records, opts) -- n * 80 (or 16, compact) and n * 64 bytes, uint8 --
    plus the flow events when RPKT_F_FLOW_EV is set."""
    torch = _torch()
    dev = batch.frames.device
    if recs is None:
        recs = torch.empty(batch.n * (REC16_BYTES if compact else REC_BYTES), dtype=torch.uint8,
                           device=dev)
    if opts is None:
        opts = torch.empty(batch.n * OPTS_BYTES, dtype=torch.uint8, device=dev)
    if flags & F_FLOW_EV and flow_ev is None:
        flow_ev = torch.empty(batch.n, dtype=torch.int64, device=dev)
    d = batch.desc()
    fn = (lib().rpkt_gpu_parse_options_batch_compact if compact
          else lib().rpkt_gpu_parse_options_batch)
    rc = fn(ctypes.byref(d), flags, recs.data_ptr(), opts.data_ptr(),
            flow_ev.data_ptr() if flow_ev is not None else None, n_buckets, _stream_ptr(stream))
    _check(rc, "rpkt_gpu_parse_options_batch%s" % ("_compact" if compact else ""))
    return (recs, opts, flow_ev) if flags & F_FLOW_EV else (recs, opts)


def layers_batch(batch, out=None, stream=None):
    """rpkt_gpu_layers_batch: the protocol stack of every frame (pktfmt-derived
    walk); returns the uint8 tensor of n * 64-byte rpkt_layers_t."""
    torch = _torch()
    if out is None:
        out = torch.empty(batch.n * LAYERS_BYTES, dtype=torch.uint8, device=batch.frames.device)
    d = batch.desc()
    rc = lib().rpkt_gpu_layers_batch(ctypes.byref(d), out.data_ptr(), _stream_ptr(stream))
    _check(rc, "rpkt_gpu_layers_batch")
    return out


def fields_batch(batch, layers, reqs, values=None, present=None, stream=None):
    """rpkt_gpu_fields_batch: header-field getters over the layer walk.  `layers` is
    rpkt_gpu_layers_batch's output on the same batch, `reqs` a FIELD_REQ_DTYPE array
    (rpkt_amd.fields.requests builds one by protocol and field name).  Returns
    (values: int64 tensor n x n_req holding the u64 bits, present: int32 tensor n,
    bit r = request r)."""
    import numpy as np
    from .records import FIELD_REQ_DTYPE
    torch = _torch()
    reqs = np.ascontiguousarray(reqs, dtype=FIELD_REQ_DTYPE)
    k = int(reqs.size)
    dev = batch.frames.device
    if values is None:
        values = torch.empty((batch.n, k), dtype=torch.int64, device=dev)   # u64 bits
    if present is None:
        present = torch.empty(batch.n, dtype=torch.int32, device=dev)
    d = batch.desc()
    rc = lib().rpkt_gpu_fields_batch(ctypes.byref(d), layers.data_ptr(),
                                     reqs.ctypes.data_as(ctypes.c_void_p), k,
                                     values.data_ptr(), present.data_ptr(),
                                     _stream_ptr(stream))
    _check(rc, "rpkt_gpu_fields_batch")
    return values, present
