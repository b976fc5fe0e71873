"""Seeded synthetic batches for the BASELINE.json configs (host C++ generator).

Config ids follow BASELINE.json `configs` (1-based like SURVEY.md §8d):
  1 benches/rpkt: 1,000 x 64 B Ether/IPv4/UDP with the rpkt_build.rs header values
  2 1,048,576 x 64 B Ether/IPv4/UDP, stride 64, 1 % bad IPv4 checksum
  3 1,048,576 x 1500 B Ether/IPv4/TCP, stride 1500, random payload, 1 % bad IP / TCP
  4 8,388,608 IMIX 64/570/1500 at 7:4:1, 50/50 TCP/UDP, packed + u32 offsets
  5 4,194,304 x U[64,1518] B, 802.1Q or QinQ, IPv4 options, TCP options, packed
  6 fuzz: every parse status, frames of 0..300 B and 1000..1600 B, packed
"""
import ctypes
import os

import numpy as np

from .build import GEN_LIB, build_gen

DEFAULT_N = {1: 1000, 2: 1 << 20, 3: 1 << 20, 4: 8 << 20, 5: 4 << 20, 6: 1 << 16}
DEFAULT_SEED = {1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6}
STRIDED = {1: 64, 2: 64, 3: 1500}
FLAGS = {1: 3, 2: 1, 3: 3, 4: 3, 5: 3, 6: 3}   # config 2 = extract + IPv4 header sum

_lib = None


def lib():
    global _lib
    if _lib is None:
        build_gen()   # no-op unless the source is newer than the library
        L = ctypes.CDLL(GEN_LIB)
        L.rpkt_gen_lengths.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_void_p]
        L.rpkt_gen_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.rpkt_gen_fill.restype = ctypes.c_int
        _lib = L
    return _lib


class HostBatch:
    """A generated batch in host memory: frames (uint8) + layout."""

    def __init__(self, config, n, seed, frames, offsets, stride, frame_len):
        self.config, self.n, self.seed = config, n, seed
        self.frames, self.offsets = frames, offsets
        self.stride, self.frame_len = stride, frame_len

    @property
    def frame_bytes(self):
        return int(self.offsets[-1]) if self.offsets is not None else self.n * self.stride

    def lens(self):
        if self.offsets is not None:
            return np.diff(self.offsets.astype(np.int64))
        return np.full(self.n, self.frame_len or self.stride, dtype=np.int64)


def make_batch(config, n=None, seed=None, threads=None, packed=None, first=0):
    """Generate frames [first, first + n) of config `config`.  packed=None uses the
    config's own layout (strided for 1-3); packed frames start at arbitrary byte
    offsets.  A shard generated with `first` equals that slice of the full batch."""
    n = DEFAULT_N[config] if n is None else n
    seed = DEFAULT_SEED[config] if seed is None else seed
    threads = threads or min(16, os.cpu_count() or 1)
    lens = np.zeros(max(n, 1), dtype=np.uint32)
    lib().rpkt_gen_lengths(config, seed, first, n, lens.ctypes.data)
    lens = lens[:n]
    use_packed = (config not in STRIDED) if packed is None else packed
    if not use_packed:
        stride = STRIDED[config]
        frames = np.zeros(n * stride, dtype=np.uint8)
        lib().rpkt_gen_fill(config, seed, first, n, lens.ctypes.data, None, stride,
                            frames.ctypes.data, threads)
        return HostBatch(config, n, seed, frames, None, stride, 0)
    slots = lens.astype(np.uint64)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(slots, out=offsets[1:])
    total = int(offsets[-1])
    if total >= (1 << 32) - 256:
        raise ValueError("batch of %d bytes exceeds the 4 GiB descriptor range" % total)
    offsets32 = offsets.astype(np.uint32)
    frames = np.zeros(total + 16, dtype=np.uint8)
    lib().rpkt_gen_fill(config, seed, first, n, lens.ctypes.data, offsets32.ctypes.data, 0,
                        frames.ctypes.data, threads)
    return HostBatch(config, n, seed, frames[:total], offsets32, 0, 0)
