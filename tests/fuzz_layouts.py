"""Random batch layouts for the layout fuzz tests (GPU parity in
test_gpu_fuzz_layouts.py, the oracle under ASan/UBSan in test_oracle_fuzz_layouts.py):
frames drawn from the reference captures and the generator's configs (valid, fuzzed,
1500-B, VLAN/option-heavy), cut at random lengths, laid out packed with random gaps,
odd phases, empty / negative / overlapping / past-the-end descriptors, or strided with
a random stride and frame length."""
import numpy as np

from rpkt_amd import gen


def frames_of(hb):
    if hb.offsets is None:
        L = hb.frame_len or hb.stride
        return [hb.frames[k * hb.stride:k * hb.stride + L].tobytes() for k in range(hb.n)]
    return [hb.frames[int(hb.offsets[k]):int(hb.offsets[k + 1])].tobytes() for k in range(hb.n)]


_POOL = None


def pool():
    global _POOL
    if _POOL is None:
        _POOL = (gen.fixture_frames() + frames_of(gen.make_batch(5, 400, seed=51)) +
                 frames_of(gen.make_batch(6, 600, seed=61)) + frames_of(gen.make_batch(3, 60, seed=31)) +
                 frames_of(gen.make_batch(2, 200, seed=21)))
    return _POOL


def packed_layout(rng, n):
    src = pool()
    picks = [src[int(k)] for k in rng.integers(0, len(src), n)]
    cut = rng.random(n) < 0.3                                  # cut some frames short
    frames = [f[:int(rng.integers(0, len(f) + 1))] if c else f for f, c in zip(picks, cut)]
    gaps = rng.integers(0, 40, n) * (rng.random(n) < 0.5)
    offs = np.zeros(n + 1, dtype=np.int64)
    blob = bytearray(int(rng.integers(0, 16)))               # odd phase at the start
    for k, f in enumerate(frames):
        blob += bytes(int(gaps[k]))
        offs[k] = len(blob)
        blob += f
    offs[n] = len(blob)
    # descriptors: a frame is [offs[k], offs[k+1]); move some starts
    m = max(1, n // 50)
    for k in rng.integers(0, n, m):                          # empty or negative length
        offs[k] = offs[k + 1] - int(rng.integers(-3, 1))
    for k in rng.integers(0, n, m):                          # overlaps the next frames
        offs[k] = max(0, offs[k] - int(rng.integers(1, 200)))
    if rng.random() < 0.5:
        offs[int(rng.integers(0, n))] = len(blob) + int(rng.integers(1, 5000))   # past the end
    buf = np.frombuffer(bytes(blob) + bytes(int(rng.integers(0, 3))), dtype=np.uint8).copy()
    offs = np.clip(offs, 0, (1 << 32) - 1).astype(np.uint32)
    return gen.HostBatch(0, n, 0, buf, offs, 0, 0)


def strided_layout(rng, n):
    src = pool()
    stride = int(rng.integers(14, 1600))
    flen = int(rng.integers(1, stride + 1)) if rng.random() < 0.5 else 0
    L = flen or stride
    buf = np.zeros(n * stride + int(rng.integers(0, 20)), dtype=np.uint8)
    for k in range(n):
        f = src[int(rng.integers(0, len(src)))][:L]
        buf[k * stride:k * stride + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return gen.HostBatch(0, n, 0, buf, None, stride, flen)
