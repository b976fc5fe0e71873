"""Receive loops of small batches, captured once as a HIP graph and replayed.

A DPDK receive loop hands the parser bursts of 32-64 frames (rpkt-dpdk/examples/
loopback_rx.rs:17, 96-121).  On the GPU a batch of tens of thousands of 64-B frames parses
in a few microseconds, about what one kernel launch costs the host, so a loop over many
small batches is launch-bound: the engine's calls are kernel launches and nothing else
(no allocation, no synchronisation, no host round trip), so a pass of the loop can be
captured as one hipGraph and replayed with one host call.

A pass that parses its slots with one rpkt_gpu_parse_ring call (`rx_pass_ring`) needs
no graph to avoid the per-batch launches: the ring's slots are one kernel.

`CapturedLoop(fn)` runs `fn` once eagerly (the warm pass, which also does the engine's
one-time per-device setup outside the capture), captures a second call of `fn` into a
graph (torch.cuda.CUDAGraph, a hipGraph on ROCm) and `replay()`s it.  `fn` issues its
engine calls on the current stream, as every rpkt_amd.engine function does by default.
The device buffers `fn` names are baked into the graph: refill the same buffers (a ring
of slots) between replays, as a NIC fills its ring.  examples/rx_graph.cpp is the same
loop for a C/C++/Rust host (hipStreamBeginCapture around the C ABI calls).
"""
from . import engine


class CapturedLoop:
    def __init__(self, fn, warm=True):
        torch = engine._torch()
        self.fn = fn
        self.graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        if warm:
            with torch.cuda.stream(side):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(self.graph):
            fn()

    def replay(self):
        """One pass of the loop: every captured engine call, on the current stream."""
        self.graph.replay()


def batch_ring(hb, slots):
    """`slots` device batches of host batch `hb`'s shape (a receive ring), each with its
    own copy of the frames."""
    return [engine.DeviceBatch.from_host(hb) for _ in range(slots)]


def rx_pass(ring, recs, ev_all, counters, ws, flags, n_buckets, streams=None):
    """One pass of the receive loop over the ring: per slot, the parse with flow events
    into its part of `ev_all`; then one flow count of the pass's events into `counters`
    (the per-queue counters of rpkt-dpdk/examples/loopback_tx.rs:176-181, summed once per
    pass).  The slots' parses are independent: given `streams`, they are forked over them
    (round robin) and joined before the count, so their kernels can overlap."""
    torch = engine._torch()
    cur = torch.cuda.current_stream()
    for s in streams or ():
        s.wait_stream(cur)
    off = 0
    for k, (db, r) in enumerate(zip(ring, recs)):
        engine.parse_batch(db, flags | engine.F_FLOW_EV, recs=r, flow_ev=ev_all[off:off + db.n],
                           n_buckets=n_buckets, stream=streams[k % len(streams)] if streams else None)
        off += db.n
    for s in streams or ():
        cur.wait_stream(s)
    engine.flow_count(ev_all[:off], off, n_buckets, counters=counters, workspace=ws)


def rx_pass_ring(slots, ev_all, n_ev, counters, ws, flags, n_buckets, compact=False):
    """The same pass with the slots parsed by one rpkt_gpu_parse_ring[_compact] call
    (engine.ring_slots(ring, recs, event views) built once per ring): one kernel for up
    to RPKT_RING_MAX_SLOTS slots instead of one per slot."""
    engine.parse_ring(slots, flags | engine.F_FLOW_EV, n_buckets, compact=compact)
    engine.flow_count(ev_all[:n_ev], n_ev, n_buckets, counters=counters, workspace=ws)
