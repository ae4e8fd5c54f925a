"""Multi-GPU work split for the front end.

The path shards with no data-path collective:

* **Independent streams** (the benchmark's mode, BASELINE config 4): stream
  s goes to rank ``s % world`` (round robin keeps per-rank load equal to
  within one stream).  Each rank owns the filter state (ns floats per
  channel) and prev_I/prev_Q of its streams; nothing is exchanged.

* **One long stream** split into contiguous segments: the reference's
  output is block-size independent (consecutive blocks == one stream, bit
  for bit, src/filter.cpp:82/139 carry the raw input tail), so a segment
  starting at sample p0 (a multiple of D) is computed exactly by a rank that
  is handed (a) the ns input samples before p0 as its ``state`` and (b) the
  decimated I/Q sample just before p0 as its ``prev``.  (b) is output
  p0/D - 1, the last output of one FIR+decimate call over [halo_lo, p0)
  with the ns samples before halo_lo as that call's state.  halo_lo =
  p0 - D*ceil(ns/D) is a multiple of D (the call runs at the stream's own
  decimation phase) and leaves the call >= ns inputs (the reference's
  n >= ns precondition).  The rank therefore reads a halo of
  D*ceil(ns/D) + ns samples before p0 -- replicated reads of the previous
  segment's data, not messages: no RCCL/xGMI traffic.
"""
from __future__ import annotations

from dataclasses import dataclass


def stream_ranks(nstreams: int, world: int) -> list[list[int]]:
    """Round-robin assignment of independent streams to ranks."""
    if world < 1:
        raise ValueError("world must be >= 1")
    return [list(range(r, nstreams, world)) for r in range(world)]


def streams_of(rank: int, nstreams: int, world: int) -> list[int]:
    return stream_ranks(nstreams, world)[rank]


@dataclass(frozen=True)
class Segment:
    rank: int
    start: int      # first input sample of the segment (p0, a multiple of D)
    stop: int       # one past the last input sample
    halo_lo: int    # first input of the prev_* recompute call (p0 - D*ceil(ns/D)); 0 for the first segment
    read_lo: int    # first input sample the rank reads: the recompute call's state (halo_lo - ns, >= 0)

    @property
    def length(self) -> int:
        return self.stop - self.start


def segment_plan(n: int, D: int, ntaps: int, ns: int, world: int) -> list[Segment]:
    """Split one stream of n samples (n % D == 0) into `world` contiguous
    segments on D-sample boundaries, each at least ns samples long (the
    reference's n >= ns precondition) and with its halo range."""
    if n % D:
        raise ValueError("n must be a multiple of D")
    if ns < ntaps - 1:
        raise ValueError("state shorter than ntaps - 1")
    nout = n // D
    bounds = [round(nout * r / world) * D for r in range(world + 1)]
    segs = []
    for r in range(world):
        a, b = bounds[r], bounds[r + 1]
        if b - a < max(ns, D):
            raise ValueError(f"segment {r} too short ({b - a} < {max(ns, D)})")
        halo_lo = max(a - D * (-(-max(ns, 1) // D)), 0) if a else 0
        segs.append(Segment(rank=r, start=a, stop=b, halo_lo=halo_lo, read_lo=max(halo_lo - ns, 0) if a else 0))
    return segs
