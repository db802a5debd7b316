"""summariseVcf: cut one VCF into summariseSlice slices.

Restates lambda/summariseVcf/lambda_function.py:69-87 (find_best_split /
next_newton_approximation, float64 slice-size model), :197-214
(partition_chunks) and :253-278 (summarise_vcf).  The chunk boundaries come
from the store (every record start of each contig, sb_store_chunk_boundaries)
instead of the CSI/TBI index (get_chunk_boundaries, :90-104): index chunk
boundaries are record starts as well, so partition_chunks sees a superset of
the index's boundaries and closes slices at the same block-distance rule.
The slices then go to the device in one sb_summarise_slices call instead of
one SNS message each (publish_slice_updates, :217-229).
"""
from __future__ import annotations

MIN_SS_TIME = 0.1  # minimum time summariseSlice will run (s)       (:21)
SS_RATE = 75000000  # processing speed of summariseSlice (B/s)     (:22)
SNS_TIME = 0.02  # time to publish a message to SNS                (:23)
MAX_CONCURRENCY = 1000  # maximum number of summariseSlice invocations (:24)


def next_newton_approximation(total_size, split_size):
    d = (-MIN_SS_TIME ** 2 / split_size ** 2 + 1 / SS_RATE ** 2
         - 2 * SNS_TIME * total_size * MIN_SS_TIME / split_size ** 3
         - SNS_TIME * total_size / split_size ** 2 / SS_RATE)
    dd = (2 * MIN_SS_TIME ** 2 / split_size ** 3 + 6 * SNS_TIME * total_size * MIN_SS_TIME / split_size ** 4
          + 2 * SNS_TIME * total_size / split_size ** 3 / SS_RATE)
    return split_size - d / dd


def find_best_split(total_size, epsilon):
    """Newton iteration from sqrt(total_size) until the extrapolated
    remaining error of the geometric-looking sequence is below epsilon."""
    seq = [total_size ** 0.5]
    while True:
        nxt = next_newton_approximation(total_size, seq[-1])
        if nxt <= 0:  # overshot into the divergent region: halve instead
            nxt = seq[-1] / 2
        if len(seq) >= 2:
            step = nxt - seq[-1]
            rate = step / (seq[-1] - seq[-2])
            if abs(rate) < 1 and abs(step / (1 - rate)) < epsilon:
                return nxt
        seq.append(nxt)


def partition_chunks(chunk_boundaries: dict, slice_size):
    """Per contig, close a slice at the first boundary whose BGZF block
    offset is >= slice_size bytes past the slice's start block."""
    out = []
    for offs in chunk_boundaries.values():
        start = offs[0]
        for v in offs:
            if (v >> 16) - (start >> 16) >= slice_size:
                out.append((start, v))
                start = v
        if offs[-1] != start:
            out.append((start, offs[-1]))
    return out


def chunk_boundaries(store, location, stride=1) -> dict:
    """{contig: sorted record-start virtual offsets (+ contig end)}."""
    out = {}
    for contig in store.contigs(location):
        b = store.chunk_boundaries(location, contig, stride)
        if b:
            out[contig] = b
    return out


def plan_slices(store, location, stride=1):
    """summarise_vcf (:253-267): the (virtual_start, virtual_end) slices."""
    cb = chunk_boundaries(store, location, stride)
    if not cb:
        return []
    first_chunk_start = min(b[0] for b in cb.values()) >> 16
    last_chunk_end = (max(b[-1] for b in cb.values()) >> 16) + 2 ** 16
    num_chunks = sum(len(b) for b in cb.values()) - 1
    total_size = last_chunk_end - first_chunk_start
    avg_chunk_size = total_size / max(num_chunks, 1)
    best = find_best_split(total_size, avg_chunk_size / 2)
    if total_size / best > MAX_CONCURRENCY:
        best = total_size / MAX_CONCURRENCY
    return partition_chunks(cb, best)


def summarise_vcf(store, location, stride=1):
    """All slices of one VCF summarised on the device; returns
    (slices, per-slice RegionStats, the VCF's totals)."""
    slices = plan_slices(store, location, stride)
    stats = store.summarise_slices([(location, a, b) for a, b in slices])
    tot = {'variantCount': 0, 'callCount': 0}
    for s in stats:
        if isinstance(s, Exception):
            raise s
        tot['variantCount'] += s['numVariants']
        tot['callCount'] += s['numCalls']
    return slices, stats, tot
