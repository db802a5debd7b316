"""summariseVcf: cut one VCF into summariseSlice slices.

Restates lambda/summariseVcf/lambda_function.py:69-87 (find_best_split /
next_newton_approximation, float64 slice-size model), :90-104
(get_chunk_boundaries over the VCF's CSI, else TBI, index: :144-156),
:197-214 (partition_chunks) and :253-278 (summarise_vcf).

The index is the one next to the VCF (``<path>.csi`` then ``<path>.tbi``,
get_vcf_index's order) or, when the VCF arrived without one, the index the
ingest writes for it (sb_index_vcf, csrc/index.cpp).  read_index parses both
formats as index_reader.py:4-125 does.  A VCF the store holds only as text
(no BGZF file) has no index; its boundaries are then every record start
(sb_store_chunk_boundaries), which partition_chunks cuts by the same
block-distance rule.  The slices go to the device in one
sb_summarise_slices call instead of one SNS message each
(publish_slice_updates, :217-229).
"""
from __future__ import annotations

import ctypes as C
import gzip
import os
import struct
import zlib

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


INDEX_FORMATS = {'csi': 0, 'tbi': 1}


def write_index(path, fmt='csi', *, min_shift=0, depth=0, save=False) -> bytes:
    """The CSI / TBI index of a BGZF VCF (sb_index_vcf); save=True also
    writes it next to the VCF as ``<path>.<fmt>``."""
    from ._lib import check, lib
    out, n = C.c_void_p(), C.c_size_t()
    check(lib().sb_index_vcf(os.fsencode(path), INDEX_FORMATS[fmt], int(min_shift), int(depth), C.byref(out),
                             C.byref(n)))
    try:
        data = C.string_at(out, n.value)
    finally:
        lib().sb_free(out)
    if save:
        with open(f'{os.fspath(path)}.{fmt}', 'wb') as f:
            f.write(data)
    return data


def read_index(data: bytes) -> dict:
    """index_reader.py:4-125 (Csi / Tbi): names, bin_limit and per reference
    the bins as (bin, [(chunk_beg, chunk_end) virtual offsets])."""
    raw = gzip.decompress(data)
    magic = raw[:4]
    at = 4

    def i32():
        nonlocal at
        (x,) = struct.unpack_from('<i', raw, at)
        at += 4
        return x

    if magic == b'CSI\x01':
        min_shift, depth = i32(), i32()
        bin_limit = ((1 << ((depth + 1) * 3)) - 1) / 7  # a float, as index_reader.py:10
        i32()  # l_aux
    elif magic == b'TBI\x01':
        min_shift, depth = 14, 5
        bin_limit = ((1 << 18) - 1) / 7
        n_ref_tbi = i32()
    else:
        raise ValueError('not a CSI or TBI index')
    conf = struct.unpack_from('<6i', raw, at)
    at += 24
    l_nm = i32()
    names_raw = raw[at:at + l_nm]
    at += l_nm
    # index_reader.py:22-30: a name is appended at each NUL (a trailing
    # unterminated name is dropped)
    names = [n.decode('latin-1') for n in names_raw.split(b'\0')[:-1]]
    n_ref = n_ref_tbi if magic == b'TBI\x01' else i32()
    refs = []
    for _ in range(n_ref):
        n_bin = i32()
        bins = []
        for _ in range(n_bin):
            (b,) = struct.unpack_from('<I', raw, at)
            at += 4
            if magic == b'CSI\x01':
                at += 8  # loffset
            n_chunk = i32()
            ch = struct.unpack_from(f'<{2 * n_chunk}Q', raw, at)
            at += 16 * n_chunk
            bins.append((b, list(zip(ch[0::2], ch[1::2]))))
        if magic == b'TBI\x01':
            n_intv = i32()
            at += 8 * n_intv
        refs.append(bins)
    return {'format': magic[:3].decode().lower(), 'min_shift': min_shift, 'depth': depth, 'bin_limit': bin_limit,
            'conf': conf, 'names': names, 'refs': refs}


def index_chunk_boundaries(data: bytes) -> dict:
    """get_chunk_boundaries (:90-104): per reference name, the sorted set of
    chunk begin/end virtual offsets of the bins below bin_limit (the
    pseudo-bins excluded)."""
    idx = read_index(data)
    lim = idx['bin_limit']
    return {name: sorted({off for b, chunks in bins if b < lim for c in chunks for off in c})
            for name, bins in zip(idx['names'], idx['refs'])}


def find_index(path):
    """get_vcf_index (:144-156): ``<path>.csi``, else ``<path>.tbi``, else None."""
    for suffix in ('.csi', '.tbi'):
        if path and os.path.exists(os.fspath(path) + suffix):
            with open(os.fspath(path) + suffix, 'rb') as f:
                return f.read()
    return None


def vcf_index(store, location):
    """The index summariseVcf reads for one VCF of the store: the one next
    to its source file, else the one the ingest writes for that file (kept
    in memory); None for a VCF ingested from text."""
    path = getattr(store, 'paths', {}).get(location)
    if path is None:
        return None
    cache = store.__dict__.setdefault('_index_cache', {})
    if location not in cache:
        data = find_index(path)
        if data is None:
            with open(path, 'rb') as f:
                bgzf = f.read(4) == b'\x1f\x8b\x08\x04'
            data = write_index(path) if bgzf else None
        cache[location] = data
    return cache[location]


def chunk_boundaries(store, location, stride=1, index=None) -> dict:
    """{contig: sorted chunk-boundary virtual offsets}: from the index
    (bytes, or 'auto' = vcf_index at stride 1) when there is one, else every
    stride-th record start (+ the contig end) from the store."""
    if isinstance(index, str) and index == 'auto':
        index = vcf_index(store, location) if stride == 1 else None
    if index is not None:
        return index_chunk_boundaries(index)
    out = {}
    for contig in store.contigs(location):
        b = store.chunk_boundaries(location, contig, stride)
        if b:
            out[contig] = b
    return out


def plan_slices(store, location, stride=1, index='auto'):
    """summarise_vcf (:253-267): the (virtual_start, virtual_end) slices."""
    return slices_from_boundaries(chunk_boundaries(store, location, stride, index))


def slices_from_boundaries(cb: dict):
    """summarise_vcf (:256-268) over get_chunk_boundaries' dict."""
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


def header_sample_count(head: bytes):
    """get_sample_count (:128-141) over the VCF's first bytes (the reference
    fetches bytes 0..first_chunk_start+65335): the tabs of the #CHROM line
    minus 8 (-1 for a header without FORMAT); ValueError at a data line
    before #CHROM; None when the bytes end first."""
    d = zlib.decompressobj(16 + zlib.MAX_WBITS)
    buf, rest = b'', head
    complete = True  # every gzip member of the bytes ended (else GzipFile hits EOFError at the cut)
    while rest:
        try:
            buf += d.decompress(rest)
        except zlib.error:
            complete = False
            break
        rest = d.unused_data
        if d.eof and rest:
            d = zlib.decompressobj(16 + zlib.MAX_WBITS)
        elif not d.eof:
            complete = False
            break
    lines = buf.split(b'\n')
    tail = lines.pop()  # after the last '\n': a line only when the stream ended cleanly
    if complete and tail:
        lines.append(tail)
    for line in lines:
        if not line.startswith(b'#'):
            raise ValueError('Incorrectly formatted file')
        if line.startswith(b'#CHROM'):
            return line.count(b'\t') - 8
    return None


def vcf_sample_count(path, first_chunk_start: int):
    with open(path, 'rb') as f:
        return header_sample_count(f.read(first_chunk_start + 65336))


def summarise_vcf(store, location, stride=1, index='auto'):
    """All slices of one VCF summarised on the device; returns
    (slices, per-slice RegionStats, the VCF's totals: variantCount,
    callCount and, for a VCF held as a file, sampleCount)."""
    cb = chunk_boundaries(store, location, stride, index)
    slices = slices_from_boundaries(cb)
    stats = store.summarise_slices([(location, a, b) for a, b in slices])
    tot = {'variantCount': 0, 'callCount': 0}
    for s in stats:
        if isinstance(s, Exception):
            raise s
        tot['variantCount'] += s['numVariants']
        tot['callCount'] += s['numCalls']
    path = getattr(store, 'paths', {}).get(location)
    if path is not None and cb:  # get_sample_count(location, first_chunk_start) (:256, :272)
        tot['sampleCount'] = vcf_sample_count(path, min(b[0] for b in cb.values()) >> 16)
    return slices, stats, tot
