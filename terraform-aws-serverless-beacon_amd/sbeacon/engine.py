"""Host-side engine: HBM variant stores and batched slice queries.

A :class:`Store` is the HBM-resident columnar image of one or more VCFs
(ingested once, replacing the per-slice ``bcftools query`` subprocess of
``lambda/performQuery/search_variants.py:42-50``).  :meth:`Store.query` takes
a list of ``PerformQueryPayload``-shaped dicts — what splitQuery would have
sent to N performQuery Lambdas — and answers all of them in one call into
``libsbeacon_hip.so``.

``registry`` maps ``vcf_location`` strings to stores so that the
reference-shaped handlers (``perform_query.py``, ``split_query.py``) can
resolve a payload's ``vcf_location`` exactly like the reference resolves it
to an S3 object.
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence
import os
from typing import Iterable

import numpy as np

from . import _lib
from ._lib import (BatchStats, BuildOpts, DedupJob, DedupStats, Query, ResultView, Slice, SliceStats, StoreInfo,
                   check, lib)
from .payloads import PerformQueryResponse

QERR = {1: UnboundLocalError, 2: IndexError, 3: ValueError, 4: AttributeError, 9: NotImplementedError}
assert 10 not in QERR  # SB_QERR_GENERAL is internal to the library (general_slice_kernel resolves it)
QERR_MSG = {
    1: "local variable 'variant_type' referenced before assignment",
    2: 'list index out of range',
    3: 'invalid literal for int() with base 10',
    4: "'NoneType' object has no attribute 'replace'",
    9: 'referenceBases contains regex metacharacters (outside the restated contract)',
}


def _b(s):
    return None if s is None else (s if isinstance(s, bytes) else str(s).encode())


_QUERY_FIELDS = ['vcf_id', 'region', 'region_len', 'end_min', 'end_max', 'reference_bases', 'reference_len',
                 'alternate_bases', 'alternate_len', 'variant_type', 'variant_type_len', 'variant_min_length',
                 'variant_max_length', 'granularity', 'include_details', 'include_samples', 'selected_samples_only',
                 'strict_variant_type', 'sample_names', 'sample_names_len']
_QUERY_FORMATS = ['u4', 'u8', 'u8', 'i8', 'i8', 'u8', 'u8', 'u8', 'u8', 'u8', 'u8', 'i8', 'i8',
                  'u1', 'u1', 'u1', 'u1', 'u1', 'u8', 'u8']
_QUERY_DTYPE = None


def _query_dtype():
    global _QUERY_DTYPE
    if _QUERY_DTYPE is None:
        _QUERY_DTYPE = np.dtype({'names': _QUERY_FIELDS, 'formats': _QUERY_FORMATS,
                                 'offsets': [getattr(Query, f).offset for f in _QUERY_FIELDS],
                                 'itemsize': C.sizeof(Query)})
    return _QUERY_DTYPE


def queries_from_payloads(payloads: list[dict], vcf_id, *, strict_variant_type: bool = False):
    """PerformQueryPayload dicts -> (ctypes Query array, keep-alive list);
    vcf_id(location) -> the store's vcf id.  Column-wise: every string goes
    into one pooled buffer (repeated values stored once) and the fields are
    filled through a numpy view of the array, so a batch of 10^5 payloads
    costs list comprehensions, not 10^6 ctypes attribute stores."""
    n = len(payloads)
    arr = (Query * max(n, 1))()
    if n == 0:
        return arr, []
    vid_cache = {}

    def vid_of(loc):
        v = vid_cache.get(loc)
        if v is None:
            v = vid_cache[loc] = vcf_id(loc)
        return v

    pts = [p.get('passthrough', {}) for p in payloads]
    for pt in pts:  # the reference calls payload.passthrough.get(...) (search_variants.py:37)
        if not isinstance(pt, dict):
            raise AttributeError(f"'{type(pt).__name__}' object has no attribute 'get'")
    em = [p.get('end_min') for p in payloads]
    ex = [p.get('end_max') for p in payloads]
    if any(x is None for x in em) or any(x is None for x in ex):
        raise TypeError("'<=' not supported between instances of 'NoneType' and 'int'")
    # pooled strings (NUL-terminated, as the bytes objects ctypes would
    # pass): offset (-1 = NULL) and length per payload; a column of few
    # distinct values (REF / ALT / variantType) stores each value once
    pool = bytearray()

    def col(vals):
        strs = [v for v in vals if v is not None]
        if len(strs) == len(vals) and all(type(v) is str for v in vals):
            joined = '\0'.join(vals)
            if joined.isascii() and len(set(vals)) * 4 > len(vals):  # mostly unique (regions): one join
                ln = np.fromiter((len(v) for v in vals), dtype=np.uint64, count=len(vals))
                off = len(pool) + np.concatenate([[0], np.cumsum(ln[:-1] + 1)]).astype(np.int64)
                pool.extend(joined.encode())
                pool.append(0)
                return off, ln
        at = {}
        for v in set(strs):
            bv = _b(v)
            at[v] = (len(pool), len(bv))
            pool.extend(bv)
            pool.append(0)
        off = np.array([at[v][0] if v is not None else -1 for v in vals], dtype=np.int64)
        ln = np.array([at[v][1] if v is not None else 0 for v in vals], dtype=np.uint64)
        return off, ln

    names = [pt.get('sampleNames', None) for pt in pts]
    cols = {
        'region': col([p['region'] for p in payloads]),
        'reference_bases': col([p.get('reference_bases') for p in payloads]),
        'alternate_bases': col([p.get('alternate_bases') for p in payloads]),
        'variant_type': col([p.get('variant_type') for p in payloads]),
        'sample_names': col([','.join(x) if x is not None else None for x in names]),
    }
    buf = C.create_string_buffer(bytes(pool), max(len(pool), 1))
    base = C.addressof(buf)
    v = np.frombuffer((C.c_char * (C.sizeof(Query) * n)).from_address(C.addressof(arr)), dtype=_query_dtype())
    lens = {'region': 'region_len', 'reference_bases': 'reference_len', 'alternate_bases': 'alternate_len',
            'variant_type': 'variant_type_len', 'sample_names': 'sample_names_len'}
    for f, (off, ln) in cols.items():
        v[f] = np.where(off >= 0, base + np.maximum(off, 0), 0).astype(np.uint64)
        v[lens[f]] = ln
    v['vcf_id'] = [vid_of(p['vcf_location']) for p in payloads]
    v['end_min'] = [int(x) for x in em]
    v['end_max'] = [int(x) for x in ex]
    v['variant_min_length'] = [int(p['variant_min_length']) for p in payloads]
    v['variant_max_length'] = [int(p['variant_max_length']) for p in payloads]
    v['granularity'] = [_lib.SB_GRAN.get(p.get('requested_granularity'), 255) for p in payloads]
    v['include_details'] = [1 if p.get('include_details') else 0 for p in payloads]
    v['include_samples'] = [1 if pt.get('includeSamples', False) else 0 for pt in pts]
    v['selected_samples_only'] = [1 if pt.get('selectedSamplesOnly', False) else 0 for pt in pts]
    v['strict_variant_type'] = 1 if strict_variant_type else 0
    return arr, [buf]


class StaleStore(Exception):
    """A persisted store whose source VCFs changed since it was saved."""

    def __init__(self, paths):
        super().__init__('stale store: ' + ', '.join(paths))
        self.paths = list(paths)


class Store:
    """An immutable HBM store built from VCF files or text."""

    def __init__(self, handle, locations, paths=None):
        self._h = handle
        self.locations = list(locations)
        self.paths = dict(paths or {})  # location -> source file (summariseVcf looks for its index there)

    # ---------------------------------------------------------------- build
    @classmethod
    def build(cls, sources, *, device: int = 0, keep_genotypes: bool = True, n_threads: int = 0):
        """``sources``: iterable of ``(vcf_location, path_or_text)``; a value
        that is an existing path is read (plain or gzip), otherwise it is
        VCF text (``str``/``bytes``) or an iterable of text chunks.  A
        3-tuple ``(vcf_location, source, (sample_names, planes))`` attaches a
        carrier bit-matrix to a sites-only VCF (``planes``: uint64
        ``[alt rows, ceil(n/64)]``, record-then-ALT order; sb_builder_attach_carriers)."""
        L = lib()
        b = C.c_void_p()
        opts = BuildOpts(1 if keep_genotypes else 0, int(n_threads))
        check(L.sb_builder_new(C.byref(opts), C.byref(b)))
        locs = []
        paths = {}
        try:
            for item in sources:
                loc, src = item[0], item[1]
                carriers = item[2] if len(item) > 2 else None
                vid = C.c_uint32()
                lb = _b(loc)
                check(L.sb_builder_begin_vcf(b, lb, len(lb), C.byref(vid)))
                locs.append(loc)
                if isinstance(src, (str, os.PathLike)) and os.path.exists(src):
                    check(L.sb_builder_add_file(b, vid.value, os.fsencode(src)))
                    paths[loc] = os.fspath(src)
                elif isinstance(src, (str, bytes)):
                    t = _b(src)
                    check(L.sb_builder_add_text(b, vid.value, t, len(t)))
                else:
                    for chunk in src:
                        t = _b(chunk)
                        check(L.sb_builder_add_text(b, vid.value, t, len(t)))
                if carriers is not None:
                    names, planes = carriers[0], carriers[1]
                    if isinstance(carriers, list):
                        carriers.clear()  # a list hands over the only reference: freed after the copy
                    nb = [_b(n) for n in names]
                    arr = (C.c_char_p * len(nb))(*nb)
                    lens = (C.c_uint32 * len(nb))(*[len(x) for x in nb])
                    planes = np.ascontiguousarray(planes, dtype=np.uint64)
                    if planes.ndim != 2 or planes.shape[1] != (len(nb) + 63) // 64:
                        raise ValueError('carrier planes must be [alt rows, ceil(n_samples / 64)] uint64')
                    check(L.sb_builder_attach_carriers(b, vid.value, arr, lens, len(nb), planes.ctypes.data,
                                                       planes.shape[0]))
                    del planes
            s = C.c_void_p()
            check(L.sb_builder_finish(b, int(device), C.byref(s)))
        finally:
            L.sb_builder_free(b)
        return cls(s, locs, paths)

    def trim(self):
        """Free the buffers cached for request batches (sb_store_trim)."""
        check(lib().sb_store_trim(self._h))

    # ---------------------------------------------------------------- persist
    def save(self, directory: str):
        """Write the store to ``directory`` (sb_store_save) with a sidecar of
        its locations and source paths."""
        import json
        check(lib().sb_store_save(self._h, os.fsencode(directory)))
        with open(os.path.join(directory, 'sbeacon.json'), 'w') as f:
            json.dump({'locations': self.locations, 'paths': self.paths}, f)

    @classmethod
    def open(cls, directory: str, *, device: int = 0):
        """Re-create a saved store (sb_store_open) without re-reading any VCF.
        Raises StaleStore (listing the changed source files) when a source
        changed since the save."""
        import json
        s = C.c_void_p()
        rc = lib().sb_store_open(os.fsencode(directory), int(device), C.byref(s))
        if rc == _lib.SB_ESTALE:
            raise StaleStore(lib().sb_last_error().decode().split('\n'))
        check(rc)
        with open(os.path.join(directory, 'sbeacon.json')) as f:
            meta = json.load(f)
        return cls(s, meta['locations'], meta['paths'])

    def candidates(self) -> tuple[int, int]:
        """(variantType candidates, bytes of their VcQ words + record ids):
        the request pass's working set (sb_store_candidates)."""
        n, b = C.c_uint64(), C.c_uint64()
        _lib.check(_lib.lib().sb_store_candidates(self.handle, C.byref(n), C.byref(b)))
        return n.value, b.value

    def close(self):
        if self._h:
            lib().sb_store_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        i = StoreInfo()
        check(lib().sb_store_get_info(self._h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in StoreInfo._fields_}

    def vcf_id(self, location: str) -> int:
        v = C.c_uint32()
        lb = _b(location)
        check(lib().sb_store_find_vcf(self._h, lb, len(lb), C.byref(v)))
        return v.value

    def sample_names(self, location: str) -> list[str]:
        vid = self.vcf_id(location)
        n = C.c_uint32()
        check(lib().sb_store_n_samples(self._h, vid, C.byref(n)))
        out = []
        p = C.c_char_p()
        ln = C.c_size_t()
        for i in range(n.value):
            check(lib().sb_store_sample_name(self._h, vid, i, C.byref(p), C.byref(ln)))
            out.append(C.string_at(p, ln.value).decode())
        return out

    # ---------------------------------------------------------------- summarise
    def summarise_slices(self, slices, *, with_timing=False):
        """slices: iterable of (vcf_location, virtual_start, virtual_end).
        Returns one RegionStats dict {numVariants, numCalls, records} per
        slice (or the exception for a slice the engine cannot represent)."""
        slices = list(slices)
        n = len(slices)
        arr = (Slice * max(n, 1))()
        for i, (loc, vs, ve) in enumerate(slices):
            arr[i].vcf_id = self.vcf_id(loc)
            arr[i].virtual_start = int(vs)
            arr[i].virtual_end = int(ve)
        out = (SliceStats * max(n, 1))()
        ms = C.c_double()
        check(lib().sb_summarise_slices(self._h, arr, n, out, C.byref(ms)))
        res = []
        for i in range(n):
            if out[i].error:
                res.append(NotImplementedError(f'slice {slices[i]} is not record-aligned / not representable'))
            else:
                res.append({'numVariants': out[i].num_variants, 'numCalls': out[i].num_calls,
                             'records': out[i].records})
        return (res, ms.value) if with_timing else res

    def region_files(self, slices, *, with_data=False):
        """summariseSlice's region files of each slice (write_data_to_s3.h):
        per slice a list of {contig, first_pos, last_pos, bytes, entries}
        dicts (+ 'data': the file's bytes -- uncompressed with
        ``with_data=True``, the reference's gzip members with
        ``with_data='gzip'``), or the exception for a slice the reference
        throws on."""
        slices = list(slices)
        n = len(slices)
        arr = (Slice * max(n, 1))()
        for i, (loc, vs, ve) in enumerate(slices):
            arr[i].vcf_id = self.vcf_id(loc)
            arr[i].virtual_start = int(vs)
            arr[i].virtual_end = int(ve)
        status = (C.c_int32 * max(n, 1))()
        h = C.c_void_p()
        mode = 2 if with_data == 'gzip' else (1 if with_data else 0)
        check(lib().sb_slice_region_files(self._h, arr, n, mode, status, C.byref(h)))
        try:
            fp = C.POINTER(_lib.RegionFile)()
            nf = C.c_size_t()
            dp = C.c_void_p()
            dl = C.c_size_t()
            check(lib().sb_region_files_get(h, C.byref(fp), C.byref(nf), C.byref(dp), C.byref(dl)))
            data = C.string_at(dp, dl.value) if mode and dl.value else b''
            contig_names = {}
            out = [[] for _ in range(n)]
            off = 0
            for k in range(nf.value):
                f = fp[k]
                loc = slices[f.slice][0]
                if loc not in contig_names:
                    contig_names[loc] = self.contigs(loc)
                d = {'contig': contig_names[loc][f.contig], 'first_pos': f.first_pos, 'last_pos': f.last_pos,
                     'bytes': f.bytes, 'entries': f.entries}
                if mode:
                    d['data'] = data[off:off + f.data_bytes]
                    off += f.data_bytes
                out[f.slice].append(d)
        finally:
            lib().sb_region_files_free(h)
        return [NotImplementedError(f'slice {slices[i]}: the reference summariseSlice throws / slice not record-'
                                    'aligned') if status[i] else out[i] for i in range(n)]

    def dedup_counts(self, jobs, *, with_stats=False):
        """jobs: iterable of (vcf_locations, contig, range_start, range_end).
        Returns the unique region-key count per job (duplicateVariantSearch's
        |uniqueVariants|), or a NotImplementedError for a job whose range
        holds a record the reference's summariseSlice throws on."""
        jobs = list(jobs)
        n = len(jobs)
        arr = (DedupJob * max(n, 1))()
        keep = []
        for i, (locs, contig, rs, re_) in enumerate(jobs):
            ids = (C.c_uint32 * max(len(locs), 1))(*[self.vcf_id(l) for l in locs])
            cb = _b(contig)
            keep.append((ids, cb))
            arr[i].vcf_ids = ids
            arr[i].n_vcf = len(locs)
            arr[i].contig = cb
            arr[i].contig_len = len(cb)
            arr[i].range_start = int(rs)
            arr[i].range_end = int(re_)
        uniq = (C.c_uint64 * max(n, 1))()
        status = (C.c_int32 * max(n, 1))()
        st = DedupStats()
        check(lib().sb_dedup_count(self._h, arr, n, uniq, status, C.byref(st)))
        res = [NotImplementedError(f'dedup job {jobs[i][1:]}: a record in range has an allele compressSeq '
                                   'rejects (the reference summariseSlice throws)') if status[i] else uniq[i]
               for i in range(n)]
        if with_stats:
            return res, {'keys': st.keys, 'collisions': st.collisions, 'device_ms': st.device_ms,
                         'path': _lib.DEDUP_PATHS[st.path], 'windows': st.windows}
        return res

    def dedup_counts_files(self, jobs, *, with_stats=False):
        """Reference-exact duplicateVariantSearch (sb_dedup_count_files).
        jobs: iterable of (files, range_start, range_end), files = list of
        (vcf_location, virtual_start, virtual_end, file index) naming region
        files by the summariseSlice slice that wrote them.  Returns the unique
        count per job, or the exception the reference raises (RuntimeError:
        its getVcfData throws; NotImplementedError: its summariseSlice throws)."""
        jobs = list(jobs)
        n = len(jobs)
        arr = (_lib.DedupFileJob * max(n, 1))()
        keep = []
        for i, (files, rs, re_) in enumerate(jobs):
            fa = (_lib.RegionRef * max(len(files), 1))()
            for k, (loc, vs, ve, fi) in enumerate(files):
                fa[k].vcf_id = self.vcf_id(loc)
                fa[k].file = int(fi)
                fa[k].virtual_start = int(vs)
                fa[k].virtual_end = int(ve)
            keep.append(fa)
            arr[i].files = fa
            arr[i].n_files = len(files)
            arr[i].range_start = int(rs)
            arr[i].range_end = int(re_)
        uniq = (C.c_uint64 * max(n, 1))()
        status = (C.c_int32 * max(n, 1))()
        st = DedupStats()
        check(lib().sb_dedup_count_files(self._h, arr, n, uniq, status, C.byref(st)))
        res = []
        for i in range(n):
            if status[i] == 5:
                res.append(RuntimeError('Invalid File Read (the reference getVcfData throws)'))
            elif status[i]:
                res.append(NotImplementedError('a region file of this job comes from a slice the reference '
                                               'summariseSlice throws on'))
            else:
                res.append(uniq[i])
        if with_stats:
            return res, {'keys': st.keys, 'collisions': st.collisions, 'device_ms': st.device_ms,
                         'path': _lib.DEDUP_PATHS[st.path], 'windows': st.windows}
        return res

    def contigs(self, location) -> list[str]:
        vid = self.vcf_id(location)
        n = C.c_uint32()
        check(lib().sb_store_n_contigs(self._h, vid, C.byref(n)))
        out = []
        p = C.c_char_p()
        ln = C.c_size_t()
        for i in range(n.value):
            check(lib().sb_store_contig_name(self._h, vid, i, C.byref(p), C.byref(ln)))
            out.append(C.string_at(p, ln.value).decode())
        return out

    def chunk_boundaries(self, location, contig, stride=1):
        """Record-start virtual offsets of one contig (+ its end), the
        stand-in for a CSI/TBI index's chunk boundaries."""
        vid = self.vcf_id(location)
        cb = _b(contig)
        n = C.c_size_t()
        check(lib().sb_store_chunk_boundaries(self._h, vid, cb, len(cb), stride, None, 0, C.byref(n)))
        arr = (C.c_uint64 * max(n.value, 1))()
        check(lib().sb_store_chunk_boundaries(self._h, vid, cb, len(cb), stride, arr, n.value, C.byref(n)))
        return list(arr[:n.value])

    def vcf_stream(self, location):
        nb, ln = C.c_uint64(), C.c_uint64()
        check(lib().sb_store_vcf_stream(self._h, self.vcf_id(location), C.byref(nb), C.byref(ln)))
        return {'blocks': nb.value, 'stream_len': ln.value}

    # ---------------------------------------------------------------- query
    def make_queries(self, payloads: list[dict], *, strict_variant_type: bool = False):
        """PerformQueryPayload dicts -> (ctypes Query array, keep-alive list)."""
        return queries_from_payloads(payloads, self.vcf_id, strict_variant_type=strict_variant_type)

    def query(self, payloads: list[dict], *, strict_variant_type: bool = False) -> 'ResultSet':
        arr, keep = self.make_queries(payloads, strict_variant_type=strict_variant_type)
        r = C.c_void_p()
        check(lib().sb_query_batch(self._h, arr, len(payloads), 0, C.byref(r)))
        del keep
        return ResultSet(r, payloads, self)

    def prepare(self, payloads: list[dict], *, strict_variant_type: bool = False) -> 'Batch':
        arr, keep = self.make_queries(payloads, strict_variant_type=strict_variant_type)
        b = C.c_void_p()
        check(lib().sb_batch_prepare(self._h, arr, len(payloads), C.byref(b)))
        del keep
        return Batch(b, payloads, self)


class Batch:
    """A device-resident query batch (inputs stay in HBM across runs)."""

    def __init__(self, handle, payloads, store):
        self._h = handle
        self.payloads = payloads
        self.store = store

    def run(self):
        check(lib().sb_batch_run(self._h))

    def sync(self):
        check(lib().sb_batch_sync(self._h))

    def timing(self):
        t, s, b = C.c_double(), C.c_double(), C.c_double()
        check(lib().sb_batch_last_timing(self._h, C.byref(t), C.byref(s), C.byref(b)))
        return {'total_ms': t.value, 'scan_ms': s.value, 'bounds_ms': b.value}

    def set_owners(self, owner, n_rows: int):
        """Query i belongs to request row owner[i] (non-decreasing)."""
        import numpy as np
        o = np.ascontiguousarray(owner, dtype=np.uint32)
        check(lib().sb_batch_set_owners(self._h, o.ctypes.data_as(C.POINTER(C.c_uint32)), len(o), int(n_rows)))

    def reduce_requests(self, dev_ptr: int):
        """Enqueue the per-request reduction into dev_ptr (n_rows x 5 int64
        on the store's device: exists, n_variants, call_count,
        all_alleles_count, errors)."""
        check(lib().sb_batch_reduce_requests(self._h, C.c_void_p(dev_ptr)))

    def compact_hits(self, hits_ptr: int, row_off_ptr: int, rec_base: int = 0, rows_ptr: int = 0):
        """Enqueue the rows' dense hit lists (sb_batch_compact_hits): hits
        (capacity ``stats()['hits']`` u64 on the device) and n_rows + 1 row
        offsets; records numbered from ``rec_base``; ``rows_ptr`` = this run's
        reduce_requests output (optional)."""
        check(lib().sb_batch_compact_hits(self._h, C.c_void_p(rows_ptr) if rows_ptr else None, C.c_void_p(hits_ptr),
                                          C.c_void_p(row_off_ptr), int(rec_base)))

    def set_stream(self, stream_ptr):
        """Run this batch's work on a caller stream (e.g.
        ``torch.cuda.current_stream().cuda_stream``); None = the store's."""
        check(lib().sb_batch_set_stream(self._h, _lib.stream_arg(stream_ptr)))

    def deliver(self, rows_ptr, hits_ptr, row_off_ptr, rec_base=0):
        """reduce_requests(rows_ptr) + compact_hits(hits_ptr, row_off_ptr,
        rec_base, rows_ptr) in one call (sb_batch_deliver)."""
        check(lib().sb_batch_deliver(self._h, C.c_void_p(rows_ptr), C.c_void_p(hits_ptr), C.c_void_p(row_off_ptr),
                                     int(rec_base)))

    def set_slice_results(self, on: bool):
        """Per-slice results of chained slices on (default) / off: off keeps
        only the request rows and hit lists (needs set_owners with every
        chain in one row); fetch() then needs a run with them on."""
        check(lib().sb_batch_set_slice_results(self._h, 1 if on else 0))

    def stats(self) -> dict:
        """Planning statistics (hits = the planned hit capacity)."""
        s = BatchStats()
        check(lib().sb_batch_get_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in BatchStats._fields_}

    def fetch(self) -> 'ResultSet':
        r = C.c_void_p()
        check(lib().sb_batch_fetch(self._h, C.byref(r)))
        return ResultSet(r, self.payloads, self.store)

    def free(self):
        if self._h:
            lib().sb_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class LazyVariants(Sequence):
    """A response's variant strings, formatted by the library on first use."""

    def __init__(self, rs, i, n):
        self._rs, self._i, self._n, self._v = rs, i, n, None

    def _load(self):
        if self._v is None:
            t = self._rs._text(lib().sb_result_variants_text, self._i)
            self._v = t.split('\n') if self._n else []
        return self._v

    def __len__(self):
        return self._n

    def __getitem__(self, k):
        return self._load()[k]

    def __iter__(self):
        return iter(self._load())

    def __eq__(self, other):
        return list(self._load()) == list(other)

    def __repr__(self):
        return repr(self._load())


class ResultSet:
    def __init__(self, handle, payloads, store):
        self._h = handle
        self.payloads = payloads
        self.store = store

    def __len__(self):
        return len(self.payloads)

    def __del__(self):
        try:
            if self._h:
                lib().sb_result_free(self._h)
                self._h = None
        except Exception:
            pass

    def stats(self) -> dict:
        s = BatchStats()
        check(lib().sb_result_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in BatchStats._fields_}

    def view(self, i: int) -> ResultView:
        v = ResultView()
        check(lib().sb_result_get(self._h, i, C.byref(v)))
        return v

    def hits(self, i: int):
        v = self.view(i)
        return [(v.hit_record[k], v.hit_alt[k]) for k in range(v.n_variants)]

    def _text(self, fn, i):
        p = C.c_void_p()
        n = C.c_size_t()
        check(fn(self._h, i, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value).decode() if n.value else ''

    def distinct_variants(self, indices) -> list[str]:
        """The distinct variant strings of the listed queries, first-seen
        order (sb_result_distinct_variants: the route aggregation)."""
        idx = np.ascontiguousarray(np.asarray(list(indices), dtype=np.uint32))
        p, n, cnt = C.c_void_p(), C.c_size_t(), C.c_uint64()
        check(lib().sb_result_distinct_variants(self._h, idx.ctypes.data_as(C.POINTER(C.c_uint32)), idx.size,
                                                C.byref(p), C.byref(n), C.byref(cnt)))
        return C.string_at(p, n.value).decode().split('\n') if cnt.value else []

    def response(self, i: int, *, lazy_variants: bool = False) -> PerformQueryResponse:
        """The reference PerformQueryResponse for query i, or raise the
        exception the reference would raise (search_variants.py:262-271).
        lazy_variants: the variant strings are formatted on first use (the
        routes aggregate them in the library instead)."""
        p = self.payloads[i]
        v = self.view(i)
        if v.error:
            raise QERR.get(v.error, RuntimeError)(QERR_MSG.get(v.error, 'error'))
        pt = p.get('passthrough') or {}
        samples_variant = bool(pt.get('selectedSamplesOnly', False))
        include_samples = bool(pt.get('includeSamples', False))
        if lazy_variants:
            variants = LazyVariants(self, i, int(v.n_variants))
        else:
            vt = self._text(lib().sb_result_variants_text, i)
            variants = vt.split('\n') if v.n_variants else []
        names_t = self._text(lib().sb_result_sample_names_text, i)
        names = names_t.split(',') if v.n_sample_indices else []
        if samples_variant:
            sample_indices = [v.sample_indices[k] for k in range(v.n_sample_indices)]
            sample_names = names
        else:
            sample_indices = []
            sample_names = names if include_samples else []
        cc, an = _lib.view_counts(v)
        r = PerformQueryResponse(
            exists=bool(v.exists), dataset_id=p.get('dataset_id'), vcf_location=p.get('vcf_location'),
            all_alleles_count=an, variants=variants, call_count=cc,
            sample_indices=sample_indices, sample_names=sample_names)
        r._src = (self, i)
        return r

    def responses(self, *, lazy_variants: bool = False) -> list:
        """All responses; an entry is the exception instance where the
        reference would have raised.  The views of every query come from one
        library call (sb_result_get_all); the per-query text calls happen only
        where there is text (variants when not lazy, sample names)."""
        n = len(self.payloads)
        if n == 0:
            return []
        views = (ResultView * n)()
        check(lib().sb_result_get_all(self._h, views, n))
        out = []
        vtext, ntext = lib().sb_result_variants_text, lib().sb_result_sample_names_text
        for i, (p, v) in enumerate(zip(self.payloads, views)):
            if v.error:
                e = QERR.get(v.error, RuntimeError)(QERR_MSG.get(v.error, 'error'))
                if not isinstance(e, (UnboundLocalError, IndexError, ValueError, AttributeError, NotImplementedError)):
                    raise e
                out.append(e)
                continue
            pt = p.get('passthrough') or {}
            nv, ns = int(v.n_variants), int(v.n_sample_indices)
            if lazy_variants:
                variants = LazyVariants(self, i, nv)
            else:
                variants = self._text(vtext, i).split('\n') if nv else []
            names = self._text(ntext, i).split(',') if ns else []
            if pt.get('selectedSamplesOnly', False):
                sample_indices = v.sample_indices[:ns] if ns else []
                sample_names = names
            else:
                sample_indices = []
                sample_names = names if pt.get('includeSamples', False) else []
            cc, an = _lib.view_counts(v)
            r = PerformQueryResponse(
                exists=bool(v.exists), dataset_id=p.get('dataset_id'), vcf_location=p.get('vcf_location'),
                all_alleles_count=an, variants=variants, call_count=cc,
                sample_indices=sample_indices, sample_names=sample_names)
            r._src = (self, i)
            out.append(r)
        return out


# ------------------------------------------------------------------ registry
class Registry:
    """vcf_location -> Store (the analogue of the S3 objects the reference reads)."""

    def __init__(self):
        self._by_loc: dict[str, Store] = {}

    def register(self, store: Store):
        for loc in store.locations:
            self._by_loc[loc] = store

    def store_for(self, location: str) -> Store:
        try:
            return self._by_loc[location]
        except KeyError:
            raise KeyError(f'no HBM store holds vcf_location {location!r}') from None

    def clear(self):
        self._by_loc.clear()

    def locations(self) -> list[str]:
        return list(self._by_loc)

    def group(self, payloads: Iterable[dict]):
        """Split payloads by store, preserving order inside each group."""
        groups: dict[int, tuple[Store, list[int]]] = {}
        for i, p in enumerate(payloads):
            s = self.store_for(p['vcf_location'])
            groups.setdefault(id(s), (s, []))[1].append(i)
        return list(groups.values())


registry = Registry()


def query_payloads(payloads: list[dict], *, strict_variant_type: bool = False, lazy_variants: bool = False) -> list:
    """Answer PerformQueryPayload dicts through the registry in as few
    device batches as there are stores.  Returns responses/exceptions in
    payload order."""
    out = [None] * len(payloads)
    for store, idx in registry.group(payloads):
        sub = [payloads[i] for i in idx]
        rs = store.query(sub, strict_variant_type=strict_variant_type)
        for j, r in zip(idx, rs.responses(lazy_variants=lazy_variants)):
            out[j] = r
    return out
