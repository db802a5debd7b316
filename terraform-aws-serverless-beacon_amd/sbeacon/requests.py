"""Request batches: the splitQuery fan-out inside the library.

One *request* is one ``SplitQueryPayload``
(``shared_resources/payloads/lambda_payloads.py:8-44``) restricted to one of
its ``vcf_locations`` -- what ``split_query_sync``
(``lambda/splitQuery/lambda_function.py:74-110``) would cut into 10 kb
``PerformQueryPayload`` slices.  ``sb_requests_prepare`` takes the requests
as a columnar array (no per-slice payload objects, no region strings) and
``sb_requests_prepare_columns`` takes the same requests as numpy-backed
columns (``request_columns``: no per-request struct, string columns as
dictionary codes); ``sb_requests_run`` answers all of them on the device, leaving one row per
request -- the route-level sums of its slices' responses
(``route_g_variants.py:144-171``: exists count, variants, call_count,
all_alleles_count, errors) -- and the rows' hit lists densely in request
order.  ``requests_array`` builds the ``sb_request`` array from numpy
columns; string columns are small dictionaries of distinct values plus a
code per request.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import Request, check, lib

_FIELDS = [f for f, _ in Request._fields_ if f != '_pad']
COMPACT_ALL, COMPACT_HITS = 1, 2  # sb_requests_set_compact modes (include/sbeacon.h)


def request_dtype() -> np.dtype:
    """numpy view of one sb_request (the C layout, padding kept)."""
    fmt = {C.c_uint32: 'u4', C.c_int64: 'i8', C.c_char_p: 'u8', C.c_size_t: 'u8', C.c_uint8: 'u1'}
    names, formats, offsets = [], [], []
    for f, t in Request._fields_:
        if f == '_pad':
            continue
        names.append(f)
        formats.append(fmt[t])
        offsets.append(getattr(Request, f).offset)
    return np.dtype({'names': names, 'formats': formats, 'offsets': offsets, 'itemsize': C.sizeof(Request)})


class _Pool:
    """Distinct strings in one ctypes buffer: value -> (address, length)."""

    def __init__(self):
        self.bufs = []

    def column(self, values: Sequence, codes, n: int):
        """values: distinct strings (None = NULL); codes: index per request
        (scalar = the same for all).  Returns (address array, length array)."""
        addr = np.zeros(len(values), dtype=np.uint64)
        ln = np.zeros(len(values), dtype=np.uint64)
        for k, v in enumerate(values):
            if v is None:
                continue
            b = v.encode() if isinstance(v, str) else bytes(v)
            buf = C.create_string_buffer(b, len(b) + 1)
            self.bufs.append(buf)
            addr[k] = C.addressof(buf)
            ln[k] = len(b)
        codes = np.broadcast_to(np.asarray(codes, dtype=np.int64), (n,))
        return addr[codes], ln[codes]


def requests_array(n: int, *, vcf_id, contig, start_min, start_max, end_min, end_max,
                   reference=('N',), reference_code=0, alternate=(None,), alternate_code=0,
                   variant_type=(None,), variant_type_code=0, variant_min_length=0, variant_max_length=-1,
                   granularity='record', include_details=True, include_samples=False,
                   selected_samples_only=False, strict_variant_type=False, sample_names=(None,),
                   sample_names_code=0):
    """sb_request array of n requests from columns (scalars broadcast).
    Returns (ctypes array, keep-alive)."""
    arr = (Request * max(n, 1))()
    keep = _Pool()
    if n == 0:
        return arr, keep
    v = np.frombuffer((C.c_char * (C.sizeof(Request) * n)).from_address(C.addressof(arr)), dtype=request_dtype())
    v['vcf_id'] = vcf_id
    v['contig'] = contig
    v['start_min'] = start_min
    v['start_max'] = start_max
    v['end_min'] = end_min
    v['end_max'] = end_max
    for f, vals, codes in (('reference_bases', reference, reference_code),
                           ('alternate_bases', alternate, alternate_code),
                           ('variant_type', variant_type, variant_type_code),
                           ('sample_names', sample_names, sample_names_code)):
        a, ln = keep.column(vals, codes, n)
        v[f] = a
        v[{'reference_bases': 'reference_len', 'alternate_bases': 'alternate_len',
           'variant_type': 'variant_type_len', 'sample_names': 'sample_names_len'}[f]] = ln
    v['variant_min_length'] = variant_min_length
    v['variant_max_length'] = variant_max_length
    g = granularity
    v['granularity'] = _lib.SB_GRAN[g] if isinstance(g, str) else g
    v['include_details'] = np.asarray(include_details, dtype=np.uint8)
    v['include_samples'] = np.asarray(include_samples, dtype=np.uint8)
    v['selected_samples_only'] = np.asarray(selected_samples_only, dtype=np.uint8)
    v['strict_variant_type'] = np.asarray(strict_variant_type, dtype=np.uint8)
    arr._keep = keep  # the buffers its pointers name live as long as it does
    return arr, keep


def request_columns(n: int, *, vcf_id, contig, start_min, start_max, end_min, end_max,
                    reference=('N',), reference_code=None, alternate=(None,), alternate_code=None,
                    variant_type=(None,), variant_type_code=None, variant_min_length=0, variant_max_length=-1,
                    granularity='record', include_details=True, include_samples=False,
                    selected_samples_only=False, strict_variant_type=False, sample_names=(None,),
                    sample_names_code=None):
    """sb_request_columns over numpy columns (no per-request struct): a
    scalar gives every request that value; string columns are the distinct
    values plus a code per request (None = every request takes values[0]).
    Returns (RequestColumns, keep-alive)."""
    c = _lib.RequestColumns()
    keep = [c]

    def arr(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        keep.append(a)
        return a.ctypes.data

    def num(field, x, dt):
        if np.ndim(x) == 0:
            setattr(c, field + '_all', int(x))
        else:
            if len(x) != n:
                raise ValueError(f'{field}: {len(x)} values for {n} requests')
            setattr(c, field, arr(x, dt))

    for f, x, dt in (('vcf_id', vcf_id, np.uint32), ('contig', contig, np.uint32), ('end_min', end_min, np.int64),
                     ('end_max', end_max, np.int64), ('variant_min_length', variant_min_length, np.int64),
                     ('variant_max_length', variant_max_length, np.int64)):
        num(f, x, dt)
    for f, x in (('start_min', start_min), ('start_max', start_max)):
        x = np.broadcast_to(np.asarray(x, dtype=np.int64), (n,))
        setattr(c, f, arr(x, np.int64))
    g = granularity
    if isinstance(g, str):
        g = _lib.SB_GRAN[g]
    for f, x in (('granularity', g), ('include_details', include_details), ('include_samples', include_samples),
                 ('selected_samples_only', selected_samples_only)):
        if np.ndim(x) == 0:
            setattr(c, f + '_all', int(x))
        else:
            setattr(c, f, arr(x, np.uint8))
    c.strict_variant_type = 1 if strict_variant_type else 0
    for f, short, vals, codes in (('reference', 'reference', reference, reference_code),
                                  ('alternate', 'alternate', alternate, alternate_code),
                                  ('variant_type', 'variant_type', variant_type, variant_type_code),
                                  ('sample_names', 'sample_names', sample_names, sample_names_code)):
        vals = list(vals)
        if all(v is None for v in vals):
            continue  # None for every request
        d = (_lib.Str * len(vals))()
        for k, v in enumerate(vals):
            if v is None:
                continue
            b = v.encode() if isinstance(v, str) else bytes(v)
            buf = C.create_string_buffer(b, len(b) + 1)
            keep.append(buf)
            d[k].p = C.addressof(buf)
            d[k].len = len(b)
        keep.append(d)
        setattr(c, f + '_dict', C.addressof(d))
        setattr(c, 'n_' + short, len(vals))
        if codes is not None:
            setattr(c, f + '_code', arr(np.broadcast_to(np.asarray(codes), (n,)), np.uint32))
    c._keep = keep  # the buffers its pointers name live as long as it does
    return c, keep


def beacon_requests(n: int, *, vcf_id: int, contig, start, end, start2=None, end2=None, contig_map=None,
                    reference='N', alternate=None, variant_type=(None,), variant_type_code=None,
                    variant_min_length=0, variant_max_length=-1, granularity='record', include_details=True):
    """sb_beacon_requests over the route's query parameters as int64 numpy
    columns (views, no conversion when they already are contiguous int64):
    contig codes (contig_map: code -> contig index in the VCF, None =
    identity), requestParameters start[0] / end[0] (start2 / end2: the second
    elements of two-element start / end), variantType as distinct values plus
    a code per request, min / max length columns or scalars.  The library
    builds each SplitQueryPayload as perform_variant_search_sync does
    (search_variants.py:179-197).  Returns (BeaconRequests, keep-alive)."""
    q = _lib.BeaconRequests()
    keep = [q]

    def col(x):
        a = np.ascontiguousarray(x, dtype=np.int64)
        if len(a) != n:
            raise ValueError(f'{len(a)} values for {n} requests')
        keep.append(a)
        return a.ctypes.data

    q.vcf_id = int(vcf_id)
    q.contig, q.start, q.end = col(contig), col(start), col(end)
    if start2 is not None:
        q.start2 = col(start2)
    if end2 is not None:
        q.end2 = col(end2)
    if contig_map is not None:
        m = np.ascontiguousarray(contig_map, dtype=np.uint32)
        keep.append(m)
        q.contig_map, q.n_contig_map = m.ctypes.data, len(m)
    for f, x in (('variant_min_length', variant_min_length), ('variant_max_length', variant_max_length)):
        if np.ndim(x) == 0:
            setattr(q, f + '_all', int(x))
        else:
            setattr(q, f, col(x))

    def text(v):
        s = _lib.Str()
        if v is not None:
            b = v.encode() if isinstance(v, str) else bytes(v)
            buf = C.create_string_buffer(b, len(b) + 1)
            keep.append(buf)
            s.p, s.len = C.addressof(buf), len(b)
        return s

    q.reference_bases, q.alternate_bases = text(reference), text(alternate)
    vals = list(variant_type)
    if not all(v is None for v in vals):
        d = (_lib.Str * len(vals))()
        for k, v in enumerate(vals):
            d[k] = text(v)
        keep.append(d)
        q.variant_type_dict, q.n_variant_type = C.addressof(d), len(vals)
        if variant_type_code is not None:
            q.variant_type_code = col(variant_type_code)
    q.granularity = _lib.SB_GRAN[granularity] if isinstance(granularity, str) else int(granularity)
    q.include_details = 1 if include_details else 0
    q._keep = keep  # the buffers its pointers name live as long as it does
    return q, keep


def requests_from_split_payloads(store, payloads: list[dict], *, strict_variant_type: bool = False,
                                 columns: bool = False):
    """SplitQueryPayload dicts -> (sb_request array, keep-alive, owners):
    one request per (payload, vcf_location) pair, owners[k] = (payload
    index, vcf_location); ``columns``: a RequestColumns (dictionary-coded
    string columns) instead of the sb_request array.  The chrom string each vcf_location maps to is
    looked up among the VCF's contigs (absent: a request with no slices, as
    bcftools emits nothing for it)."""
    rows = []
    for i, p in enumerate(payloads):
        for loc, chrom in p['vcf_locations'].items():
            rows.append((i, loc, chrom))
    n = len(rows)
    contig_idx = {}

    def cidx(loc, chrom):
        key = (loc, chrom)
        if key not in contig_idx:
            names = store.contigs(loc)
            contig_idx[key] = names.index(chrom) if chrom in names else 0xffffffff
        return contig_idx[key]

    def codes(vals):
        d = {}
        out = np.empty(len(vals), dtype=np.int64)
        for k, x in enumerate(vals):
            out[k] = d.setdefault(x, len(d))
        return list(d), out

    P = [payloads[i] for i, _, _ in rows]
    ref_v, ref_c = codes([p.get('reference_bases') for p in P])
    alt_v, alt_c = codes([p.get('alternate_bases') for p in P])
    vt_v, vt_c = codes([p.get('variant_type') for p in P])
    pts = [p.get('passthrough') or {} for p in P]
    sn_v, sn_c = codes([','.join(pt['sampleNames']) if pt.get('sampleNames') is not None else None for pt in pts])
    make = request_columns if columns else requests_array
    arr, keep = make(
        n, vcf_id=[store.vcf_id(loc) for _, loc, _ in rows], contig=[cidx(loc, c) for _, loc, c in rows],
        start_min=[int(p['start_min']) for p in P], start_max=[int(p['start_max']) for p in P],
        end_min=[int(p['end_min']) for p in P], end_max=[int(p['end_max']) for p in P],
        reference=ref_v, reference_code=ref_c, alternate=alt_v, alternate_code=alt_c,
        variant_type=vt_v, variant_type_code=vt_c,
        variant_min_length=[int(p['variant_min_length']) for p in P],
        variant_max_length=[int(p['variant_max_length']) for p in P],
        granularity=[_lib.SB_GRAN.get(p.get('requested_granularity'), 255) for p in P],
        include_details=[1 if p.get('include_datasets') in ('HIT', 'ALL') else 0 for p in P],
        include_samples=[1 if pt.get('includeSamples', False) else 0 for pt in pts],
        selected_samples_only=[1 if pt.get('selectedSamplesOnly', False) else 0 for pt in pts],
        strict_variant_type=1 if strict_variant_type else 0, sample_names=sn_v, sample_names_code=sn_c)
    return arr, keep, [(i, loc) for i, loc, _ in rows]


class RequestBatch:
    """A prepared request batch (sb_requests_prepare) on the store's device."""

    def __init__(self, store, arr, n: int, core=None):
        """arr: an sb_request array (requests_array), RequestColumns
        (request_columns) or BeaconRequests (beacon_requests; core: the
        shard's ShardCore, None = every slice)."""
        self.store = store
        self.n = n
        h = C.c_void_p()
        if isinstance(arr, _lib.BeaconRequests):
            check(lib().sb_requests_prepare_beacon(store.handle, C.byref(arr), n,
                                                   C.byref(core) if core is not None else None, C.byref(h)))
        elif isinstance(arr, _lib.RequestColumns):
            check(lib().sb_requests_prepare_columns(store.handle, C.byref(arr), n, C.byref(h)))
        else:
            check(lib().sb_requests_prepare(store.handle, C.cast(arr, C.c_void_p), n, C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def run(self, rows_ptr: int, hits_ptr: int, row_off_ptr: int, rec_base: int = 0):
        """Enqueue one pass: rows (n x 5 int64: exists, n_variants, call_count,
        all_alleles_count, errors), dense hits, n + 1 row offsets."""
        check(lib().sb_requests_run(self._h, C.c_void_p(rows_ptr), C.c_void_p(hits_ptr), C.c_void_p(row_off_ptr),
                                    int(rec_base)))

    def sync(self):
        check(lib().sb_batch_sync(self._h))

    def timing(self):
        t, s, b = C.c_double(), C.c_double(), C.c_double()
        check(lib().sb_batch_last_timing(self._h, C.byref(t), C.byref(s), C.byref(b)))
        return {'total_ms': t.value, 'scan_ms': s.value}

    def time_eval(self, on: bool):
        """Events around every pass's request_eval_kernel (measurement);
        timing()['scan_ms'] then reports that kernel alone."""
        check(lib().sb_requests_time_eval(self._h, 1 if on else 0))

    def set_replan(self, on: bool):
        """Every pass first re-runs the device planning kernels from the
        packed requests kept in HBM (sb_requests_set_replan; device-planned
        batches only)."""
        check(lib().sb_requests_set_replan(self._h, 1 if on else 0))

    def plan_fused(self) -> bool:
        """True when the last pass planned its runs inside request_eval_kernel
        (sb_requests_plan_fused: a re-planning pass of a fixed-stride batch)."""
        f = C.c_int()
        check(lib().sb_requests_plan_fused(self._h, C.byref(f)))
        return bool(f.value)

    def set_compact(self, on):
        """Narrow outputs (sb_requests_set_compact).  True / COMPACT_ALL:
        rows [n, 4] uint32 (exists, n_variants, call_count,
        all_alleles_count), n + 1 uint32 row offsets, uint32 hits (record +
        rec_base) | ALT label << 29.  COMPACT_HITS: wide rows and offsets,
        uint32 hits.  False / 0: wide."""
        mode = COMPACT_ALL if on is True else int(on)
        check(lib().sb_requests_set_compact(self._h, mode))
        self.compact = mode

    def escape_flags(self) -> tuple[bool, bool]:
        """(rows escaped, hit labels escaped) by the compact passes up to the
        last sync (sb_requests_escapes)."""
        r, h = C.c_int(), C.c_int()
        check(lib().sb_requests_escapes(self._h, C.byref(r), C.byref(h)))
        return bool(r.value), bool(h.value)

    def escapes(self, rows32=None, hits32=None):
        """After a compact pass and its sync: the answers the compact form
        could not hold (sb_requests_escapes).  Returns (wide, labels):
        wide = (row indices, [k, 5] int64 wide rows) of the rows written as
        SB_ROW32_ESCAPED, labels = (hit positions, ALT indices) of the hits
        with the escape label -- either None when the passes wrote none."""
        r, h = C.c_int(), C.c_int()
        check(lib().sb_requests_escapes(self._h, C.byref(r), C.byref(h)))
        wide = labels = None
        if r.value and rows32 is not None:
            idx = np.ascontiguousarray(np.flatnonzero(np.asarray(rows32).view(np.uint32).reshape(-1, 4)[:, 0] ==
                                                      ROW32_ESCAPED), dtype=np.uint32)
            out = np.zeros((len(idx), 5), dtype=np.int64)
            check(lib().sb_requests_wide_rows(self._h, idx.ctypes.data, len(idx), out.ctypes.data))
            wide = (idx, out)
        if h.value and hits32 is not None:
            pos = np.ascontiguousarray(np.flatnonzero((np.asarray(hits32).view(np.uint32) >> 29) == HIT32_LABEL_ESCAPE),
                                       dtype=np.uint64)
            lab = np.zeros(len(pos), dtype=np.uint32)
            check(lib().sb_requests_hit_labels(self._h, pos.ctypes.data, len(pos), lab.ctypes.data))
            labels = (pos, lab)
        return wide, labels

    def inexact_rows(self) -> np.ndarray:
        """After a pass: True for rows whose call_count / all_alleles_count
        are not exact in int64 (low 64 bits held; sb_requests_inexact_rows)."""
        f = np.zeros(max(self.n, 1), dtype=np.uint8)
        check(lib().sb_requests_inexact_rows(self._h, f.ctypes.data))
        return f[:self.n].astype(bool)

    def stats(self) -> dict:
        st = _lib.BatchStats()
        check(lib().sb_batch_get_stats(self._h, C.byref(st)))
        return {f: getattr(st, f) for f, _ in _lib.BatchStats._fields_}

    def set_stream(self, stream_ptr):
        check(lib().sb_batch_set_stream(self._h, _lib.stream_arg(stream_ptr)))

    def free(self):
        if self._h:
            lib().sb_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def answer(self, rec_base: int = 0, device=None, raw: bool = False):
        """One pass, rows + hit lists copied to the host (torch tensors on
        the store's device as staging): (rows [n, 5] int64, hits uint64,
        row_off [n + 1] int64) -- in the wide form whichever output form the
        batch writes (compact outputs widened by widen_compact).  raw: the
        outputs as the batch writes them, (rows, hits, row_off, compact) --
        compact = True: [n, 4] uint32 rows, uint32 hits and offsets."""
        import torch
        dev = device if device is not None else torch.device('cuda', self.store.info()['device'])
        mode = getattr(self, 'compact', 0)
        if mode == COMPACT_HITS:
            rows = torch.zeros((max(self.n, 1), 5), dtype=torch.int64, device=dev)
            hits = torch.zeros(max(int(self.stats()['hits']), 1), dtype=torch.int32, device=dev)
            row_off = torch.zeros(self.n + 1, dtype=torch.int64, device=dev)
            self.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            self.run(rows.data_ptr(), hits.data_ptr(), row_off.data_ptr(), rec_base)
            self.sync()
            ro = row_off.cpu().numpy()
            h32 = hits[:int(ro[-1])].cpu().numpy()
            _, labels = self.escapes(None, h32)
            return (rows[:self.n].cpu().numpy(), widen_hits(h32, labels), ro) + ((False,) if raw else ())
        if mode:
            rows = torch.zeros((max(self.n, 1), 4), dtype=torch.int32, device=dev)
            hits = torch.zeros(max(int(self.stats()['hits']), 1), dtype=torch.int32, device=dev)
            row_off = torch.zeros(self.n + 1, dtype=torch.int32, device=dev)
            self.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            self.run(rows.data_ptr(), hits.data_ptr(), row_off.data_ptr(), rec_base)
            self.sync()
            ro = row_off.cpu().numpy().view(np.uint32)
            r32 = rows[:self.n].cpu().numpy().view(np.uint32)
            h32 = hits[:int(ro[-1])].cpu().numpy().view(np.uint32)
            wide, labels = self.escapes(r32, h32)
            if raw and wide is None and labels is None:
                return r32, h32, ro, True
            out = widen_compact(r32, h32, ro, wide=wide, labels=labels)
            return out + (False,) if raw else out
        rows = torch.zeros((max(self.n, 1), 5), dtype=torch.int64, device=dev)
        hits = torch.zeros(max(int(self.stats()['hits']), 1), dtype=torch.int64, device=dev)
        row_off = torch.zeros(self.n + 1, dtype=torch.int64, device=dev)
        self.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        self.run(rows.data_ptr(), hits.data_ptr(), row_off.data_ptr(), rec_base)
        self.sync()
        ro = row_off.cpu().numpy()
        if raw:
            return rows[:self.n].cpu().numpy(), hits[:int(ro[-1])].cpu().numpy().view(np.uint64), ro, False
        return rows[:self.n].cpu().numpy(), hits[:int(ro[-1])].cpu().numpy().view(np.uint64), ro


ROW32_ESCAPED = 0xffffffff  # SB_ROW32_ESCAPED
HIT32_LABEL_ESCAPE = 7       # SB_HIT32_LABEL_ESCAPE


def widen_hits(hits32, labels=None):
    """uint32 hits ((record + rec_base) | ALT label << 29) as the wide form's
    uint64 record | ALT label << 32; labels = (positions, ALT indices) of the
    escaped labels (RequestBatch.escapes)."""
    h = np.asarray(hits32).view(np.uint32).astype(np.uint64)
    out = (h & np.uint64((1 << 29) - 1)) | ((h >> np.uint64(29)) << np.uint64(32))
    if labels is not None:
        pos, lab = labels
        out[pos] = (out[pos] & np.uint64(0xffffffff)) | (np.asarray(lab, dtype=np.uint64) << np.uint64(32))
    return out


def widen_rows(rows32, wide=None):
    """Compact rows (sb_request_row32: u32 exists, n_variants, call_count,
    all_alleles_count) as the wide [n, 5] int64 rows with a zero error count;
    wide = (row indices, wide rows) of the escaped rows (RequestBatch.escapes)."""
    rows32 = np.asarray(rows32).view(np.uint32).reshape(-1, 4)
    rows = np.zeros((len(rows32), 5), dtype=np.int64)
    rows[:, :4] = rows32
    if wide is not None:
        idx, w = wide
        rows[np.asarray(idx, dtype=np.int64)] = w
    return rows


def widen_compact(rows32, hits32, row_off32, wide=None, labels=None):
    """Compact request outputs (sb_requests_set_compact) in the wide form:
    (rows [n, 5] int64 with a zero error count, hits uint64 = record | ALT
    label << 32, row_off int64), escapes resolved (RequestBatch.escapes)."""
    return widen_rows(rows32, wide), widen_hits(hits32, labels), np.asarray(row_off32).view(np.uint32).astype(np.int64)
