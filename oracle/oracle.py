"""ctypes wrapper around the C oracle (oracle/sbeacon_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.

``OracleVcf(path).perform_query(payload_dict)`` returns the dict the reference
``PerformQueryResponse.dump()`` would return
(``shared_resources/payloads/lambda_responses.py:14-23``) or raises the Python
exception class the reference raises on the same input.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liboracle.so')

GRAN = {'boolean': 0, 'count': 1, 'aggregated': 2, 'record': 3}
ERRORS = {1: UnboundLocalError, 2: IndexError, 3: ValueError, 4: AttributeError,
          9: NotImplementedError}


class OrcQuery(C.Structure):
    _fields_ = [('region', C.c_char_p), ('end_min', C.c_int64), ('end_max', C.c_int64),
                ('reference_bases', C.c_char_p), ('alternate_bases', C.c_char_p),
                ('variant_type', C.c_char_p), ('include_details', C.c_int32),
                ('granularity', C.c_int32), ('variant_min_length', C.c_int64),
                ('variant_max_length', C.c_int64), ('include_samples', C.c_int32),
                ('selected_samples_only', C.c_int32), ('sample_names', C.c_char_p),
                ('patched', C.c_int32)]


class OrcResult(C.Structure):
    _fields_ = [('error', C.c_int32), ('exists', C.c_int32), ('call_count', C.c_int64),
                ('all_alleles_count', C.c_int64), ('variants', C.c_void_p),
                ('n_variants', C.c_int64), ('sample_indices', C.POINTER(C.c_int32)),
                ('n_sample_indices', C.c_int64), ('sample_names', C.c_void_p),
                ('n_sample_names', C.c_int64), ('call_count_hex', C.c_char_p),
                ('all_alleles_count_hex', C.c_char_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_load_vcf.restype = C.c_void_p
        L.orc_load_vcf.argtypes = [C.c_char_p, C.c_int]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_n_records.restype = C.c_int64
        L.orc_n_records.argtypes = [C.c_void_p]
        L.orc_n_samples.restype = C.c_int32
        L.orc_n_samples.argtypes = [C.c_void_p]
        L.orc_query_one.argtypes = [C.c_void_p, C.POINTER(OrcQuery), C.POINTER(OrcResult)]
        L.orc_query_batch.argtypes = [C.c_void_p, C.POINTER(OrcQuery), C.c_int64,
                                      C.POINTER(OrcResult), C.c_int]
        L.orc_result_free.argtypes = [C.POINTER(OrcResult)]
        L.orc_records_in_region.restype = C.c_int64
        L.orc_records_in_region.argtypes = [C.c_void_p, C.c_char_p]
        _lib = L
    return _lib


def build():
    import subprocess
    subprocess.check_call(['make', '-s', '-C', HERE])


def _b(s):
    return None if s is None else str(s).encode()


def make_query(p: dict, patched: bool = False):
    """PerformQueryPayload dict -> OrcQuery (keeps the encoded strings alive)."""
    pt = p.get('passthrough') or {}
    names = pt.get('sampleNames', None)
    keep = [_b(p['region']), _b(p.get('reference_bases')), _b(p.get('alternate_bases')),
            _b(p.get('variant_type')), _b(','.join(names)) if names is not None else None]
    q = OrcQuery(keep[0], int(p['end_min']), int(p['end_max']), keep[1], keep[2], keep[3],
                 1 if p.get('include_details') else 0, GRAN.get(p.get('requested_granularity'), -1),
                 int(p['variant_min_length']), int(p['variant_max_length']),
                 1 if pt.get('includeSamples', False) else 0,
                 1 if pt.get('selectedSamplesOnly', False) else 0, keep[4], 1 if patched else 0)
    return q, keep


def _result_dict(r: OrcResult, p: dict):
    pt = p.get('passthrough') or {}
    samples_variant = bool(pt.get('selectedSamplesOnly', False))
    variants = C.string_at(r.variants).decode() if r.variants else ''
    names = C.string_at(r.sample_names).decode() if r.sample_names else ''
    return {
        'exists': bool(r.exists),
        'vcf_location': p.get('vcf_location'),
        'dataset_id': p.get('dataset_id'),
        'all_alleles_count': int(r.all_alleles_count_hex, 16) if r.all_alleles_count_hex else int(r.all_alleles_count),
        'variants': variants.split('\n') if r.n_variants else [],
        'call_count': int(r.call_count_hex, 16) if r.call_count_hex else int(r.call_count),
        'sample_indices': [r.sample_indices[i] for i in range(r.n_sample_indices)] if samples_variant else [],
        'sample_names': names.split(',') if r.n_sample_names else [],
    }


class OracleVcf:
    def __init__(self, path: str, load_gt: bool = True):
        self.path = path
        self.h = lib().orc_load_vcf(path.encode(), 1 if load_gt else 0)
        if not self.h:
            raise FileNotFoundError(path)

    def close(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_records(self):
        return lib().orc_n_records(self.h)

    def perform_query(self, payload: dict, patched: bool = False) -> dict:
        q, _keep = make_query(payload, patched)
        r = OrcResult()
        lib().orc_query_one(self.h, C.byref(q), C.byref(r))
        try:
            if r.error:
                raise ERRORS.get(r.error, RuntimeError)(f'oracle error {r.error}')
            return _result_dict(r, payload)
        finally:
            lib().orc_result_free(C.byref(r))

    def perform_query_batch(self, payloads, patched=False, threads=0, want_results=True):
        """Run many queries (OpenMP); returns list of dict | Exception class."""
        n = len(payloads)
        arr = (OrcQuery * n)()
        keep = []
        for i, p in enumerate(payloads):
            q, k = make_query(p, patched)
            arr[i] = q
            keep.append(k)
        res = (OrcResult * n)()
        lib().orc_query_batch(self.h, arr, n, res, int(threads))
        out = []
        for i in range(n):
            if want_results:
                if res[i].error:
                    out.append(ERRORS.get(res[i].error, RuntimeError))
                else:
                    out.append(_result_dict(res[i], payloads[i]))
            lib().orc_result_free(C.byref(res[i]))
        return out

    def time_batch(self, payloads, patched=False, threads=0, min_seconds=0.0, max_passes=10000):
        """CPU-baseline timing: the payloads are converted once, then the C
        restatement runs over the whole batch (OpenMP x threads) pass after
        pass until min_seconds of C time have accumulated.  Returns
        (seconds inside the C calls, passes)."""
        import time
        n = len(payloads)
        arr = (OrcQuery * n)()
        keep = []
        for i, p in enumerate(payloads):
            q, k = make_query(p, patched)
            arr[i] = q
            keep.append(k)
        res = (OrcResult * n)()
        total, passes = 0.0, 0
        while passes < max_passes and (passes == 0 or total < min_seconds):
            t = time.perf_counter()
            lib().orc_query_batch(self.h, arr, n, res, int(threads))
            total += time.perf_counter() - t
            passes += 1
            for i in range(n):
                lib().orc_result_free(C.byref(res[i]))
        return total, passes

    def records_in_region(self, region: str) -> int:
        return lib().orc_records_in_region(self.h, region.encode())


# ------------------------------------------------------------ summariseSlice
def _summ_lib():
    L = lib()
    if not hasattr(L, '_summ_ready'):
        L.orc_bgzf_open.restype = C.c_void_p
        L.orc_bgzf_open.argtypes = [C.c_char_p]
        L.orc_bgzf_close.argtypes = [C.c_void_p]
        L.orc_bgzf_ulen.restype = C.c_int64
        L.orc_bgzf_ulen.argtypes = [C.c_void_p]
        L.orc_bgzf_nblocks.restype = C.c_int64
        L.orc_bgzf_nblocks.argtypes = [C.c_void_p]
        L.orc_bgzf_voff_to_u.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.orc_summarise_slice.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_region_stats.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]
        L.orc_slice_region_files.restype = C.c_int64
        L.orc_slice_region_files.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64), C.c_int64,
                                             C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        L._summ_ready = True
    return L


def region_stats(text: bytes):
    """getRegionStats (summariseSlice/source/main.cpp:195-245) over raw text."""
    L = _summ_lib()
    nv, nc, rec = C.c_uint64(), C.c_uint64(), C.c_uint64()
    rc = L.orc_region_stats(text, len(text), C.byref(nv), C.byref(nc), C.byref(rec))
    if rc:
        raise ValueError(f'unsupported record (oracle rc={rc})')
    return {'numVariants': nv.value, 'numCalls': nc.value, 'records': rec.value}


class OracleBgzf:
    """A BGZF file decompressed in memory; summarise_slice restates one
    summariseSlice invocation {location, virtual_start, virtual_end}."""

    def __init__(self, path):
        self.h = _summ_lib().orc_bgzf_open(os.fsencode(path))
        if not self.h:
            raise ValueError(f'not a BGZF file: {path}')

    def close(self):
        if self.h:
            _summ_lib().orc_bgzf_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ulen(self):
        return _summ_lib().orc_bgzf_ulen(self.h)

    def voff_to_u(self, voff):
        u = C.c_uint64()
        if _summ_lib().orc_bgzf_voff_to_u(self.h, voff, C.byref(u)):
            raise ValueError(voff)
        return u.value

    def region_files(self, vstart, vend, with_data=False):
        """The slice's region files [(first, last, bytes, entries)] (+ the
        concatenated uncompressed bytes); ValueError where the reference
        throws."""
        L = _summ_lib()
        cap = 4096
        rows = (C.c_uint64 * (4 * cap))()
        dcap = max(1 << 16, 2 * self.ulen) if with_data else 0
        data = C.create_string_buffer(dcap) if with_data else None
        dl = C.c_int64()
        n = L.orc_slice_region_files(self.h, vstart, vend, rows, cap, data, dcap, C.byref(dl))
        if n < 0:
            raise ValueError(f'region files: oracle rc={n}')
        files = [tuple(rows[4 * i:4 * i + 4]) for i in range(n)]
        return (files, data.raw[:dl.value]) if with_data else files

    def summarise_slice(self, vstart, vend):
        nv, nc, rec = C.c_uint64(), C.c_uint64(), C.c_uint64()
        rc = _summ_lib().orc_summarise_slice(self.h, vstart, vend, C.byref(nv), C.byref(nc), C.byref(rec))
        if rc:
            raise ValueError(f'unsupported slice (oracle rc={rc})')
        return {'numVariants': nv.value, 'numCalls': nc.value, 'records': rec.value}


# ---------------------------------------------------- duplicateVariantSearch
def dedup_count(texts, contig: str, range_start: int, range_end: int):
    """|{to_string(pos) + ref'_alt'}| over the region entries of `contig` in
    the VCF texts with range_start <= pos <= range_end
    (duplicateVariantSearch.cpp:31-84; intended range semantics).
    Raises ValueError where the reference's summariseSlice throws."""
    L = lib()
    if not hasattr(L, '_dedup_ready'):
        L.orc_dedup_count.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_int64), C.c_int, C.c_char_p, C.c_int64,
                                      C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
        L._dedup_ready = True
    texts = [t if isinstance(t, bytes) else t.encode() for t in texts]
    arr = (C.c_char_p * max(len(texts), 1))(*texts)
    lens = (C.c_int64 * max(len(texts), 1))(*[len(t) for t in texts])
    cb = contig.encode()
    u = C.c_uint64()
    if L.orc_dedup_count(arr, lens, len(texts), cb, len(cb), range_start, range_end, C.byref(u)):
        raise ValueError('a record in range makes summariseSlice throw (compressSeq)')
    return u.value
