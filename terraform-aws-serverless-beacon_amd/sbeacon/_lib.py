"""ctypes binding of libsbeacon_hip.so (declared in include/sbeacon.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, importing the engine raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_NAME = 'libsbeacon_hip.so'
LIB_PATH = os.environ.get('SBEACON_LIB', os.path.join(PKG_ROOT, LIB_NAME))

SB_OK = 0
SB_GRAN = {'boolean': 0, 'count': 1, 'aggregated': 2, 'record': 3}


SB_EINVAL = -1  # malformed argument / payload (and compact outputs a batch cannot fit)
SB_ESTALE = -7  # sb_store_open: a source VCF changed since the save
SB_EINTERNAL = -8  # a device pass failed its own consistency checks
SB_HOST_ONLY = -1  # sb_builder_finish / sb_store_open: no device image


class SbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f'sbeacon error {code}: {msg}')
        self.code = code


class BuildOpts(C.Structure):
    _fields_ = [('keep_genotypes', C.c_int32), ('n_threads', C.c_int32)]


class StoreInfo(C.Structure):
    _fields_ = [('n_records', C.c_uint64), ('n_alt_rows', C.c_uint64), ('n_vcfs', C.c_uint32),
                ('n_segments', C.c_uint32), ('device_bytes', C.c_uint64), ('max_samples', C.c_uint32),
                ('device', C.c_int32)]


class Query(C.Structure):
    _fields_ = [('vcf_id', C.c_uint32), ('_pad0', C.c_uint32),
                ('region', C.c_char_p), ('region_len', C.c_size_t),
                ('end_min', C.c_int64), ('end_max', C.c_int64),
                ('reference_bases', C.c_char_p), ('reference_len', C.c_size_t),
                ('alternate_bases', C.c_char_p), ('alternate_len', C.c_size_t),
                ('variant_type', C.c_char_p), ('variant_type_len', C.c_size_t),
                ('variant_min_length', C.c_int64), ('variant_max_length', C.c_int64),
                ('granularity', C.c_uint8), ('include_details', C.c_uint8),
                ('include_samples', C.c_uint8), ('selected_samples_only', C.c_uint8),
                ('strict_variant_type', C.c_uint8), ('_pad1', C.c_uint8 * 3),
                ('sample_names', C.c_char_p), ('sample_names_len', C.c_size_t)]


class Request(C.Structure):
    """sb_request: one SplitQueryPayload x one of its VCFs (include/sbeacon.h)."""
    _fields_ = [('vcf_id', C.c_uint32), ('contig', C.c_uint32),
                ('start_min', C.c_int64), ('start_max', C.c_int64), ('end_min', C.c_int64), ('end_max', C.c_int64),
                ('reference_bases', C.c_char_p), ('reference_len', C.c_size_t),
                ('alternate_bases', C.c_char_p), ('alternate_len', C.c_size_t),
                ('variant_type', C.c_char_p), ('variant_type_len', C.c_size_t),
                ('variant_min_length', C.c_int64), ('variant_max_length', C.c_int64),
                ('granularity', C.c_uint8), ('include_details', C.c_uint8), ('include_samples', C.c_uint8),
                ('selected_samples_only', C.c_uint8), ('strict_variant_type', C.c_uint8), ('_pad', C.c_uint8 * 3),
                ('sample_names', C.c_char_p), ('sample_names_len', C.c_size_t)]


class Str(C.Structure):
    """sb_str: p == NULL is None."""
    _fields_ = [('p', C.c_void_p), ('len', C.c_size_t)]


class RequestColumns(C.Structure):
    """sb_request_columns (include/sbeacon.h): requests as columns."""
    _fields_ = [('vcf_id', C.c_void_p), ('vcf_id_all', C.c_uint32),
                ('contig', C.c_void_p), ('contig_all', C.c_uint32),
                ('start_min', C.c_void_p), ('start_max', C.c_void_p),
                ('end_min', C.c_void_p), ('end_min_all', C.c_int64),
                ('end_max', C.c_void_p), ('end_max_all', C.c_int64),
                ('variant_min_length', C.c_void_p), ('variant_min_length_all', C.c_int64),
                ('variant_max_length', C.c_void_p), ('variant_max_length_all', C.c_int64),
                ('reference_dict', C.c_void_p), ('reference_code', C.c_void_p), ('n_reference', C.c_uint32),
                ('alternate_dict', C.c_void_p), ('alternate_code', C.c_void_p), ('n_alternate', C.c_uint32),
                ('variant_type_dict', C.c_void_p), ('variant_type_code', C.c_void_p), ('n_variant_type', C.c_uint32),
                ('sample_names_dict', C.c_void_p), ('sample_names_code', C.c_void_p), ('n_sample_names', C.c_uint32),
                ('granularity', C.c_void_p), ('granularity_all', C.c_uint8),
                ('include_details', C.c_void_p), ('include_details_all', C.c_uint8),
                ('include_samples', C.c_void_p), ('include_samples_all', C.c_uint8),
                ('selected_samples_only', C.c_void_p), ('selected_samples_only_all', C.c_uint8),
                ('strict_variant_type', C.c_uint8)]


class BeaconRequests(C.Structure):
    """sb_beacon_requests (include/sbeacon.h): the route's query parameters
    as int64 columns, one VCF."""
    _fields_ = [('vcf_id', C.c_uint32), ('contig', C.c_void_p), ('contig_map', C.c_void_p),
                ('n_contig_map', C.c_uint32), ('start', C.c_void_p), ('start2', C.c_void_p),
                ('end', C.c_void_p), ('end2', C.c_void_p),
                ('variant_type_code', C.c_void_p), ('variant_type_dict', C.c_void_p), ('n_variant_type', C.c_uint32),
                ('variant_min_length', C.c_void_p), ('variant_min_length_all', C.c_int64),
                ('variant_max_length', C.c_void_p), ('variant_max_length_all', C.c_int64),
                ('reference_bases', Str), ('alternate_bases', Str),
                ('granularity', C.c_uint8), ('include_details', C.c_uint8)]


class ShardCore(C.Structure):
    """sb_shard_core: [(contig_lo, pos_lo), (contig_hi, pos_hi)) in one VCF."""
    _fields_ = [('contig_lo', C.c_uint32), ('pos_lo', C.c_int64), ('contig_hi', C.c_uint32), ('pos_hi', C.c_int64)]


class ResultView(C.Structure):
    _fields_ = [('error', C.c_int32), ('exists', C.c_int32), ('call_count', C.c_int64),
                ('all_alleles_count', C.c_int64), ('n_variants', C.c_uint64),
                ('hit_record', C.POINTER(C.c_uint32)), ('hit_alt', C.POINTER(C.c_uint32)),
                ('n_sample_indices', C.c_uint64), ('sample_indices', C.POINTER(C.c_uint32)),
                ('big_limbs', C.c_uint32), ('_pad', C.c_uint32),
                ('big_call_count', C.POINTER(C.c_uint32)), ('big_all_alleles_count', C.POINTER(C.c_uint32))]


def big_int(limbs, n: int) -> int:
    """n 32-bit two's complement limbs (little-endian) -> Python int."""
    return int.from_bytes(C.string_at(limbs, 4 * n), 'little', signed=True)


def view_counts(v) -> tuple[int, int]:
    """(call_count, all_alleles_count) of a ResultView, exact past 64 bits."""
    if v.big_limbs:
        return big_int(v.big_call_count, v.big_limbs), big_int(v.big_all_alleles_count, v.big_limbs)
    return int(v.call_count), int(v.all_alleles_count)


class BatchStats(C.Structure):
    _fields_ = [('n_queries', C.c_uint64), ('records_scanned', C.c_uint64), ('hits', C.c_uint64),
                ('device_ms', C.c_double), ('chained_slices', C.c_uint64), ('chains', C.c_uint64),
                ('cand_loaded', C.c_uint64), ('cand_window', C.c_uint64), ('cand_unique', C.c_uint64)]


class Slice(C.Structure):
    _fields_ = [('vcf_id', C.c_uint32), ('_pad', C.c_uint32), ('virtual_start', C.c_uint64),
                ('virtual_end', C.c_uint64)]


class SliceStats(C.Structure):
    _fields_ = [('error', C.c_int32), ('_pad', C.c_int32), ('num_variants', C.c_uint64),
                ('num_calls', C.c_uint64), ('records', C.c_uint64)]


class RegionFile(C.Structure):
    _fields_ = [('slice', C.c_uint32), ('contig', C.c_uint32), ('first_pos', C.c_uint64), ('last_pos', C.c_uint64),
                ('bytes', C.c_uint64), ('entries', C.c_uint64), ('data_bytes', C.c_uint64)]


class DedupJob(C.Structure):
    _fields_ = [('vcf_ids', C.POINTER(C.c_uint32)), ('n_vcf', C.c_uint32), ('contig_len', C.c_uint32),
                ('contig', C.c_char_p), ('range_start', C.c_uint64), ('range_end', C.c_uint64)]


class RegionRef(C.Structure):
    _fields_ = [('vcf_id', C.c_uint32), ('file', C.c_uint32), ('virtual_start', C.c_uint64),
                ('virtual_end', C.c_uint64)]


class DedupFileJob(C.Structure):
    _fields_ = [('files', C.POINTER(RegionRef)), ('n_files', C.c_uint32), ('_pad', C.c_uint32),
                ('range_start', C.c_uint64), ('range_end', C.c_uint64)]


class DedupStats(C.Structure):
    _fields_ = [('keys', C.c_uint64), ('collisions', C.c_uint64), ('device_ms', C.c_double),
                ('path', C.c_uint32), ('windows', C.c_uint32)]


class RouteEvent(C.Structure):
    """sb_route_event: one /g_variants event over its request rows."""
    _fields_ = [('row_lo', C.c_uint32), ('row_hi', C.c_uint32), ('granularity', C.c_uint8), ('check_all', C.c_uint8),
                ('_pad', C.c_uint8 * 2), ('assembly', C.c_uint32), ('pagination', C.c_uint32)]


class RouteInput(C.Structure):
    """sb_route_input (include/sbeacon.h)."""
    _fields_ = [('events', C.c_void_p), ('n_events', C.c_size_t),
                ('row_vcf', C.c_void_p), ('vcf_all', C.c_uint32),
                ('row_contig', C.c_void_p), ('contig_all', C.c_uint32),
                ('compact', C.c_int32), ('_pad', C.c_uint32),
                ('rows', C.c_void_p), ('hits', C.c_void_p), ('row_off', C.c_void_p), ('rec_base', C.c_uint64),
                ('assembly_dict', C.c_void_p), ('n_assembly', C.c_uint32),
                ('pagination_dict', C.c_void_p), ('n_pagination', C.c_uint32),
                ('beacon_id', Str), ('api_version', Str)]


DEDUP_PATHS = ('windows', 'buckets', 'radix')


# every exported symbol of include/sbeacon.h: name -> (restype, argtypes)
P = C.c_void_p
SIGNATURES = {
    'sb_last_error': (C.c_char_p, []),
    'sb_abi_version': (C.c_int, []),
    'sb_builder_new': (C.c_int, [C.POINTER(BuildOpts), C.POINTER(P)]),
    'sb_builder_begin_vcf': (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint32)]),
    'sb_builder_add_text': (C.c_int, [P, C.c_uint32, C.c_char_p, C.c_size_t]),
    'sb_builder_add_file': (C.c_int, [P, C.c_uint32, C.c_char_p]),
    'sb_builder_attach_carriers': (C.c_int, [P, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32),
                                             C.c_uint32, C.c_void_p, C.c_uint64]),
    'sb_builder_finish': (C.c_int, [P, C.c_int, C.POINTER(P)]),
    'sb_builder_free': (None, [P]),
    'sb_store_close': (None, [P]),
    'sb_store_get_info': (C.c_int, [P, C.POINTER(StoreInfo)]),
    'sb_store_find_vcf': (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint32)]),
    'sb_store_candidates': (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    'sb_store_n_samples': (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint32)]),
    'sb_store_sample_name': (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_char_p),
                                       C.POINTER(C.c_size_t)]),
    'sb_query_batch': (C.c_int, [P, C.POINTER(Query), C.c_size_t, C.c_uint32, C.POINTER(P)]),
    'sb_result_get': (C.c_int, [P, C.c_size_t, C.POINTER(ResultView)]),
    'sb_result_get_all': (C.c_int, [P, C.POINTER(ResultView), C.c_size_t]),
    'sb_result_variants_text': (C.c_int, [P, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    'sb_result_sample_names_text': (C.c_int, [P, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    'sb_result_stats': (C.c_int, [P, C.POINTER(BatchStats)]),
    'sb_result_free': (None, [P]),
    'sb_batch_prepare': (C.c_int, [P, C.POINTER(Query), C.c_size_t, C.POINTER(P)]),
    'sb_batch_run': (C.c_int, [P]),
    'sb_batch_sync': (C.c_int, [P]),
    'sb_batch_last_timing': (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    'sb_batch_get_stats': (C.c_int, [P, C.POINTER(BatchStats)]),
    'sb_batch_fetch': (C.c_int, [P, C.POINTER(P)]),
    'sb_batch_free': (None, [P]),
    'sb_batch_set_owners': (C.c_int, [P, C.POINTER(C.c_uint32), C.c_size_t, C.c_uint32]),
    'sb_batch_reduce_requests': (C.c_int, [P, C.c_void_p]),
    'sb_batch_compact_hits': (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    'sb_batch_set_stream': (C.c_int, [P, C.c_void_p]),
    'sb_batch_set_slice_results': (C.c_int, [P, C.c_int]),
    'sb_batch_deliver': (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    'sb_summarise_slices': (C.c_int, [P, C.POINTER(Slice), C.c_size_t, C.POINTER(SliceStats),
                                      C.POINTER(C.c_double)]),
    'sb_slice_region_files': (C.c_int, [P, C.POINTER(Slice), C.c_size_t, C.c_int, C.POINTER(C.c_int32),
                                        C.POINTER(P)]),
    'sb_region_files_get': (C.c_int, [P, C.POINTER(C.POINTER(RegionFile)), C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    'sb_region_files_free': (None, [P]),
    'sb_dedup_count': (C.c_int, [P, C.POINTER(DedupJob), C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_int32),
                                 C.POINTER(DedupStats)]),
    'sb_dedup_count_files': (C.c_int, [P, C.POINTER(DedupFileJob), C.c_size_t, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_int32), C.POINTER(DedupStats)]),
    'sb_store_n_contigs': (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint32)]),
    'sb_store_contig_name': (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t)]),
    'sb_store_chunk_boundaries': (C.c_int, [P, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint32,
                                            C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_size_t)]),
    'sb_store_vcf_stream': (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    'sb_index_vcf': (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                               C.POINTER(C.c_size_t)]),
    'sb_free': (None, [P]),
    'sb_result_distinct_variants': (C.c_int, [P, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_size_t), C.POINTER(C.c_uint64)]),
    'sb_builder_set_record_range': (C.c_int, [P, C.c_uint32, C.c_uint64, C.c_uint64]),
    'sb_vcf_scan_file': (C.c_int, [C.c_char_p, C.POINTER(P)]),
    'sb_vcf_scan_info': (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_void_p)]),
    'sb_vcf_scan_contig': (C.c_int, [P, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    'sb_vcf_scan_free': (None, [P]),
    'sb_requests_prepare': (C.c_int, [P, C.c_void_p, C.c_size_t, C.POINTER(P)]),
    'sb_requests_run': (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    'sb_requests_prepare_columns': (C.c_int, [P, C.c_void_p, C.c_size_t, C.POINTER(P)]),
    'sb_requests_prepare_beacon': (C.c_int, [P, C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(P)]),
    'sb_requests_time_eval': (C.c_int, [P, C.c_int]),
    'sb_requests_set_replan': (C.c_int, [P, C.c_int]),
    'sb_requests_plan_fused': (C.c_int, [P, C.POINTER(C.c_int)]),
    'sb_requests_set_compact': (C.c_int, [P, C.c_int]),
    'sb_requests_inexact_rows': (C.c_int, [P, P]),
    'sb_requests_escapes': (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    'sb_requests_wide_rows': (C.c_int, [P, C.c_void_p, C.c_size_t, C.c_void_p]),
    'sb_requests_hit_labels': (C.c_int, [P, C.c_void_p, C.c_size_t, C.c_void_p]),
    'sb_store_trim': (C.c_int, [P]),
    'sb_store_save': (C.c_int, [P, C.c_char_p]),
    'sb_store_open': (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    'sb_perform_query_events': (C.c_int, [C.POINTER(P), C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32,
                                          C.POINTER(P)]),
    'sb_json_out_get': (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                  C.POINTER(C.c_void_p)]),
    'sb_json_out_free': (None, [P]),
    'sb_route_bodies': (C.c_int, [P, C.POINTER(RouteInput), C.POINTER(P)]),
}

_lib = None


def lib():
    """Load libsbeacon_hip.so (raises OSError if it is missing: no fallback)."""
    global _lib
    if _lib is None:
        try:
            # torch bundles its own libamdhip64.so.7 (same soname as ROCm's):
            # load it first so the process has ONE HIP runtime whichever of
            # torch / this library the caller touches first
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f'{LIB_PATH} not found: build it with `python -c "import __graft_entry__ as g; g.build()"`')
        L = C.CDLL(LIB_PATH)
        variant = 'SBEACON_LIB' in os.environ  # an A/B build of another revision: bind what it has
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None) if variant else getattr(L, name)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != SB_OK:
        msg = lib().sb_last_error()
        raise SbError(rc, msg.decode() if msg else '')
    return rc


HIP_STREAM_LEGACY = 1  # hipStreamLegacy: the null stream, which torch's default stream is


def stream_arg(stream_ptr):
    """The ``void *stream`` of sb_batch_set_stream for a caller stream
    handle: None -> NULL (the store's own stream); 0 -> hipStreamLegacy.

    torch reports its default stream as ``cuda_stream == 0``.  Passed as
    NULL, the batch would run on the store's non-blocking stream, unordered
    with the caller's default-stream copies of its outputs (a D2H copy then
    reads rows while request_eval_kernel is still writing them)."""
    if stream_ptr is None:
        return None
    return C.c_void_p(int(stream_ptr) if int(stream_ptr) else HIP_STREAM_LEGACY)
