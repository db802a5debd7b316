"""BASELINE.json workloads: 1000G-shape synthetic stores and their query mixes.

Config 2: chr22-shape store, 1,103,547 records x 2,504
samples (seed 22); 10,000 Beacon requests (seed 1022): 5,000 range requests
(start uniform over the span, width uniform 1-100,000 bp, ref = alt = 'N',
granularity record, includeResultsetResponses HIT) and 5,000 point ref/alt
requests (70 % drawn from existing rows, 30 % random SNVs; start=[POS-1],
end=[POS-1+len(alt)] as route_g_variants_id.py builds them).  Each request is
converted exactly as shared_resources/variantutils/search_variants.py:179-199
and sliced as lambda/splitQuery/lambda_function.py:82-106, so the unit the
device answers is the reference's PerformQueryPayload.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import PKG_ROOT
from .payloads import SplitQueryPayload
from .split_query import split_payloads

SYNTH_PATH = os.path.join(PKG_ROOT, 'libsbeacon_synth.so')
_syn = None


def synth_lib():
    global _syn
    if _syn is None:
        L = C.CDLL(SYNTH_PATH)
        L.sbs_new.restype = C.c_void_p
        L.sbs_new.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_double, C.c_char_p]
        L.sbs_free.argtypes = [C.c_void_p]
        L.sbs_positions.argtypes = [C.c_void_p, C.c_void_p]
        L.sbs_alleles.restype = C.c_int
        L.sbs_alleles.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.sbs_header.restype = C.c_void_p
        L.sbs_header.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]
        L.sbs_records.restype = C.c_void_p
        L.sbs_records.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_size_t)]
        L.sbs_free_text.argtypes = [C.c_void_p]
        L.sbs_new_member.restype = C.c_void_p
        L.sbs_new_member.argtypes = [C.c_void_p, C.c_uint64, C.c_double, C.c_uint32]
        L.sbs_set_an_sites.argtypes = [C.c_void_p, C.c_uint32]
        L.sbs_alt_rows.restype = C.c_uint64
        L.sbs_alt_rows.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int]
        L.sbs_carrier_planes.restype = C.c_int
        L.sbs_carrier_planes.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_void_p, C.c_uint64]
        L.sbs_bgzf_compress.restype = C.c_void_p
        L.sbs_bgzf_compress.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_size_t)]
        _syn = L
    return _syn


def bgzf_compress(data: bytes, *, level=6, eof=True, threads=0) -> bytes:
    """bgzip-compatible BGZF (0xff00-byte blocks + EOF block)."""
    n = C.c_size_t()
    p = synth_lib().sbs_bgzf_compress(data, len(data), level, 1 if eof else 0, threads, C.byref(n))
    out = C.string_at(p, n.value)
    synth_lib().sbs_free_text(p)
    return out


def write_bgzf(path, chunks, *, level=6, threads=0):
    """Stream text chunks into one BGZF file (block boundaries fall every
    0xff00 bytes of the concatenated text, as bgzip places them)."""
    pending = b''
    with open(path, 'wb') as f:
        for c in chunks:
            pending += c
            cut = len(pending) - len(pending) % 0xff00
            if cut:
                f.write(bgzf_compress(pending[:cut], level=level, eof=False, threads=threads))
                pending = pending[cut:]
        f.write(bgzf_compress(pending, level=level, eof=True, threads=threads))
    return path


CHR22_SPAN = (16050075, 51244237)


class SyntheticVcf:
    """Seeded 1000G-shape VCF (records are pure functions of seed + index)."""

    def __init__(self, *, seed=22, n_records=1103547, n_samples=2504, start=CHR22_SPAN[0],
                 mean_gap=(CHR22_SPAN[1] - CHR22_SPAN[0]) / (1103547 - 1), contig='22'):
        self.seed, self.n_records, self.n_samples, self.contig = seed, n_records, n_samples, contig
        self._h = synth_lib().sbs_new(seed, n_records, n_samples, start, float(mean_gap), contig.encode())
        self._pos = None

    def __del__(self):
        try:
            synth_lib().sbs_free(self._h)
        except Exception:
            pass

    def _take(self, p, n):
        b = C.string_at(p, n.value)
        synth_lib().sbs_free_text(p)
        return b

    def header(self, sites_only=False) -> bytes:
        n = C.c_size_t()
        return self._take(synth_lib().sbs_header(self._h, 1 if sites_only else 0, C.byref(n)), n)

    def records(self, lo, hi, sites_only=False, threads=0) -> bytes:
        n = C.c_size_t()
        return self._take(synth_lib().sbs_records(self._h, lo, hi, 1 if sites_only else 0, threads, C.byref(n)), n)

    def chunks(self, sites_only=False, chunk=1 << 16, threads=0):
        yield self.header(sites_only)
        for lo in range(0, self.n_records, chunk):
            yield self.records(lo, min(lo + chunk, self.n_records), sites_only, threads)

    def write(self, path, sites_only=True, threads=0):
        with open(path, 'wb') as f:
            for c in self.chunks(sites_only, threads=threads):
                f.write(c)
        return path

    def positions(self) -> np.ndarray:
        if self._pos is None:
            a = np.empty(self.n_records, dtype=np.uint32)
            synth_lib().sbs_positions(self._h, a.ctypes.data)
            self._pos = a
        return self._pos

    def member(self, own_seed, *, share=0.7, n_samples=None):
        """A cohort member (config 4): the same positions, record i taken
        from this generator with probability `share`, else from own_seed."""
        m = SyntheticVcf.__new__(SyntheticVcf)
        m.seed, m.n_records, m.contig = own_seed, self.n_records, self.contig
        m.n_samples = self.n_samples if n_samples is None else n_samples
        m._h = synth_lib().sbs_new_member(self._h, own_seed, float(share), m.n_samples)
        m._pos = self._pos
        return m

    def set_an_sites(self, an: int):
        """Config 5: every record's INFO AN = an (AC drawn over it); GT
        carriers over the n_samples cohort scale with 2 n_samples / an."""
        synth_lib().sbs_set_an_sites(self._h, int(an))
        return self

    def sample_names(self) -> list[str]:
        return [f'HG{i + 96:05d}' for i in range(self.n_samples)]

    def alt_rows(self, lo=0, hi=None, threads=0) -> int:
        hi = self.n_records if hi is None else hi
        return int(synth_lib().sbs_alt_rows(self._h, lo, hi, threads))

    def carrier_planes(self, lo=0, hi=None, threads=0, out=None) -> np.ndarray:
        """Carrier bit-matrix of records [lo, hi), the genotypes records()
        renders as GT text: uint64 [alt rows, ceil(n_samples / 64)]."""
        hi = self.n_records if hi is None else hi
        words = (self.n_samples + 63) // 64
        if out is None:
            out = np.empty((self.alt_rows(lo, hi, threads), words), dtype=np.uint64)
        n = out.shape[0]
        if out.shape[1] != words or not out.flags['C_CONTIGUOUS']:
            raise ValueError('out must be a C-contiguous [alt rows, words] uint64 array')
        if synth_lib().sbs_carrier_planes(self._h, lo, hi, threads, out.ctypes.data, n) != 0:
            raise RuntimeError('carrier plane generation failed')
        return out

    def alleles(self, i):
        ref = C.create_string_buffer(256)
        alt = C.create_string_buffer(256)
        n = synth_lib().sbs_alleles(self._h, i, ref, 256, alt, 256)
        return ref.value.decode(), alt.value.decode(), n

    def build_store(self, location, *, device=0, keep_genotypes=True, threads=0, sites_only=False):
        from .engine import Store
        return Store.build([(location, self.chunks(sites_only=sites_only, threads=threads))], device=device,
                           keep_genotypes=keep_genotypes, n_threads=threads)


def beacon_request_payloads(*, vcf_location, chrom, start, end, reference_bases, alternate_bases,
                            granularity='record', include='HIT', variant_type=None, vmin=0, vmax=-1,
                            passthrough=None, dataset_id='synthetic', query_id='bench'):
    """One Beacon request -> its PerformQueryPayloads (search_variants.py:179-238
    + splitQuery)."""
    if len(start) == 2:
        start_min, start_max = start
    else:
        start_min = start[0]
    if len(end) == 2:
        end_min, end_max = end
    else:
        end_min, end_max = start_min, end[0]
    if len(start) != 2:
        start_max = end_max
    sp = SplitQueryPayload(passthrough=passthrough or {}, dataset_id=dataset_id, query_id=query_id,
                           reference_bases=reference_bases, start_min=start_min + 1, start_max=start_max + 1,
                           end_min=end_min + 1, end_max=end_max + 1, alternate_bases=alternate_bases,
                           variant_type=variant_type, include_datasets=include, vcf_locations={vcf_location: chrom},
                           vcf_groups=[], requested_granularity=granularity, variant_min_length=vmin,
                           variant_max_length=vmax)
    return split_payloads(sp)


def config2_requests(gen: SyntheticVcf, *, n_range=5000, n_point=5000, seed=1022):
    """The 10k-request mix of config 2 as (kind, request-kwargs) tuples."""
    rng = np.random.default_rng(seed)
    pos = gen.positions()
    lo, hi = int(pos[0]), int(pos[-1])
    reqs = []
    starts = rng.integers(lo, hi, n_range)
    widths = rng.integers(1, 100001, n_range)
    for s, w in zip(starts, widths):
        reqs.append(dict(start=[int(s) - 1], end=[int(s) - 1 + int(w)], reference_bases='N',
                         alternate_bases='N'))
    for k in range(n_point):
        if rng.random() < 0.7:
            i = int(rng.integers(0, gen.n_records))
            p = int(pos[i])
            ref, alt, _ = gen.alleles(i)
            ref, alt = ref.upper(), alt.upper()
        else:
            p = int(rng.integers(lo, hi))
            b = rng.choice(list('ACGT'), 2, replace=False)
            ref, alt = str(b[0]), str(b[1])
        reqs.append(dict(start=[p - 1], end=[p - 1 + len(alt)], reference_bases=ref, alternate_bases=alt))
    return reqs


def requests_to_payloads(reqs, *, vcf_location, chrom):
    """Flatten requests into slice payloads; returns (payloads, owner) where
    owner[j] = request index of payload j."""
    payloads, owner = [], []
    for ri, r in enumerate(reqs):
        ps = beacon_request_payloads(vcf_location=vcf_location, chrom=chrom, **r)
        payloads.extend(ps)
        owner.extend([ri] * len(ps))
    return payloads, owner


def config4_cohort(*, n_datasets=50, n_records=1103547, seed=4, share=0.7, n_samples=250):
    """Config 4: datasets over one shared chr22-shape site
    pool.  Dataset d holds two VCFs (a vcfGroup split by samples, 250 + 250)
    with the same sites: each record is the pool's with probability `share`,
    else a private one at the same position.  Returns
    (pool, [(dataset_id, [(vcf_location, SyntheticVcf), ...]), ...])."""
    pool = SyntheticVcf(seed=seed, n_records=n_records, n_samples=n_samples)
    out = []
    for d in range(n_datasets):
        m = pool.member(seed * 1000 + d + 1, share=share, n_samples=n_samples)
        out.append((f'ds{d:02d}', [(f's3://cohort/ds{d:02d}/part{k}.vcf.gz', m) for k in (0, 1)]))
    return pool, out
