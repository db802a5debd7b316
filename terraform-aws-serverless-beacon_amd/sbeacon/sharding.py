"""Sharding a store across the GPUs of one node.

A :class:`ShardPlan` cuts the records of any ``Store.build`` input (VCF
files: plain, gzip or BGZF) into ``world`` record-balanced *cores* in
(VCF, contig, POS) order -- the order splitQuery's fan-out walks
(``lambda/splitQuery/lambda_function.py:74-110``) -- plus a right *halo* of
``halo`` bp on the contig where the next core starts, so that every
performQuery slice (at most 10 kb, ``SPLIT_SIZE``) is answered WHOLE by the
rank whose core holds its first base: the reference's order-dependent
per-slice semantics (cumulative call_count, early exits,
``search_variants.py:229-254``) never need a cross-GPU exchange.  Cuts never
split a run of records with one POS.

* :meth:`ShardPlan.build_store` -- rank r's store: each VCF ingested with
  ``sb_builder_set_record_range`` (its core + halo records only).
* :meth:`ShardPlan.route` / :meth:`route_payloads` -- the rank answering a
  slice ``chrom:a-b`` of a VCF: the core holding (VCF, contig, a).  A contig
  the VCF lacks (bcftools emits nothing) goes to the VCF's first rank.
* :meth:`ShardPlan.split_requests` -- the request-level fan-out: each
  SplitQueryPayload x VCF cut into the runs of its slices each rank answers
  (sub-requests of ``sb_requests_prepare``), one row per request on every
  rank; the rows of one request sum over ranks (route_g_variants.py:144-171).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib

SPLIT_SIZE = 10000  # lambda/splitQuery/lambda_function.py:12


@dataclass
class VcfLayout:
    location: str
    path: str
    contigs: list          # [(name, lo, hi)] records [lo, hi) in file order
    pos: np.ndarray        # POS of every record (uint32)

    @property
    def n(self) -> int:
        return len(self.pos)


def scan_vcf(location: str, path: str) -> VcfLayout:
    """CHROM / POS of every record (sb_vcf_scan_file, C++, no store)."""
    L = lib()
    h = C.c_void_p()
    check(L.sb_vcf_scan_file(os.fsencode(path), C.byref(h)))
    try:
        n, nc, p = C.c_uint64(), C.c_uint32(), C.c_void_p()
        check(L.sb_vcf_scan_info(h, C.byref(n), C.byref(nc), C.byref(p)))
        pos = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(n.value,)).copy() if n.value \
            else np.zeros(0, dtype=np.uint32)
        contigs = []
        name, ln, lo, hi = C.c_char_p(), C.c_size_t(), C.c_uint64(), C.c_uint64()
        for i in range(nc.value):
            check(L.sb_vcf_scan_contig(h, i, C.byref(name), C.byref(ln), C.byref(lo), C.byref(hi)))
            contigs.append((C.string_at(name, ln.value).decode(), lo.value, hi.value))
    finally:
        L.sb_vcf_scan_free(h)
    return VcfLayout(location, os.fspath(path), contigs, pos)


class ShardPlan:
    """Record-balanced (VCF, contig, POS) shards of a set of VCF files."""

    def __init__(self, layouts: list[VcfLayout], world: int, halo: int = SPLIT_SIZE):
        if world < 1:
            raise ValueError('world >= 1')
        self.layouts, self.world, self.halo = layouts, world, halo
        self.vcf_index = {l.location: i for i, l in enumerate(layouts)}
        self._cidx = [{c[0]: k for k, c in enumerate(l.contigs)} for l in layouts]
        sizes = np.array([l.n for l in layouts], dtype=np.int64)
        self.vcf_base = np.concatenate([[0], np.cumsum(sizes)])
        N = int(self.vcf_base[-1])
        # cuts: global record ordinals, moved forward off any run of one POS
        cuts = [0]
        for r in range(1, world):
            g = max(r * N // world, cuts[-1])
            g = self._pos_boundary(g)
            cuts.append(max(g, cuts[-1]))
        cuts.append(N)
        self.cuts = cuts
        # routing keys: rank r >= 1 owns (vcf, contig, a) >= key[r]
        keys = [(0, 0, 0)]
        for r in range(1, world):
            keys.append(self._key_of(cuts[r]))
        self.keys = keys
        self._kv = np.array([k[0] for k in keys], dtype=np.int64)
        self._kc = np.array([k[1] for k in keys], dtype=np.int64)
        self._kp = np.array([k[2] for k in keys], dtype=np.int64)

    @classmethod
    def from_sources(cls, sources, world: int, halo: int = SPLIT_SIZE):
        """sources: [(vcf_location, path)] as Store.build takes them."""
        return cls([scan_vcf(loc, path) for loc, path in sources], world, halo)

    # ---------------------------------------------------------------- cuts
    def _locate(self, g: int):
        """global ordinal -> (vcf, record in vcf, contig index)."""
        v = int(np.searchsorted(self.vcf_base, g, side='right') - 1)
        v = min(v, len(self.layouts) - 1)
        i = g - int(self.vcf_base[v])
        L = self.layouts[v]
        for k, (_, lo, hi) in enumerate(L.contigs):
            if lo <= i < hi:
                return v, i, k
        return v, i, len(L.contigs)

    def _pos_boundary(self, g: int) -> int:
        N = int(self.vcf_base[-1])
        if g <= 0 or g >= N:
            return g
        v, i, k = self._locate(g)
        L = self.layouts[v]
        if k >= len(L.contigs):
            return g
        lo, hi = L.contigs[k][1], L.contigs[k][2]
        if i == lo:
            return g
        p = L.pos[i - 1]
        seg = L.pos[i:hi]
        j = int(np.searchsorted(seg, p, side='right'))  # first record past the run of POS p
        return g + j

    def _key_of(self, g: int):
        N = int(self.vcf_base[-1])
        if g >= N:
            return (len(self.layouts), 0, 0)
        v, i, k = self._locate(g)
        L = self.layouts[v]
        if i == L.contigs[k][1]:
            # a core that starts a contig owns the contig from base 0 -- and the
            # whole VCF when it starts the VCF (contigs it lacks route there)
            return (v, 0, 0) if i == 0 else (v, k, 0)
        return (v, k, int(L.pos[i]))

    def record_range(self, rank: int, v: int):
        """Records [lo, hi) of VCF v that rank r's store holds: its core plus
        the halo on the contig where the next core starts."""
        a, b = self.cuts[rank], self.cuts[rank + 1]
        base, n = int(self.vcf_base[v]), self.layouts[v].n
        lo, hi = min(max(a - base, 0), n), min(max(b - base, 0), n)
        if hi <= lo:
            if not (base <= b < base + n and a < b):
                return lo, lo
        if rank + 1 < self.world and base <= b < base + n:
            v2, i, k = self._locate(b)
            L = self.layouts[v]
            clo, chi = L.contigs[k][1], L.contigs[k][2]
            if clo < i:  # the next core starts inside this contig: halo of records with POS < P + halo
                p = int(L.pos[i]) + self.halo
                hi = max(hi, i + int(np.searchsorted(L.pos[i:chi], p, side='left')))
        return lo, hi

    # ---------------------------------------------------------------- stores
    def build_store(self, rank: int, *, device: int = 0, keep_genotypes: bool = True, n_threads: int = 0,
                    text=None, carriers=None):
        """Rank r's store: every VCF of the plan restricted to its record range.
        ``text(v, lo, hi)``, when given, yields VCF v's header + records
        [lo, hi) as text chunks (a generated VCF) instead of reading its file;
        ``carriers(v, lo, hi)``, when given, returns (sample names, planes) --
        the carrier bit-matrix of a sites-only text, uint64 [ALT rows of
        records lo..hi, ceil(n/64)] (sb_builder_attach_carriers) -- or None."""
        from ._lib import BuildOpts
        from .engine import Store
        L = lib()
        b = C.c_void_p()
        check(L.sb_builder_new(C.byref(BuildOpts(1 if keep_genotypes else 0, int(n_threads))), C.byref(b)))
        try:
            for v, lay in enumerate(self.layouts):
                vid = C.c_uint32()
                lb = lay.location.encode()
                check(L.sb_builder_begin_vcf(b, lb, len(lb), C.byref(vid)))
                lo, hi = self.record_range(rank, v)
                if text is None:
                    check(L.sb_builder_set_record_range(b, vid.value, lo, hi))
                    check(L.sb_builder_add_file(b, vid.value, os.fsencode(lay.path)))
                else:
                    for chunk in text(v, lo, hi):
                        check(L.sb_builder_add_text(b, vid.value, chunk, len(chunk)))
                car = carriers(v, lo, hi) if carriers is not None else None
                if car is not None:
                    names = [n.encode() for n in car[0]]
                    planes = np.ascontiguousarray(car[1], dtype=np.uint64)
                    del car
                    if planes.ndim != 2 or planes.shape[1] != (len(names) + 63) // 64:
                        raise ValueError('carrier planes must be [alt rows, ceil(n_samples / 64)] uint64')
                    arr = (C.c_char_p * len(names))(*names)
                    lens = (C.c_uint32 * len(names))(*[len(x) for x in names])
                    check(L.sb_builder_attach_carriers(b, vid.value, arr, lens, len(names), planes.ctypes.data,
                                                       planes.shape[0]))
                    del planes
            s = C.c_void_p()
            check(L.sb_builder_finish(b, int(device), C.byref(s)))
        finally:
            L.sb_builder_free(b)
        return Store(s, [l.location for l in self.layouts],
                     {l.location: l.path for l in self.layouts if text is None})

    def record_base(self, rank: int, v: int = 0) -> int:
        """Ordinal within VCF v of the first record rank r's store holds."""
        return self.record_range(rank, v)[0]

    # ---------------------------------------------------------------- routing
    def contig_index(self, v: int, chrom: str) -> int:
        """Index of chrom among VCF v's contigs (file order); absent = len."""
        return self._cidx[v].get(chrom, len(self.layouts[v].contigs))

    def route(self, v, c, a):
        """Rank answering slices with first base a on contig index c of VCF v
        (numpy arrays or scalars): the last rank whose key <= (v, c, a)."""
        v, c, a = (np.asarray(x, dtype=np.int64) for x in (v, c, a))
        ge = ((v[..., None] > self._kv) | ((v[..., None] == self._kv) & (
            (c[..., None] > self._kc) | ((c[..., None] == self._kc) & (a[..., None] >= self._kp)))))
        return ge.sum(axis=-1) - 1

    def route_payloads(self, payloads: list[dict]) -> np.ndarray:
        """Rank of every PerformQueryPayload (its region's first base).  A
        region that does not parse raises in performQuery before any record
        is read, so any rank answers it (rank 0).  A region wider than the
        halo that reaches the next core's records cannot be answered by one
        shard: rank -1 (callers raise)."""
        out = np.zeros(len(payloads), dtype=np.int64)
        for j, p in enumerate(payloads):
            reg = p['region']
            v = self.vcf_index.get(p['vcf_location'])
            if v is None:
                raise KeyError(f"vcf_location {p['vcf_location']!r} is not in the shard plan")
            try:
                chrom = reg[:reg.find(':')]
                a = int(reg[reg.find(':') + 1:reg.find('-')])
                b = int(reg[reg.find('-') + 1:])
            except ValueError:
                continue
            c = self.contig_index(v, chrom)
            r = int(self.route(v, c, a))
            if b - a + 1 > self.halo and r + 1 < self.world and int(self.route(v, c, b)) != r:
                r = -1
            out[j] = r
        return out

    def slice_runs(self, rank: int, v, c, smin, smax):
        """Vectorised splitQuery cut (lambda/splitQuery/lambda_function.py:74-110)
        of requests [smin, smax] on contig index c of VCF v: the sub-request
        [a, b] of the slices (a = smin + 10000 k, k in [k0, k1)) whose first
        base rank r's core holds; b < a when it holds none."""
        v, c, smin, smax = (np.asarray(x, dtype=np.int64) for x in (v, c, smin, smax))
        nsl = np.where(smax >= smin, (smax - smin) // SPLIT_SIZE + 1, 0)

        # slice k's first base smin + 10000 k is routed monotonically in k: the
        # run on rank r is [k0, k1) = slices routed >= r minus those routed > r
        def first_k(rk):
            """first slice index routed to rank >= rk (nsl if none)."""
            if rk <= 0:
                return np.zeros_like(nsl)
            if rk >= self.world:
                return nsl.copy()
            kv, kc, kp = self.keys[rk]
            out = np.where((v > kv) | ((v == kv) & (c > kc)), 0, nsl)
            same = (v == kv) & (c == kc)
            need = -((-(kp - smin)) // SPLIT_SIZE)  # ceil((kp - smin) / 10000)
            return np.where(same, np.clip(need, 0, nsl), out)

        k0, k1 = first_k(rank), first_k(rank + 1)
        k1 = np.maximum(k1, k0)
        a = smin + SPLIT_SIZE * k0
        b = np.minimum(smax, smin + SPLIT_SIZE * k1 - 1)
        return a, np.where(k1 > k0, b, a - 1)

    def core(self, rank: int, v: int = 0):
        """Rank r's core in VCF v as the library's sb_shard_core (slice_runs
        inside sb_requests_prepare_beacon): slices whose (contig, first base)
        lies in [key r, key r+1) restricted to VCF v."""
        from ._lib import ShardCore
        NONE, LO = 0xffffffff, -(1 << 62)
        c = ShardCore()
        if rank <= 0:
            c.contig_lo, c.pos_lo = 0, LO
        else:
            kv, kc, kp = self.keys[rank]
            if kv < v:
                c.contig_lo, c.pos_lo = 0, LO
            elif kv > v:
                c.contig_lo, c.pos_lo = NONE, 0
            else:
                c.contig_lo, c.pos_lo = kc, kp
        if rank + 1 >= self.world:
            c.contig_hi, c.pos_hi = NONE, 0
        else:
            kv, kc, kp = self.keys[rank + 1]
            if kv > v:
                c.contig_hi, c.pos_hi = NONE, 0
            elif kv < v:
                c.contig_hi, c.pos_hi = 0, LO
            else:
                c.contig_hi, c.pos_hi = kc, kp
        return c

    def split_requests(self, split_payloads: list[dict], rank: int):
        """The request-level fan-out on rank r: one sb_request per
        (SplitQueryPayload, vcf_location) pair -- every rank gets the same
        rows -- each cut to the run of its slices whose first base rank r's
        core holds (an empty run: a row with no slices).  Returns (sb_request
        array, keep-alive, owners [(payload index, vcf_location)])."""
        from .requests import requests_array
        rows = [(i, loc, chrom) for i, p in enumerate(split_payloads) for loc, chrom in p['vcf_locations'].items()]
        n = len(rows)
        P = [split_payloads[i] for i, _, _ in rows]
        v = np.array([self.vcf_index[loc] for _, loc, _ in rows], dtype=np.int64)
        c = np.array([self.contig_index(int(v[k]), chrom) for k, (_, _, chrom) in enumerate(rows)], dtype=np.int64)
        smin = np.array([int(p['start_min']) for p in P], dtype=np.int64)
        smax = np.array([int(p['start_max']) for p in P], dtype=np.int64)
        a, b = self.slice_runs(rank, v, c, smin, smax)

        def codes(vals):
            d = {}
            out = np.empty(len(vals), dtype=np.int64)
            for k, x in enumerate(vals):
                out[k] = d.setdefault(x, len(d))
            return list(d), out

        ref_v, ref_c = codes([p.get('reference_bases') for p in P])
        alt_v, alt_c = codes([p.get('alternate_bases') for p in P])
        vt_v, vt_c = codes([p.get('variant_type') for p in P])
        pts = [p.get('passthrough') or {} for p in P]
        sn_v, sn_c = codes([','.join(pt['sampleNames']) if pt.get('sampleNames') is not None else None for pt in pts])
        nc = np.array([len(self.layouts[int(x)].contigs) for x in v], dtype=np.int64)
        arr, keep = requests_array(
            n, vcf_id=v, contig=np.where(c < nc, c, 0xffffffff), start_min=a, start_max=b,
            end_min=[int(p['end_min']) for p in P], end_max=[int(p['end_max']) for p in P],
            reference=ref_v, reference_code=ref_c, alternate=alt_v, alternate_code=alt_c,
            variant_type=vt_v, variant_type_code=vt_c,
            variant_min_length=[int(p['variant_min_length']) for p in P],
            variant_max_length=[int(p['variant_max_length']) for p in P],
            granularity=[_lib.SB_GRAN.get(p.get('requested_granularity'), 255) for p in P],
            include_details=[1 if p.get('include_datasets') in ('HIT', 'ALL') else 0 for p in P],
            include_samples=[1 if pt.get('includeSamples', False) else 0 for pt in pts],
            selected_samples_only=[1 if pt.get('selectedSamplesOnly', False) else 0 for pt in pts],
            sample_names=sn_v, sample_names_code=sn_c)
        return arr, keep, [(i, loc) for i, loc, _ in rows]

    # ---------------------------------------------------------------- text (tests)
    def shard_text(self, rank: int, v: int) -> bytes:
        """VCF text of rank r's part of VCF v (header + its record range):
        what its store holds, for CPU-side checks."""
        import gzip
        path = self.layouts[v].path
        opener = gzip.open if open(path, 'rb').read(2) == b'\x1f\x8b' else open
        lo, hi = self.record_range(rank, v)
        out, r = [], 0
        with opener(path, 'rb') as f:
            for line in f:
                if line.startswith(b'#'):
                    out.append(line)
                    continue
                if not line.strip():
                    continue
                if lo <= r < hi:
                    out.append(line)
                r += 1
        return b''.join(out)
