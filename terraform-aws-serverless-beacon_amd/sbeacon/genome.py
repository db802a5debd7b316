"""Whole-genome workload and contig sharding (BASELINE.json configs[2];
SURVEY.md §8d config 3, §8e).

Store: a 1000 Genomes-shape whole genome — ~85 M records over contigs 1-22,
X, Y, counts proportional to contig length (``chrom_matching.py:12-38``),
one synthetic generator per contig (seed ``1000 * seed + contig index``),
generated as sites-only text; the bench store carries the generator's
2,504-sample carrier bit-matrix beside it (``build_shard_store(genotypes=
True)``: the planes the GT columns would give, attached through
``sb_builder_attach_carriers``) -- the HBM-resident store north_star
describes, although the config-3 queries never read genotypes.

Sharding (one rank per GPU).  The genome's records, in (contig, POS) order,
are cut into ``world`` ranges of equal record count; rank r's *core* is
``[cut_r, cut_{r+1})`` in (contig index, POS) order.  A performQuery slice
(``splitQuery``: ``[a, min(a + 9999, start_max)]``, one contig) is answered
by the rank whose core holds ``(contig, a)``.  Its records lie in
``[a, a + 9999]``, so every rank also holds a right *halo* of 10,000 bp past
its core: each slice is answered whole by one GPU and the reference's
order-dependent per-slice semantics (cumulative call_count, early exits)
need no cross-GPU exchange.  A request whose slices fall on several ranks
is combined at the route level (exists OR, counts summed —
``route_g_variants.py:144-171``), which is what the RCCL step carries.

Requests (config 3): ``n`` Beacon requests, seed 1003 + 0: contig drawn
proportional to length, start uniform over the contig's populated span,
width uniform 1-100,000 bp, ``referenceBases='N'``, ``alternateBases=None``,
``variantType`` in {DEL, INS, DUP, DUP:TANDEM, CNV} with length bounds,
granularity ``record``, ``includeResultsetResponses='HIT'``.  They are
ordered by (contig, start) so every rank's requests form one contiguous
window of request rows (the router keeps the permutation to the arrival
order).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .chrom_matching import CHROMOSOME_LENGTHS
from .workload import SyntheticVcf

CONTIGS = [c for c in CHROMOSOME_LENGTHS if c != 'MT']
SPLIT_SIZE = 10000  # lambda/splitQuery/lambda_function.py:12
HALO = SPLIT_SIZE
EDGE = 10000  # records start EDGE bp into each contig and stop EDGE bp before its end
LOCATION = 'synthetic/wgs-1000g-shape.vcf.gz'
VARIANT_TYPES = ['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV']
VMIN = [0, 0, 1, 5]
VMAX = [-1, -1, 10, 50, 1000]


class _GenomePositions:
    """POS of every genome record, in genome order, read from the contig
    generators on demand (index or slice; a slice within one contig is a
    view)."""

    def __init__(self, shape):
        self.shape = shape

    def __len__(self):
        return int(self.shape.n_total)

    def _contig(self, g):
        return int(np.searchsorted(self.shape.offsets, g, side='right') - 1)

    def __getitem__(self, k):
        off = self.shape.offsets
        if isinstance(k, slice):
            a, b, step = k.indices(len(self))
            assert step == 1
            if b <= a:
                return np.zeros(0, dtype=np.uint32)
            out = []
            while a < b:
                ci = self._contig(a)
                e = min(b, int(off[ci + 1]))
                out.append(self.shape.gen(ci).positions()[a - int(off[ci]):e - int(off[ci])])
                a = e
            return out[0] if len(out) == 1 else np.concatenate(out)
        g = int(k)
        ci = self._contig(g)
        return self.shape.gen(ci).positions()[g - int(off[ci])]


class GenomeShape:
    def __init__(self, *, n_total: int = 85_000_000, seed: int = 3, n_samples: int = 2504):
        self.seed, self.n_total, self.n_samples = seed, n_total, n_samples
        lens = np.array([CHROMOSOME_LENGTHS[c] for c in CONTIGS], dtype=np.float64)
        counts = np.floor(n_total * lens / lens.sum()).astype(np.int64)
        counts[0] += n_total - counts.sum()
        self.counts = counts
        self.offsets = np.concatenate([[0], np.cumsum(counts)])  # global record index of each contig's first
        self._gens: dict[int, SyntheticVcf] = {}

    def gen(self, ci: int) -> SyntheticVcf:
        g = self._gens.get(ci)
        if g is None:
            c = CONTIGS[ci]
            n = int(self.counts[ci])
            span = CHROMOSOME_LENGTHS[c] - 2 * EDGE
            g = SyntheticVcf(seed=1000 * self.seed + ci, n_records=n, n_samples=self.n_samples, start=EDGE,
                             mean_gap=span / max(n - 1, 1), contig=c)
            self._gens[ci] = g
        return g

    def span(self, ci: int):
        p = self.gen(ci).positions()
        return int(p[0]), int(p[-1])

    # ------------------------------------------------------------- sharding
    # The genome is one VCF (LOCATION) of the contigs in order; it is cut by
    # the product sharder, sbeacon.sharding.ShardPlan, over a layout whose POS
    # column is read lazily from the generators (the plan only reads it at
    # the cut contigs), so a deployment over real VCF files and this bench
    # run the same cuts, routing, halo and sub-request split.
    def layout(self):
        from .sharding import VcfLayout
        contigs = [(c, int(self.offsets[ci]), int(self.offsets[ci + 1])) for ci, c in enumerate(CONTIGS)]
        return VcfLayout(LOCATION, LOCATION, contigs, _GenomePositions(self))

    def plan(self, world: int):
        """The ShardPlan of `world` ranks (cached)."""
        plans = self.__dict__.setdefault('_plans', {})
        p = plans.get(world)
        if p is None:
            from .sharding import ShardPlan
            p = plans[world] = ShardPlan([self.layout()], world, HALO)
        return p

    def cuts(self, world: int):
        """world + 1 cut points (contig index, POS): rank r's core is
        [cuts[r], cuts[r + 1]) in lexicographic order (the plan's keys)."""
        keys = self.plan(world).keys
        return [(0, 0)] + [(int(k[1]), int(k[2])) for k in keys[1:]] + [(len(CONTIGS), 0)]

    def shard_pieces(self, world: int, rank: int):
        """[(contig index, record lo, record hi)] of rank's store: its core
        plus the right halo (ShardPlan.record_range)."""
        lo, hi = self.plan(world).record_range(rank, 0)
        pieces = []
        for ci in range(len(CONTIGS)):
            a, b = max(lo, int(self.offsets[ci])), min(hi, int(self.offsets[ci + 1]))
            if b > a:
                pieces.append((ci, a - int(self.offsets[ci]), b - int(self.offsets[ci])))
        return pieces

    def text(self, lo: int, hi: int, chunk=1 << 20, threads=0, progress=None):
        """VCF text (header + records [lo, hi) in genome order, sites only) in
        large chunks: the builder parses each chunk with all its threads."""
        first = True
        done = 0
        for ci in range(len(CONTIGS)):
            a, b = max(lo, int(self.offsets[ci])), min(hi, int(self.offsets[ci + 1]))
            if first:
                yield self.gen(ci).header(sites_only=True)
                first = False
            if b <= a:
                continue
            g = self.gen(ci)
            a, b = a - int(self.offsets[ci]), b - int(self.offsets[ci])
            for x in range(a, b, chunk):
                y = min(x + chunk, b)
                yield g.records(x, y, sites_only=True, threads=threads)
                done += y - x
                if progress:
                    progress(CONTIGS[ci], done)

    def shard_chunks(self, world: int, rank: int, chunk=1 << 20, threads=0, progress=None):
        """VCF text of rank's shard (one VCF, contigs in order, sites only)."""
        lo, hi = self.plan(world).record_range(rank, 0)
        return self.text(lo, hi, chunk, threads, progress)

    def build_shard_store(self, world: int, rank: int, *, device=0, threads=0, progress=None, genotypes=False):
        """Rank's store, built by ShardPlan.build_store from the generated
        text (sites only); ``genotypes``: with the generator's n_samples
        carrier bit-matrix attached (the rows the GT columns would give,
        SyntheticVcf.carrier_planes: ~320 B per ALT row at 2,504 samples)."""
        return self.plan(world).build_store(
            rank, device=device, keep_genotypes=False, n_threads=threads,
            text=lambda v, lo, hi: self.text(lo, hi, threads=threads, progress=progress),
            carriers=(lambda v, lo, hi: self.carriers(lo, hi, threads)) if genotypes and self.n_samples else None)

    def carriers(self, lo: int, hi: int, threads: int = 0):
        """(sample names, carrier planes) of genome records [lo, hi),
        record-then-ALT order."""
        pieces = []
        for ci in range(len(CONTIGS)):
            a, b = max(lo, int(self.offsets[ci])), min(hi, int(self.offsets[ci + 1]))
            if b > a:
                pieces.append((ci, a - int(self.offsets[ci]), b - int(self.offsets[ci])))
        rows = [self.gen(ci).alt_rows(a, b, threads) for ci, a, b in pieces]
        out = np.empty((sum(rows), (self.n_samples + 63) // 64), dtype=np.uint64)
        r = 0
        for (ci, a, b), n in zip(pieces, rows):
            self.gen(ci).carrier_planes(a, b, threads, out=out[r:r + n])
            r += n
        return self.gen(0).sample_names(), out

    def shard_records(self, world: int, rank: int) -> int:
        return sum(hi - lo for _, lo, hi in self.shard_pieces(world, rank))


@dataclass
class Requests:
    """Config-3 requests, ordered by (contig, start); Beacon 0-based start."""
    ci: np.ndarray     # contig index
    start: np.ndarray  # requestParameters.start[0] (0-based)
    width: np.ndarray  # end[0] - start[0]
    vt: np.ndarray     # index into VARIANT_TYPES
    vmin: np.ndarray
    vmax: np.ndarray

    def __len__(self):
        return len(self.ci)

    @property
    def end(self) -> np.ndarray:
        """requestParameters.end[0] (computed once)."""
        e = self.__dict__.get('_end')
        if e is None:
            e = self.__dict__['_end'] = self.start + self.width
        return e

    def rows(self, a: int, b: int) -> 'Requests':
        """Requests [a, b) as views (the end column too)."""
        sub = Requests(self.ci[a:b], self.start[a:b], self.width[a:b], self.vt[a:b], self.vmin[a:b], self.vmax[a:b])
        sub.__dict__['_end'] = self.end[a:b]
        return sub


def config3_requests(shape: GenomeShape, n: int = 1_000_000, seed: int = 1003) -> Requests:
    rng = np.random.default_rng(seed)
    lens = np.array([CHROMOSOME_LENGTHS[c] for c in CONTIGS], dtype=np.float64)
    ci = rng.choice(len(CONTIGS), size=n, p=lens / lens.sum())
    width = rng.integers(1, 100001, n)
    lo = np.array([shape.span(c)[0] for c in range(len(CONTIGS))])
    hi = np.array([shape.span(c)[1] for c in range(len(CONTIGS))])
    u = rng.random(n)
    start = (lo[ci] - 1 + u * (hi[ci] - lo[ci])).astype(np.int64)
    vt = rng.integers(0, len(VARIANT_TYPES), n)
    vmin = np.array(VMIN)[rng.integers(0, len(VMIN), n)]
    vmax = np.array(VMAX)[rng.integers(0, len(VMAX), n)]
    order = np.lexsort((start, ci))
    return Requests(ci[order], start[order], width[order], vt[order], vmin[order], vmax[order])


@dataclass
class ShardSlices:
    """The performQuery slices one rank answers: request row (relative to
    row_lo), contig, [a, b], the request's end bracket and filters."""
    row_lo: int
    n_rows: int
    req: np.ndarray
    ci: np.ndarray
    a: np.ndarray
    b: np.ndarray
    end_min: np.ndarray
    end_max: np.ndarray
    vt: np.ndarray
    vmin: np.ndarray
    vmax: np.ndarray

    def __len__(self):
        return len(self.a)


def request_slices(reqs: Requests):
    """Every slice of every request, as perform_variant_search_sync +
    split_query build them (search_variants.py:179-199: start=[s], end=[e]
    -> start_min = s+1, start_max = end_max = e+1, end_min = s+1;
    splitQuery: a = start_min + 10000 k, b = min(a + 9999, start_max))."""
    smin = reqs.start + 1
    smax = reqs.start + reqs.width + 1
    nsl = (smax - smin) // SPLIT_SIZE + 1
    req = np.repeat(np.arange(len(reqs), dtype=np.int64), nsl)
    first = np.repeat(np.cumsum(nsl) - nsl, nsl)
    k = np.arange(len(req), dtype=np.int64) - first
    a = smin[req] + SPLIT_SIZE * k
    b = np.minimum(a + SPLIT_SIZE - 1, smax[req])
    return req, a, b, smin[req], smax[req]


def rank_of_slices(shape: GenomeShape, world: int, ci: np.ndarray, a: np.ndarray) -> np.ndarray:
    """Rank answering slices with first base a on contig ci (ShardPlan.route)."""
    ci = np.asarray(ci, dtype=np.int64)
    return shape.plan(world).route(np.zeros_like(ci), ci, a)


def shard_slices(shape: GenomeShape, reqs: Requests, world: int, rank: int) -> ShardSlices:
    # only requests whose [start_min, start_max] reaches this rank's core are expanded
    smin = reqs.start + 1
    smax = reqs.start + reqs.width + 1
    near = (rank_of_slices(shape, world, reqs.ci, smin) <= rank) & (rank_of_slices(shape, world, reqs.ci, smax) >= rank)
    idx = np.flatnonzero(near)
    sub = Requests(reqs.ci[idx], reqs.start[idx], reqs.width[idx], reqs.vt[idx], reqs.vmin[idx], reqs.vmax[idx])
    req, a, b, emin, emax = request_slices(sub)
    req = idx[req] if len(idx) else req
    ci = reqs.ci[req]
    mine = rank_of_slices(shape, world, ci, a) == rank
    req, a, b, emin, emax, ci = req[mine], a[mine], b[mine], emin[mine], emax[mine], ci[mine]
    if len(req):
        row_lo, n_rows = int(req[0]), int(req[-1]) - int(req[0]) + 1
    else:
        row_lo, n_rows = 0, 0
    return ShardSlices(row_lo, n_rows, (req - row_lo).astype(np.uint32), ci, a, b, emin, emax,
                       reqs.vt[req], reqs.vmin[req], reqs.vmax[req])


def slice_payloads(sl: ShardSlices, lo=0, hi=None):
    """PerformQueryPayload dicts of slices [lo, hi) (tests / small batches)."""
    hi = len(sl) if hi is None else hi
    out = []
    for j in range(lo, hi):
        out.append(dict(passthrough={}, dataset_id='wgs', query_id='genome', region=f'{CONTIGS[sl.ci[j]]}:'
                        f'{sl.a[j]}-{sl.b[j]}', reference_bases='N', end_min=int(sl.end_min[j]),
                        end_max=int(sl.end_max[j]), alternate_bases=None, variant_type=VARIANT_TYPES[sl.vt[j]],
                        include_details=True, requested_granularity='record',
                        variant_min_length=int(sl.vmin[j]), variant_max_length=int(sl.vmax[j]),
                        vcf_location=LOCATION))
    return out


def shard_query_array(sl: ShardSlices, vid: int):
    """Vectorised sb_query array for a rank's slices: the same field values
    slice_payloads + engine.queries_from_payloads produce, without
    per-query Python objects.  Returns (array, keep-alive buffers)."""
    from . import _lib
    from ._lib import Query
    n = len(sl)
    arr = (Query * max(n, 1))()
    keep = []
    if n:
        regions = '\n'.join(f'{CONTIGS[c]}:{a}-{b}' for c, a, b in zip(sl.ci.tolist(), sl.a.tolist(),
                                                                        sl.b.tolist())).encode() + b'\n'
        rbuf = C.create_string_buffer(regions, len(regions))
        nl = np.flatnonzero(np.frombuffer(regions, dtype=np.uint8) == 10)
        starts = np.concatenate([[0], nl[:-1] + 1])
        lens = nl - starts
        consts = {k: C.create_string_buffer(k.encode(), len(k)) for k in ['N'] + VARIANT_TYPES}
        caddr = {k: C.addressof(v) for k, v in consts.items()}
        keep += [rbuf, consts]
        dt = np.dtype({'names': ['vcf_id', 'region', 'region_len', 'end_min', 'end_max', 'reference_bases',
                                 'reference_len', 'alternate_bases', 'alternate_len', 'variant_type',
                                 'variant_type_len', 'variant_min_length', 'variant_max_length', 'granularity',
                                 'include_details', 'include_samples', 'selected_samples_only',
                                 'strict_variant_type', 'sample_names', 'sample_names_len'],
                       'formats': ['u4', 'u8', 'u8', 'i8', 'i8', 'u8', 'u8', 'u8', 'u8', 'u8', 'u8', 'i8', 'i8',
                                   'u1', 'u1', 'u1', 'u1', 'u1', 'u8', 'u8'],
                       'offsets': [getattr(Query, f).offset for f in
                                   ['vcf_id', 'region', 'region_len', 'end_min', 'end_max', 'reference_bases',
                                    'reference_len', 'alternate_bases', 'alternate_len', 'variant_type',
                                    'variant_type_len', 'variant_min_length', 'variant_max_length', 'granularity',
                                    'include_details', 'include_samples', 'selected_samples_only',
                                    'strict_variant_type', 'sample_names', 'sample_names_len']],
                       'itemsize': C.sizeof(Query)})
        v = np.frombuffer((C.c_char * (C.sizeof(Query) * n)).from_address(C.addressof(arr)), dtype=dt)
        v['vcf_id'] = vid
        v['region'] = C.addressof(rbuf) + starts
        v['region_len'] = lens
        v['end_min'] = sl.end_min
        v['end_max'] = sl.end_max
        v['reference_bases'] = caddr['N']
        v['reference_len'] = 1
        v['alternate_bases'] = 0
        v['alternate_len'] = 0
        vt_addr = np.array([caddr[k] for k in VARIANT_TYPES], dtype=np.uint64)
        vt_len = np.array([len(k) for k in VARIANT_TYPES], dtype=np.uint64)
        v['variant_type'] = vt_addr[sl.vt]
        v['variant_type_len'] = vt_len[sl.vt]
        v['variant_min_length'] = sl.vmin
        v['variant_max_length'] = sl.vmax
        v['granularity'] = _lib.SB_GRAN['record']
        v['include_details'] = 1
        v['include_samples'] = 0
        v['selected_samples_only'] = 0
        v['strict_variant_type'] = 0
        v['sample_names'] = 0
        v['sample_names_len'] = 0
    return arr, keep


def prepare_shard_batch(store, sl: ShardSlices):
    """The rank's slices prepared on its device, request rows attached."""
    from ._lib import check, lib
    from .engine import Batch
    arr, keep = shard_query_array(sl, store.vcf_id(LOCATION))
    h = C.c_void_p()
    check(lib().sb_batch_prepare(store.handle, arr, len(sl), C.byref(h)))
    del keep
    batch = Batch(h, None, store)
    batch.set_owners(sl.req, sl.n_rows)
    return batch


def union_rows(shape: GenomeShape, sl: ShardSlices) -> int:
    """Records inside the union of the slices' [a, b] windows (each record
    counted once however many slices scan it): the unique rows a step must
    bring in from HBM at least once."""
    total = 0
    for ci in np.unique(sl.ci):
        m = sl.ci == ci
        a, b = sl.a[m].astype(np.int64), sl.b[m].astype(np.int64)
        o = np.argsort(a, kind='stable')
        a, b = a[o], b[o]
        # merge overlapping windows
        reach = np.maximum.accumulate(b)
        start = np.ones(len(a), dtype=bool)
        start[1:] = a[1:] > reach[:-1] + 1
        ids = np.cumsum(start) - 1
        ua = a[start]
        ub = np.zeros(len(ua), dtype=np.int64)
        np.maximum.at(ub, ids, b)
        pos = shape.gen(int(ci)).positions().astype(np.int64)
        total += int((np.searchsorted(pos, ub, side='right') - np.searchsorted(pos, ua, side='left')).sum())
    return total


def first_rank_of_rows(shape: GenomeShape, reqs: Requests, world: int, sl: ShardSlices) -> np.ndarray:
    """Rank holding the first slice of each of the window's request rows (the
    request's host-facing rank in ResultExchange 'first' mode)."""
    rows = sl.row_lo + np.arange(sl.n_rows)
    return rank_of_slices(shape, world, reqs.ci[rows], reqs.start[rows] + 1)


def shard_record_base(shape: GenomeShape, world: int, rank: int) -> int:
    """Global record index (contig order) of the first record of rank's shard
    store: shard record i is global record base + i (its pieces are
    consecutive in that order)."""
    return shape.plan(world).record_base(rank, 0)


@dataclass
class ShardRequests:
    """The sub-requests one rank answers (request batch): row w = request
    row_lo + w; its slices on this rank are slice indices [k0, k1) of the
    request's splitQuery slices, i.e. the sub-request [start_min + 10000 k0,
    min(start_max, start_min + 10000 k1 - 1)] (end bounds unchanged)."""
    row_lo: int
    n_rows: int
    ci: np.ndarray
    start_min: np.ndarray
    start_max: np.ndarray   # < start_min: no slice of the request on this rank
    end_min: np.ndarray
    end_max: np.ndarray
    vt: np.ndarray
    vmin: np.ndarray
    vmax: np.ndarray

    def __len__(self):
        return self.n_rows


def shard_requests(shape: GenomeShape, reqs: Requests, world: int, rank: int) -> ShardRequests:
    """Vectorised: each request's slices whose first base is in rank's core
    [cuts[rank], cuts[rank + 1]) form one run of slice indices.  Requests are
    ordered by (contig, start), so the rank's rows are one range and only the
    rows of the two cut contigs can lose slices (the others keep every slice:
    their columns are views)."""
    cuts = shape.cuts(world)
    (c0, p0), (c1, p1) = cuts[rank], cuts[rank + 1]
    r0 = int(np.searchsorted(reqs.ci, c0, side='left'))
    r1 = int(np.searchsorted(reqs.ci, c1, side='right'))
    ci = reqs.ci[r0:r1]
    smin = reqs.start[r0:r1] + 1
    smax = smin + reqs.width[r0:r1]
    n = len(smin)
    e0 = int(np.searchsorted(ci, c0, side='right'))  # rows [0, e0): contig c0
    s1 = int(np.searchsorted(ci, c1, side='left'))   # rows [s1, n): contig c1
    plan = shape.plan(world)
    segs = [(0, n)] if c0 == c1 else [(0, e0), (s1, n)]
    cut = []  # (x0, has, a, b) of each cut contig's rows: the plan's splitQuery cut
    for x0, x1 in segs:
        if x1 <= x0:
            continue
        aa, bb = plan.slice_runs(rank, 0, ci[x0:x1], smin[x0:x1], smax[x0:x1])
        cut.append((x0, bb >= aa, aa, bb))
    # the first and last rows with a slice here (rows between the cut contigs have all of theirs)
    firsts, lasts = [], []
    for x0, has, _, _ in cut:
        if has.any():
            firsts.append(x0 + int(np.argmax(has)))
            lasts.append(x0 + len(has) - int(np.argmax(has[::-1])))
    if e0 < s1 and c0 != c1:
        firsts.append(e0)
        lasts.append(s1)
    if not firsts:
        e = np.zeros(0, dtype=np.int64)
        return ShardRequests(0, 0, e, e, e, e, e, e, e, e)
    lo, hi = min(firsts), max(lasts)
    a, b = smin[lo:hi], smax[lo:hi]
    changed = [(x0, aa, bb) for x0, _, aa, bb in cut
               if not (np.array_equal(aa, smin[x0:x0 + len(aa)]) and np.array_equal(bb, smax[x0:x0 + len(bb)]))]
    if changed:
        a, b = a.copy(), b.copy()
        for x0, aa, bb in changed:
            y0, y1 = max(x0, lo), min(x0 + len(aa), hi)
            if y1 > y0:
                a[y0 - lo:y1 - lo] = aa[y0 - x0:y1 - x0]
                b[y0 - lo:y1 - lo] = bb[y0 - x0:y1 - x0]
    w = slice(r0 + lo, r0 + hi)
    return ShardRequests(r0 + lo, hi - lo, ci[lo:hi], a, b, smin[lo:hi], smax[lo:hi], reqs.vt[w], reqs.vmin[w],
                         reqs.vmax[w])


def shard_rows(shape: GenomeShape, reqs: Requests, world: int, rank: int) -> tuple[int, int]:
    """Rows [lo, hi) of the requests with at least one slice on rank (the
    ShardRequests row range): requests are ordered by (contig, start), so
    only the rows of the two cut contigs go through the plan's splitQuery
    cut; the library cuts every row itself (sb_requests_prepare_beacon)."""
    cuts = shape.cuts(world)
    (c0, _), (c1, _) = cuts[rank], cuts[rank + 1]
    r0 = int(np.searchsorted(reqs.ci, c0, side='left'))
    r1 = int(np.searchsorted(reqs.ci, c1, side='right'))
    ci = reqs.ci[r0:r1]
    n = len(ci)
    e0 = int(np.searchsorted(ci, c0, side='right'))
    s1 = int(np.searchsorted(ci, c1, side='left'))
    plan = shape.plan(world)
    firsts, lasts = [], []

    def has(x0, x1):  # rows [x0, x1) of the cut contig's rows: a slice on rank?
        smin = reqs.start[r0 + x0:r0 + x1] + 1
        aa, bb = plan.slice_runs(rank, 0, ci[x0:x1], smin, smin + reqs.width[r0 + x0:r0 + x1])
        return bb >= aa

    for x0, x1 in ([(0, n)] if c0 == c1 else [(0, e0), (s1, n)]):
        if x1 <= x0:
            continue
        # only the first and the last row with a slice matter: grow a window
        # from each end (a pipelined caller prepares ~125 k-row chunks, and
        # the whole cut contig through slice_runs cost ~0.3 ms per chunk)
        k, f = 64, None
        while f is None:
            hh = has(x0, min(x1, x0 + k))
            if hh.any():
                f = x0 + int(np.argmax(hh))
            elif x0 + k >= x1:
                break
            k *= 4
        if f is None:
            continue
        k, l = 64, None
        while l is None:
            a = max(f, x1 - k)
            hh = has(a, x1)
            if hh.any():
                l = a + len(hh) - int(np.argmax(hh[::-1]))
            k *= 4
        firsts.append(f)
        lasts.append(l)
    if e0 < s1 and c0 != c1:
        firsts.append(e0)
        lasts.append(s1)
    if not firsts:
        return r0, r0
    return r0 + min(firsts), r0 + max(lasts)


def prepare_beacon_shard(store, shape: GenomeShape, reqs: Requests, world: int, rank: int, rows=None):
    """The rank's request batch straight from the Beacon request columns:
    (row_lo, n_rows, RequestBatch).  The library builds each request's
    SplitQueryPayload and cuts it to the rank's core (the plan's
    sb_shard_core) while packing -- the same batch as prepare_shard_requests
    over shard_requests, with no per-request numpy work here."""
    from .requests import RequestBatch, beacon_requests
    lo, hi = rows if rows is not None else shard_rows(shape, reqs, world, rank)
    n = hi - lo
    cache = store.__dict__.setdefault('_genome_cmap', {})
    cmap = cache.get(LOCATION)
    if cmap is None:
        at = {c: i for i, c in enumerate(store.contigs(LOCATION))}
        cmap = cache[LOCATION] = np.array([at.get(c, 0xffffffff) for c in CONTIGS], dtype=np.uint32)
    q, keep = beacon_requests(
        n, vcf_id=store.vcf_id(LOCATION), contig=reqs.ci[lo:hi], contig_map=cmap, start=reqs.start[lo:hi],
        end=reqs.end[lo:hi], reference='N', alternate=None, variant_type=VARIANT_TYPES,
        variant_type_code=reqs.vt[lo:hi], variant_min_length=reqs.vmin[lo:hi], variant_max_length=reqs.vmax[lo:hi],
        granularity='record', include_details=True)
    batch = RequestBatch(store, q, n, core=shape.plan(world).core(rank, 0))
    del keep
    return lo, n, batch


def prepare_shard_requests(store, sr: ShardRequests):
    """The rank's request batch (sbeacon.requests.RequestBatch)."""
    from .requests import RequestBatch, request_columns
    names = store.contigs(LOCATION)
    at = {c: i for i, c in enumerate(names)}
    cmap = np.array([at.get(c, 0xffffffff) for c in CONTIGS], dtype=np.uint32)
    arr, keep = request_columns(
        sr.n_rows, vcf_id=store.vcf_id(LOCATION), contig=cmap[sr.ci] if sr.n_rows else np.zeros(0, np.uint32),
        start_min=sr.start_min, start_max=sr.start_max, end_min=sr.end_min, end_max=sr.end_max,
        reference=('N',), alternate=(None,), variant_type=VARIANT_TYPES, variant_type_code=sr.vt,
        variant_min_length=sr.vmin, variant_max_length=sr.vmax, granularity='record', include_details=1)
    batch = RequestBatch(store, arr, sr.n_rows)
    del keep
    return batch
