"""gnomAD-shape sites workload (BASELINE.json configs[4]; SURVEY.md §8d
config 5): AC/AN aggregation and sample-subset genotype masks.

Store: ~750 M sites over contigs 1-22, X, Y (counts proportional to contig
length, as config 3), INFO ``AC``/``AN`` over a gnomAD-size cohort (every
record ``AN = 152,312``, AC drawn over it), plus a 2,504-sample genotype
carrier bit-matrix (one bit per sample per ALT) attached through
``sb_builder_attach_carriers``.  The matrix is the one the synthetic
generator renders as GT text (``SyntheticVcf.carrier_planes`` ==
GT columns of ``SyntheticVcf.records(sites_only=False)``), so the CPU oracle
reads exactly the genotypes the device holds.

Sharding: the genome is cut into ``SHARDS = 8`` record-balanced shards
(GenomeShape.cuts, 10 kb right halo), one per GPU of an 8 x MI355X node
(~94 M sites + ~30 GB of carrier planes per GPU).  Rank r answers shard r's
requests only (weak scaling: per-GPU work is fixed, no data-path
collective); requests that would straddle a shard cut are dropped when the
request set is drawn.

Requests (seed 1005), half of each kind:
  * AC/AN aggregation: ``referenceBases='N'``, ``alternateBases='N'``,
    granularity ``record``, ``includeResultsetResponses='HIT'`` over a range
    of 1-10,000 bp (``search_variants.py:170-176,195-250``);
  * sample subset: the same over 1-2,000 bp with
    ``passthrough.selectedSamplesOnly`` and ``sampleNames`` = one of 64 fixed
    subsets of 10-2,504 samples (log-uniform size), ``includeSamples``
    (``search_variants_in_samples.py:31-295``): the kernel ORs the carrier
    rows of every hit ALT and ANDs the subset mask.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .chrom_matching import CHROMOSOME_LENGTHS
from .genome import CONTIGS, GenomeShape, SPLIT_SIZE

GNOMAD_RECORDS = 750_000_000
SHARDS = 8
AN_SITES = 152_312
LOCATION = 'synthetic/gnomad-shape-sites.vcf.gz'
N_SUBSETS = 64


class GnomadShape(GenomeShape):
    def __init__(self, *, n_total: int = GNOMAD_RECORDS, seed: int = 5, n_samples: int = 2504,
                 an_sites: int = AN_SITES, shards: int = SHARDS):
        super().__init__(n_total=n_total, seed=seed, n_samples=n_samples)
        self.an_sites, self.shards = an_sites, shards

    def gen(self, ci: int):
        fresh = ci not in self._gens
        g = super().gen(ci)
        if fresh:
            g.set_an_sites(self.an_sites)
        return g

    def sample_names(self) -> list[str]:
        return self.gen(0).sample_names()

    def shard_carriers(self, rank: int, threads: int = 0) -> np.ndarray:
        """Carrier planes of shard `rank`, record-then-ALT order."""
        pieces = self.shard_pieces(self.shards, rank)
        rows = [self.gen(ci).alt_rows(lo, hi, threads) for ci, lo, hi in pieces]
        out = np.empty((sum(rows), (self.n_samples + 63) // 64), dtype=np.uint64)
        r = 0
        for (ci, lo, hi), n in zip(pieces, rows):
            self.gen(ci).carrier_planes(lo, hi, threads, out=out[r:r + n])
            r += n
        return out

    def build_gnomad_store(self, rank: int, *, device=0, threads=0, progress=None):
        from .engine import Store
        car = [self.sample_names(), self.shard_carriers(rank, threads)]
        if progress:
            progress('carriers', 0)
        src = (LOCATION, self.shard_chunks(self.shards, rank, threads=threads, progress=progress), car)
        return Store.build([src], device=device, keep_genotypes=False, n_threads=threads)


def sample_subsets(n_samples: int, names: list[str], seed: int = 1005, n: int = N_SUBSETS) -> list[str]:
    """n ','-joined sampleNames lists, sizes log-uniform in [10, n_samples]."""
    rng = np.random.default_rng(seed + 1)
    out = []
    for _ in range(n):
        k = int(round(np.exp(rng.uniform(np.log(10), np.log(n_samples)))))
        pick = rng.choice(n_samples, size=min(max(k, 10), n_samples), replace=False)
        out.append(','.join(names[i] for i in pick))
    return out


@dataclass
class GnomadSlices:
    """Shard `rank`'s slices: owning request, contig, [a, b], end bracket,
    kind (0 = AC/AN aggregation, 1 = sample subset), subset id."""
    req: np.ndarray
    ci: np.ndarray
    a: np.ndarray
    b: np.ndarray
    end_min: np.ndarray
    end_max: np.ndarray
    kind: np.ndarray
    subset: np.ndarray
    n_requests: int

    def __len__(self):
        return len(self.a)


def config5_slices(shape: GnomadShape, rank: int, n_requests: int, seed: int = 1005) -> GnomadSlices:
    """n_requests requests drawn inside shard `rank` (contig, start uniform
    over the shard's core), split into slices as splitQuery does."""
    rng = np.random.default_rng(seed * 1000 + rank)
    cuts = shape.cuts(shape.shards)
    (c0, p0), (c1, p1) = cuts[rank], cuts[rank + 1]
    # the core's extent per contig
    spans = []
    for ci in range(c0, min(c1, len(CONTIGS) - 1) + 1):
        lo_c, hi_c = shape.span(ci)
        lo = max(p0, lo_c) if ci == c0 else lo_c
        hi = (p1 - 1) if ci == c1 else hi_c
        if hi > lo:
            spans.append((ci, lo, hi))
    w = np.array([hi - lo for _, lo, hi in spans], dtype=np.float64)
    pick = rng.choice(len(spans), size=n_requests, p=w / w.sum())
    kind = (rng.random(n_requests) < 0.5).astype(np.uint8)
    width = np.where(kind == 1, rng.integers(1, 2001, n_requests), rng.integers(1, 10001, n_requests))
    sp_ci = np.array([s[0] for s in spans])
    sp_lo = np.array([s[1] for s in spans], dtype=np.int64)
    sp_hi = np.array([s[2] for s in spans], dtype=np.int64)
    ci = sp_ci[pick]
    start = (sp_lo[pick] - 1 + rng.random(n_requests) * (sp_hi[pick] - sp_lo[pick])).astype(np.int64)
    # keep requests whose last base stays inside the core (no shard straddling)
    keep = start + width + 1 <= sp_hi[pick]
    ci, start, width, kind = ci[keep], start[keep], width[keep], kind[keep]
    subset = rng.integers(0, N_SUBSETS, len(ci)).astype(np.int64)
    order = np.lexsort((start, ci))
    ci, start, width, kind, subset = ci[order], start[order], width[order], kind[order], subset[order]
    # perform_variant_search_sync + split_query (start=[s], end=[e])
    smin = start + 1
    smax = start + width + 1
    nsl = (smax - smin) // SPLIT_SIZE + 1
    req = np.repeat(np.arange(len(ci), dtype=np.int64), nsl)
    first = np.repeat(np.cumsum(nsl) - nsl, nsl)
    k = np.arange(len(req), dtype=np.int64) - first
    a = smin[req] + SPLIT_SIZE * k
    b = np.minimum(a + SPLIT_SIZE - 1, smax[req])
    return GnomadSlices(req, ci[req], a, b, smin[req], smax[req], kind[req], subset[req], len(ci))


def slice_payloads(sl: GnomadSlices, subsets: list[str], idx=None) -> list[dict]:
    """PerformQueryPayload dicts of the slices (all, or the indices `idx`)."""
    idx = range(len(sl)) if idx is None else idx
    out = []
    for j in idx:
        samp = sl.kind[j] == 1
        pt = {}
        if samp:
            pt = {'sampleNames': subsets[int(sl.subset[j]) % len(subsets)].split(','), 'selectedSamplesOnly': True,
                  'includeSamples': True}
        out.append(dict(passthrough=pt, dataset_id='gnomad', query_id='gnomad',
                        region=f'{CONTIGS[sl.ci[j]]}:{sl.a[j]}-{sl.b[j]}', reference_bases='N',
                        end_min=int(sl.end_min[j]), end_max=int(sl.end_max[j]), alternate_bases='N',
                        variant_type=None, include_details=True, requested_granularity='record',
                        variant_min_length=0, variant_max_length=-1, vcf_location=LOCATION))
    return out


def contig_length(ci: int) -> int:
    return CHROMOSOME_LENGTHS[CONTIGS[ci]]
