"""Config 5 (gnomAD-shape sites + a carrier bit-matrix; sbeacon/gnomad.py).

CPU: the synthetic carrier planes are the genotypes the generator renders as
GT text (the set search_variants.py:233-236 collects), and
sb_builder_attach_carriers rejects inputs the reference could not answer from
a carrier matrix.  GPU: a shard store built from sites text + attached planes
answers AC/AN aggregation and sample-subset slices exactly as the C oracle
does on the same records' full GT text, and exactly as a store ingested from
that GT text."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import normalise


def _planes_from_text(text: str, words: int):
    rows = []
    for line in text.splitlines():
        f = line.split('\t')
        for k in range(len(f[4].split(','))):
            row = np.zeros(words, dtype=np.uint64)
            for s, gt in enumerate(f[9:]):
                if str(k + 1) in re.split(r'[|/]', gt):
                    row[s >> 6] |= np.uint64(1) << np.uint64(s & 63)
            rows.append(row)
    return np.array(rows, dtype=np.uint64).reshape(-1, words)


@pytest.mark.parametrize('an', [0, 152_312])
def test_carrier_planes_are_the_gt_text(an):
    from sbeacon.workload import SyntheticVcf
    g = SyntheticVcf(seed=5, n_records=1500, n_samples=130, start=100, mean_gap=4.0, contig='7')
    if an:
        g.set_an_sites(an)
    planes = g.carrier_planes(threads=4)
    text = g.records(0, 1500).decode()
    assert np.array_equal(planes, _planes_from_text(text, 3))
    if an:
        assert f'AN={an};' in text
    # chunked generation into a preallocated array gives the same rows
    out = np.empty_like(planes)
    n0 = g.alt_rows(0, 700)
    g.carrier_planes(0, 700, 2, out=out[:n0])
    g.carrier_planes(700, 1500, 3, out=out[n0:])
    assert np.array_equal(out, planes)


def _builder(text: bytes):
    from sbeacon._lib import BuildOpts, lib
    L = lib()
    b = C.c_void_p()
    assert L.sb_builder_new(C.byref(BuildOpts(0, 2)), C.byref(b)) == 0
    vid = C.c_uint32()
    assert L.sb_builder_begin_vcf(b, b'x.vcf', 5, C.byref(vid)) == 0
    assert L.sb_builder_add_text(b, vid.value, text, len(text)) == 0
    return L, b, vid.value


def _attach(L, b, vid, names, planes):
    nb = [n.encode() for n in names]
    arr = (C.c_char_p * len(nb))(*nb)
    lens = (C.c_uint32 * len(nb))(*[len(x) for x in nb])
    planes = np.ascontiguousarray(planes, dtype=np.uint64)
    return L.sb_builder_attach_carriers(b, vid, arr, lens, len(nb), planes.ctypes.data, planes.shape[0])


def test_attach_carriers_validation():
    from sbeacon._lib import lib
    from sbeacon.workload import SyntheticVcf
    g = SyntheticVcf(seed=6, n_records=200, n_samples=70, start=100, mean_gap=4.0, contig='2')
    text = g.header(sites_only=True) + g.records(0, 200, sites_only=True)
    planes = g.carrier_planes()
    names = g.sample_names()
    L, b, vid = _builder(text)
    try:
        assert _attach(L, b, vid, names, planes[:-1]) < 0  # one row short
        assert b'rows' in lib().sb_last_error()
        assert _attach(L, b, vid, names, planes) == 0
        assert _attach(L, b, vid, names, planes) < 0  # already has samples
    finally:
        L.sb_builder_free(b)
    # a record without AN: the reference would count GT tokens (:244-250)
    lines = text.decode().split('\n')
    i = next(k for k, ln in enumerate(lines) if ln and not ln.startswith('#'))
    lines[i] = lines[i].replace(';AN=', ';XN=')
    L, b, vid = _builder('\n'.join(lines).encode())
    try:
        assert _attach(L, b, vid, names, planes) < 0
        assert b'AC and AN' in lib().sb_last_error()
    finally:
        L.sb_builder_free(b)


def test_config5_slices_stay_in_their_shard():
    from sbeacon.genome import rank_of_slices
    from sbeacon.gnomad import GnomadShape, config5_slices
    shape = GnomadShape(n_total=400_000, n_samples=64)
    for r in (0, 3, 7):
        sl = config5_slices(shape, r, 500)
        assert sl.n_requests > 400 and len(sl) >= sl.n_requests
        assert (rank_of_slices(shape, 8, sl.ci, sl.a) == r).all()
        assert set(np.unique(sl.kind)) == {0, 1}
        assert ((sl.b - sl.a) < 10000).all()


@pytest.fixture(scope='module')
def small_gnomad(tmp_path_factory):
    from sbeacon.gnomad import GnomadShape, config5_slices, sample_subsets, slice_payloads
    shape = GnomadShape(n_total=2_000_000, n_samples=100)
    sl = config5_slices(shape, 0, 1500)
    subsets = sample_subsets(100, shape.sample_names(), n=8)
    payloads = slice_payloads(sl, subsets)
    path = str(tmp_path_factory.mktemp('gnomad') / 'shard0.vcf')
    with open(path, 'wb') as f:
        for k, (ci, lo, hi) in enumerate(shape.shard_pieces(8, 0)):
            g = shape.gen(ci)
            if k == 0:
                f.write(g.header(sites_only=False))
            f.write(g.records(lo, hi, sites_only=False, threads=4))
    return shape, sl, payloads, path


@pytest.mark.gpu
def test_attached_carriers_match_oracle_and_gt_store(small_gnomad):
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    from sbeacon.gnomad import LOCATION
    shape, sl, payloads, path = small_gnomad
    store = shape.build_gnomad_store(0, device=0, threads=4)
    rs = store.query(payloads)
    orc = OracleVcf(path)
    exp = orc.perform_query_batch(payloads)
    gt_store = Store.build([(LOCATION, path)], device=0)
    rs2 = gt_store.query(payloads)
    n_samp = 0
    for i, (p, e) in enumerate(zip(payloads, exp)):
        got = normalise(rs.response(i).dump())
        assert got == normalise(e), (p['region'], p['passthrough'].keys())
        assert normalise(rs2.response(i).dump()) == got
        n_samp += bool(got['sample_indices'])
    assert n_samp > 150  # the sample-subset path was exercised


@pytest.mark.gpu
def test_flat_carrier_rows_2504_samples(tmp_path):
    """40-word carrier rows (2,504 samples) take the flattened sample path
    (8 rows = 5 full-wave loads, query_kernels.hip scan_slice); every
    includeSamples / sample-subset response equals the oracle's on the GT text."""
    import random

    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    from sbeacon.workload import SyntheticVcf, config2_requests, requests_to_payloads
    gen = SyntheticVcf(seed=41, n_records=3000, n_samples=2504, mean_gap=60.0)
    path = str(tmp_path / 'wide.vcf')
    gen.write(path, sites_only=False)
    store = Store.build([('w.vcf', path)], device=0)
    reqs = config2_requests(gen, n_range=200, n_point=0, seed=78)
    payloads, _ = requests_to_payloads(reqs, vcf_location='w.vcf', chrom='22')
    names = gen.sample_names()
    rng = random.Random(9)
    for p in payloads:
        if rng.random() < 0.5:
            p['passthrough'] = {'includeSamples': True}
        else:
            pick = rng.sample(names, rng.choice([10, 300, 2504]))
            p['passthrough'] = {'sampleNames': pick, 'selectedSamplesOnly': True, 'includeSamples': True}
        p['requested_granularity'] = 'record'
        p['include_details'] = True
    exp = OracleVcf(path).perform_query_batch(payloads)
    rs = store.query(payloads)
    n_samp = 0
    for i, (p, e) in enumerate(zip(payloads, exp)):
        got = normalise(rs.response(i).dump())
        assert got == normalise(e), (p['region'], p['passthrough'].keys())
        n_samp += len(got['sample_indices']) > 64
    assert n_samp > 20  # rows past the first 64 samples were collected
