"""Slice chains on the device (chain_kernel): every 10 kb slice splitQuery cut
a variantType request into, answered by one wave per request, must equal the
C oracle per slice and the per-slice path (SBEACON_NO_CHAINS=1) bit for bit,
including the host-filled n_scanned.  Two VCFs whose slices interleave (as
split_payloads emits them), requests longer than a chain (kChainMax slices),
short last slices, every variantType, length bounds, END brackets, and
slices that must stay on the per-slice path (boolean / count granularities,
include_details False, a window holding an AC-less record = VT_SLOW)."""
import random

import pytest

from conftest import normalise

pytestmark = pytest.mark.gpu

VTYPES = ['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV', 'SNP']


def _requests(rng, span_lo, span_hi, n):
    out = []
    for _ in range(n):
        width = rng.choice([1, 50, 9999, 10000, 10001, 25000, 99999, 180000, 330000, 420000])
        s = rng.randrange(span_lo - 20000, span_hi)
        smin, smax = s + 1, s + width + 1
        u = rng.random()
        if u < 0.6:
            emin, emax = smin, smax
        elif u < 0.8:
            emin, emax = 0, 10**9
        else:
            emin = smin + rng.randrange(0, width + 1)
            emax = emin + rng.randrange(0, 3000)
        if rng.random() < 0.7:
            vmin, vmax = 0, -1
        else:
            vmin, vmax = rng.choice([0, 1, 2, 3]), rng.choice([-1, 1, 2, 5, 100])
        g = rng.random()
        gran, inc = ('record', 'HIT') if g < 0.8 else rng.choice([('boolean', 'HIT'), ('count', 'HIT'),
                                                                    ('record', 'NONE')])
        out.append(dict(passthrough={}, dataset_id='ds', query_id='c', reference_bases='N', start_min=smin,
                        start_max=smax, end_min=emin, end_max=emax, alternate_bases=None,
                        variant_type=rng.choice(VTYPES), include_datasets=inc, requested_granularity=gran,
                        variant_min_length=vmin, variant_max_length=vmax, vcf_groups=[]))
    return out


@pytest.fixture(scope='module')
def two_vcfs(tmp_path_factory):
    from sbeacon import synth
    d = tmp_path_factory.mktemp('chains')
    a, b = str(d / 'a.vcf'), str(d / 'b.vcf')
    synth.make_fixture(a, n_records=20000, n_samples=8, seed=21, quirks=False)
    synth.make_fixture(b, n_records=12000, n_samples=8, seed=22, quirks=True)
    return {'a.vcf': a, 'b.vcf': b}


def _payloads(two_vcfs):
    from sbeacon.split_query import split_payloads
    rng = random.Random(2024)
    pls = []
    for sp in _requests(rng, 16050075, 16050075 + 640000, 260):
        sp['vcf_locations'] = {'a.vcf': '22', 'b.vcf': '22'}
        pls += split_payloads(sp)
    return pls


def test_chains_vs_oracle_and_per_slice_path(two_vcfs, monkeypatch):
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    store = Store.build(list(two_vcfs.items()), device=0)
    pls = _payloads(two_vcfs)
    assert len(pls) > 2000
    got = store.query(pls)
    monkeypatch.setenv('SBEACON_NO_CHAINS', '1')
    ref = store.query(pls)
    monkeypatch.delenv('SBEACON_NO_CHAINS')
    assert got.stats()['records_scanned'] == ref.stats()['records_scanned']
    assert got.stats()['hits'] == ref.stats()['hits'] > 0
    orcs = {k: OracleVcf(v) for k, v in two_vcfs.items()}  # GT text: the AC-less fallback counts it
    exp = [None] * len(pls)
    for loc, orc in orcs.items():
        idx = [i for i, p in enumerate(pls) if p['vcf_location'] == loc]
        for i, e in zip(idx, orc.perform_query_batch([pls[i] for i in idx], patched=True)):
            exp[i] = e
    st = got.stats()
    assert st['chained_slices'] > len(pls) // 2 and ref.stats()['chained_slices'] == 0
    n_exists = 0
    gr, rr = got.responses(), ref.responses()
    for p, g, r, e in zip(pls, gr, rr, exp):
        if isinstance(e, type):
            assert isinstance(g, e) and isinstance(r, e), p
            continue
        assert not isinstance(g, Exception) and not isinstance(r, Exception), (p, g, r)
        assert g.dump() == r.dump(), p
        assert normalise(g.dump()) == normalise(e), p
        n_exists += bool(e['exists'])
    assert n_exists > 200
