"""Pin the C oracle (oracle/sbeacon_oracle.c) to the reference goldens.

The goldens were produced by running the reference performQuery modules
themselves (tests/golden/make_goldens.py); the oracle must reproduce every
response and every exception class bit for bit.
"""
import os

import pytest

from conftest import FIXTURES, normalise

pytestmark = pytest.mark.filterwarnings('ignore')


@pytest.fixture(scope='module')
def oracles():
    from oracle.oracle import OracleVcf
    return {n: OracleVcf(os.path.join(FIXTURES, n + '.vcf')) for n in ('tiny22', 'quirk22')}


def test_golden_inventory(goldens):
    kinds = {(c['fixture'], c['oracle'], c['error']) for c in goldens}
    assert ('tiny22', 'reference', None) in kinds
    assert ('tiny22', 'reference', 'UnboundLocalError') in kinds
    assert ('quirk22', 'reference', 'IndexError') in kinds
    assert ('tiny22', 'patched-oracle', None) in kinds
    assert len(goldens) > 1000


def test_oracle_matches_reference_goldens(goldens, oracles):
    bad = []
    for i, c in enumerate(goldens):
        o = oracles[c['fixture']]
        try:
            got, err = o.perform_query(c['payload'], patched=c['oracle'] == 'patched-oracle'), None
        except Exception as e:  # noqa: BLE001 - the exception class is the contract
            got, err = None, type(e).__name__
        if err != c['error']:
            bad.append((i, 'error', err, c['error']))
        elif got is not None and normalise(got) != normalise(c['response']):
            bad.append((i, 'response'))
    assert not bad, bad[:5]


def test_oracle_matches_general_goldens(general_goldens):
    """General records (> 64 ALTs, AC / AN past int32 / int64 up to 4300
    digits, GT fallbacks with ploidy > 3, alleles >= 8 whose variants come in
    CPython set order, huge GT tokens): the oracle against the reference."""
    from oracle.oracle import OracleVcf
    o = OracleVcf(os.path.join(FIXTURES, 'general22.vcf'))
    kinds = {c['error'] for c in general_goldens}
    assert {None, 'IndexError', 'ValueError'} <= kinds
    assert any(isinstance((c['response'] or {}).get('call_count'), dict) for c in general_goldens)
    bad = []
    for i, c in enumerate(general_goldens):
        try:
            got, err = o.perform_query(c['payload'], patched=c['oracle'] == 'patched-oracle'), None
        except Exception as e:  # noqa: BLE001
            got, err = None, type(e).__name__
        if err != c['error']:
            bad.append((i, 'error', err, c['error']))
        elif got is not None and normalise(got) != normalise(c['response']):
            bad.append((i, 'response'))
    assert not bad, bad[:5]


def test_oracle_region_count(oracles):
    o = oracles['tiny22']
    assert o.records_in_region('22:1-10') == 0
    assert o.records_in_region('22:1-100000000') == o.n_records
