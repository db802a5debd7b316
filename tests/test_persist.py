"""Persisted stores on the CPU (host-only stores, SB_HOST_ONLY): save and
re-open give the same host side (contigs, request plans), a changed source
file makes the saved store stale (SB_ESTALE naming it), and a StoreSet
re-ingests only the groups whose files changed.  The device image round
trip is tests/test_gpu_persist.py."""
import os
import random
import shutil

import pytest

from conftest import FIXTURES

HOST_ONLY = -1


def _copy(tmp_path, name):
    p = tmp_path / name
    shutil.copy(os.path.join(FIXTURES, name), p)
    return str(p)


def _plan_stats(store, loc, seed=4):
    from payload_gen import read_records
    from sbeacon.requests import RequestBatch, requests_from_split_payloads
    recs, _ = read_records(store.paths[loc])
    rng = random.Random(seed)
    sps = []
    for _ in range(200):
        pos = recs[rng.randrange(len(recs))][1]
        w = rng.choice([0, 10, 5000, 25000, 300000])
        sps.append(dict(passthrough={}, dataset_id='d', query_id='q', reference_bases='N', start_min=max(1, pos - w),
                        start_max=pos + w, end_min=0, end_max=10**9, alternate_bases=None,
                        variant_type=rng.choice(['DEL', 'INS', 'DUP', 'CNV', None]), include_datasets='HIT',
                        vcf_locations={loc: '22'}, vcf_groups=[], requested_granularity='record',
                        variant_min_length=0, variant_max_length=-1))
    arr, keep, owners = requests_from_split_payloads(store, sps)
    b = RequestBatch(store, arr, len(owners))
    st = b.stats()
    b.free()
    return st


def test_host_only_store_round_trip(tmp_path):
    from sbeacon.engine import Store
    src = _copy(tmp_path, 'tiny22.vcf')
    st = Store.build([('tiny22.vcf', src)], device=HOST_ONLY)
    st.save(str(tmp_path / 'store'))
    assert os.path.getsize(tmp_path / 'store' / 'device.bin') == 0
    again = Store.open(str(tmp_path / 'store'), device=HOST_ONLY)
    assert again.locations == st.locations and again.paths == st.paths
    assert again.contigs('tiny22.vcf') == st.contigs('tiny22.vcf')
    a, b = _plan_stats(st, 'tiny22.vcf'), _plan_stats(again, 'tiny22.vcf')
    assert a == b and a['chains'] > 0
    # a host-only image cannot serve a device
    from sbeacon._lib import SbError
    with pytest.raises(SbError):
        Store.open(str(tmp_path / 'store'), device=0)


def test_changed_source_makes_the_store_stale(tmp_path):
    from sbeacon.engine import StaleStore, Store
    src = _copy(tmp_path, 'tiny22.vcf')
    st = Store.build([('tiny22.vcf', src)], device=HOST_ONLY)
    st.save(str(tmp_path / 'store'))
    with open(src, 'ab') as f:  # one more record
        f.write(b'22\t99999999\t.\tA\tC\t.\t.\tAC=1;AN=2\tGT\t0|1\n')
    with pytest.raises(StaleStore) as e:
        Store.open(str(tmp_path / 'store'), device=HOST_ONLY)
    assert e.value.paths == [src]


def test_store_set_rebuilds_only_changed_groups(tmp_path):
    from sbeacon.persist import StoreSet
    a = _copy(tmp_path, 'tiny22.vcf')
    b = _copy(tmp_path, 'quirk22.vcf')
    groups = {'ds_a': [('tiny22.vcf', a)], 'ds_b': [('quirk22.vcf', b)]}
    ss = StoreSet(str(tmp_path / 'stores'))
    ss.load(groups, device=HOST_ONLY)
    assert sorted(ss.rebuilt) == ['ds_a', 'ds_b'] and ss.opened == []
    ss.load(groups, device=HOST_ONLY)
    assert ss.rebuilt == [] and sorted(ss.opened) == ['ds_a', 'ds_b']
    text = open(b, 'rb').read()
    with open(b, 'wb') as f:  # the same size, other bytes: the sample hash catches it
        f.write(text.replace(b'AN=', b'AM=', 1))
    ss.load(groups, device=HOST_ONLY)
    assert ss.rebuilt == ['ds_b'] and ss.opened == ['ds_a']


def test_store_set_rebuilds_a_repointed_location(tmp_path):
    """A location re-pointed to another file (the old one unchanged, so its
    saved fingerprint still matches) is a rebuild, not a re-open of the old
    file's data."""
    from sbeacon.persist import StoreSet
    a = _copy(tmp_path, 'tiny22.vcf')
    other = str(tmp_path / 'tiny22_v2.vcf')
    text = open(a, 'rb').read()
    with open(other, 'wb') as f:
        f.write(text.replace(b'AN=', b'AM=', 1))
    ss = StoreSet(str(tmp_path / 'stores'))
    ss.load({'ds': [('tiny22.vcf', a)]}, device=HOST_ONLY)
    assert ss.rebuilt == ['ds']
    ss.load({'ds': [('tiny22.vcf', other)]}, device=HOST_ONLY)
    assert ss.rebuilt == ['ds'] and ss.opened == []
    assert ss.stores['ds'].paths['tiny22.vcf'] == other
    ss.load({'ds': [('tiny22.vcf', other)]}, device=HOST_ONLY)
    assert ss.rebuilt == [] and ss.opened == ['ds']


def test_save_replaces_the_directory_whole(tmp_path):
    """sb_store_save writes into DIR.tmp and renames it into place (ADVICE
    round 4): a second save over the first leaves one complete directory and
    no temporary or previous copy; the re-opened store is the saved one."""
    from sbeacon.engine import Store
    src = _copy(tmp_path, 'tiny22.vcf')
    st = Store.build([('tiny22.vcf', src)], device=HOST_ONLY)
    d = str(tmp_path / 'store')
    st.save(d)
    st.save(d + '/')
    assert sorted(os.listdir(d)) == ['device.bin', 'host.bin', 'manifest.json', 'sbeacon.json']
    assert not os.path.exists(d + '.tmp') and not os.path.exists(d + '.old')
    again = Store.open(d, device=HOST_ONLY)
    assert again.contigs('tiny22.vcf') == st.contigs('tiny22.vcf')
