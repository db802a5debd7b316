"""The dataset ingest pipeline on the device (summariseVcf -> summariseSlice
counts + region files -> initDuplicateVariantSearch range splits ->
duplicateVariantSearch), checked stage by stage against the C restatements:
slice counts and region files vs oracle/summarise_oracle.c, range splits by
construction (tests/test_range_splits.py pins them to the reference), per-range
distinct counts vs orc_dedup_count."""
import pytest

pytestmark = pytest.mark.gpu


def test_summarise_dataset_pipeline(tmp_path):
    from oracle.oracle import OracleBgzf, dedup_count
    from sbeacon.engine import Store
    from sbeacon.summarise import summarise_dataset
    from sbeacon.summarise_vcf import plan_slices
    from sbeacon.workload import SyntheticVcf, write_bgzf
    # sparse positions: region files split on POS gaps > 100,000, so the
    # contig is cut into several ranges
    pool = SyntheticVcf(seed=4, n_records=4000, n_samples=6, mean_gap=40000)
    datasets = [(f'ds{d}', [(f's3://bkt/ds{d}/part{k}.vcf.gz', pool.member(400 + 10 * d + k, share=0.7))
                            for k in (0, 1)]) for d in range(2)]
    files = []
    for ds, parts in datasets:
        for loc, gen in parts:
            path = str(tmp_path / (loc.replace('/', '_') + '.gz'))
            write_bgzf(path, gen.chunks(threads=4), threads=4)
            files.append((ds, loc, path))
    store = Store.build([(loc, path) for _, loc, path in files], device=0)
    for ds, parts in datasets:
        locs = [loc for loc, _ in parts]
        # a small abs_max so the contig is cut into several ranges
        # the intended-range extension (strict=False) against the intended-range oracle
        counts, messages, per_range = summarise_dataset(store, ds, locs, abs_max=20_000, strict=False)
        assert len(messages) > 3
        exp_v = exp_c = 0
        for loc in locs:
            path = next(p for d, l, p in files if l == loc)
            o = OracleBgzf(path)
            for a, b in plan_slices(store, loc):
                e = o.summarise_slice(a, b)
                exp_v += e['numVariants']
                exp_c += e['numCalls']
        assert (counts['variantCount'], counts['callCount']) == (exp_v, exp_c)
        texts = [b''.join(gen.chunks()) for _, gen in parts]
        for m, got in zip(messages, per_range):
            assert got == dedup_count(texts, m['contig'], m['rangeStart'], m['rangeEnd']), m
        assert counts['uniqueVariants'] == sum(per_range)


def test_region_files_gzip_and_strict_dedup(tmp_path, monkeypatch):
    """Region files as the reference stores them (gzip members, level 9) and
    duplicateVariantSearch in the reference-exact mode: every target file is
    read by ReadVcfData::getVcfData's loop over the REFERENCE gzip reader
    (oracle/_ref, built from lambda/shared/gzip/gzip.cpp); the device count of
    each range must equal |union of those key sets|, reference throws included."""
    import zlib
    from oracle import ref
    from test_ref_pinned import deflate9, gzip_payload
    if ref.lib() is None:
        pytest.skip('oracle/_ref missing')
    # every (job, file) pair's entries from the file profile are also read by
    # the reader walk and compared (the library raises on a difference)
    monkeypatch.setenv('SBEACON_STRICT_CHECK', '1')
    from sbeacon.dedup import dedup_batch, init_duplicate_variant_search
    from sbeacon.engine import Store
    from sbeacon.summarise import _single_store_registry, region_file_keys, summarise_dataset
    from sbeacon.summarise_vcf import plan_slices
    from sbeacon.workload import SyntheticVcf, write_bgzf
    pool = SyntheticVcf(seed=8, n_records=6000, n_samples=4, mean_gap=25000)
    parts = [(f's3://bkt/dsS/p{k}.vcf.gz', pool.member(800 + k, share=0.6)) for k in (0, 1)]
    paths = []
    for loc, gen in parts:
        path = str(tmp_path / (loc.replace('/', '_') + '.gz'))
        write_bgzf(path, gen.chunks(threads=4), threads=4)
        paths.append((loc, path))
    locs = [l for l, _ in paths]
    store = Store.build(paths, device=0)
    gz_files, refs, keys = {}, {}, []
    for loc in locs:
        slices = plan_slices(store, loc)
        keys += region_file_keys(store, loc, slices, refs)
        raw = store.region_files([(loc, a, b) for a, b in slices], with_data=True)
        gz = store.region_files([(loc, a, b) for a, b in slices], with_data='gzip')
        for (a, b), fr, fg in zip(slices, raw, gz):
            assert len(fr) == len(fg)
            for i, (x, y) in enumerate(zip(fr, fg)):
                assert zlib.decompress(y['data'], 16 + zlib.MAX_WBITS) == x['data']
                assert gzip_payload(y['data']) == gzip_payload(ref.gzip_deflate(x['data'], 9)) \
                    == gzip_payload(deflate9(x['data']))
                gz_files[(loc, a, b, i)] = y['data']
    assert all(r in gz_files for r in refs.values())
    reg = _single_store_registry(store)
    for abs_max in (10_000, 10**9):  # many ranges (files overlap range starts) / one range per contig
        messages = init_duplicate_variant_search('dsS', locs, keys, abs_max=abs_max)
        assert messages
        per_range = dedup_batch(messages, registry=reg, file_refs=refs)
        again = dedup_batch(messages, registry=reg, file_refs=refs)  # the region files from the store's cache
        norm = lambda rs: [r if isinstance(r, int) else type(r) for r in rs]  # noqa: E731
        assert norm(again) == norm(per_range)
        n_throw = 0
        for m, got in zip(messages, per_range):
            exp = set()
            for p in m['targetFilepaths']:
                kf = ref.region_keys(gz_files[refs[p]], m['rangeStart'], m['rangeEnd'])
                if isinstance(kf, Exception):
                    exp = kf
                    break
                exp |= set(kf)
            if isinstance(exp, Exception):
                n_throw += 1
                assert isinstance(got, RuntimeError), m
            else:
                assert got == len(exp), m
        if abs_max == 10**9:
            assert n_throw == 0
            counts, _, pr = summarise_dataset(store, 'dsS', locs, abs_max=abs_max, strict=True)
            assert counts['uniqueVariants'] == sum(pr) == sum(per_range)


def test_sns_handler_answers_the_reference_count(tmp_path):
    """The drop-in duplicateVariantSearch handler, default mode: the
    messages initDuplicateVariantSearch fans out, each delivered as an SNS
    event to dedup.lambda_handler with nothing but its keys -- each count
    equals |union of the REFERENCE reader's key sets| over the target files
    (oracle/_ref: ReadVcfData::getVcfData's loop over gzip.cpp), and a
    reference throw is the handler's exception."""
    import json
    from oracle import ref
    if ref.lib() is None:
        pytest.skip('oracle/_ref missing')
    from sbeacon import dedup, engine
    from sbeacon.engine import Store
    from sbeacon.summarise import region_file_keys
    from sbeacon.summarise_vcf import plan_slices
    from sbeacon.workload import SyntheticVcf, write_bgzf
    pool = SyntheticVcf(seed=18, n_records=5000, n_samples=4, mean_gap=20000)
    parts = [(f's3://bkt/dsH/p{k}.vcf.gz', pool.member(900 + k, share=0.6)) for k in (0, 1, 2)]
    paths = []
    for loc, gen in parts:
        path = str(tmp_path / (loc.replace('/', '_') + '.gz'))
        write_bgzf(path, gen.chunks(threads=4), threads=4)
        paths.append((loc, path))
    locs = [l for l, _ in paths]
    store = Store.build(paths, device=0)
    gz_files, refs, keys = {}, {}, []
    for loc in locs:
        slices = plan_slices(store, loc)
        keys += region_file_keys(store, loc, slices, refs)
        gz = store.region_files([(loc, a, b) for a, b in slices], with_data='gzip')
        for (a, b), fg in zip(slices, gz):
            for i, y in enumerate(fg):
                gz_files[(loc, a, b, i)] = y['data']
    # a fresh store: the handler resolves every key through its own map
    store2 = Store.build(paths, device=0)
    engine.registry.register(store2)
    try:
        n_ok = n_throw = 0
        for abs_max in (8_000, 10**9):
            tally = dedup.DuplicateTally()
            messages = dedup.init_duplicate_variant_search('dsH', locs, keys, abs_max=abs_max, tally=tally)
            assert messages
            for m in messages:
                exp = set()
                for p in m['targetFilepaths']:
                    kf = ref.region_keys(gz_files[refs[p]], m['rangeStart'], m['rangeEnd'])
                    if isinstance(kf, Exception):
                        exp = kf
                        break
                    exp |= set(kf)
                ev = {'Records': [{'Sns': {'Message': json.dumps(m)}}]}
                if isinstance(exp, Exception):
                    n_throw += 1
                    with pytest.raises(RuntimeError):
                        dedup.lambda_handler(ev, tally=tally)
                else:
                    n_ok += 1
                    r = dedup.lambda_handler(ev, tally=tally)
                    assert r['statusCode'] == 200 and r['body'] == 'Success'
                    assert r['uniqueVariants'] == len(exp), m
            # the intended-range extension stays available on request
            alt = dedup.dedup_batch(messages, strict=False)
            assert all(isinstance(x, int) for x in alt)
        assert n_ok > 5
        # a key no summary of the store writes: the message fails (the S3 download would)
        bad = dict(messages[0], targetFilepaths=[messages[0]['targetFilepaths'][0].rsplit('/', 1)[0] + '/1-2-3'])
        with pytest.raises(KeyError):
            dedup.lambda_handler({'Records': [{'Sns': {'Message': json.dumps(bad)}}]})
    finally:
        engine.registry.clear()
