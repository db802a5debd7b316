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
        counts, messages, per_range = summarise_dataset(store, ds, locs, abs_max=20_000)
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
