#!/usr/bin/env python3
"""Compare the packed chain kernel against the chain-sequential one on the
chain test's payloads; print the first differing slices."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'), REPO, os.path.join(REPO, 'tests')]


def main():
    import tempfile
    import test_gpu_chains as T
    from sbeacon import synth
    from sbeacon.engine import Store
    d = tempfile.mkdtemp()
    a, b = os.path.join(d, 'a.vcf'), os.path.join(d, 'b.vcf')
    synth.make_fixture(a, n_records=20000, n_samples=8, seed=21, quirks=False)
    synth.make_fixture(b, n_records=12000, n_samples=8, seed=22, quirks=True)
    two = {'a.vcf': a, 'b.vcf': b}
    store = Store.build(list(two.items()), device=0)
    pls = T._payloads(two)
    got = store.query(pls)
    os.environ['SBEACON_CHAIN_KERNEL'] = 'seq'
    ref = store.query(pls)
    print('hits', got.stats()['hits'], ref.stats()['hits'])
    n = 0
    for i, p in enumerate(pls):
        g, r = got.view(i), ref.view(i)
        if (g.error, g.exists, g.call_count, g.all_alleles_count, g.n_variants) != (r.error, r.exists, r.call_count, r.all_alleles_count, r.n_variants):
            n += 1
            if n <= 12:
                gv = set(got.hits(i)); rv = set(ref.hits(i))
                print(i, p['region'], p['variant_type'], p['vcf_location'], (g.error, g.exists, g.call_count, g.n_variants),
                      (r.error, r.exists, r.call_count, r.n_variants), 'missing', sorted(rv - gv)[:4], 'extra', sorted(gv - rv)[:4])
    print('differing slices', n, 'of', len(pls))


if __name__ == '__main__':
    main()
