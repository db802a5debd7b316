"""Seeded random PerformQueryPayload generator for parity tests (no
reference dependency; mirrors the mix used by tests/golden/make_goldens.py)."""
import random

VTYPES = ['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV', 'SNP', None]
GRANS = ['boolean', 'count', 'aggregated', 'record']


def read_records(path):
    recs, names = [], []
    with open(path) as f:
        for line in f:
            if line.startswith('##'):
                continue
            if line.startswith('#CHROM'):
                names = line.rstrip('\n').split('\t')[9:]
                continue
            c = line.rstrip('\n').split('\t', 5)
            recs.append((c[0], int(c[1]), c[3], c[4].split(',')))
    return recs, names


def random_payload(rng: random.Random, recs, names, vcf_location, *, alt_none_p=0.2, samples_p=0.55):
    chrom, pos, ref, alts = recs[rng.randrange(len(recs))]
    width = rng.choice([1, 1, 2, 10, 100, 1000, 5000, 10000, 10000, 10000])
    a = max(1, pos - rng.randrange(0, width))
    b = a + width - 1
    u = rng.random()
    if u < 0.6:
        end_min, end_max = a, b + rng.choice([0, 0, 1, 20, 10**6])
    elif u < 0.8:
        end_min, end_max = 0, 10**9
    else:
        end_min = a + rng.randrange(0, width)
        end_max = end_min + rng.randrange(0, 40)
    u = rng.random()
    if u < 0.5:
        rb = 'N'
    elif u < 0.75:
        rb = ref.upper()
    elif u < 0.8:
        rb = ref.lower()
    elif u < 0.9:
        rb = ''.join(rng.choice('ACGT') for _ in range(rng.choice([1, 1, 2, 3])))
    else:
        r = list(ref.upper())
        r[rng.randrange(len(r))] = 'N'
        rb = ''.join(r)
    u = rng.random()
    vt = None
    if u < alt_none_p:
        ab = None
        vt = rng.choice(VTYPES)
    elif u < 0.55:
        ab = 'N'
    elif u < 0.85:
        ab = rng.choice(alts).upper()
    elif u < 0.9:
        ab = rng.choice(alts).lower()
    else:
        ab = ''.join(rng.choice('ACGT') for _ in range(rng.choice([1, 2])))
    if rng.random() < 0.7:
        vmin, vmax = 0, -1
    else:
        vmin, vmax = rng.choice([0, 1, 2, 3]), rng.choice([-1, 1, 2, 5, 100])
    u = rng.random()
    if u < 1 - samples_p:
        pt = {}
    elif u < 1 - samples_p / 2:
        pt = {'includeSamples': True}
    else:
        k = rng.randrange(1, len(names) + 1) if names else 1
        pt = {'sampleNames': rng.sample(names, k) if names else ['_'], 'selectedSamplesOnly': True}
        if rng.random() < 0.5:
            pt['includeSamples'] = True
    return dict(passthrough=pt, dataset_id='ds', query_id='t', region=f'{chrom}:{a}-{b}', reference_bases=rb,
                end_min=end_min, end_max=end_max, alternate_bases=ab, variant_type=vt,
                include_details=rng.random() < 0.6, requested_granularity=rng.choice(GRANS),
                variant_min_length=vmin, variant_max_length=vmax, vcf_location=vcf_location)
