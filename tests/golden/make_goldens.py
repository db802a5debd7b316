#!/usr/bin/env python3
"""Generate golden performQuery vectors by running the REFERENCE code.

TEST INFRASTRUCTURE — runs only in the build container, where the read-only
reference checkout exists at ``/root/reference``.  Nothing on the GPU box or in
the product path imports this file; the outputs it writes
(``tests/golden/*.json`` + ``tests/golden/fixtures/*.vcf``) are plain data.

How the reference is driven:

* ``lambda/performQuery/search_variants.py`` and
  ``search_variants_in_samples.py`` are imported unmodified.  Their AWS imports
  (``boto3``, ``botocore.exceptions``, ``jsons``, ``dynamodb.variant_queries``)
  are replaced by inert ``sys.modules`` stubs — no network, nothing executed from
  the stubs on the query path (``is_async=False``).
* ``bcftools`` on ``PATH`` is ``fake_bcftools.py`` (see its docstring for the
  restated contract; parity at that boundary is unpinned).
* ``perform_query`` is called directly with the dispatch rule of
  ``lambda/performQuery/lambda_function.py:43-46`` (``lambda_handler`` itself
  deletes ``/tmp/*``, so it is not called).
* ``alternate_bases=None`` (variantType) queries crash in the reference with
  ``UnboundLocalError`` (``search_variants.py:101`` reads ``variant_type``
  before ``:193`` assigns it).  Those payloads are recorded twice: once with the
  reference's real outcome (the error), and once against an in-memory
  *patched-oracle* copy of the source in which the branch selector
  ``variant_type ==`` at ``:101,112,123,134,145`` reads ``payload.variant_type``
  (the evident intent).

Usage:  python tests/golden/make_goldens.py   (rewrites the golden files)
"""
from __future__ import annotations

import dataclasses
import json
import os
import random
import stat
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))

from sbeacon import synth  # noqa: E402

FIX = os.path.join(HERE, 'fixtures')


# --------------------------------------------------------------------------- stubs
def install_stubs():
    boto3 = types.ModuleType('boto3')

    class _Client:
        def __getattr__(self, name):
            raise RuntimeError(f'boto3 stub: {name} must not be called on the sync path')

    boto3.client = lambda *a, **k: _Client()
    boto3.resource = lambda *a, **k: _Client()
    botocore = types.ModuleType('botocore')
    botocore_exc = types.ModuleType('botocore.exceptions')

    class ClientError(Exception):
        pass

    botocore_exc.ClientError = ClientError
    botocore.exceptions = botocore_exc

    jsons = types.ModuleType('jsons')

    class JsonSerializable:
        def dump(self):
            if dataclasses.is_dataclass(self):
                return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}
            return dict(self.__dict__)

        def dumps(self):
            return json.dumps(self.dump())

    jsons.JsonSerializable = JsonSerializable
    jsons.dumps = lambda obj: json.dumps(obj.dump() if hasattr(obj, 'dump') else obj)
    jsons.load = lambda d, cls: cls(**d)
    jsons.loads = lambda s, cls: cls(**json.loads(s))

    dyn = types.ModuleType('dynamodb')
    dyn.__path__ = []
    vq = types.ModuleType('dynamodb.variant_queries')
    dyn.variant_queries = vq
    sys.modules.update({
        'boto3': boto3, 'botocore': botocore, 'botocore.exceptions': botocore_exc,
        'jsons': jsons, 'dynamodb': dyn, 'dynamodb.variant_queries': vq,
    })
    os.environ.setdefault('VARIANTS_BUCKET', 'stub-bucket')


def install_fake_bcftools(tmpdir):
    exe = os.path.join(tmpdir, 'bcftools')
    with open(exe, 'w') as f:
        f.write(f'#!/bin/sh\nexec {sys.executable} {os.path.join(HERE, "fake_bcftools.py")} "$@"\n')
    os.chmod(exe, os.stat(exe).st_mode | stat.S_IEXEC)
    os.environ['PATH'] = tmpdir + os.pathsep + os.environ['PATH']


def import_reference():
    pq = os.path.join(REF, 'lambda', 'performQuery')
    sys.path.insert(0, pq)
    import search_variants  # noqa: F401
    import search_variants_in_samples  # noqa: F401
    from payloads.lambda_payloads import PerformQueryPayload
    return sys.modules['search_variants'], sys.modules['search_variants_in_samples'], PerformQueryPayload


def patched_module(mod, name):
    """In-memory patched-oracle copy: branch on payload.variant_type."""
    src = open(mod.__file__).read()
    n_if = src.count('if variant_type == ')
    src2 = src.replace('if variant_type == ', 'if payload.variant_type == ')
    assert n_if == 5, n_if
    m = types.ModuleType(name)
    m.__file__ = mod.__file__ + ' (patched-oracle)'
    exec(compile(src2, m.__file__, 'exec'), m.__dict__)
    return m


# --------------------------------------------------------------------------- payloads
def read_records(path):
    recs = []
    names = []
    with open(path) as f:
        for line in f:
            if line.startswith('##'):
                continue
            if line.startswith('#CHROM'):
                names = line.rstrip('\n').split('\t')[9:]
                continue
            c = line.rstrip('\n').split('\t')
            recs.append((int(c[1]), c[3], c[4].split(',')))
    return recs, names


VTYPES = ['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV', 'SNP', None]
GRANS = ['boolean', 'count', 'aggregated', 'record']


def random_payload(rng: random.Random, recs, names, vcf_location, *, force_alt_none=False):
    lo, hi = recs[0][0], recs[-1][0]
    anchor = recs[rng.randrange(len(recs))]
    width = rng.choice([1, 1, 2, 10, 100, 1000, 5000, 10000, 10000])
    a = max(1, anchor[0] - rng.randrange(0, width))
    if rng.random() < 0.05:
        a = rng.choice([lo - 500, hi + 10])
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
        ref = 'N'
    elif u < 0.75:
        ref = anchor[1].upper()
    elif u < 0.8:
        ref = anchor[1].lower()
    elif u < 0.9:
        ref = ''.join(rng.choice('ACGT') for _ in range(rng.choice([1, 1, 2, 3])))
    else:
        r = list(anchor[1].upper())
        r[rng.randrange(len(r))] = 'N'
        ref = ''.join(r)
    u = rng.random()
    vt = None
    if force_alt_none or u < 0.2:
        alt = None
        vt = rng.choice(VTYPES)
    elif u < 0.55:
        alt = 'N'
    elif u < 0.85:
        alt = rng.choice(anchor[2]).upper()
    elif u < 0.9:
        alt = rng.choice(anchor[2]).lower()
    else:
        alt = ''.join(rng.choice('ACGT') for _ in range(rng.choice([1, 2])))
    if rng.random() < 0.7:
        vmin, vmax = 0, -1
    else:
        vmin = rng.choice([0, 1, 2, 3])
        vmax = rng.choice([-1, 1, 2, 5, 100])
    gran = rng.choice(GRANS)
    include_details = rng.random() < 0.6
    u = rng.random()
    if u < 0.45:
        passthrough = {}
    elif u < 0.75:
        passthrough = {'includeSamples': True}
    else:
        k = rng.randrange(1, len(names) + 1)
        subset = rng.sample(names, k)
        passthrough = {'sampleNames': subset, 'selectedSamplesOnly': True}
        if rng.random() < 0.5:
            passthrough['includeSamples'] = True
    return dict(passthrough=passthrough, dataset_id='ds-1', query_id='golden',
                region=f'22:{a}-{b}', reference_bases=ref, end_min=end_min, end_max=end_max,
                alternate_bases=alt, variant_type=vt, include_details=include_details,
                requested_granularity=gran, variant_min_length=vmin, variant_max_length=vmax,
                vcf_location=vcf_location)


def split_payloads(recs, vcf_location):
    """Payloads exactly as splitQuery builds them (lambda/splitQuery/lambda_function.py:74-110)."""
    out = []
    lo, hi = recs[0][0], recs[-1][0]
    for gran in GRANS:
        for check_all in (True, False):
            for ref, alt in (('N', 'N'), ('N', 'T'), ('A', 'N'), ('C', 'G')):
                start_min, start_max = lo - 100, hi + 100
                s = start_min
                while s <= start_max:
                    e = min(s + 10000 - 1, start_max)
                    out.append(dict(passthrough={}, dataset_id='ds-1', query_id='golden',
                                    region=f'22:{s}-{e}', reference_bases=ref,
                                    end_min=start_min, end_max=start_max,
                                    alternate_bases=alt, variant_type=None,
                                    include_details=check_all, requested_granularity=gran,
                                    variant_min_length=0, variant_max_length=-1,
                                    vcf_location=vcf_location))
                    s += 10000
    return out


def run_one(sv, svs, PQP, p):
    payload = PQP(**p)
    mod = svs if payload.passthrough.get('selectedSamplesOnly', False) else sv
    try:
        resp = mod.perform_query(payload, False)
        d = resp.dump()
        return {'response': d, 'error': None}
    except Exception as e:  # the reference's own failure modes are part of the contract
        return {'response': None, 'error': type(e).__name__}


def main():
    install_stubs()
    tmp = tempfile.mkdtemp(prefix='sbeacon-golden-')
    install_fake_bcftools(tmp)
    sv, svs, PQP = import_reference()
    sv_p = patched_module(sv, 'search_variants_patched')
    svs_p = patched_module(svs, 'search_variants_in_samples_patched')

    os.makedirs(FIX, exist_ok=True)
    fixtures = {
        'tiny22': dict(n_records=2000, n_samples=16, seed=1, quirks=False),
        'quirk22': dict(n_records=600, n_samples=12, seed=7, quirks=True),
    }
    for name, kw in fixtures.items():
        synth.make_fixture(os.path.join(FIX, name + '.vcf'), **kw)

    rng = random.Random(20250117)
    cases = []
    # 1) tiny22: splitQuery-shaped payloads + random payloads (reference as-is)
    for name, n_random in (('tiny22', 450), ('quirk22', 250)):
        path = os.path.join(FIX, name + '.vcf')
        recs, names = read_records(path)
        payloads = (split_payloads(recs, path) if name == 'tiny22' else []) + \
            [random_payload(rng, recs, names, path) for _ in range(n_random)]
        # sample-path focused payloads (search_variants.py:233-236, :257-258)
        for _ in range(100 if name == 'tiny22' else 50):
            p = random_payload(rng, recs, names, path)
            p['requested_granularity'] = rng.choice(['record', 'aggregated'])
            p['include_details'] = True
            if not p['passthrough']:
                p['passthrough'] = {'includeSamples': True}
            if p['alternate_bases'] is None or rng.random() < 0.5:
                p['alternate_bases'] = 'N'
            if rng.random() < 0.5:
                p['reference_bases'] = 'N'
            payloads.append(p)
        for p in payloads:
            r = run_one(sv, svs, PQP, p)
            cases.append({'fixture': name, 'oracle': 'reference', 'payload': p, **r})
        # 2) variantType payloads against the patched-oracle copy
        for _ in range(150 if name == 'tiny22' else 60):
            p = random_payload(rng, recs, names, path, force_alt_none=True)
            r_ref = run_one(sv, svs, PQP, p)
            cases.append({'fixture': name, 'oracle': 'reference', 'payload': p, **r_ref})
            r = run_one(sv_p, svs_p, PQP, p)
            cases.append({'fixture': name, 'oracle': 'patched-oracle', 'payload': p, **r})

    # vcf_location is stored relative to the fixture dir so the file is portable
    for c in cases:
        c['payload']['vcf_location'] = os.path.basename(c['payload']['vcf_location'])
        if c['response']:
            c['response']['vcf_location'] = os.path.basename(c['response']['vcf_location'])
    out = os.path.join(HERE, 'perform_query_golden.json')
    with open(out, 'w') as f:
        json.dump({'generator': 'tests/golden/make_goldens.py',
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17',
                   'cases': cases}, f, separators=(',', ':'))
    n_err = sum(1 for c in cases if c['error'])
    n_exists = sum(1 for c in cases if c['response'] and c['response']['exists'])
    print(f'wrote {len(cases)} cases ({n_err} reference errors, {n_exists} exists=True) -> {out}')


if __name__ == '__main__':
    main()
