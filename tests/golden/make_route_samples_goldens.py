#!/usr/bin/env python3
"""Golden responses of the sample-path routes ``/g_variants/{id}/individuals``
and ``/g_variants/{id}/biosamples``, made by running the REFERENCE routes.

TEST INFRASTRUCTURE — runs only in the build container (reads
/root/reference); writes ``route_samples_golden.json`` (events in,
status/body or error class out, plus the metadata tables the stub served).

The chain route -> perform_variant_search_sync -> splitQuery -> performQuery
-> fake bcftools runs unmodified in process with the stubs of
make_route_goldens.py.  In addition the Athena entity models are stubbed:
``Individual.get_by_query`` / ``Biosample.get_by_query`` answer the
reference's UNION of ``get_record_query`` parts from in-memory tables (rows
keyed by dataset and VCF sample name; SQL UNION drops whole-row duplicates)
and ``jsons.dump(objs, strip_privates=True)`` drops ``_``-prefixed
attributes.  The routes walk Python sets of sample names, so the run pins
PYTHONHASHSEED=0 (re-executing itself) and the golden records it.

Usage:  python tests/golden/make_route_samples_goldens.py
"""
from __future__ import annotations

import base64
import json
import os
import random
import re
import sys
import tempfile
import threading
import types

if __name__ == '__main__' and os.environ.get('PYTHONHASHSEED') != '0':
    # set iteration order must be reproducible: rerun as a child with the
    # seed fixed (a child process, never an exec of this one)
    import subprocess
    sys.exit(subprocess.run([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED='0')).returncode)

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_goldens as mg  # noqa: E402
import make_route_goldens as mrg  # noqa: E402

ASSEMBLY = mrg.ASSEMBLY


def metadata(spec):
    """Rows per (kind, dataset, sample).  Every 5th sample has two analyses
    of one individual / biosample (identical rows: UNION keeps one), every
    7th shares its individual with the previous sample."""
    tables = {'individuals': {}, 'biosamples': {}}
    for d in spec:
        names = []
        for v in d['vcfLocations']:
            _, n = mg.read_records(v)
            names += [x for x in n if x not in names]
        ind, bio = {}, {}
        for k, s in enumerate(names):
            owner = names[k - 1] if k % 7 == 6 else s
            irow = {'id': f'{d["id"]}-ind-{owner}', 'sex': {'id': 'NCIT:C16576' if k % 2 else 'NCIT:C20197',
                                                            'label': 'female' if k % 2 else 'male'},
                    'karyotypicSex': 'XX' if k % 2 else 'XY', '_datasetId': d['id'], '_cohortId': 'c1'}
            brow = {'id': f'{d["id"]}-bio-{s}', 'individualId': irow['id'],
                    'biosampleStatus': {'id': 'EFO:0009654', 'label': 'reference sample'},
                    'sampleOriginType': {'id': 'UBERON:0000178', 'label': 'blood'}, '_datasetId': d['id']}
            ind[s] = [irow, dict(irow)] if k % 5 == 0 else [irow]
            bio[s] = [brow, dict(brow)] if k % 5 == 0 else [brow]
        tables['individuals'][d['id']] = ind
        tables['biosamples'][d['id']] = bio
    return tables


def install_entity_stubs(tables):
    os.environ.update(INDIVIDUALS_TABLE='individuals', BIOSAMPLES_TABLE='biosamples')

    def model(kind):
        class Model:
            def __init__(self, row):
                self.__dict__.update(row)

            @classmethod
            def get_by_query(cls, query, queue=None, execution_parameters=None):
                rows, seen = [], set()
                for part in query.split(' UNION '):
                    ds = re.search(r"_datasetid='([^']*)'", part).group(1)
                    names = re.findall(r"'([^']*)'", part.split(' IN ')[1])
                    for n in names:
                        for r in tables[kind].get(ds, {}).get(n, []):
                            key = json.dumps(r, sort_keys=True)
                            if key not in seen:
                                seen.add(key)
                                rows.append(cls(r))
                return rows
        return Model

    ind = types.ModuleType('athena.individual')
    ind.Individual = model('individuals')
    bio = types.ModuleType('athena.biosample')
    bio.Biosample = model('biosamples')
    sys.modules.update({'athena.individual': ind, 'athena.biosample': bio})
    jsons = sys.modules['jsons']

    def dump(obj, strip_privates=False, **kw):
        if isinstance(obj, list):
            return [dump(o, strip_privates) for o in obj]
        d = dict(obj.__dict__) if hasattr(obj, '__dict__') else obj
        return {k: v for k, v in d.items() if not (strip_privates and k.startswith('_'))}

    jsons.dump = dump


def make_events(rng, recs, resource):
    events = []
    for i in range(60):
        pos, ref, alts = recs[rng.randrange(len(recs))]
        alt = rng.choice(alts)
        if rng.random() < 0.15:
            alt = rng.choice('ACGT')
        vid = base64.b64encode(f'{ASSEMBLY}\t22\t{pos}\t{ref}\t{alt}'.encode()).decode()
        gran = rng.choice(['boolean', 'count', 'record', 'record', 'aggregated', None])
        path = resource.replace('{id}', vid)
        if rng.random() < 0.4:
            q = {} if gran is None else {'requestedGranularity': gran}
            if rng.random() < 0.15:
                q.update(skip='2', limit='3')  # strings, as API Gateway passes them
            events.append({'resource': resource, 'httpMethod': 'GET', 'path': path, 'pathParameters': {'id': vid},
                           'queryStringParameters': q or None})
        else:
            query = {} if gran is None else {'requestedGranularity': gran}
            if rng.random() < 0.6:
                query['pagination'] = {'skip': rng.choice([0, 0, 2, 5, 30]), 'limit': rng.choice([3, 4, 100])}
            events.append({'resource': resource, 'httpMethod': 'POST', 'path': path, 'pathParameters': {'id': vid},
                           'queryStringParameters': None, 'body': json.dumps({'query': query})})
    return events


def main():
    mg.install_stubs()
    tmp = tempfile.mkdtemp(prefix='sbeacon-route-samples-')
    mg.install_fake_bcftools(tmp)
    spec = mrg.catalog(mg.FIX)
    handlers = {}
    mrg.install_route_stubs(spec, handlers)
    tables = metadata(spec)
    install_entity_stubs(tables)
    sv, svs, PQP = mg.import_reference()
    gv = os.path.join(mg.REF, 'lambda', 'getGenomicVariants')
    sys.path.insert(0, gv)
    sq = mrg.load_by_path('ref_split_query', os.path.join(mg.REF, 'lambda', 'splitQuery', 'lambda_function.py'))
    from payloads.lambda_payloads import SplitQueryPayload
    gate = threading.Semaphore(8)

    def perform(event):
        payload = PQP(**event)
        mod = svs if payload.passthrough.get('selectedSamplesOnly', False) else sv
        with gate:
            return mod.perform_query(payload, False).dump()

    handlers.update({'performQuery': perform,
                     'splitQuery': lambda ev: sq.split_query_sync(SplitQueryPayload(**ev))})
    routes = {
        '/g_variants/{id}/individuals': mrg.load_by_path(
            'ref_route_ind', os.path.join(gv, 'route_g_variants_id_individuals.py')).route,
        '/g_variants/{id}/biosamples': mrg.load_by_path(
            'ref_route_bio', os.path.join(gv, 'route_g_variants_id_biosamples.py')).route,
    }
    hq = mrg.load_by_path('ref_request_hash', os.path.join(mg.REF, 'shared_resources', 'apiutils',
                                                           'request_hash.py'))
    recs, _ = mg.read_records(os.path.join(mg.FIX, 'tiny22.vcf'))
    rng = random.Random(20250120)
    cases = []
    for resource, fn in routes.items():
        for ev in make_events(rng, recs, resource):
            qid = hq.hash_query(ev)
            try:
                cases.append({'event': ev, 'query_id': qid, 'error': None, 'response': fn(ev, qid)})
            except Exception as e:  # noqa: BLE001 - the reference's failure is the contract
                cases.append({'event': ev, 'query_id': qid, 'error': type(e).__name__, 'response': None})
    cat = json.loads(json.dumps(spec).replace(mg.FIX + os.sep, ''))
    out = os.path.join(HERE, 'route_samples_golden.json')
    with open(out, 'w') as f:
        json.dump({'generator': 'tests/golden/make_route_samples_goldens.py',
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17',
                   'pythonhashseed': '0', 'env': {k: mrg.ENV[k] for k in ('BEACON_API_VERSION', 'BEACON_ID')},
                   'datasets': cat, 'metadata': tables, 'cases': cases}, f, separators=(',', ':'))
    n_err = sum(1 for c in cases if c['error'])
    print(f'wrote {len(cases)} sample-route cases ({n_err} reference errors) -> {out}')


if __name__ == '__main__':
    main()
