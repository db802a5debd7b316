#!/usr/bin/env python3
"""Generate golden g_variants ROUTE responses by running the REFERENCE code.

TEST INFRASTRUCTURE — runs only in the build container, where the read-only
reference checkout exists at ``/root/reference``.  Nothing on the GPU box or in
the product path imports this file; its output (``route_golden.json``) is
plain data: route events in, reference status/body (or error class) out.

The whole reference call chain runs unmodified, in process:
``route_g_variants.route`` / ``route_g_variants_id.route``
(lambda/getGenomicVariants) -> ``variantutils.search_variants.
perform_variant_search_sync`` -> ``local_utils.split_query_sync`` ->
[lambda invoke] -> ``lambda/splitQuery/lambda_function.split_query_sync`` ->
[lambda invoke] -> ``lambda/performQuery`` ``perform_query`` (dispatch rule of
``lambda_function.py:43-46``) -> ``bcftools`` = ``fake_bcftools.py``.

Stubbed (no network, nothing from the stubs is on the compute path):
``boto3`` (a ``lambda`` client whose ``invoke`` calls the two handlers above
in process and returns their JSON payload, or the Lambda error payload
``{'errorMessage', 'errorType'}`` when the handler raises), ``botocore``,
``jsons``, ``smart_open``, ``dynamodb.variant_queries`` (``get_job_status``
-> NEW), and the Athena modules (``new_entity_search_conditions`` -> no
conditions; ``Dataset.get_by_query`` -> the in-memory datasets below).

Usage:  python tests/golden/make_route_goldens.py
"""
from __future__ import annotations

import base64
import importlib.util
import io
import json
import os
import random
import sys
import tempfile
import threading
import types
from enum import Enum

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_goldens as mg  # noqa: E402  (stubs, fake bcftools, fixture reader)

REF = mg.REF
FIX = mg.FIX
ASSEMBLY = 'GRCh38'

ENV = {
    'BEACON_API_VERSION': 'v2.0.0', 'BEACON_ID': 'au.csiro-serverless.beacon',
    'DATASETS_TABLE': 'datasets', 'ANALYSES_TABLE': 'analyses', 'METADATA_DATABASE': 'metadata',
    'METADATA_BUCKET': 'stub-metadata', 'SPLIT_QUERY_LAMBDA': 'splitQuery',
    'SPLIT_QUERY_TOPIC_ARN': 'arn:stub:splitQuery', 'PERFORM_QUERY_LAMBDA': 'performQuery',
    'PERFORM_QUERY_TOPIC_ARN': 'arn:stub:performQuery', 'VARIANTS_BUCKET': 'stub-bucket',
    'DYNAMO_VARIANT_QUERIES_TABLE': 'q', 'DYNAMO_VARIANT_QUERY_RESPONSES_TABLE': 'r',
}


def catalog(fix):
    """The datasets the stubbed Athena returns (vcf paths absolute here,
    basenames in the golden file)."""
    tiny, quirk = os.path.join(fix, 'tiny22.vcf'), os.path.join(fix, 'quirk22.vcf')
    return [
        dict(id='ds-tiny', assemblyId=ASSEMBLY, vcfLocations=[tiny],
             vcfChromosomeMap=[{'vcf': tiny, 'chromosomes': ['22']}]),
        dict(id='ds-both', assemblyId=ASSEMBLY, vcfLocations=[tiny, quirk],
             vcfChromosomeMap=[{'vcf': tiny, 'chromosomes': ['22']}, {'vcf': quirk, 'chromosomes': ['22']}]),
        dict(id='ds-37', assemblyId='GRCh37', vcfLocations=[tiny],
             vcfChromosomeMap=[{'vcf': tiny, 'chromosomes': ['22']}]),
    ]


def install_route_stubs(datasets_spec, handlers):
    os.environ.update(ENV)
    botocore = sys.modules['botocore']
    cfg = types.ModuleType('botocore.config')

    class Config:
        def __init__(self, **kw):
            self.kw = kw

    cfg.Config = Config
    botocore.config = cfg
    sys.modules['botocore.config'] = cfg

    class LambdaClient:
        def invoke(self, FunctionName, InvocationType, Payload):
            try:
                out = handlers[FunctionName](json.loads(Payload))
            except Exception as e:  # a failed synchronous invoke returns the error payload
                out = {'errorMessage': str(e), 'errorType': type(e).__name__}
            return {'Payload': io.BytesIO(json.dumps(out).encode())}

    class Inert:
        def __getattr__(self, name):
            raise RuntimeError(f'boto3 stub: {name} must not be called on the sync route path')

    boto3 = sys.modules['boto3']
    boto3.client = lambda name, *a, **k: LambdaClient() if name == 'lambda' else Inert()
    session = types.SimpleNamespace(Session=lambda: types.SimpleNamespace(region_name='stub'))
    boto3.session = session

    so = types.ModuleType('smart_open')
    so.open = lambda *a, **k: (_ for _ in ()).throw(RuntimeError('smart_open stub'))
    sys.modules['smart_open'] = so

    vq = sys.modules['dynamodb.variant_queries']

    class JobStatus(Enum):
        NEW = 1
        RUNNING = 2
        COMPLETED = 3

    vq.JobStatus = JobStatus
    vq.get_job_status = lambda query_id: JobStatus.NEW
    vq.VariantQuery = vq.VariantResponse = type('Model', (), {})
    vq.get_current_time_utc = lambda: None

    athena = types.ModuleType('athena')
    athena.__path__ = []
    common = types.ModuleType('athena.common')
    common.entity_search_conditions = lambda *a, **k: ('', [])
    common.run_custom_query = lambda *a, **k: (_ for _ in ()).throw(RuntimeError('athena stub'))
    dataset = types.ModuleType('athena.dataset')

    class Dataset:
        def __init__(self, *, id, assemblyId, vcfLocations, vcfChromosomeMap):
            self.id = id
            self._assemblyId = assemblyId
            self._vcfLocations = vcfLocations
            self._vcfChromosomeMap = vcfChromosomeMap

        @classmethod
        def get_by_query(cls, query, execution_parameters=None):
            # datasets_query_fast(assembly_id): WHERE _assemblyid='<id>'
            asm = query.split("_assemblyid='")[1].split("'")[0]
            return [cls(**d) for d in datasets_spec if d['assemblyId'] == asm]

    dataset.Dataset = Dataset
    dataset.parse_datasets_with_samples = lambda *a, **k: (_ for _ in ()).throw(RuntimeError('athena stub'))
    ff = types.ModuleType('athena.filter_functions')
    ff.new_entity_search_conditions = lambda filters, *a, **k: ('', [])
    sys.modules.update({'athena': athena, 'athena.common': common, 'athena.dataset': dataset,
                        'athena.filter_functions': ff})


def load_by_path(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def make_events(rng, recs, names):
    lo, hi = recs[0][0], recs[-1][0]
    events = []

    def one(method, rp, gran, irr, extra_q=None):
        if method == 'GET':
            q = {'start': ','.join(str(x) for x in rp['start']), 'end': ','.join(str(x) for x in rp['end'])}
            for k in ('assemblyId', 'referenceName', 'referenceBases', 'alternateBases', 'variantType'):
                if rp.get(k) is not None:
                    q[k] = rp[k]
            if gran is not None:
                q['requestedGranularity'] = gran
            if irr is not None:
                q['includeResultsetResponses'] = irr
            q.update(extra_q or {})
            return {'resource': '/g_variants', 'httpMethod': 'GET', 'path': '/g_variants',
                    'pathParameters': None, 'queryStringParameters': q}
        query = {'requestParameters': {k: v for k, v in rp.items() if v is not None}}
        if gran is not None:
            query['requestedGranularity'] = gran
        if irr is not None:
            query['includeResultsetResponses'] = irr
        if rng.random() < 0.3:
            query['pagination'] = {'skip': rng.choice([0, 10]), 'limit': rng.choice([10, 100])}
        return {'resource': '/g_variants', 'httpMethod': 'POST', 'path': '/g_variants',
                'pathParameters': None, 'queryStringParameters': None,
                'body': json.dumps({'meta': {'apiVersion': 'v2.0'}, 'query': query})}

    for _ in range(170):
        anchor = recs[rng.randrange(len(recs))]
        width = rng.choice([1, 10, 200, 5000, 15000, 30000])
        s0 = max(0, anchor[0] - 1 - rng.randrange(0, width))
        u = rng.random()
        if u < 0.55:
            start, end = [s0], [s0 + width]
        elif u < 0.8:
            start, end = [s0, s0 + width], [s0, s0 + width + rng.choice([0, 10, 1000])]
        elif u < 0.95:
            start, end = [s0], [s0 + rng.randrange(0, 50), s0 + width]
        else:
            start, end = [rng.choice([lo - 20000, hi + 10])], [rng.choice([lo - 10000, hi + 5000])]
        u = rng.random()
        if u < 0.45:
            ref, alt = 'N', 'N'
        elif u < 0.75:
            ref, alt = anchor[1].upper(), rng.choice(anchor[2]).upper()
        elif u < 0.85:
            ref, alt = 'N', rng.choice('ACGT')
        else:
            ref, alt = rng.choice(['N', anchor[1].upper()]), None
        rp = {'assemblyId': rng.choice([ASSEMBLY] * 9 + ['GRCh37']),
              'referenceName': rng.choice(['22'] * 12 + ['X']),
              'referenceBases': ref, 'alternateBases': alt, 'start': start, 'end': end,
              'variantType': rng.choice(['DEL', 'SNP', 'INS']) if alt is None else None}
        gran = rng.choice(['boolean', 'count', 'record', 'aggregated', None])
        irr = rng.choice(['HIT', 'ALL', 'NONE', 'MISS', None, 'HIT'])
        events.append(one(rng.choice(['GET', 'POST']), rp, gran, irr))
    # error-shaped requests the reference handles its own way
    rp = {'assemblyId': ASSEMBLY, 'referenceName': '22', 'referenceBases': 'N', 'alternateBases': 'N',
          'start': [lo], 'end': []}
    events.append(one('POST', rp, 'count', 'HIT'))  # missing end -> (False, []) iterated
    # /g_variants/{id}: existing and absent variants
    for _ in range(40):
        pos, ref, alts = recs[rng.randrange(len(recs))]
        alt = rng.choice(alts)
        if rng.random() < 0.2:
            alt = rng.choice('ACGT')
        vid = base64.b64encode(f'{ASSEMBLY}\t22\t{pos}\t{ref}\t{alt}'.encode()).decode()
        gran = rng.choice(['boolean', 'count', 'record', 'aggregated', None])
        if rng.random() < 0.5:
            q = {} if gran is None else {'requestedGranularity': gran}
            events.append({'resource': '/g_variants/{id}', 'httpMethod': 'GET', 'path': f'/g_variants/{vid}',
                           'pathParameters': {'id': vid}, 'queryStringParameters': q or None})
        else:
            query = {} if gran is None else {'requestedGranularity': gran}
            events.append({'resource': '/g_variants/{id}', 'httpMethod': 'POST', 'path': f'/g_variants/{vid}',
                           'pathParameters': {'id': vid}, 'queryStringParameters': None,
                           'body': json.dumps({'query': query})})
    return events


def main():
    mg.install_stubs()
    tmp = tempfile.mkdtemp(prefix='sbeacon-route-golden-')
    mg.install_fake_bcftools(tmp)
    spec = catalog(FIX)
    handlers = {}
    install_route_stubs(spec, handlers)
    sv, svs, PQP = mg.import_reference()
    gv = os.path.join(REF, 'lambda', 'getGenomicVariants')
    sys.path.insert(0, gv)
    sq = load_by_path('ref_split_query', os.path.join(REF, 'lambda', 'splitQuery', 'lambda_function.py'))
    from payloads.lambda_payloads import SplitQueryPayload
    gate = threading.Semaphore(8)  # bound concurrent fake-bcftools processes

    def perform(event):
        payload = PQP(**event)
        mod = svs if payload.passthrough.get('selectedSamplesOnly', False) else sv
        with gate:
            return mod.perform_query(payload, False).dump()

    def split(event):
        return sq.split_query_sync(SplitQueryPayload(**event))

    handlers.update({'performQuery': perform, 'splitQuery': split})
    rg = load_by_path('ref_route_g_variants', os.path.join(gv, 'route_g_variants.py'))
    rgi = load_by_path('ref_route_g_variants_id', os.path.join(gv, 'route_g_variants_id.py'))
    hq = load_by_path('ref_request_hash', os.path.join(REF, 'shared_resources', 'apiutils', 'request_hash.py'))

    recs, names = mg.read_records(os.path.join(FIX, 'tiny22.vcf'))
    events = make_events(random.Random(20250118), recs, names)
    cases = []
    for i, ev in enumerate(events):
        qid = hq.hash_query(ev)
        fn = rg.route if ev['resource'] == '/g_variants' else rgi.route
        try:
            out = fn(ev, qid)
            case = {'event': ev, 'query_id': qid, 'error': None, 'response': out}
        except Exception as e:  # noqa: BLE001 - the reference's failure is the contract
            case = {'event': ev, 'query_id': qid, 'error': type(e).__name__, 'response': None}
        cases.append(case)
        if i % 20 == 0:
            print(f'{i}/{len(events)}', file=sys.stderr, flush=True)
    # dataset catalog with basenames (paths are only meaningful to fake bcftools)
    cat = json.loads(json.dumps(spec).replace(FIX + os.sep, ''))
    out = os.path.join(HERE, 'route_golden.json')
    with open(out, 'w') as f:
        json.dump({'generator': 'tests/golden/make_route_goldens.py',
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17',
                   'env': {k: ENV[k] for k in ('BEACON_API_VERSION', 'BEACON_ID')},
                   'datasets': cat, 'cases': cases}, f, separators=(',', ':'))
    n_err = sum(1 for c in cases if c['error'])
    print(f'wrote {len(cases)} route cases ({n_err} reference errors) -> {out}')


if __name__ == '__main__':
    main()
