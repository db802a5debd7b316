"""getGenomicVariants routes over the HBM engine.

``route`` restates ``lambda/getGenomicVariants/route_g_variants.py:49-208``
and ``route_id`` restates ``route_g_variants_id.py:45-170``: the same GET /
POST parameter parsing and defaults, the same fan-out
(:func:`sbeacon.variant_search.perform_variant_search_sync`, which sends every
slice of every dataset to the device as one batch), the same aggregation
(``exists`` OR, ``variants`` set, one ``get_variant_entry`` per distinct
``assembly\\tchrom\\tpos\\tref\\talt``) and the same envelopes
(:mod:`sbeacon.responses`).

The reference iterates the performQuery responses in thread-completion order;
here they arrive in (dataset, slice, VCF) order, so ``results`` may be listed
in a different order — every count and every set is the same.  Dataset
resolution (Athena) and the job-status table (DynamoDB) are the
:mod:`sbeacon.catalog` hooks.  ``lambda_handler`` dispatches like
``lambda_function.py:18-52`` without the jsonschema request validation
(jsonschema is not part of this image).
"""
from __future__ import annotations

import base64
import json

from . import responses
from .catalog import JobStatus, catalog as default_catalog
from .variant_search import perform_variant_search_sync


def _params(event):
    """route_g_variants.py:50-111 -> dict of the parsed request."""
    if event['httpMethod'] == 'GET':
        params = event['queryStringParameters'] or dict()
        filters_list = []
        filters_str = params.get('filters', filters_list)
        if isinstance(filters_str, str):
            filters_list = filters_str.split(',')
        return dict(
            apiVersion=params.get('apiVersion', responses.BEACON_API_VERSION),
            skip=params.get('skip', 0), limit=params.get('limit', 100),
            includeResultsetResponses=params.get('includeResultsetResponses', 'NONE'),
            start=[int(a) for a in params['start'].split(',')],
            end=[int(a) for a in params['end'].split(',')],
            assemblyId=params.get('assemblyId', None), referenceName=params.get('referenceName', None),
            referenceBases=params.get('referenceBases', None), alternateBases=params.get('alternateBases', None),
            variantMinLength=params.get('variantMinLength', 0), variantMaxLength=params.get('variantMaxLength', -1),
            variantType=params.get('variantType', None),
            filters=[{'id': f} for f in filters_list],
            requestedGranularity=params.get('requestedGranularity', 'boolean'))
    if event['httpMethod'] == 'POST':
        params = json.loads(event['body']) or dict()
        meta = params.get('meta', dict())
        query = params.get('query', dict()) or dict()
        pagination = query.get('pagination', dict())
        rp = query.get('requestParameters', dict())
        return dict(
            apiVersion=meta.get('apiVersion', responses.BEACON_API_VERSION),
            skip=pagination.get('skip', 0), limit=pagination.get('limit', 100),
            includeResultsetResponses=query.get('includeResultsetResponses', 'NONE'),
            start=rp.get('start', []), end=rp.get('end', []),
            assemblyId=rp.get('assemblyId', None), referenceName=rp.get('referenceName', None),
            referenceBases=rp.get('referenceBases', None), alternateBases=rp.get('alternateBases', None),
            variantMinLength=rp.get('variantMinLength', 0), variantMaxLength=rp.get('variantMaxLength', -1),
            variantType=rp.get('variantType', None),
            filters=query.get('filters', []),
            requestedGranularity=query.get('requestedGranularity', 'boolean'))
    # neither GET nor POST: the reference reads unbound locals next
    raise UnboundLocalError("local variable 'includeResultsetResponses' referenced before assignment")


def aggregate(query_responses, *, granularity, check_all, assembly_id):
    """route_g_variants.py:144-171: returns (exists, variants, results).

    Responses answered by the device carry their result set (``_src``): their
    variant strings are deduplicated in the library
    (sb_result_distinct_variants) and only the distinct strings reach
    Python.  ``results`` follows first-seen order per result set (the
    reference's is thread-completion order)."""
    variants = set()
    results = []
    found = set()
    exists = False
    by_set = {}  # id(result set) -> (result set, [query indices])

    def add(strings):
        variants.update(strings)
        for variant in strings:
            chrom, pos, ref, alt, typ = variant.split('\t')
            internal_id = f'{assembly_id}\t{chrom}\t{pos}\t{ref}\t{alt}'
            if internal_id not in found:
                results.append(responses.get_variant_entry(
                    base64.b64encode(internal_id.encode()).decode(), assembly_id, ref, alt,
                    int(pos), int(pos) + len(alt), typ))
                found.add(internal_id)

    for query_response in query_responses:
        exists = exists or query_response.exists
        if exists:
            if granularity == 'boolean':
                break
            if check_all:
                src = getattr(query_response, '_src', None)
                if src is not None:
                    by_set.setdefault(id(src[0]), (src[0], []))[1].append(src[1])
                else:
                    add(query_response.variants)
    for rs, idx in by_set.values():
        add(rs.distinct_variants(idx))
    return exists, variants, results


def _finish(granularity, exists, variants, results, query_id, pagination=None):
    """route_g_variants.py:179-198 (None for any other granularity, as there)."""
    if granularity == 'boolean':
        return responses.bundle_response(200, responses.get_boolean_response(exists=exists), query_id)
    if granularity == 'count':
        return responses.bundle_response(200, responses.get_counts_response(exists=exists, count=len(variants)),
                                         query_id)
    if granularity in ('record', 'aggregated'):
        kw = {} if pagination is None else {'reqPagination': pagination}
        return responses.bundle_response(200, responses.get_result_sets_response(
            setType='genomicVariant', exists=exists, total=len(variants), results=results, **kw), query_id)
    return None


def _not_new(status, query_id, catalog):
    """route_g_variants.py:200-208."""
    if status == JobStatus.RUNNING:
        return responses.bundle_response(200, responses.get_boolean_response(
            exists=False, info={'message': 'Query still running.'}))
    return responses.bundle_response(200, catalog.cache[query_id])


def route(event, query_id, *, catalog=None):
    """GET/POST /g_variants."""
    catalog = catalog or default_catalog
    p = _params(event)
    check_all = p['includeResultsetResponses'] in ('HIT', 'ALL')
    status = catalog.job_status(query_id)
    if status != JobStatus.NEW:
        return _not_new(status, query_id, catalog)
    datasets, samples = catalog.resolve(p['filters'], p['assemblyId'])
    query_responses = perform_variant_search_sync(
        datasets=datasets, referenceName=p['referenceName'], referenceBases=p['referenceBases'],
        alternateBases=p['alternateBases'], start=p['start'], end=p['end'], variantType=p['variantType'],
        variantMinLength=p['variantMinLength'], variantMaxLength=p['variantMaxLength'],
        requestedGranularity=p['requestedGranularity'], includeResultsetResponses=p['includeResultsetResponses'],
        query_id=query_id, dataset_samples=samples)
    exists, variants, results = aggregate(query_responses, granularity=p['requestedGranularity'],
                                          check_all=check_all, assembly_id=p['assemblyId'])
    return _finish(p['requestedGranularity'], exists, variants, results, query_id,
                   responses.get_pagination_object(p['skip'], p['limit']))


def route_id(event, query_id, *, catalog=None):
    """GET/POST /g_variants/{id} (route_g_variants_id.py:45-170): the id is
    base64('assembly\\tchrom\\tpos\\tref\\talt'); the point query is
    start=[pos-1], end=[pos-1+len(alt)], includeResultsetResponses='ALL'."""
    catalog = catalog or default_catalog
    if event['httpMethod'] == 'GET':
        params = event.get('queryStringParameters', dict()) or dict()
        granularity = params.get('requestedGranularity', 'boolean')
        filters_str = params.get('filters', [])
        filters = [{'id': f} for f in (filters_str.split(',') if isinstance(filters_str, str) else [])]
    elif event['httpMethod'] == 'POST':
        params = json.loads(event.get('body', '{}')) or dict()
        query = params.get('query', dict())
        granularity = query.get('requestedGranularity', 'boolean')
        filters = query.get('filters', [])
    else:
        raise UnboundLocalError("local variable 'requestedGranularity' referenced before assignment")
    variant_id = event['pathParameters'].get('id', None)
    dataset_hash = base64.b64decode(variant_id.encode()).decode()
    assembly_id, reference_name, pos, reference_bases, alternate_bases = dataset_hash.split('\t')
    pos = int(pos) - 1
    status = catalog.job_status(query_id)
    if status != JobStatus.NEW:
        return _not_new(status, query_id, catalog)
    datasets, samples = catalog.resolve(filters, assembly_id)
    query_responses = perform_variant_search_sync(
        datasets=datasets, referenceName=reference_name, referenceBases=reference_bases,
        alternateBases=alternate_bases, start=[pos], end=[pos + len(alternate_bases)], variantType=None,
        variantMinLength=0, variantMaxLength=-1, requestedGranularity=granularity,
        includeResultsetResponses='ALL', query_id=query_id, dataset_samples=samples)
    exists, variants, results = aggregate(query_responses, granularity=granularity, check_all=True,
                                          assembly_id=assembly_id)
    return _finish(granularity, exists, variants, results, query_id)


def lambda_handler(event, context=None, *, catalog=None):
    """lambda_function.py:18-52 route dispatch (query_id = request hash)."""
    from .request_hash import hash_query
    if event['httpMethod'] == 'POST':
        try:
            json.loads(event.get('body') or '{}')
        except ValueError:
            return responses.bad_request(errorMessage='Error parsing request body, Expected JSON.')
    event_hash = hash_query(event)
    if event['resource'] == '/g_variants':
        return route(event, event_hash, catalog=catalog)
    if event['resource'] == '/g_variants/{id}':
        return route_id(event, event_hash, catalog=catalog)
    if event['resource'] in ('/g_variants/{id}/individuals', '/g_variants/{id}/biosamples'):
        from .route_g_variants_samples import route_biosamples, route_individuals
        fn = route_individuals if event['resource'].endswith('individuals') else route_biosamples
        return fn(event, event_hash, catalog=catalog)
    return None
