"""Sample-path routes of one variant: ``/g_variants/{id}/individuals`` and
``/g_variants/{id}/biosamples`` over the HBM engine.

Restates ``lambda/getGenomicVariants/route_g_variants_id_individuals.py:
86-238`` and ``route_g_variants_id_biosamples.py:116-266``: the same GET /
POST parsing (GET ``skip`` / ``limit`` stay strings, as there), the same
variant-id decoding (base64 ``assembly\\tchrom\\tpos\\tref\\talt``, point query
``start=[pos-1]``, ``end=[pos-1+len(alt)]``), the same carrier search
(:func:`sbeacon.variant_search.perform_variant_search_sync` with
``requestedGranularity='record'``, ``includeResultsetResponses='ALL'`` and
``passthrough={'includeSamples': True}``: the device sample path ORs the
carrier bit-planes of every hit allele), the same per-dataset sample sets
(``dataset_samples[id].update(sorted(names))``; individuals walks the
datasets sorted by id, biosamples in first-hit order), the same skip / limit
walk over each set and the same envelopes.

The reference then reads the chosen samples' rows from Athena
(``get_record_query``: ``INDIVIDUALS_TABLE`` / ``BIOSAMPLES_TABLE`` joined to
``ANALYSES_TABLE`` on ``_vcfsampleid``, the parts UNION-ed).  The metadata
store is out of scope; the rows come from
``catalog.entities(kind, dataset_id, sample_names)`` (in-memory tables by
default), UNION-deduplicated over whole rows and dumped without their
``_``-prefixed attributes (``jsons.dump(..., strip_privates=True)``).

Set iteration order: the reference walks a Python ``set`` of sample names,
so which samples a ``skip`` / ``limit`` window picks depends on the
interpreter's string-hash seed (``PYTHONHASHSEED``); the same set is built
here, so under the same seed and response order the same samples are picked.
"""
from __future__ import annotations

import base64
import json
from collections import OrderedDict, defaultdict

from . import responses
from .catalog import JobStatus, catalog as default_catalog
from .route_g_variants import _not_new
from .variant_search import perform_variant_search_sync


def _params(event):
    """(granularity, skip, limit, filters) as :86-120 / :116-150 read them."""
    if event['httpMethod'] == 'GET':
        params = event.get('queryStringParameters', dict()) or dict()
        filters_list = []
        filters_str = params.get('filters', filters_list)
        if isinstance(filters_str, str):
            filters_list = filters_str.split(',')
        return (params.get('requestedGranularity', 'boolean'), params.get('skip', 0), params.get('limit', 100),
                [{'id': f} for f in filters_list])
    if event['httpMethod'] == 'POST':
        params = json.loads(event.get('body', '{}')) or dict()
        query = params.get('query', dict())
        pagination = query.get('pagination', dict())
        return (query.get('requestedGranularity', 'boolean'), pagination.get('skip', 0), pagination.get('limit', 100),
                query.get('filters', []))
    raise UnboundLocalError("local variable 'requestedGranularity' referenced before assignment")


def _decode(event):
    """The variant id of :122-128 -> (assembly, chrom, pos0, ref, alt)."""
    variant_id = event['pathParameters'].get('id', None)
    dataset_hash = base64.b64decode(variant_id.encode()).decode()
    assembly_id, reference_name, pos, reference_bases, alternate_bases = dataset_hash.split('\t')
    return assembly_id, reference_name, int(pos) - 1, reference_bases, alternate_bases


def _carrier_sets(granularity, filters, variant, query_id, catalog):
    """The variant search of :132-169 -> (exists, {dataset_id: set(sample names)})."""
    assembly_id, reference_name, pos, reference_bases, alternate_bases = variant
    datasets, samples = catalog.resolve(filters, assembly_id)
    query_responses = perform_variant_search_sync(
        datasets=datasets, referenceName=reference_name, referenceBases=reference_bases,
        alternateBases=alternate_bases, start=[pos], end=[pos + len(alternate_bases)], variantType=None,
        variantMinLength=0, variantMaxLength=-1, requestedGranularity='record', includeResultsetResponses='ALL',
        query_id=query_id, dataset_samples=samples, passthrough={'includeSamples': True})
    dataset_samples = defaultdict(set)
    exists = False
    for query_response in query_responses:
        exists = exists or query_response.exists
        if query_response.exists:
            if granularity == 'boolean':
                break
            dataset_samples[query_response.dataset_id].update(sorted(query_response.sample_names))
    return exists, dataset_samples


def _union_rows(rows):
    """SQL UNION: whole-row duplicates dropped (first occurrence kept)."""
    out, seen = [], set()
    for r in rows:
        k = json.dumps(r, sort_keys=True, default=str)
        if k not in seen:
            seen.add(k)
            out.append(r)
    return out


def _strip_privates(rows):
    return [{k: v for k, v in r.items() if not k.startswith('_')} for r in rows]


def _route(event, query_id, catalog, kind, ordered):
    catalog = catalog or default_catalog
    granularity, skip, limit, filters = _params(event)
    variant = _decode(event)
    status = catalog.job_status(query_id)
    if status != JobStatus.NEW:
        return _not_new(status, query_id, catalog)
    exists, dataset_samples = _carrier_sets(granularity, filters, variant, query_id, catalog)
    items = OrderedDict(sorted(dataset_samples.items())) if ordered else dataset_samples
    chosen = []  # (dataset_id, [sample names]) -> one get_record_query each
    iterated = 0
    picked = 0
    for dataset_id, sample_names in items.items():
        if len(sample_names) > 0:
            if granularity == 'count':
                iterated += len(sample_names)
            elif granularity in ('record', 'aggregated'):
                chosen_samples = []
                for sample_name in sample_names:
                    iterated += 1
                    if iterated > skip and picked < limit:
                        chosen_samples.append(sample_name)
                        picked += 1
                    if picked == limit:
                        break
                if len(chosen_samples) > 0:
                    chosen.append((dataset_id, chosen_samples))
    if granularity == 'boolean':
        return responses.bundle_response(200, responses.get_boolean_response(exists=exists), query_id)
    if granularity == 'count':
        return responses.bundle_response(200, responses.get_counts_response(exists=iterated > 0, count=iterated),
                                         query_id)
    if granularity in ('record', 'aggregated'):
        rows = []
        for dataset_id, names in chosen:
            rows.extend(catalog.entities(kind, dataset_id, names))
        rows = _union_rows(rows) if chosen else []
        return responses.bundle_response(200, responses.get_result_sets_response(
            setType=kind, reqPagination=responses.get_pagination_object(skip=skip, limit=limit),
            exists=len(rows) > 0, total=len(rows), results=_strip_privates(rows)), query_id)
    return None


def route_individuals(event, query_id, *, catalog=None):
    """GET/POST /g_variants/{id}/individuals (route_g_variants_id_individuals.py:86-238)."""
    return _route(event, query_id, catalog, 'individuals', ordered=True)


def route_biosamples(event, query_id, *, catalog=None):
    """GET/POST /g_variants/{id}/biosamples (route_g_variants_id_biosamples.py:116-266)."""
    return _route(event, query_id, catalog, 'biosamples', ordered=False)
