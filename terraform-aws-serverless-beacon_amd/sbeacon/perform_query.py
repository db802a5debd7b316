"""performQuery handler, backed by the HBM store instead of bcftools.

Mirrors ``lambda/performQuery/lambda_function.py:23-49`` (event handling and
the ``selectedSamplesOnly`` dispatch) and the two query modules
``search_variants.perform_query`` (``search_variants.py:33-271``) and
``search_variants_in_samples.perform_query`` (``search_variants_in_samples.py:31-259``):
same payload, same ``PerformQueryResponse``, same exception class where the
reference raises.  The dispatch on ``passthrough.selectedSamplesOnly`` happens
inside the engine (one flag per query), so a batch may mix both variants.

``STRICT_VARIANT_TYPE``: the reference raises ``UnboundLocalError`` for every
``alternate_bases=None`` (variantType) query that reaches a record
(``search_variants.py:101``).  By default the engine answers such queries
with the evident intent (branch on ``payload.variant_type``; SURVEY.md
§8a.1-4); set ``SBEACON_STRICT_VARIANT_TYPE=1`` to reproduce the crash.

The async path (``is_async``: the SNS-delivered event; ``:273-317``) also
records the response for the route's fan-in: a response number, the body
and ``markFinished`` on the query's record (``sbeacon.variant_queries``,
in process instead of DynamoDB/S3).
"""
from __future__ import annotations

import json
import os

from .engine import query_payloads
from .payloads import PerformQueryPayload, PerformQueryResponse

STRICT_VARIANT_TYPE = os.environ.get('SBEACON_STRICT_VARIANT_TYPE', '0') == '1'


def _as_dict(payload) -> dict:
    return payload.dump() if hasattr(payload, 'dump') else dict(payload)


def perform_query(payload, is_async=False) -> PerformQueryResponse:
    d = _as_dict(payload)
    res = query_payloads([d], strict_variant_type=STRICT_VARIANT_TYPE)[0]
    if isinstance(res, Exception):
        raise res
    if is_async:
        from .variant_queries import record_response
        record_response(d.get('query_id', 'test'), res)
    return res


def perform_query_batch(payloads, *, lazy_variants=False) -> list:
    """Batched entry: one device pass for many PerformQueryPayloads.
    Entries are responses or the exception the reference would raise."""
    return query_payloads([_as_dict(p) for p in payloads], strict_variant_type=STRICT_VARIANT_TYPE,
                          lazy_variants=lazy_variants)


def lambda_handler(event, context):
    is_async = False
    try:  # lambda_function.py:33-39 SNS unwrap
        event = json.loads(event['Records'][0]['Sns']['Message'])
        is_async = True
    except Exception:
        is_async = False
    payload = PerformQueryPayload.load(event)
    # lambda_function.py:43: a passthrough that is not an object raises here
    payload.passthrough.get('selectedSamplesOnly', False)
    return perform_query(payload, is_async).dump()
