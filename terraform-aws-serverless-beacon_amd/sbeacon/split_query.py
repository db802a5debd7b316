"""splitQuery handler: cut [start_min, start_max] into 10 kb slices.

Mirrors ``lambda/splitQuery/lambda_function.py:74-128``.  The reference
invokes one performQuery Lambda per (slice x VCF) over a 32-thread pool and
returns their responses in completion order; here every slice payload is
built the same way and the whole fan-out is answered by ONE batched device
call, returned in deterministic (slice, VCF) order.  A slice whose query the
reference would crash on is returned as the Lambda error payload
(``{'errorMessage', 'errorType'}``) a failed synchronous invoke yields.
"""
from __future__ import annotations

import json

from .payloads import PerformQueryPayload, SplitQueryPayload
from .perform_query import perform_query_batch

SPLIT_SIZE = 10000  # lambda_function.py:12


def _as_obj(p):
    if isinstance(p, SplitQueryPayload):
        return p
    return SplitQueryPayload.load(p)


def split_payloads(split_payload) -> list[dict]:
    """The PerformQueryPayloads of lambda_function.py:82-106, in order."""
    sp = _as_obj(split_payload)
    check_all = sp.include_datasets in ('HIT', 'ALL')
    out = []
    split_start = sp.start_min
    while split_start <= sp.start_max:
        split_end = min(split_start + SPLIT_SIZE - 1, sp.start_max)
        for vcf_location, chrom in sp.vcf_locations.items():
            out.append(PerformQueryPayload(
                passthrough=sp.passthrough, dataset_id=sp.dataset_id, query_id=sp.query_id,
                reference_bases=sp.reference_bases, end_min=sp.end_min, end_max=sp.end_max,
                alternate_bases=sp.alternate_bases, variant_type=sp.variant_type,
                requested_granularity=sp.requested_granularity,
                variant_min_length=sp.variant_min_length, variant_max_length=sp.variant_max_length,
                include_details=check_all, region=f'{chrom}:{split_start}-{split_end}',
                vcf_location=vcf_location).dump())
        split_start += SPLIT_SIZE
    return out


def lambda_error(e: Exception) -> dict:
    return {'errorMessage': str(e), 'errorType': type(e).__name__}


def split_query_sync(split_payload) -> list[dict]:
    payloads = split_payloads(split_payload)
    if not payloads:
        return []
    res = perform_query_batch(payloads)
    return [lambda_error(r) if isinstance(r, Exception) else r.dump() for r in res]


def lambda_handler(event, context):
    try:  # SNS (async) events publish to performQuery; here they run synchronously too
        event = json.loads(event['Records'][0]['Sns']['Message'])
    except Exception:
        pass
    return split_query_sync(SplitQueryPayload.load(event))
