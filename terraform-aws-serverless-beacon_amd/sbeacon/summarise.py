"""summariseSlice handler backed by the HBM store.

Mirrors ``lambda/summariseSlice/source/main.cpp:440-467``: the SNS message
``{"location", "virtual_start", "virtual_end"}`` names one BGZF virtual-offset
slice of a VCF; the result is that slice's ``RegionStats`` (``numVariants`` =
sum over visited records of 1 + commas in INFO/AC, ``numCalls`` = sum of
INFO/AN, ``main.cpp:43-109``), including the reference's skip heuristic
(``main.cpp:226,234-235``).  The DynamoDB ``ADD variantCount, callCount`` and
the region-file upload (``write_data_to_s3.h``) are storage plumbing and out of
scope; the counts are returned instead.  Many slices go to the device in one
call (``summarise_batch``) — the analogue of summariseVcf's SNS fan-out
(``lambda/summariseVcf/lambda_function.py:217-229``).
"""
from __future__ import annotations

import json

from .engine import registry


def summarise_batch(messages):
    """messages: dicts {location, virtual_start, virtual_end} -> RegionStats dicts."""
    groups = {}
    for i, m in enumerate(messages):
        s = registry.store_for(m['location'])
        groups.setdefault(id(s), (s, []))[1].append(i)
    out = [None] * len(messages)
    for store, idx in groups.values():
        res = store.summarise_slices([(messages[i]['location'], messages[i]['virtual_start'],
                                       messages[i]['virtual_end']) for i in idx])
        for i, r in zip(idx, res):
            out[i] = r
    return out


def summarise_slice(location, virtual_start, virtual_end):
    r = summarise_batch([{'location': location, 'virtual_start': virtual_start, 'virtual_end': virtual_end}])[0]
    if isinstance(r, Exception):
        raise r
    return {'numVariants': r['numVariants'], 'numCalls': r['numCalls']}


def lambda_handler(event, context=None):
    msg = event
    try:  # main.cpp:446-453: Records[0].Sns.Message is a JSON string
        msg = json.loads(event['Records'][0]['Sns']['Message'])
    except (KeyError, IndexError, TypeError):
        pass
    return summarise_slice(msg['location'], int(msg['virtual_start']), int(msg['virtual_end']))
