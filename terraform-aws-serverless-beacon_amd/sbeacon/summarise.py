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


def region_file_keys(store, location, slices, refs=None):
    """The S3 keys summariseSlice writes for these slices of one VCF
    (write_data_to_s3.h:93-101: vcf-summaries/contig/{CHROM}/{bucket%key}/
    regions/{first}-{last}-{bytes}), in slice then file order.  Each key's
    file -- (location, virtual_start, virtual_end, file index), what a
    duplicateVariantSearch of the key reads -- goes into the store's region
    file map (sbeacon.dedup.region_file_refs; a later file with the same key
    replaces it, as an S3 PUT does) and into ``refs`` when given."""
    from .dedup import bucket_key
    bk = bucket_key(location)
    known = store.__dict__.setdefault('_region_refs', {})
    keys = []
    for sl, files in zip(slices, store.region_files([(location, a, b) for a, b in slices])):
        if isinstance(files, Exception):
            raise files
        for i, f in enumerate(files):
            k = f"vcf-summaries/contig/{f['contig']}/{bk}/regions/{f['first_pos']}-{f['last_pos']}-{f['bytes']}"
            keys.append(k)
            known[k] = (location, sl[0], sl[1], i)
            if refs is not None:
                refs[k] = known[k]
    return keys


def strict_dedup_default() -> bool:
    """duplicateVariantSearch reads the region files exactly as the
    reference does (sb_dedup_count_files) unless SBEACON_STRICT_DEDUP=0,
    which counts the intended inclusive range instead (sb_dedup_count)."""
    from .dedup import strict_default
    return strict_default()


def summarise_dataset(store, dataset, locations, *, tally=None, abs_max=None, strict=None, vcf_groups=None):
    """The ingest pipeline of one dataset on the device: summariseVcf's slice
    plan + summariseSlice counts for every VCF (lambda/summariseVcf,
    lambda/summariseSlice), the region-file keys those slices write, then
    initDuplicateVariantSearch's range splits (lambda/summariseDataset/
    initDuplicateVariantSearch.py:235-255) answered by duplicateVariantSearch
    (one batched device call).  Returns the dataset's counts:
    variantCount / callCount from the summaries (summariseDataset
    lambda_function.py:102-125) and uniqueVariants = the sum of the ranges'
    distinct counts (the DATASETS_TABLE variantCount duplicateVariantSearch
    leaves, duplicateVariantSearch.cpp:76-84).  strict (default: unless
    SBEACON_STRICT_DEDUP=0): the reference's file-reading semantics.
    sampleCount is counted once per VCF group (summariseDataset
    lambda_function.py:118-124; vcf_groups defaults to one group of all the
    locations, submitDataset lambda_function.py:93)."""
    from .dedup import DuplicateTally, dedup_batch, init_duplicate_variant_search
    from .summarise_vcf import summarise_vcf
    strict = strict_dedup_default() if strict is None else strict
    tally = tally or DuplicateTally()
    counts = {'variantCount': 0, 'callCount': 0}
    keys = []
    refs = {}
    group_of = {loc: i for i, grp in enumerate(vcf_groups or [list(locations)]) for loc in grp}
    counted = set()
    for loc in locations:
        slices, _, tot = summarise_vcf(store, loc)
        counts['variantCount'] += tot['variantCount']
        counts['callCount'] += tot['callCount']
        if 'sampleCount' in tot and group_of[loc] not in counted:
            counts['sampleCount'] = counts.get('sampleCount', 0) + tot['sampleCount']
            counted.add(group_of[loc])
        keys += region_file_keys(store, loc, slices, refs)
    messages = init_duplicate_variant_search(dataset, locations, keys, tally=tally, abs_max=abs_max)
    per_range = dedup_batch(messages, tally=tally, registry=_single_store_registry(store),
                            file_refs=refs, strict=strict) if messages else []
    for r in per_range:
        if isinstance(r, Exception):
            raise r
    counts['uniqueVariants'] = tally.dataset_counts.get(dataset, 0)
    counts['ranges'] = len(messages)
    return counts, messages, per_range


def _single_store_registry(store):
    from .engine import Registry
    reg = Registry()
    reg.register(store)
    return reg
