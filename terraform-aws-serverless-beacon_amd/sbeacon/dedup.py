"""duplicateVariantSearch handler over the HBM store.

Mirrors lambda/duplicateVariantSearch/source/main.cpp:31-43 (the SNS message
{"bucket", "rangeStart", "rangeEnd", "contig", "targetFilepaths", "dataset"})
and duplicateVariantSearch.cpp:31-84 (unique region keys of the range, then
the two DynamoDB updates).  The region files named in ``targetFilepaths``
are not read: each names the VCF it summarises
(``vcf-summaries/contig/{CHROM}/{bucket%key}/regions/...``,
write_data_to_s3.h:39-101, summariseSlice main.cpp), and that VCF's region
keys are already resident in the store, so the unique count is one device
call (``sb_dedup_count``).  Many messages go to the device together through
:func:`dedup_batch`.

The two DynamoDB tables the reference updates are modelled by
:class:`DuplicateTally` (VARIANT_DUPLICATES_TABLE: per (contig, dataset) an
``ADD variantCount`` + ``DELETE toUpdate`` of the finished range, conditional
on the range still being listed) and its ``dataset_counts`` (DATASETS_TABLE
``ADD variantCount`` once every range of the contig has reported,
duplicateVariantSearch.cpp:76-84,86-200).
"""
from __future__ import annotations

import json

from . import engine


def bucket_key(location: str) -> str:
    """writeDataToS3's s3BucketKey: the location minus its first 5 ("s3://")
    and last 7 (".vcf.gz") characters, '/' -> '%' (write_data_to_s3.h:137-142)."""
    return location[5:5 + max(len(location) - 12, 0)].replace('/', '%')


def region_path_bucket_key(path: str) -> str:
    """The {bucket%key} component of a region-file key
    vcf-summaries/contig/{CHROM}/{bucket%key}/regions/{first}-{last}
    (write_data_to_s3.h:94-101)."""
    parts = path.split('/')
    if len(parts) < 6 or parts[0] != 'vcf-summaries' or parts[1] != 'contig' or parts[-2] != 'regions':
        raise ValueError(f'not a region-file key: {path!r}')
    return parts[-3]


def message_job(msg: dict, locations):
    """SNS message -> (vcf_locations, contig, range_start, range_end); each
    target file is resolved to the registered VCF it summarises."""
    by_key = {}
    for l in locations:
        by_key.setdefault(bucket_key(l), []).append(l)
    locs = []
    for p in msg['targetFilepaths']:
        k = region_path_bucket_key(p)
        if len(by_key.get(k, ())) != 1:
            raise KeyError(f'region file {p!r} names {len(by_key.get(k, ()))} registered VCFs (need exactly 1)')
        if by_key[k][0] not in locs:
            locs.append(by_key[k][0])
    return locs, msg['contig'], int(msg['rangeStart']), int(msg['rangeEnd'])


class DuplicateTally:
    """In-memory stand-in for VARIANT_DUPLICATES_TABLE + DATASETS_TABLE."""

    def __init__(self):
        self.items = {}           # (contig, dataset) -> {'variantCount': int, 'toUpdate': set}
        self.dataset_counts = {}  # dataset -> variantCount

    def expect(self, contig, dataset, ranges):
        """What initDuplicateVariantSearch writes before fanning out
        (summariseDataset/initDuplicateVariantSearch.py)."""
        self.items[(contig, dataset)] = {'variantCount': 0, 'toUpdate': {(int(a), int(b)) for a, b in ranges}}

    def update_duplicates(self, contig, dataset, rs, re_, count) -> int:
        """updateVariantDuplicates: -1 until the last range reports, then the
        contig's total (duplicateVariantSearch.cpp:125-200)."""
        item = self.items.get((contig, dataset))
        if item is None or (rs, re_) not in item['toUpdate']:
            return -1  # ConditionalCheckFailed -> not retried
        item['variantCount'] += count
        item['toUpdate'].discard((rs, re_))
        return -1 if item['toUpdate'] else item['variantCount']

    def update_counts(self, dataset, final_tally):
        self.dataset_counts[dataset] = self.dataset_counts.get(dataset, 0) + final_tally


def dedup_batch(messages, *, tally: DuplicateTally | None = None, registry=None):
    """Answer many duplicateVariantSearch messages with one device call per
    store.  Returns the unique count per message (or the exception)."""
    reg = registry or engine.registry
    known = reg.locations()
    jobs = [message_job(m, known) for m in messages]
    by_store = {}
    for i, (locs, contig, rs, re_) in enumerate(jobs):
        stores = {id(reg.store_for(l)): reg.store_for(l) for l in locs}
        if len(stores) > 1:
            raise ValueError('a dedup job spans several stores; shard datasets whole')
        st = next(iter(stores.values())) if stores else None
        by_store.setdefault(id(st), (st, []))[1].append(i)
    out = [None] * len(jobs)
    for st, idx in by_store.values():
        if st is None:
            for i in idx:
                out[i] = 0
            continue
        res = st.dedup_counts([jobs[i] for i in idx])
        for i, r in zip(idx, res):
            out[i] = r
    if tally is not None:
        for m, (locs, contig, rs, re_), r in zip(messages, jobs, out):
            if isinstance(r, Exception):
                continue
            final = tally.update_duplicates(contig, m['dataset'], rs, re_, r)
            if final >= 0:
                tally.update_counts(m['dataset'], final)
    return out


def lambda_handler(event, context=None, *, tally: DuplicateTally | None = None):
    """SNS event -> the reference's bundleResponse("Success", 200)
    (duplicateVariantSearch/source/main.cpp:11-47)."""
    rec = event['Records'][0]['Sns']['Message'] if 'Records' in event else event
    msg = json.loads(rec) if isinstance(rec, str) else rec
    r = dedup_batch([msg], tally=tally)[0]
    if isinstance(r, Exception):
        raise r
    return {'headers': {'Access-Control-Allow-Origin': '*'}, 'statusCode': 200, 'body': 'Success',
            'uniqueVariants': r}
