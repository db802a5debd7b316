"""duplicateVariantSearch handler over the HBM store.

Mirrors lambda/duplicateVariantSearch/source/main.cpp:31-43 (the SNS message
{"bucket", "rangeStart", "rangeEnd", "contig", "targetFilepaths", "dataset"})
and duplicateVariantSearch.cpp:31-84 (unique region keys of the range, then
the two DynamoDB updates).  Each key in ``targetFilepaths`` names the VCF it
summarises (``vcf-summaries/contig/{CHROM}/{bucket%key}/regions/...``,
write_data_to_s3.h:39-101) and one region file of it; that VCF's region keys
are already resident in the store, so the unique count is one device call.
Many messages go to the device together through :func:`dedup_batch`.

Default (the reference's answer): every target file is read as
``ReadVcfData::getVcfData`` reads it (readVcfData.cpp:15-35 over the gzip
reader of gzip.cpp:61-144: entries from the first POS >= rangeStart up to the
first one past rangeEnd inside the reader's final refill, a throw when a
skipped entry straddles its 1 KiB buffer), on the device
(``sb_dedup_count_files``).  The key resolves to its file through the region
files summariseSlice writes for the VCF's summariseVcf slices
(:func:`region_file_refs`).  ``SBEACON_STRICT_DEDUP=0`` (or ``strict=False``)
selects an extension instead: the distinct keys of the intended inclusive
range ``[rangeStart, rangeEnd]`` (``sb_dedup_count``), with no dependence on
how the region files were cut.

The two DynamoDB tables the reference updates are modelled by
:class:`DuplicateTally` (VARIANT_DUPLICATES_TABLE: per (contig, dataset) an
``ADD variantCount`` + ``DELETE toUpdate`` of the finished range, conditional
on the range still being listed) and its ``dataset_counts`` (DATASETS_TABLE
``ADD variantCount`` once every range of the contig has reported,
duplicateVariantSearch.cpp:76-84,86-200).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

from . import engine

# main.tf:16,128 (maximum_load_file_size -> ABS_MAX_DATA_SPLIT)
ABS_MAX_DATA_SPLIT = int(os.environ.get('ABS_MAX_DATA_SPLIT', 750_000_000))


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


# ------------------------------------------------ initDuplicateVariantSearch
# lambda/summariseDataset/initDuplicateVariantSearch.py: the (contig, range,
# region files) jobs a dataset's duplicate search fans out, planned from the
# region-file keys summariseSlice wrote (sbeacon.summarise.region_file_keys).
@dataclass
class VcfRegionData:  # :21-27
    filepath: str
    filename: str
    filesize: int
    startRange: int
    endRange: int


@dataclass
class BasePairRange:  # :30-34
    start: int
    end: int
    filePaths: list = field(default_factory=list)


def get_file_name_info(filepath: str) -> VcfRegionData:
    """:77-89 — .../{filename}/regions/{first}-{last}-{bytes}."""
    parts = filepath.split('/')
    rng = parts[-1].split('-')
    return VcfRegionData(filepath, parts[-3], int(rng[2]), int(rng[0]), int(rng[1]))


def filter_range(region_data, start, end):
    """:92-99 — the files overlapping [start, end] and their summed size."""
    files = [rd for rd in region_data if rd.startRange <= end and rd.endRange >= start]
    return sum(rd.filesize for rd in files), files


def add_range(region_data, start_range, end_range, range_slices, abs_max=None):
    """:103-125 — shrink the range end to a file end until the overlapping
    files fit abs_max (or nothing smaller exists), record it, and return the
    next start and the index after its last file."""
    abs_max = ABS_MAX_DATA_SPLIT if abs_max is None else abs_max
    size, files = filter_range(region_data, start_range, end_range)
    while size > abs_max:
        try:
            new_end = max(f.endRange for f in files if f.endRange < end_range)
            size, files = filter_range(files, start_range, new_end)
        except ValueError:  # no smaller end: keep the range (the reference prints and continues)
            new_end = end_range
        if end_range == new_end:
            break
        end_range = new_end
    range_slices.append(BasePairRange(start_range, end_range, [f.filepath for f in files]))
    return end_range + 1, region_data.index(files[-1]) + 1


def calc_range_splits(region_data, abs_max=None, max_iterations=10_000_000):
    """:171-191 — greedy ranges of region files whose summed size stays under
    abs_max.  The reference loops until the range start passes the last
    file's end; inputs on which it never does (it would spin until the
    Lambda times out) raise RuntimeError after max_iterations."""
    abs_max = ABS_MAX_DATA_SPLIT if abs_max is None else abs_max
    range_slices = []
    running_total = 0
    start_range = region_data[0].startRange
    item_inc = 0
    min_data_split = abs_max - region_data[0].filesize * 2
    it = 0
    while start_range - 1 != region_data[-1].endRange:
        it += 1
        if it > max_iterations:
            raise RuntimeError('calcRangeSplits does not terminate on this input (the reference spins)')
        element = region_data[item_inc]
        if running_total < min_data_split:
            running_total += element.filesize
            item_inc = item_inc + 1 if item_inc + 1 < len(region_data) else item_inc
        else:
            start_range, item_inc = add_range(region_data, start_range, element.endRange, range_slices, abs_max)
            running_total = 0
    if running_total != 0:
        add_range(region_data, start_range, max(r.endRange for r in region_data), range_slices, abs_max)
    return range_slices


def init_duplicate_variant_search(dataset, filepaths, region_keys, *, bucket='variants', tally=None,
                                  abs_max=None):
    """:235-255 — for every contig with region files of the dataset's VCFs
    (``region_keys``: every region-file key of the variants bucket, the
    listing retrieveS3Objects does), the range splits as
    duplicateVariantSearch SNS messages; with a DuplicateTally, the
    mark_updating / clearDatasetVariantCount writes too."""
    filenames = ['/' + fn[5:-7].replace('/', '%') + '/' for fn in filepaths]
    by_contig = {}
    for k in region_keys:
        parts = k.split('/')
        if len(parts) >= 6 and parts[0] == 'vcf-summaries' and parts[1] == 'contig':
            by_contig.setdefault(parts[2], []).append(k)
    if tally is not None:
        tally.dataset_counts[dataset] = 0
    messages = []
    for contig, keys in by_contig.items():
        region = [get_file_name_info(k) for k in keys if any(fn in k for fn in filenames)]
        if not region:
            continue
        region.sort(key=lambda x: x.startRange)
        splits = calc_range_splits(region, abs_max)
        if tally is not None:
            tally.expect(contig, dataset, [(s.start, s.end) for s in splits])
        for s in splits:
            messages.append({'bucket': bucket, 'rangeStart': s.start, 'rangeEnd': s.end, 'contig': contig,
                             'targetFilepaths': s.filePaths, 'dataset': dataset})
    return messages


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


def strict_default() -> bool:
    """The reference's file-reading semantics unless SBEACON_STRICT_DEDUP=0."""
    return os.environ.get('SBEACON_STRICT_DEDUP', '1') != '0'


def region_file_refs(store, location) -> dict:
    """region-file key -> (location, virtual_start, virtual_end, file index)
    for every region file summariseSlice writes for ``location``
    (write_data_to_s3.h:39-101) over the slices summariseVcf plans for it
    (summarise_vcf.plan_slices); built once per store and VCF.  Keys that
    sbeacon.summarise.region_file_keys produced for other slices of the store
    are in the same map (a later file with the same key replaces the earlier,
    as an S3 PUT does)."""
    refs = store.__dict__.setdefault('_region_refs', {})
    planned = store.__dict__.setdefault('_region_refs_planned', set())
    if location not in planned:
        from .summarise import region_file_keys
        from .summarise_vcf import plan_slices
        region_file_keys(store, location, plan_slices(store, location))
        planned.add(location)
    return refs


def dedup_batch(messages, *, tally: DuplicateTally | None = None, registry=None, file_refs=None, strict=None):
    """Answer many duplicateVariantSearch messages with one device call per
    store.  Returns the unique count per message (or the exception).

    strict (default :func:`strict_default`): the reference's count -- each
    target file read as ReadVcfData::getVcfData reads it
    (sb_dedup_count_files); its key resolves through ``file_refs`` (key ->
    (location, virtual_start, virtual_end, file index),
    summarise.region_file_keys) or else the store's :func:`region_file_refs`;
    a key naming no region file the store's summaries write is that
    message's KeyError (the reference's S3 download would fail).  strict
    False: the intended inclusive range (sb_dedup_count)."""
    strict = strict_default() if strict is None else strict
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
        if not strict:
            res = st.dedup_counts([jobs[i] for i in idx])
            for i, r in zip(idx, res):
                out[i] = r
            continue
        calls, call_idx = [], []
        for i in idx:
            refs = []
            try:
                for p in messages[i]['targetFilepaths']:
                    fr = file_refs.get(p) if file_refs is not None else None
                    if fr is None:
                        fr = region_file_refs(st, _location_of(p, jobs[i][0])).get(p)
                    if fr is None:
                        raise KeyError(f'no region file {p!r} in the summaries of the store')
                    refs.append(fr)
            except KeyError as e:
                out[i] = e
                continue
            calls.append((refs, jobs[i][2], jobs[i][3]))
            call_idx.append(i)
        if calls:
            for i, r in zip(call_idx, st.dedup_counts_files(calls)):
                out[i] = r
    if tally is not None:
        for m, (locs, contig, rs, re_), r in zip(messages, jobs, out):
            if isinstance(r, Exception):
                continue
            final = tally.update_duplicates(contig, m['dataset'], rs, re_, r)
            if final >= 0:
                tally.update_counts(m['dataset'], final)
    return out


def _location_of(path, locations):
    k = region_path_bucket_key(path)
    for l in locations:
        if bucket_key(l) == k:
            return l
    raise KeyError(path)


def lambda_handler(event, context=None, *, tally: DuplicateTally | None = None, strict=None):
    """SNS event -> the reference's bundleResponse("Success", 200)
    (duplicateVariantSearch/source/main.cpp:11-47); the count the reference
    adds to its tables rides along as ``uniqueVariants``.  A reader throw
    (gzip.cpp:97 "proccesData input invalid") is raised, as the Lambda
    fails."""
    rec = event['Records'][0]['Sns']['Message'] if 'Records' in event else event
    msg = json.loads(rec) if isinstance(rec, str) else rec
    r = dedup_batch([msg], tally=tally, strict=strict)[0]
    if isinstance(r, Exception):
        raise r
    return {'headers': {'Access-Control-Allow-Origin': '*'}, 'statusCode': 200, 'body': 'Success',
            'uniqueVariants': r}
