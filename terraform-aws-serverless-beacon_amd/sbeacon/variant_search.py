"""Variant-search fan-out (``shared_resources/variantutils/search_variants.py:158-244``).

Same coordinate conversion (Beacon 0-based start/end -> 1-based bracket,
``:179-199``), same chromosome matching, same per-dataset ``SplitQueryPayload``
(including the ``sampleNames`` / ``selectedSamplesOnly`` passthrough when
``dataset_samples`` is given, ``:213-218``).  Instead of a 500-thread pool of
synchronous splitQuery invokes, every slice of every dataset goes to the
device in one batch per store.
"""
from __future__ import annotations

import copy

from .chrom_matching import get_matching_chromosome
from .payloads import PerformQueryResponse, SplitQueryPayload
from .perform_query import perform_query_batch
from .split_query import split_payloads


def split_query_payloads(*, datasets, referenceName, referenceBases, alternateBases, start, end, variantType,
                         variantMinLength, variantMaxLength, requestedGranularity, includeResultsetResponses,
                         query_id='TEST', passthrough=dict(), dataset_samples=[]):
    """The SplitQueryPayload of each dataset (search_variants.py:176-238),
    or None where the reference takes its ``except`` branch (:192-194)."""
    try:
        vcf_chromosomes = {vcfm['vcf']: get_matching_chromosome(vcfm['chromosomes'], referenceName)
                           for dataset in datasets for vcfm in dataset._vcfChromosomeMap}
        if len(start) == 2:
            start_min, start_max = start
        else:
            start_min = start[0]
        if len(end) == 2:
            end_min, end_max = end
        else:
            end_min = start_min
            end_max = end[0]
        if len(start) != 2:
            start_max = end_max
    except Exception as e:  # :192-194 (the caller then iterates the tuple)
        print('Error occured ', e)
        return None
    start_min += 1
    start_max += 1
    end_min += 1
    end_max += 1

    out = []
    for n, dataset in enumerate(datasets):
        vcf_locations = {vcf: vcf_chromosomes[vcf] for vcf in dataset._vcfLocations if vcf_chromosomes[vcf]}
        event_passthrough = copy.deepcopy(passthrough)
        if len(dataset_samples) == len(datasets) and len(dataset_samples[n]) > 0:
            event_passthrough['sampleNames'] = dataset_samples[n]
            event_passthrough['selectedSamplesOnly'] = True
        out.append(SplitQueryPayload(
            passthrough=event_passthrough, dataset_id=dataset.id, query_id=query_id,
            vcf_locations=vcf_locations, vcf_groups=[], reference_bases=referenceBases,
            start_min=start_min, start_max=start_max, end_min=end_min, end_max=end_max,
            alternate_bases=alternateBases, variant_type=variantType,
            include_datasets=includeResultsetResponses, requested_granularity=requestedGranularity,
            variant_min_length=variantMinLength, variant_max_length=variantMaxLength))
    return out


def perform_variant_search_sync(*, datasets, referenceName, referenceBases, alternateBases, start, end,
                                variantType, variantMinLength, variantMaxLength, requestedGranularity,
                                includeResultsetResponses, query_id='TEST', passthrough=dict(),
                                dataset_samples=[]):
    sps = split_query_payloads(
        datasets=datasets, referenceName=referenceName, referenceBases=referenceBases, alternateBases=alternateBases,
        start=start, end=end, variantType=variantType, variantMinLength=variantMinLength,
        variantMaxLength=variantMaxLength, requestedGranularity=requestedGranularity,
        includeResultsetResponses=includeResultsetResponses, query_id=query_id, passthrough=passthrough,
        dataset_samples=dataset_samples)
    if sps is None:
        return False, []
    payloads = []
    for sp in sps:
        payloads.extend(split_payloads(sp))
    if not payloads:
        return []
    out = []
    for r in perform_query_batch(payloads, lazy_variants=True):
        if isinstance(r, Exception):
            raise r  # the reference fails loading a Lambda error payload here (:244)
        out.append(r)
    return out
