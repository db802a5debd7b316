"""Wire types of the variant query path, field-for-field identical to the
reference (``shared_resources/payloads/lambda_payloads.py:8-77`` and
``lambda_responses.py:14-23``), without the ``jsons`` dependency: ``dump()``
returns the same dict ``jsons`` produced and ``load()`` accepts it back.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, fields


class _Serializable:
    def dump(self) -> dict:
        return dict(self.__dict__)

    def dumps(self) -> str:
        return json.dumps(self.dump())

    @classmethod
    def load(cls, d: dict):
        return cls(**d)

    @classmethod
    def loads(cls, s: str):
        return cls.load(json.loads(s))


class SplitQueryPayload(_Serializable):
    """lambda_payloads.py:8-44."""

    def __init__(self, *, passthrough={}, dataset_id, query_id, reference_bases, start_min, start_max,
                 end_min, end_max, alternate_bases, variant_type, include_datasets, vcf_locations,
                 vcf_groups, requested_granularity, variant_min_length, variant_max_length):
        self.passthrough = passthrough
        self.dataset_id = dataset_id
        self.query_id = query_id
        self.reference_bases = reference_bases
        self.start_min = start_min
        self.start_max = start_max
        self.end_min = end_min
        self.end_max = end_max
        self.alternate_bases = alternate_bases
        self.variant_type = variant_type
        self.include_datasets = include_datasets
        self.vcf_locations = vcf_locations
        self.vcf_groups = vcf_groups
        self.requested_granularity = requested_granularity
        self.variant_min_length = variant_min_length
        self.variant_max_length = variant_max_length


class PerformQueryPayload(_Serializable):
    """lambda_payloads.py:46-77."""

    def __init__(self, *, passthrough={}, dataset_id=None, query_id='test', region=None,
                 reference_bases=None, end_min=None, end_max=None, alternate_bases=None,
                 variant_type=None, include_details=None, requested_granularity=None,
                 variant_min_length=None, variant_max_length=None, vcf_location=None):
        self.passthrough = passthrough
        self.dataset_id = dataset_id
        self.query_id = query_id
        self.region = region
        self.reference_bases = reference_bases
        self.end_min = end_min
        self.end_max = end_max
        self.alternate_bases = alternate_bases
        self.variant_type = variant_type
        self.include_details = include_details
        self.requested_granularity = requested_granularity
        self.variant_min_length = variant_min_length
        self.variant_max_length = variant_max_length
        self.vcf_location = vcf_location


@dataclass
class PerformQueryResponse(_Serializable):
    """lambda_responses.py:14-23."""
    exists: bool
    vcf_location: str
    dataset_id: str
    all_alleles_count: int
    variants: list
    call_count: int
    sample_indices: list = field(default_factory=list)
    sample_names: list = field(default_factory=list)

    def dump(self) -> dict:
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        if not isinstance(d['variants'], list):  # engine.LazyVariants
            d['variants'] = list(d['variants'])
        return d
