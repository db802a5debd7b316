"""Dataset catalog: the slice of the reference's metadata layer the variant
routes read.

The reference resolves an ``assemblyId`` (and optional Beacon ``filters``) to
datasets with an Athena query (``route_g_variants.py:28-47,119-128``;
``athena/dataset.py:21-66`` holds ``id``, ``_vcfLocations``,
``_vcfChromosomeMap``).  The Athena/S3/DynamoDB metadata plumbing is out of
scope, so datasets are registered here in memory with the same
attribute names, and ``filters`` resolution is a pluggable hook
(``filter_resolver(filters, assembly_id) -> {dataset_id: [sample names]}``,
the ``ARRAY_AGG(A._vcfsampleid)`` of ``datasets_query``).
"""
from __future__ import annotations

from enum import Enum


class JobStatus(Enum):
    """dynamodb/variant_queries.py JobStatus."""
    NEW = 1
    RUNNING = 2
    COMPLETED = 3


class Dataset:
    """athena/dataset.py:21-66 (fields the variant path reads)."""

    def __init__(self, *, id='', assemblyId='', vcfLocations=(), vcfChromosomeMap=()):
        self.id = id
        self._assemblyId = assemblyId
        self._vcfLocations = list(vcfLocations)
        self._vcfChromosomeMap = list(vcfChromosomeMap)

    def __eq__(self, other):
        return isinstance(other, Dataset) and self.id == other.id

    def __hash__(self):
        return hash(self.id)

    def __repr__(self):
        return f'Dataset(id={self.id!r}, vcfs={len(self._vcfLocations)})'


class Catalog:
    def __init__(self):
        self._datasets: list[Dataset] = []
        self.filter_resolver = None
        self.job_status = lambda query_id: JobStatus.NEW
        self.cache: dict[str, dict] = {}  # fetch_from_cache stand-in (query-responses/{id}.json)
        self._entities: dict[str, dict] = {}  # kind -> dataset_id -> sample name -> [rows]
        self.entity_provider = None

    def add_entities(self, kind: str, dataset_id: str, rows: dict):
        """Metadata rows of one dataset (``kind`` = 'individuals' /
        'biosamples'), keyed by the VCF sample name that analyses map them
        from (``ANALYSES_TABLE._vcfsampleid``).  A value is one row or a list
        of rows (a sample with several analyses)."""
        tab = self._entities.setdefault(kind, {}).setdefault(dataset_id, {})
        for name, row in rows.items():
            tab.setdefault(name, []).extend(row if isinstance(row, list) else [row])

    def entities(self, kind: str, dataset_id: str, sample_names) -> list:
        """get_record_query(dataset_id, sample_names) of the sample routes
        (route_g_variants_id_individuals.py:64-83, _biosamples.py:95-113):
        the rows joined to the analyses of those samples.  A custom store is
        plugged in through ``entity_provider(kind, dataset_id, names)``."""
        if self.entity_provider is not None:
            return list(self.entity_provider(kind, dataset_id, list(sample_names)))
        tab = self._entities.get(kind, {}).get(dataset_id, {})
        return [dict(r) for n in sample_names for r in tab.get(n, [])]

    def add(self, dataset: Dataset):
        self._datasets = [d for d in self._datasets if d.id != dataset.id] + [dataset]
        return dataset

    def clear(self):
        self._datasets.clear()
        self.filter_resolver = None
        self.entity_provider = None
        self.cache.clear()
        self._entities.clear()

    def datasets_fast(self, assembly_id):
        """datasets_query_fast: every dataset of the assembly, no samples."""
        return [d for d in self._datasets if d._assemblyId == assembly_id]

    def resolve(self, filters, assembly_id):
        """(datasets, samples) as route_g_variants.py:119-128 builds them."""
        if filters:
            if self.filter_resolver is None:
                raise NotImplementedError('Beacon filters need the metadata store (Athena), which is out of '
                                          'scope; set catalog.filter_resolver')
            hits = self.filter_resolver(filters, assembly_id)
            ds = [d for d in self._datasets if d._assemblyId == assembly_id and d.id in hits]
            return ds, [list(hits[d.id]) for d in ds]
        return self.datasets_fast(assembly_id), []


catalog = Catalog()
