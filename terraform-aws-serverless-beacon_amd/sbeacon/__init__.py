"""sbeacon — MI355X-native engine for sBeacon's genomic-variant query path.

Host-side mirror of the reference's operator interface
(splitQuery -> performQuery) over ``libsbeacon_hip.so``.
"""
from .payloads import PerformQueryPayload, PerformQueryResponse, SplitQueryPayload  # noqa: F401

__all__ = ['PerformQueryPayload', 'PerformQueryResponse', 'SplitQueryPayload']
