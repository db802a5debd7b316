"""The async variant-search fan-in, in process.

The reference's asynchronous path publishes one SNS message per dataset to
splitQuery, each performQuery Lambda stores its response under the query id
and bumps the query record, and the route polls that record until every
slice has answered:

* ``shared_resources/dynamodb/variant_queries.py:29-59`` -- ``VariantQuery``
  (fanOut, responses, responsesCounter, start/end/elapsed time, a 5-minute
  TTL) with the atomic ``getResponseNumber`` / ``markFinished`` updates, and
  ``VariantResponse`` rows keyed by (query id, response number);
* ``lambda/performQuery/search_variants.py:273-317`` -- an async performQuery
  takes a response number, stores its JSON body (S3 above 300 KB, with
  ``checkS3``), then marks itself finished;
* ``shared_resources/variantutils/search_variants.py:27-155`` --
  ``perform_variant_search`` records the query, publishes, adds the fan-out
  (``get_split_query_fan_out`` x VCFs per dataset) and polls until
  ``fanOut == 0`` (``REQUEST_TIMEOUT``), then yields the responses in
  response-number order.

Here the tables are a locked in-process registry (the same fields and
atomic updates; bodies of any size stay in memory, ``checkS3`` still says
which ones the reference would have put in S3), "publishing" hands the
whole fan-out to a background worker that answers every slice of every
dataset in ONE device batch (``perform_query_batch``) and records each
response as its Lambda would, and the poll waits on a condition variable
instead of sleeping 0.5 s between reads.
"""
from __future__ import annotations

import json
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timedelta, timezone

REQUEST_TIMEOUT = 600        # search_variants.py:20 (seconds)
S3_BODY_LIMIT = 1024 * 300   # performQuery search_variants.py:283: larger bodies go to S3
TTL = timedelta(minutes=5)   # variant_queries.py:40 timeToExist


def _now():
    return datetime.now(timezone.utc)


class VariantQuery:
    """variant_queries.py:29-59: one query's fan-in record."""

    def __init__(self, id='test'):
        self.id = id
        self.responsesCounter = 0
        self.responses = 0
        self.fanOut = 0
        self.startTime = _now()
        self.endTime = None
        self.elapsedTime = -1
        self.complete = False
        self.timeToExist = self.startTime + TTL

    # the table operations (one lock for the whole table: every update is
    # atomic, as the DynamoDB update expressions are)
    def save(self):
        with _table.cv:
            _table.queries[self.id] = self
            _table.cv.notify_all()

    def refresh(self):
        with _table.cv:
            q = _table.queries.get(self.id)
            if q is None:
                raise KeyError(f'query {self.id!r} does not exist')
            self.__dict__.update(q.__dict__)

    def _row(self):
        """The stored record (an update of a missing item creates it, as
        DynamoDB's update_item does).  Call under the table lock."""
        q = _table.queries.get(self.id)
        if q is None:
            q = _table.queries[self.id] = VariantQuery(self.id)
        return q

    def add_fan_out(self, n: int):
        """``VariantQuery.fanOut.set(VariantQuery.fanOut + n)``"""
        with _table.cv:
            self._row().fanOut += n
            _table.cv.notify_all()

    def getResponseNumber(self) -> int:
        with _table.cv:
            q = self._row()
            q.responsesCounter += 1
            self.responsesCounter = q.responsesCounter
            return q.responsesCounter

    def markFinished(self):
        with _table.cv:
            q = self._row()
            q.responses += 1
            q.fanOut -= 1
            q.endTime = _now()
            _table.cv.notify_all()


class VariantResponse:
    """variant_queries.py (VariantResponse): one performQuery body."""

    def __init__(self, id, responseNumber=0, result=None, checkS3=False):
        self.id = id
        self.responseNumber = responseNumber
        self.result = result      # the response JSON (response.dumps())
        self.checkS3 = checkS3    # True where the reference stores the body in S3

    def save(self):
        with _table.cv:
            _table.responses[(self.id, self.responseNumber)] = self

    @staticmethod
    def batch_get(keys):
        with _table.cv:
            return [_table.responses[k] for k in keys if k in _table.responses]


class _Table:
    def __init__(self):
        self.cv = threading.Condition()
        self.queries: dict[str, VariantQuery] = {}
        self.responses: dict[tuple, VariantResponse] = {}

    def expire(self):
        """Drop the records whose TTL has passed (DynamoDB's TTL sweep)."""
        now = _now()
        with self.cv:
            gone = [k for k, q in self.queries.items() if q.timeToExist < now]
            for k in gone:
                del self.queries[k]
            if gone:
                self.responses = {k: v for k, v in self.responses.items() if k[0] not in gone}


_table = _Table()
_publisher = ThreadPoolExecutor(max_workers=2, thread_name_prefix='sbeacon-fanout')


def record_response(query_id: str, response) -> VariantResponse:
    """The async tail of performQuery (search_variants.py:273-317): a
    response number, the body, then markFinished."""
    _table.expire()
    query = VariantQuery(query_id)
    result = VariantResponse(query_id)
    result.responseNumber = query.getResponseNumber()
    body = response.dumps()
    result.result = body
    result.checkS3 = len(body) >= S3_BODY_LIMIT
    result.save()
    query.markFinished()
    return result


def perform_query_batch_async(payloads: list[dict]):
    """Every payload as an async performQuery: one device batch, then each
    response recorded under its payload's query id (in payload order).  A
    payload the reference's Lambda would fail on records nothing, as the
    failed invocation does (its slice never finishes: the poll times out)."""
    from .perform_query import perform_query_batch
    for p, r in zip(payloads, perform_query_batch(payloads, lazy_variants=True)):
        if isinstance(r, Exception):
            continue
        record_response(p['query_id'], r)


def get_split_query_fan_out(start_min: int, start_max: int) -> int:
    """variantutils/local_utils.py:19-25: the slices splitQuery cuts."""
    from .split_query import SPLIT_SIZE
    return max(0, (start_max - start_min) // SPLIT_SIZE + 1) if start_max >= start_min else 0


def perform_variant_search(*, datasets, referenceName, referenceBases, alternateBases, start, end, variantType,
                           variantMinLength, variantMaxLength, requestedGranularity, includeResultsetResponses,
                           query_id='TEST', passthrough=dict(), dataset_samples=[], timeout=REQUEST_TIMEOUT):
    """search_variants.py:27-155 (a generator of PerformQueryResponse)."""
    import copy
    from .chrom_matching import get_matching_chromosome
    from .payloads import PerformQueryResponse, SplitQueryPayload
    from .split_query import split_payloads
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
    except Exception as e:  # :60-62: the generator then yields nothing
        print('Error occured ', e)
        return
    start_min += 1
    start_max += 1
    end_min += 1
    end_max += 1
    query_record = VariantQuery(query_id)
    query_record.save()
    split_query_fan_out = get_split_query_fan_out(start_min, start_max)
    perform_query_fan_out = 0
    payloads = []
    for n, dataset in enumerate(datasets):
        vcf_locations = {vcf: vcf_chromosomes[vcf] for vcf in dataset._vcfLocations if vcf_chromosomes[vcf]}
        event_passthrough = copy.deepcopy(passthrough)
        if len(dataset_samples) == len(datasets) and len(dataset_samples[n]) > 0:
            event_passthrough['sampleNames'] = dataset_samples[n]
            event_passthrough['selectedSamplesOnly'] = True
        perform_query_fan_out += split_query_fan_out * len(vcf_locations)
        sp = SplitQueryPayload(
            passthrough=event_passthrough, dataset_id=dataset.id, query_id=query_id,
            vcf_locations=vcf_locations, vcf_groups=[], reference_bases=referenceBases,
            start_min=start_min, start_max=start_max, end_min=end_min, end_max=end_max,
            alternate_bases=alternateBases, variant_type=variantType,
            include_datasets=includeResultsetResponses, requested_granularity=requestedGranularity,
            variant_min_length=variantMinLength, variant_max_length=variantMaxLength)
        payloads.extend(split_payloads(sp))
    # "publish": the whole fan-out as one device batch on the worker
    if payloads:
        _publisher.submit(perform_query_batch_async, payloads)
    query_record.add_fan_out(perform_query_fan_out)
    # poll (:130-142): until every slice has finished or the timeout
    deadline = time.monotonic() + timeout
    query_results = {}
    with _table.cv:
        while True:
            q = _table.queries.get(query_id)
            if q is not None and q.fanOut == 0:
                q.complete = True
                q.elapsedTime = (q.endTime - q.startTime).total_seconds() if q.endTime else 0
                n_resp = q.responses
                break
            left = deadline - time.monotonic()
            if left <= 0:
                n_resp = None
                break
            _table.cv.wait(min(left, 0.5))
    if n_resp is not None:
        for item in VariantResponse.batch_get([(query_id, k) for k in range(1, n_resp + 1)]):
            query_results[item.responseNumber] = item
    for _, var_response in query_results.items():
        yield PerformQueryResponse.load(json.loads(var_response.result))
