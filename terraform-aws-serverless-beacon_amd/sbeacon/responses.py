"""Beacon v2 response envelopes of the g_variants routes.

Same dict shapes, key order and values as the reference helpers:
``shared_resources/apiutils/entries.py:1-24`` (get_variant_entry),
``shared_resources/apiutils/responses.py:145-254`` (pagination, result sets,
counts, boolean) and ``shared_resources/apiutils/api_response.py:37-67``
(bundle_response, bad_request).  ``BEACON_API_VERSION`` / ``BEACON_ID`` come
from the environment as in the reference (which requires them; defaults are
given here so the library imports without Lambda configuration).
"""
from __future__ import annotations

import json
import os

BEACON_API_VERSION = os.environ.get('BEACON_API_VERSION', 'v2.0.0')
BEACON_ID = os.environ.get('BEACON_ID', 'au.csiro-serverless.beacon')
HEADERS = {'Access-Control-Allow-Origin': '*'}
SCHEMA = 'https://json-schema.org/draft/2020-12/schema'


def _meta(granularity, req_api, req_granularity, pagination):
    return {
        'beaconId': BEACON_ID,
        'apiVersion': BEACON_API_VERSION,
        'returnedSchemas': [{'entityType': 'info', 'schema': 'beacon-map-v2.0.0'}],
        'returnedGranularity': granularity,
        'receivedRequestSummary': {
            'apiVersion': req_api,
            'requestedSchemas': [],
            'pagination': pagination,
            'requestedGranularity': req_granularity,
        },
    }


def get_variant_entry(internal_id, seq_id, ref, alt, start, end, typ):
    """entries.py:1-24."""
    return {
        'variantInternalId': internal_id,
        'variation': {
            'referenceBases': ref,
            'alternateBases': alt,
            'location': {
                'interval': {
                    'start': {'type': 'Number', 'value': start},
                    'end': {'type': 'Number', 'value': end},
                    'type': 'SequenceInterval',
                },
                'sequence_id': seq_id,
                'type': 'SequenceLocation',
            },
            'variantType': typ,
        },
    }


def get_pagination_object(skip, limit):
    """responses.py:145-149."""
    return {'limit': limit, 'skip': skip}


def get_result_sets_response(*, reqAPI=None, reqPagination=None, results=None, setType=None, info=None,
                             exists=False, total=0):
    """responses.py:160-203: one 'redacted' result set; returnedGranularity
    is always 'record' (:166)."""
    results = [] if results is None else results
    return {
        '$schema': SCHEMA,
        'info': {} if info is None else info,
        'meta': _meta('record', BEACON_API_VERSION if reqAPI is None else reqAPI, 'record',
                      {} if reqPagination is None else reqPagination),
        'response': {
            'resultSets': [{
                'exists': len(results) > 0,
                'id': 'redacted',
                'results': results,
                'resultsCount': len(results),
                'resultsHandovers': [],
                'setType': setType,
            }],
        },
        'responseSummary': {'exists': exists, 'numTotalResults': total},
    }


def get_counts_response(*, reqAPI=None, reqGranularity='count', exists=False, count=0, info=None):
    """responses.py:206-231."""
    return {
        '$schema': SCHEMA,
        'info': {} if info is None else info,
        'meta': _meta('count', BEACON_API_VERSION if reqAPI is None else reqAPI, reqGranularity, {}),
        'responseSummary': {'exists': exists, 'numTotalResults': count},
    }


def get_boolean_response(*, reqAPI=None, reqGranularity='boolean', exists=False, info=None):
    """responses.py:234-254."""
    return {
        '$schema': SCHEMA,
        'info': {} if info is None else info,
        'meta': _meta('boolean', BEACON_API_VERSION if reqAPI is None else reqAPI, reqGranularity, {}),
        'responseSummary': {'exists': exists},
    }


def bundle_response(status_code, body, query_id=None):
    """api_response.py:37-46 (the S3 response cache is a TODO there too)."""
    return {'statusCode': status_code, 'headers': HEADERS, 'body': json.dumps(body)}


def bad_request(*, apiVersion=None, errorMessage=None, filters=None, pagination=None, requestParameters=None,
                requestedSchemas=None):
    """api_response.py:13-34."""
    body = {
        '$schema': SCHEMA,
        'error': {'errorCode': 400, 'errorMessage': f'{errorMessage}'},
        'meta': {
            'apiVersion': BEACON_API_VERSION,
            'beaconId': BEACON_ID,
            'receivedRequestSummary': {
                'apiVersion': apiVersion,
                'filters': [] if filters is None else filters,
                'pagination': {} if pagination is None else pagination,
                'requestParameters': requestParameters,
                'requestedSchemas': requestedSchemas,
            },
            'returnedSchemas': [],
        },
    }
    return bundle_response(400, body)
