"""Query id of a route event (shared_resources/apiutils/request_hash.py:6-15):
md5 of the sorted-key JSON of the hashed event attributes, the body parsed."""
from __future__ import annotations

import hashlib
import json

_HASH_ATTR = ('body', 'httpMethod', 'path', 'pathParameters', 'queryStringParameters')


def hash_query(event) -> str:
    h = {a: event.get(a, None) for a in _HASH_ATTR}
    if h.get('body'):
        h['body'] = json.loads(h['body'])
    return hashlib.md5(json.dumps(h, sort_keys=True).encode()).hexdigest()
