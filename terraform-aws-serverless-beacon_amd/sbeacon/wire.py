"""performQuery at the wire: a batch of Lambda events (JSON text) in, the
JSON text of each handler result out.

The reference's performQuery Lambda (``lambda/performQuery/lambda_function.py:23-49``)
takes one event -- a ``PerformQueryPayload`` or its SNS envelope -- and
returns ``response.dump()``, which the Lambda runtime serialises with
``json.dumps``.  ``perform_query_events`` answers many such events in one
library call (``sb_perform_query_events``): the events are parsed in C++,
each store's events go to the device in one batch, and every response is
written in C++ as the exact text ``json.dumps(response.dump())`` gives.  An
event the C++ fast path does not type (status 1) is answered here by
``perform_query.lambda_handler`` -- the same code the single-event handler
runs -- so its result, or the exception it raises, is the reference's.
Raised exceptions are rendered as the Lambda runtime reports them,
``{"errorMessage": str(e), "errorType": type(e).__name__}``.
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import perform_query
from ._lib import check, lib
from .engine import registry


def _error_text(e: BaseException) -> str:
    return json.dumps({'errorMessage': str(e), 'errorType': type(e).__name__})


def _python_handler(text) -> str:
    """One event through the Python handler; ``text`` is str or UTF-8 bytes
    (decoded here, so an invalid event is its own error response)."""
    try:
        if not isinstance(text, str):
            text = bytes(text).decode()
        return json.dumps(perform_query.lambda_handler(json.loads(text), None))
    except Exception as e:  # the Lambda runtime reports the raised exception
        return _error_text(e)


class EventResponses:
    """The response texts of one event batch as JSON lines: response i is
    ``buf[offsets[i]:offsets[i + 1] - 1]`` (each line ends with '\\n');
    ``fallback`` marks the events the Python handler answered.  ``buf`` is a
    read-only view of the library's buffer (no copy), valid while this
    object lives."""

    def __init__(self, buf, offsets: np.ndarray, fallback: np.ndarray, handle=None):
        self.buf, self.offsets, self.fallback, self._h = buf, offsets, fallback, handle

    def __del__(self):
        h, self._h = getattr(self, '_h', None), None
        if h:
            try:
                self.buf = None
                lib().sb_json_out_free(h)
            except Exception:
                pass

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, i: int) -> str:
        return bytes(self.buf[int(self.offsets[i]):int(self.offsets[i + 1]) - 1]).decode()

    def texts(self) -> list[str]:
        return bytes(self.buf).decode().split('\n')[:-1] if len(self) else []


def pack_events(events) -> tuple[bytes, np.ndarray]:
    """Event texts (str / bytes) -> one buffer + n + 1 offsets."""
    bs = [e.encode() if isinstance(e, str) else bytes(e) for e in events]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs])
    return b''.join(bs), off


def perform_query_events_packed(buf: bytes, offsets: np.ndarray, *, stores=None,
                                strict_variant_type=None) -> EventResponses:
    """Events already packed (``pack_events``): the response texts joined by
    '\\n' in one buffer (JSON text holds no raw newline)."""
    if stores is None:
        seen = {}
        for loc in registry.locations():
            s = registry.store_for(loc)
            seen.setdefault(id(s), s)
        stores = list(seen.values())
    strict = perform_query.STRICT_VARIANT_TYPE if strict_variant_type is None else strict_variant_type
    n = len(offsets) - 1
    if n <= 0:
        return EventResponses(b'', np.zeros(1, dtype=np.uint64), np.zeros(0, dtype=np.uint8))
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    handles = (C.c_void_p * max(len(stores), 1))(*[s.handle for s in stores])
    src = C.c_char_p(bytes(buf))  # the bytes object's own storage (no copy for bytes input)
    out = C.c_void_p()
    check(lib().sb_perform_query_events(handles, len(stores), C.cast(src, C.c_void_p), offsets.ctypes.data, n,
                                        1 if strict else 0, C.byref(out)))
    p, ln, po, ps = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_void_p()
    try:
        check(lib().sb_json_out_get(out, C.byref(p), C.byref(ln), C.byref(po), C.byref(ps)))
    except Exception:
        lib().sb_json_out_free(out)
        raise
    view = memoryview((C.c_char * max(ln.value, 1)).from_address(p.value)).cast('B')[:ln.value] if ln.value \
        else memoryview(b'')
    roff = np.ctypeslib.as_array(C.cast(po, C.POINTER(C.c_uint64)), shape=(n + 1,))
    status = np.ctypeslib.as_array(C.cast(ps, C.POINTER(C.c_uint8)), shape=(n,)).copy()
    fb = np.flatnonzero(status)
    if not len(fb):  # zero copy: the view stays valid while the result object holds the handle
        return EventResponses(view.toreadonly(), roff, status, out)
    # events outside the typed fast path: the Python handler
    try:
        parts = [bytes(view[int(roff[i]):int(roff[i + 1])]) for i in range(n)]
    finally:
        lib().sb_json_out_free(out)
    raw = buf if isinstance(buf, bytes) else bytes(buf)
    for i in fb.tolist():
        parts[i] = _python_handler(raw[int(offsets[i]):int(offsets[i + 1])]).encode() + b'\n'
    roff = np.zeros(n + 1, dtype=np.uint64)
    roff[1:] = np.cumsum([len(x) for x in parts])
    return EventResponses(memoryview(b''.join(parts)), roff, status)


def perform_query_events(events, *, stores=None, strict_variant_type=None) -> list[str]:
    """Event texts -> the JSON text of each handler result, in order."""
    buf, off = pack_events(events)
    return perform_query_events_packed(buf, off, stores=stores, strict_variant_type=strict_variant_type).texts()
