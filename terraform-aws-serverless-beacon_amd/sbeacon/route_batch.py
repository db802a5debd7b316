"""GET / POST /g_variants for a batch of events over the request path.

``route`` (:mod:`sbeacon.route_g_variants`) restates
``lambda/getGenomicVariants/route_g_variants.py:49-208`` one event at a
time and answers its fan-out with one per-slice device batch.  ``route_batch``
answers MANY events the way a serving front end receives them: every event's
fan-out -- one request per (dataset, VCF), the SplitQueryPayloads of
``perform_variant_search_sync`` (``shared_resources/variantutils/
search_variants.py:158-244``) -- becomes one row of ONE request batch
(``sb_requests_prepare_columns``: splitQuery's 10 kb cut in the library,
variantType requests as chains on ``request_eval_kernel``), one pass answers
them all (``sb_requests_run``), and ``sb_route_bodies`` folds each event's
rows and hit lists into the route's response body in C++: ``exists`` OR,
the distinct variant strings (``count = len(variants)``), one
``get_variant_entry`` per distinct internal id, the envelope of
``responses.py:160-254`` written as ``json.dumps`` writes it.

Each entry of the result is what ``route(event)`` returns -- the
``bundle_response`` dict -- or the exception it raises.  Events outside the
batched form (another resource or method, a job that is not NEW, request
values of unexpected types, VCFs spread over several stores, a VCF with
negative AC, a slice that raises, text that is not UTF-8) are answered by
``route`` itself, so their result is the per-event path's.  ``results`` is
listed in (dataset, VCF, hit) order; the reference's is thread-completion
order (its tests compare it as a set).

:func:`route_bodies` is the library call on its own: request rows and hit
lists of a pass (wide or compact, host memory) + per-event parameters ->
response bodies.  The bench times requests -> bodies with it
(``bench_genome.route_bodies_passes``).
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import _lib, responses
from .catalog import JobStatus, catalog as default_catalog
from .route_g_variants import _not_new, _params, route

GRAN_CODE = {'boolean': _lib.SB_GRAN['boolean'], 'count': _lib.SB_GRAN['count'],
             'aggregated': _lib.SB_GRAN['aggregated'], 'record': _lib.SB_GRAN['record']}
OTHER_GRAN = 255


class Bodies:
    """sb_route_bodies output: ``text(i)`` the body of event i (status 0),
    ``status[i]``: 0 body, 1 answer through ``route``, 2 the route returns None."""

    def __init__(self, handle):
        self._h = handle
        buf, ln, off, st = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_void_p()
        _lib.check(_lib.lib().sb_json_out_get(handle, C.byref(buf), C.byref(ln), C.byref(off), C.byref(st)))
        self.n_bytes = ln.value
        self._buf = buf.value
        self._n = None
        self._off_p, self._st_p = off.value, st.value

    def bind(self, n: int):
        self._n = n
        self.offsets = np.ctypeslib.as_array((C.c_uint64 * (n + 1)).from_address(self._off_p)) if n else \
            np.zeros(1, np.uint64)
        self.status = np.ctypeslib.as_array((C.c_uint8 * n).from_address(self._st_p)) if n else np.zeros(0, np.uint8)
        return self

    def raw(self) -> memoryview:
        """The JSON lines (each body followed by '\\n'), without a copy."""
        if not self.n_bytes:
            return memoryview(b'')
        return memoryview((C.c_char * self.n_bytes).from_address(self._buf)).cast('B')

    def text(self, i: int) -> str:
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return C.string_at(self._buf + a, b - a - 1).decode('ascii')

    def free(self):
        if self._h:
            _lib.lib().sb_json_out_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _strs(values):
    """distinct values -> (sb_str array, keep-alive); None -> NULL."""
    arr = (_lib.Str * max(len(values), 1))()
    keep = [arr]
    for k, v in enumerate(values):
        if v is None:
            continue
        b = v.encode() if isinstance(v, str) else bytes(v)
        buf = C.create_string_buffer(b, len(b) + 1)
        keep.append(buf)
        arr[k].p, arr[k].len = C.addressof(buf), len(b)
    return arr, keep


def route_bodies(store, *, rows, hits, row_off, compact: bool, rec_base: int = 0, row_lo, row_hi,
                 granularity, check_all, assembly=('GRCh38',), assembly_code=0,
                 pagination=('{"limit": 100, "skip": 0}',), pagination_code=0, row_vcf=0, row_contig=0) -> Bodies:
    """sb_route_bodies over a pass's outputs in host memory.

    rows / hits / row_off: the pass's outputs (wide: [n, 5] int64, uint64,
    int64; compact: [n, 4] uint32, uint32, uint32).  Per event: its rows
    [row_lo, row_hi), granularity (SB_GRAN code or 255), check_all,
    an assembly and a pagination index into the dictionaries (pagination: the
    JSON text of get_pagination_object); scalars broadcast.  row_vcf /
    row_contig: per request row, or a scalar."""
    n_ev = len(row_lo)
    ev = np.zeros(n_ev, dtype=np.dtype([('row_lo', '<u4'), ('row_hi', '<u4'), ('granularity', 'u1'),
                                        ('check_all', 'u1'), ('_pad', 'u1', 2), ('assembly', '<u4'),
                                        ('pagination', '<u4')]))
    assert ev.dtype.itemsize == C.sizeof(_lib.RouteEvent)
    ev['row_lo'] = row_lo
    ev['row_hi'] = row_hi
    ev['granularity'] = granularity
    ev['check_all'] = check_all
    ev['assembly'] = assembly_code
    ev['pagination'] = pagination_code
    q = _lib.RouteInput()
    keep = [ev]
    q.events, q.n_events = ev.ctypes.data, n_ev

    def col(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        keep.append(a)
        return a.ctypes.data

    if np.ndim(row_vcf) == 0:
        q.vcf_all = int(row_vcf)
    else:
        q.row_vcf = col(row_vcf, np.uint32)
    if np.ndim(row_contig) == 0:
        q.contig_all = int(row_contig)
    else:
        q.row_contig = col(row_contig, np.uint32)
    if compact:
        q.compact = 1
        q.rows, q.hits, q.row_off = col(rows, np.uint32), col(hits, np.uint32), col(row_off, np.uint32)
    else:
        q.rows, q.hits, q.row_off = col(rows, np.int64), col(hits, np.uint64), col(row_off, np.int64)
    q.rec_base = int(rec_base)
    ad, k1 = _strs(list(assembly))
    pd, k2 = _strs(list(pagination))
    keep += k1 + k2
    q.assembly_dict, q.n_assembly = C.addressof(ad), len(assembly)
    q.pagination_dict, q.n_pagination = C.addressof(pd), len(pagination)
    (bid, bl), (api, al) = [(C.create_string_buffer(v.encode()), len(v.encode()))
                            for v in (responses.BEACON_ID, responses.BEACON_API_VERSION)]
    keep += [bid, api]
    q.beacon_id.p, q.beacon_id.len = C.addressof(bid), bl
    q.api_version.p, q.api_version.len = C.addressof(api), al
    h = C.c_void_p()
    _lib.check(_lib.lib().sb_route_bodies(store.handle, C.byref(q), C.byref(h)))
    return Bodies(h).bind(n_ev)


def _route_one(ev, qid, catalog):
    """The per-event path, dispatched on the resource as lambda_function.py:
    18-52 does (route_g_variants_lambda_handler)."""
    from .route_g_variants import route_id
    res = ev.get('resource')
    if res == '/g_variants/{id}':
        return route_id(ev, qid, catalog=catalog)
    if res in ('/g_variants/{id}/individuals', '/g_variants/{id}/biosamples'):
        from .route_g_variants_samples import route_biosamples, route_individuals
        return (route_individuals if res.endswith('individuals') else route_biosamples)(ev, qid, catalog=catalog)
    return route(ev, qid, catalog=catalog)


def _id_params(ev):
    """route_g_variants_id.py:45-107 as the parameters _params gives: the
    point query of the id base64('assembly\\tchrom\\tpos\\tref\\talt'),
    start=[pos-1], end=[pos-1+len(alt)], includeResultsetResponses='ALL'."""
    import base64
    if ev['httpMethod'] == 'GET':
        params = ev.get('queryStringParameters', dict()) or dict()
        granularity = params.get('requestedGranularity', 'boolean')
        filters_str = params.get('filters', [])
        filters = [{'id': f} for f in (filters_str.split(',') if isinstance(filters_str, str) else [])]
    else:
        params = json.loads(ev.get('body', '{}')) or dict()
        query = params.get('query', dict())
        granularity = query.get('requestedGranularity', 'boolean')
        filters = query.get('filters', [])
    variant_id = ev['pathParameters'].get('id', None)
    assembly_id, reference_name, pos, reference_bases, alternate_bases = \
        base64.b64decode(variant_id.encode()).decode().split('\t')
    pos = int(pos) - 1
    return dict(requestedGranularity=granularity, assemblyId=assembly_id, filters=filters,
                referenceName=reference_name, referenceBases=reference_bases, alternateBases=alternate_bases,
                start=[pos], end=[pos + len(alternate_bases)], variantType=None, variantMinLength=0,
                variantMaxLength=-1, includeResultsetResponses='ALL', skip=0, limit=100)


def _is_int(x) -> bool:
    return isinstance(x, int) and not isinstance(x, bool)


def _plan_event(ev, qid, catalog, strict):
    """(granularity, check_all, assembly, pagination JSON, [SplitQueryPayload
    dicts]) of one event on the batched form, or None: answer it with route()."""
    from .variant_search import split_query_payloads
    res = ev.get('resource', '/g_variants')
    if res not in ('/g_variants', '/g_variants/{id}') or ev.get('httpMethod') not in ('GET', 'POST'):
        return None
    try:
        p = _params(ev) if res == '/g_variants' else _id_params(ev)
    except Exception:
        return None
    g = p['requestedGranularity']
    asm = p['assemblyId']
    if not (asm is None or isinstance(asm, str)) or not isinstance(g, str):
        return None
    for k in ('referenceBases', 'alternateBases', 'variantType'):
        if not (p[k] is None or isinstance(p[k], str)):
            return None
    try:
        datasets, samples = catalog.resolve(p['filters'], asm)
        sps = split_query_payloads(
            datasets=datasets, referenceName=p['referenceName'], referenceBases=p['referenceBases'],
            alternateBases=p['alternateBases'], start=p['start'], end=p['end'], variantType=p['variantType'],
            variantMinLength=p['variantMinLength'], variantMaxLength=p['variantMaxLength'],
            requestedGranularity=g, includeResultsetResponses=p['includeResultsetResponses'], query_id=qid,
            dataset_samples=samples)
    except Exception:
        return None
    if sps is None:
        return None
    pl = []
    for sp in sps:
        d = sp.dump()
        if not all(_is_int(d[k]) for k in ('start_min', 'start_max', 'end_min', 'end_max', 'variant_min_length',
                                             'variant_max_length')):
            return None
        if d['vcf_locations']:
            pl.append(d)
    code = GRAN_CODE.get(g, OTHER_GRAN)
    pag = '{}'  # (route_id's record body has no reqPagination: {})
    if res == '/g_variants' and code in (GRAN_CODE['record'], GRAN_CODE['aggregated']):
        try:
            pag = json.dumps(responses.get_pagination_object(p['skip'], p['limit']))
        except Exception:
            return None
    return code, 1 if p['includeResultsetResponses'] in ('HIT', 'ALL') else 0, asm, pag, pl


def _device_answer(store, payloads, owners, cols, n_rows):
    """One request pass over the batch's rows (wide outputs, host copies).
    payloads / owners: the SplitQueryPayload dicts and each row's (payload,
    vcf_location) -- unused here; the CPU tests answer from them with the
    oracle instead."""
    from .requests import RequestBatch
    batch = RequestBatch(store, cols, n_rows)
    try:
        if COMPACT:
            try:
                batch.set_compact(True)
            except _lib.SbError:
                pass  # (a batch with a per-slice part answers wide)
        return batch.answer(raw=True)
    finally:
        batch.free()


_answer = _device_answer
COMPACT = True  # the narrow outputs (16 B rows, u32 hits) where the batch allows them
last_stats = {'batched': 0, 'route': 0}


def route_batch(events, query_ids=None, *, catalog=None) -> list:
    """``route(event, query_id)`` for every event, the fan-outs answered by
    one request pass per store.  Entry i: the bundle_response dict, None (the
    route's other-granularity case) or the exception route() raises."""
    from . import engine
    from .perform_query import STRICT_VARIANT_TYPE
    from .request_hash import hash_query
    from .requests import requests_from_split_payloads
    catalog = catalog or default_catalog
    n = len(events)
    qids = list(query_ids) if query_ids is not None else [hash_query(e) for e in events]
    out = [None] * n
    slow = []
    plans = {}  # store id -> (store, [(event index, plan)])
    for i, ev in enumerate(events):
        try:
            status = catalog.job_status(qids[i])
        except Exception:
            slow.append(i)
            continue
        if status != JobStatus.NEW:
            out[i] = _not_new(status, qids[i], catalog)
            continue
        plan = _plan_event(ev, qids[i], catalog, STRICT_VARIANT_TYPE)
        if plan is None:
            slow.append(i)
            continue
        stores = set()
        try:
            for d in plan[4]:
                for loc in d['vcf_locations']:
                    stores.add(engine.registry.store_for(loc))
        except KeyError:
            slow.append(i)
            continue
        if len(stores) > 1:
            slow.append(i)
            continue
        st = next(iter(stores)) if stores else None
        if st is None:  # no VCF to ask: every store answers it alike (no rows)
            st = next(iter(plans.values()))[0] if plans else None
            if st is None:
                locs = engine.registry.locations()
                st = engine.registry.store_for(locs[0]) if locs else None
        if st is None:
            slow.append(i)
            continue
        plans.setdefault(id(st), (st, []))[1].append((i, plan))
    for store, items in plans.values():
        payloads, row_lo, row_hi = [], [], []
        asm_vals, asm_code, pag_vals, pag_code = {}, [], {}, []
        for i, (code, chk, asm, pag, pl) in items:
            row_lo.append(sum(len(d['vcf_locations']) for d in payloads))
            payloads.extend(pl)
            row_hi.append(row_lo[-1] + sum(len(d['vcf_locations']) for d in pl))
            asm_code.append(asm_vals.setdefault(asm, len(asm_vals)))
            pag_code.append(pag_vals.setdefault(pag, len(pag_vals)))
        n_rows = row_hi[-1] if row_hi else 0
        if n_rows:
            cols, keep, owners = requests_from_split_payloads(store, payloads, strict_variant_type=STRICT_VARIANT_TYPE,
                                                              columns=True)
            res = _answer(store, payloads, owners, cols, n_rows)
            rows, hits, row_off = res[:3]
            compact = bool(res[3]) if len(res) > 3 else False
            vcf = np.fromiter((store.vcf_id(loc) for _, loc in owners), dtype=np.uint32, count=n_rows)
            contig = np.frombuffer(C.string_at(cols.contig, 4 * n_rows), dtype=np.uint32) if cols.contig else \
                np.full(n_rows, cols.contig_all, np.uint32)
            bad = contig == 0xffffffff  # a chrom the VCF lacks: no slices, no hits (any contig will do)
            contig = np.where(bad, 0, contig)
        else:
            rows, hits, row_off = np.zeros((1, 5), np.int64), np.zeros(0, np.uint64), np.zeros(1, np.int64)
            compact = False
            vcf = contig = 0
        bodies = route_bodies(store, rows=rows, hits=hits, row_off=row_off, compact=compact, row_lo=row_lo,
                              row_hi=row_hi, granularity=[it[1][0] for it in items],
                              check_all=[it[1][1] for it in items], assembly=list(asm_vals), assembly_code=asm_code,
                              pagination=list(pag_vals), pagination_code=pag_code, row_vcf=vcf, row_contig=contig)
        for j, (i, _) in enumerate(items):
            s = int(bodies.status[j])
            if s == 0:
                out[i] = {'statusCode': 200, 'headers': responses.HEADERS, 'body': bodies.text(j)}
            elif s == 2:
                out[i] = None
            else:
                slow.append(i)
        bodies.free()
    last_stats['route'] = len(slow)
    last_stats['batched'] = n - len(slow)
    for i in sorted(slow):
        try:
            out[i] = _route_one(events[i], qids[i], catalog)
        except Exception as e:  # noqa: BLE001
            out[i] = e
    return out
