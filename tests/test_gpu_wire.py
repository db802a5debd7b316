"""performQuery at the wire (sb_perform_query_events): event JSON text in,
response JSON text out.  Every reference golden as an event (direct and
SNS-wrapped), general-record goldens (AC/AN past int64, > 64 ALTs), random
payloads with sample names, and events outside the C++ fast path (which the
Python handler answers): the parsed response equals the reference golden /
the Python handler's result, and the text equals json.dumps of it."""
import json
import os
import random

import pytest

from conftest import FIXTURES, normalise
from payload_gen import random_payload, read_records

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def stores():
    from sbeacon.engine import Store
    return {n: Store.build([(n + '.vcf', os.path.join(FIXTURES, n + '.vcf'))], device=0)
            for n in ('tiny22', 'quirk22', 'general22')}


def _python(ev):
    from sbeacon.wire import _python_handler
    return _python_handler(json.dumps(ev))


@pytest.mark.parametrize('wrap', ['sync', 'sns'])
def test_wire_reference_goldens(goldens, general_goldens, stores, wrap, monkeypatch):
    from sbeacon import engine, perform_query
    from sbeacon.wire import perform_query_events_packed, pack_events
    monkeypatch.setattr(perform_query, 'STRICT_VARIANT_TYPE', True)
    for s in stores.values():
        engine.registry.register(s)
    try:
        cases = [c for c in goldens + general_goldens if c['oracle'] == 'reference' and c['fixture'] in stores]
        assert len(cases) > 1000
        evs = [c['payload'] if wrap == 'sync' else {'Records': [{'Sns': {'Message': json.dumps(c['payload'])}}]}
               for c in cases]
        buf, off = pack_events([json.dumps(e) for e in evs])
        out = perform_query_events_packed(buf, off, strict_variant_type=True)
        assert len(out) == len(cases)
        assert not out.fallback.any()  # every golden event is on the typed fast path
        n_digits = 0
        for i, c in enumerate(cases):
            text = out[i]
            # byte-exact: the text json.dumps gives for the Python handler's result
            assert text == _python(evs[i]), c['payload']
            got = json.loads(text)
            if c['error']:
                assert got['errorType'] == c['error'], (c['payload'], got)
            elif 'errorType' in got:  # a count past CPython's 4300-digit str() limit: json.dumps raises
                assert got['errorType'] == 'ValueError' and 'integer string conversion' in got['errorMessage']
                n_digits += 1
            else:
                assert normalise(got) == normalise(c['response']), c['payload']
        assert n_digits < 10
    finally:
        engine.registry.clear()


def test_wire_random_and_fallback_events(stores):
    """Random payloads (sample names, every granularity) and events the C++
    parser leaves to the Python handler, mixed in one batch."""
    from sbeacon import engine
    from sbeacon.wire import perform_query_events_packed, pack_events
    for s in stores.values():
        engine.registry.register(s)
    try:
        rng = random.Random(11)
        evs = []
        for fx in ('tiny22', 'quirk22'):
            recs, names = read_records(os.path.join(FIXTURES, fx + '.vcf'))
            for _ in range(300):
                evs.append(random_payload(rng, recs, names, fx + '.vcf'))
        base = dict(evs[0])
        odd = [dict(base, dataset_id=7),                        # non-string dataset_id: echoed as an int
               dict(base, end_min='5'),                         # str vs int comparison: TypeError
               dict(base, unexpected=1),                        # PerformQueryPayload(**event): TypeError
               dict(base, vcf_location='nowhere.vcf'),          # no store holds it: KeyError
               dict(base, dataset_id='dé\U0001F600"\\'),   # escapes + a non-BMP character (fast path)
               dict(base, passthrough=None),                    # passthrough.get: AttributeError (:43)
               dict(base, passthrough=False),                   # the same
               {'Records': {'0': 1}}]                           # an envelope that does not unwrap
        evs.extend(odd)
        texts = [json.dumps(e) for e in evs]
        # a duplicated keyword: json.loads keeps the last value (dict
        # semantics), so the fast path must too
        dup = json.dumps(dict(base, end_max='not an int'))[:-1] + ', "end_max": ' + str(base['end_max']) + '}'
        texts.append(dup)
        evs.append(json.loads(dup))
        buf, off = pack_events(texts)
        out = perform_query_events_packed(buf, off)
        fb = out.fallback.tolist()
        assert fb[-9:] == [1, 1, 1, 1, 0, 1, 1, 1, 0]
        assert not any(fb[:-9])
        assert 'AttributeError' in out[len(evs) - 4] and 'AttributeError' in out[len(evs) - 3]
        for i, ev in enumerate(evs):
            assert out[i] == _python(ev), (ev, out[i])
        assert out.texts() == [out[i] for i in range(len(evs))]
    finally:
        engine.registry.clear()
