"""Host side of the wire path (no device): with no store every event leaves
the C++ fast path, so each response is the Python handler's -- including the
exception it raises, rendered as the Lambda runtime reports it -- and the
JSON-lines packing / offsets of sb_perform_query_events hold for malformed,
empty and non-ASCII events alike."""
import json

from sbeacon.wire import _python_handler, pack_events, perform_query_events, perform_query_events_packed


def test_every_event_falls_back_without_stores():
    evs = ['{"region": 1}', '[1]', '{}', 'not json', '{"vcf_location": "x.vcf", "region": "22:1-2"}',
           json.dumps({'Records': [{'Sns': {'Message': json.dumps({'vcf_location': 'é.vcf'})}}]}), '""']
    buf, off = pack_events(evs)
    out = perform_query_events_packed(buf, off, stores=[])
    assert out.fallback.tolist() == [1] * len(evs)
    for i, e in enumerate(evs):
        assert out[i] == _python_handler(e)
        assert json.loads(out[i])['errorType']
    assert out.texts() == [out[i] for i in range(len(evs))]
    assert perform_query_events([], stores=[]) == []
