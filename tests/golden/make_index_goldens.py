#!/usr/bin/env python3
"""Golden vectors for summariseVcf over CSI / TBI indexes, made by running
the REFERENCE handler.

TEST INFRASTRUCTURE — runs only in the build container (reads
/root/reference).  Writes ``index/<fixture>.<fmt>`` (the indexes sb_index_vcf
writes for the fixtures of index_fixtures.py; plain data) and
``index_golden.json``.

``lambda/summariseVcf/lambda_function.py`` and ``index_reader.py`` are
imported unmodified with inert ``boto3`` / ``botocore`` stubs; the stub
clients answer the handler's calls from memory: ``s3.get_object`` serves the
index (``.csi``; for a "tbi" case the ``.csi`` lookup raises ClientError so
get_vcf_index falls back to ``.tbi``, :144-156) and the VCF's first bytes
(get_sample_count's Range request); ``dynamodb.update_item`` and
``sns.publish`` record what the handler writes.  Per case the golden holds
the SNS slice messages (publish_slice_updates, :217-229), the ``toUpdate``
slice strings (mark_updating, :159-186) and the sampleCount
(update_sample_count, :281-297), plus get_chunk_boundaries' dict (:90-104)
and partition_chunks at three finer slice sizes.

Usage:  python tests/golden/make_index_goldens.py
"""
from __future__ import annotations

import importlib.util
import io
import json
import os
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference/lambda/summariseVcf'
sys.path.insert(0, HERE)
from index_fixtures import FIXTURES, write_fixture  # noqa: E402


class _Calls:
    def __init__(self):
        self.files = {}
        self.published = []
        self.updates = []


CALLS = _Calls()


def install_stubs():
    boto3 = types.ModuleType('boto3')
    botocore = types.ModuleType('botocore')
    exc = types.ModuleType('botocore.exceptions')

    class ClientError(Exception):
        def __init__(self, response, op):
            super().__init__(op)
            self.response = response

    class Client:
        def get_object(self, Bucket, Key, Range=None):
            data = CALLS.files.get(Key)
            if data is None:
                raise ClientError({'Error': {'Code': 'NoSuchKey'}}, 'GetObject')
            if Range:
                a, b = Range[len('bytes='):].split('-')
                data = data[int(a):int(b) + 1]
            return {'Body': io.BytesIO(data)}

        def list_objects_v2(self, **kw):
            return {'IsTruncated': False}

        def delete_objects(self, **kw):
            return {}

        def update_item(self, **kw):
            CALLS.updates.append(kw)
            return {}

        def publish(self, **kw):
            CALLS.published.append(json.loads(kw['Message']))
            return {}

    boto3.client = lambda *a, **k: Client()
    exc.ClientError = ClientError
    botocore.exceptions = exc
    sys.modules.update({'boto3': boto3, 'botocore': botocore, 'botocore.exceptions': exc})
    os.environ.update(SUMMARISE_SLICE_SNS_TOPIC_ARN='arn:stub', VARIANTS_BUCKET='variants',
                      DYNAMO_VCF_SUMMARIES_TABLE='summaries')


def load_reference():
    sys.path.insert(0, REF)  # `from index_reader import Csi, Tbi`
    spec = importlib.util.spec_from_file_location('ref_summarise_vcf', os.path.join(REF, 'lambda_function.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    install_stubs()
    ref = load_reference()
    from sbeacon.summarise_vcf import write_index
    os.makedirs(os.path.join(HERE, 'index'), exist_ok=True)
    cases = []
    with tempfile.TemporaryDirectory() as tmp:
        for name, (*_, formats) in FIXTURES.items():
            path = write_fixture(name, tmp)
            vcf = open(path, 'rb').read()
            for fmt in formats:
                idx = write_index(path, fmt)
                with open(os.path.join(HERE, 'index', f'{name}.{fmt}'), 'wb') as f:
                    f.write(idx)
                key = f'vcfs/{name}.vcf.gz'
                CALLS.files = {key: vcf, f'{key}.{fmt}': idx}
                CALLS.published, CALLS.updates = [], []
                ref.lambda_handler({'Records': [{'Sns': {'Message': f's3://bucket/{key}'}}]}, None)
                to_update = CALLS.updates[0]['ExpressionAttributeValues'][':toUpdate']['SS']
                sample = int(CALLS.updates[1]['ExpressionAttributeValues'][':sampleCount']['N'])
                # partition_chunks (:197-214) over the reference's own
                # get_chunk_boundaries at finer slice sizes (more cuts)
                cb = ref.get_chunk_boundaries(f's3://bucket/{key}')
                parts = {str(sz): [list(c) for c in ref.partition_chunks(cb, sz)] for sz in (20000, 65536, 250000)}
                cases.append({'fixture': name, 'format': fmt,
                              'slices': [[m['virtual_start'], m['virtual_end']] for m in CALLS.published],
                              'boundaries': cb, 'partitions': parts,
                              'to_update': to_update, 'sample_count': sample,
                              'vcf_bytes': len(vcf), 'index_bytes': len(idx)})
                print(f'{name}.{fmt}: {len(cases[-1]["slices"])} slices, sampleCount {sample}')
    with open(os.path.join(HERE, 'index_golden.json'), 'w') as f:
        json.dump({'generator': 'tests/golden/make_index_goldens.py',
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17', 'cases': cases}, f,
                  separators=(',', ':'))


if __name__ == '__main__':
    main()
