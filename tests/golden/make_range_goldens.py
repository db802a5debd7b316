#!/usr/bin/env python3
"""Golden vectors for initDuplicateVariantSearch's range planning, made by
running the REFERENCE functions.

TEST INFRASTRUCTURE — runs only in the build container (reads
/root/reference); writes ``range_golden.json`` (plain data: region-file key
lists in, range splits out).

``lambda/summariseDataset/initDuplicateVariantSearch.py`` is imported
unmodified with inert ``boto3`` / ``botocore`` stubs (module-level clients are
created but never called on this path) and the environment it reads at import
(``ABS_MAX_DATA_SPLIT`` etc.).  For each case the region-file keys
``vcf-summaries/contig/{c}/{vcf}/regions/{first}-{last}-{bytes}`` go through
the reference's own ``getFileNameInfo`` + sort + ``calcRangeSplits``
(``:77-89,171-191``, with ``addRange`` / ``filterRange`` ``:93-125``).  A case
on which ``calcRangeSplits`` does not terminate within 2 s is recorded as
``"timeout"`` (the Lambda would spin until its own timeout).

Usage:  python tests/golden/make_range_goldens.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import signal
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
ABS_MAX = 750_000_000  # main.tf:16 maximum_load_file_size


def install_stubs():
    boto3 = types.ModuleType('boto3')
    boto3.client = lambda *a, **k: object()
    botocore = types.ModuleType('botocore')
    exc = types.ModuleType('botocore.exceptions')

    class ClientError(Exception):
        pass

    exc.ClientError = ClientError
    botocore.exceptions = exc
    sys.modules.update({'boto3': boto3, 'botocore': botocore, 'botocore.exceptions': exc})
    os.environ.update(ABS_MAX_DATA_SPLIT=str(ABS_MAX), DUPLICATE_VARIANT_SEARCH_SNS_TOPIC_ARN='arn:stub',
                      DYNAMO_VARIANT_DUPLICATES_TABLE='dups', VARIANTS_BUCKET='variants',
                      DYNAMO_DATASETS_TABLE='datasets')


def load_reference():
    path = os.path.join(REF, 'lambda', 'summariseDataset', 'initDuplicateVariantSearch.py')
    spec = importlib.util.spec_from_file_location('ref_init_dup', path)
    m = importlib.util.module_from_spec(spec)
    sys.modules['ref_init_dup'] = m  # dataclasses resolve annotations through sys.modules
    spec.loader.exec_module(m)
    return m


def random_keys(rng):
    """Region-file keys of 1-3 VCFs on one contig: consecutive slices of each
    VCF, files split by gaps, sizes drawn so ranges need 1..n splits."""
    keys = []
    n_vcf = rng.choice([1, 2, 2, 3])
    for v in range(n_vcf):
        pos = rng.randrange(1, 5000)
        for _ in range(rng.randrange(1, 25)):
            first = pos + rng.randrange(0, 200000)
            last = first + rng.randrange(0, 3_000_000)
            size = rng.choice([rng.randrange(1000, 10_000_000), rng.randrange(10_000_000, 400_000_000),
                               rng.randrange(400_000_000, 900_000_000)])
            keys.append(f'vcf-summaries/contig/22/bkt%ds%part{v}/regions/{first}-{last}-{size}')
            pos = last + 1
    return keys


class Timeout(Exception):
    pass


def main():
    install_stubs()
    ref = load_reference()
    rng = random.Random(20250119)

    def alarm(*_):
        raise Timeout()

    signal.signal(signal.SIGALRM, alarm)
    cases = []
    for _ in range(300):
        keys = random_keys(rng)
        region = [ref.getFileNameInfo(k) for k in keys]
        region.sort(key=lambda x: x.startRange)
        signal.alarm(2)
        try:
            splits = ref.calcRangeSplits(region)
            out = [{'start': s.start, 'end': s.end, 'filePaths': s.filePaths} for s in splits]
            err = None
        except Timeout:
            out, err = None, 'timeout'
        except Exception as e:  # noqa: BLE001
            out, err = None, type(e).__name__
        finally:
            signal.alarm(0)
        cases.append({'keys': keys, 'splits': out, 'error': err})
    with open(os.path.join(HERE, 'range_golden.json'), 'w') as f:
        json.dump({'generator': 'tests/golden/make_range_goldens.py', 'abs_max_data_split': ABS_MAX,
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17', 'cases': cases}, f,
                  separators=(',', ':'))
    print(f'wrote {len(cases)} cases ({sum(1 for c in cases if c["error"])} reference errors/timeouts)')


if __name__ == '__main__':
    main()
