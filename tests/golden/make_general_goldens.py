#!/usr/bin/env python3
"""Goldens for *general records* -- VCF records the packed device words cannot
hold -- made by running the REFERENCE performQuery code.

TEST INFRASTRUCTURE -- runs only in the build container (needs the read-only
reference at /root/reference).  It reuses make_goldens.py's stubs, fake
bcftools and payload generator; the outputs (fixtures/general22.vcf,
general_golden.json) are plain data.

What the fixture exercises (lambda/performQuery/search_variants.py:97-254,
search_variants_in_samples.py:82-245):

* ALT lists longer than 64 (``alts = all_alts.split(',')`` has no bound, :97);
* INFO AC / AN integers beyond int32, beyond int64 and up to CPython's 4300
  digit ``int()`` limit (``int(...)`` at :199, :206 is unbounded below it;
  a 4301-digit value raises ValueError), with '_' separators and signs;
* GT fallbacks (no AC / no AN, :215-226, :244-250) with ploidy > 3, allele
  numbers >= 8 (the variant order is CPython's iteration order of
  ``set(all_calls) & hit_set``, :223, not ascending), allele numbers >= 255,
  leading-zero and 20+-digit GT tokens, a token equal to 2**61 (hash(2**61) ==
  hash(1)), and a 4301-digit token (``int(g)`` raises ValueError);
* sample collection over > 99 alleles (multi-digit hit_string regex, :233-236).

Usage:  python tests/golden/make_general_goldens.py
"""
from __future__ import annotations

import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

import make_goldens as mg  # noqa: E402

FIX = os.path.join(HERE, 'fixtures')
N_SAMPLES = 6
NAMES = [f'G{i}' for i in range(N_SAMPLES)]
BASES = 'ACGT'


def _alts(rng, ref, n):
    """n ALT strings: mostly distinct sequences, a few single bases / symbolic /
    REF repeats so that every hit predicate has something to match."""
    out = []
    for k in range(n):
        u = rng.random()
        if u < 0.15:
            out.append(rng.choice('ACGTN'))
        elif u < 0.2:
            out.append(rng.choice(['<DEL>', '<INS>', '<DUP>', '<CN0>', '<CN2>', '<DUP:TANDEM>', '<INV>']))
        elif u < 0.25:
            out.append(ref * rng.choice([0, 2, 3]) or '.')
        else:
            out.append(rng.choice(BASES) + ''.join(rng.choice(BASES) for _ in range(rng.randrange(1, 6))))
        if rng.random() < 0.1:
            out[-1] = out[-1].lower()
    return out


def _big(rng, kind):
    if kind == 'i32':
        return str(rng.choice([2**31, 2**31 + 7, 3 * 10**9, -(2**31) - 5]))
    if kind == 'i64':
        return str(rng.choice([2**63 - 1, 2**63, 2**64 + 3, 10**20, -(2**63) - 1]))
    if kind == 'huge':
        return str(rng.randrange(10**38, 10**45))
    if kind == 'under':
        return '1_000_000_000_000'
    if kind == 'max':
        return '9' * 4300
    if kind == 'over':
        return '1' * 4301
    return str(rng.randrange(0, 50))


def _gt(rng, n_alt, ploidy, extra):
    """One sample's GT text: ploidy tokens drawn from 0..n_alt (+ extras)."""
    toks = []
    for _ in range(ploidy):
        u = rng.random()
        if u < 0.1:
            toks.append('.')
        elif u < 0.1 + extra and n_alt >= 1:
            toks.append(rng.choice(['0' + str(rng.randrange(1, n_alt + 1)), str(2**61), str(2**61 + 2),
                                    str(rng.randrange(10**20, 10**22)), str(n_alt + 1), str(n_alt + 300)]))
        else:
            toks.append(str(rng.randrange(0, n_alt + 1)))
    return rng.choice('|/').join(toks)


def make_fixture(path, seed=9):
    rng = random.Random(seed)
    lines = ['##fileformat=VCFv4.2', '##source=make_general_goldens.py',
             '#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t' + '\t'.join(NAMES)]
    pos = 20000
    kinds = ['normal', 'many_alts', 'big_ac', 'big_an', 'fb_order', 'fb_ploidy', 'fb_many', 'no_an',
             'fb_big_tok', 'mixed']
    for r in range(260):
        pos += rng.randrange(1, 120)
        kind = kinds[r % len(kinds)] if r % 3 else 'normal'
        ref = rng.choice(BASES) + ''.join(rng.choice(BASES) for _ in range(rng.choice([0, 0, 0, 1, 2])))
        if kind == 'normal':
            n_alt = rng.choice([1, 1, 2, 3])
        elif kind in ('many_alts', 'fb_many'):
            n_alt = rng.choice([65, 70, 100, 130, 300])
        elif kind in ('fb_order', 'fb_big_tok'):
            n_alt = rng.choice([8, 9, 10, 12, 17, 20, 33])
        else:
            n_alt = rng.choice([1, 2, 4, 9])
        alts = _alts(rng, ref, n_alt)
        info = []
        has_ac = kind not in ('fb_order', 'fb_ploidy', 'fb_many', 'fb_big_tok') or rng.random() < 0.1
        has_an = kind != 'no_an' and rng.random() < 0.93
        if has_ac:
            ac_kind = {'big_ac': rng.choice(['i32', 'i64', 'huge', 'under', 'max', 'small']),
                       'mixed': rng.choice(['i32', 'small', 'huge'])}.get(kind, 'small')
            n_ac = n_alt if rng.random() < 0.92 else max(1, n_alt - rng.randrange(1, 3))
            acs = [_big(rng, ac_kind) if rng.random() < 0.4 else str(rng.choice([0, 0, 1, 2, 5, 17]))
                   for _ in range(n_ac)]
            if kind == 'big_ac' and rng.random() < 0.08:
                acs[rng.randrange(n_ac)] = _big(rng, 'over')
            info.append('AC=' + ','.join(acs))
        info.append('AF=0.5')
        if has_an:
            an_kind = {'big_an': rng.choice(['i32', 'i64', 'huge', 'under', 'max']),
                       'mixed': 'i32'}.get(kind, 'small')
            an = _big(rng, an_kind) if an_kind != 'small' else str(rng.randrange(2, 40))
            if kind == 'big_an' and rng.random() < 0.08:
                an = _big(rng, 'over')
            info.append('AN=' + an)
        if rng.random() < 0.5:
            info.append('VT=' + rng.choice(['SNP', 'INDEL', 'SV']))
        ploidy = {'fb_ploidy': rng.choice([4, 5, 6]), 'fb_order': rng.choice([2, 3, 4])}.get(kind, 2)
        extra = 0.35 if kind in ('fb_big_tok', 'fb_order') else 0.0
        gts = [_gt(rng, n_alt, ploidy if rng.random() < 0.8 else rng.choice([1, 2, 3]), extra)
               for _ in range(N_SAMPLES)]
        if kind == 'fb_big_tok' and rng.random() < 0.15:
            gts[rng.randrange(N_SAMPLES)] = '1' * 4301 + '|0'
        lines.append(f'22\t{pos}\t.\t{ref}\t{",".join(alts)}\t50\tPASS\t{";".join(info)}\tGT\t' + '\t'.join(gts))
    with open(path, 'w') as f:
        f.write('\n'.join(lines) + '\n')


def targeted_payloads(recs, path, rng):
    """Payloads aimed at each record: its exact POS window (and a window around
    it), every ALT predicate family, sample collection and subsets."""
    out = []
    base = dict(dataset_id='ds-g', query_id='golden', vcf_location=path, variant_type=None,
                variant_min_length=0, variant_max_length=-1)
    for pos, ref, alts in recs:
        for _ in range(2):
            w = rng.choice([0, 0, 30, 200])
            a, b = pos - rng.randrange(0, w + 1), pos + rng.randrange(0, w + 1)
            u = rng.random()
            if u < 0.35:
                alt, vt = 'N', None
            elif u < 0.6:
                alt, vt = rng.choice(alts).upper(), None
            else:
                alt, vt = None, rng.choice(['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV'])
            pt_u = rng.random()
            if pt_u < 0.35:
                pt = {}
            elif pt_u < 0.7:
                pt = {'includeSamples': True}
            else:
                pt = {'sampleNames': rng.sample(NAMES, rng.randrange(1, N_SAMPLES + 1)), 'selectedSamplesOnly': True}
            out.append(dict(base, passthrough=pt, region=f'22:{a}-{b}', end_min=0, end_max=10**9,
                            reference_bases=rng.choice(['N', 'N', ref.upper()]), alternate_bases=alt, variant_type=vt,
                            include_details=rng.random() < 0.75,
                            requested_granularity=rng.choice(['record', 'record', 'aggregated', 'count', 'boolean'])))
    return out


def main():
    mg.install_stubs()
    tmp = tempfile.mkdtemp(prefix='sbeacon-golden-')
    mg.install_fake_bcftools(tmp)
    sv, svs, PQP = mg.import_reference()
    sv_p = mg.patched_module(sv, 'search_variants_patched')
    svs_p = mg.patched_module(svs, 'search_variants_in_samples_patched')
    path = os.path.join(FIX, 'general22.vcf')
    make_fixture(path)
    recs, names = mg.read_records(path)
    rng = random.Random(20261017)
    payloads = targeted_payloads(recs, path, rng)
    payloads += [mg.random_payload(rng, recs, names, path) for _ in range(300)]
    lo, hi = recs[0][0], recs[-1][0]
    for gran in mg.GRANS:  # splitQuery-shaped 10 kb slices over the whole fixture
        for ref, alt in (('N', 'N'), ('N', 'A')):
            s = lo - 100
            while s <= hi + 100:
                payloads.append(dict(passthrough={'includeSamples': True}, dataset_id='ds-g', query_id='golden',
                                     region=f'22:{s}-{min(s + 9999, hi + 100)}', reference_bases=ref,
                                     end_min=0, end_max=10**9, alternate_bases=alt, variant_type=None,
                                     include_details=True, requested_granularity=gran, variant_min_length=0,
                                     variant_max_length=-1, vcf_location=path))
                s += 10000
    cases = []
    for p in payloads:
        if p['alternate_bases'] is None:
            r = mg.run_one(sv_p, svs_p, PQP, p)
            cases.append({'fixture': 'general22', 'oracle': 'patched-oracle', 'payload': p, **r})
        else:
            r = mg.run_one(sv, svs, PQP, p)
            cases.append({'fixture': 'general22', 'oracle': 'reference', 'payload': p, **r})
    for c in cases:
        c['payload']['vcf_location'] = os.path.basename(c['payload']['vcf_location'])
        if c['response']:
            c['response']['vcf_location'] = os.path.basename(c['response']['vcf_location'])
            # integers beyond JSON's double range stay exact as hex text (str()
            # of an int past 4300 digits raises in this CPython)
            for k in ('call_count', 'all_alleles_count'):
                v = c['response'][k]
                if abs(v) >= 2**53:
                    c['response'][k] = {'hex': hex(v)}
    out = os.path.join(HERE, 'general_golden.json')
    with open(out, 'w') as f:
        json.dump({'generator': 'tests/golden/make_general_goldens.py',
                   'reference': 'Yatish0833/terraform-aws-serverless-beacon @ 2025-01-17',
                   'python': sys.version.split()[0], 'cases': cases}, f, separators=(',', ':'))
    n_err = sum(1 for c in cases if c['error'])
    n_ex = sum(1 for c in cases if c['response'] and c['response']['exists'])
    print(f'wrote {len(cases)} cases ({n_err} reference errors, {n_ex} exists=True) -> {out}')


if __name__ == '__main__':
    sys.setrecursionlimit(10000)
    main()
