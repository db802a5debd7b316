"""Seeded synthetic VCF generator for parity fixtures and plumbing runs.

The reference ships no VCF, no index and no golden output for the variant query
path, so every fixture is generated here.  This module writes
small, edge-case-dense VCF 4.2 text files shaped like a 1000 Genomes chr22
release: the same INFO layout (``AC;AF;AN;NS;DP;EAS_AF;...;AA;VT``), phased
diploid GTs, plus the cases the reference query loop branches on
(``lambda/performQuery/search_variants.py:84-254``):

* multiallelic ALTs, insertions, deletions, MNPs, tandem-repeat ALTs
  (``(REF){2,}`` for the DUP/CNV regexes at ``:124,146``),
* symbolic ALTs ``<DEL> <DUP> <DUP:TANDEM> <INS> <CN0> <CN1> <CN2> <CN3> <INV>``,
* lower-case REF/ALT (the reference upper-cases before comparing, ``:94,173,180``),
* ``.`` ALT, ``*`` ALT, REF containing ``N``,
* unphased, haploid, missing and half-missing GTs (the GT regex at ``:233-236``),
* AC entries equal to zero (the ``alt_counts[i] != 0`` filter at ``:212``),
* same-POS records, ``AC_AFR=`` look-alike tags (exact ``startswith`` at ``:196``).

``quirks=True`` additionally writes records without ``INFO/AC`` and/or
``INFO/AN``, duplicated ``AC=`` tags and ``INFO=.`` — the genotype fallback
branches at ``:215-226`` and ``:244-250``.

This is the fixture generator only; the 1000G-shape bench stores are produced
by the C++ generator (``csrc/synth.cpp``) because Python cannot emit
1.1 M x 2,504 genotypes in reasonable time.
"""
from __future__ import annotations

import numpy as np

SYMBOLIC = ['<DEL>', '<DUP>', '<DUP:TANDEM>', '<INS>', '<CN0>', '<CN1>', '<CN2>',
            '<CN3>', '<INV>', '<DEL:ME:ALU>', '<INS:ME>']
BASES4 = 'ACGT'


def sample_names(n: int) -> list[str]:
    return [f'HG{i + 96:05d}' for i in range(n)]


def _rand_seq(rng, n, alphabet=BASES4):
    return ''.join(alphabet[i] for i in rng.integers(0, len(alphabet), n))


def _genotypes(rng, n_samples, n_alt, haploid_mask):
    """Return list of GT strings plus per-allele counts (index 0 = REF)."""
    # allele frequencies: mostly rare, 1/k-like
    freqs = rng.dirichlet(np.ones(n_alt + 1) * 0.3)
    freqs[0] += 1.5  # make REF dominant
    freqs /= freqs.sum()
    gts = []
    counts = np.zeros(n_alt + 1, dtype=np.int64)
    for s in range(n_samples):
        u = rng.random()
        if haploid_mask[s]:
            if u < 0.05:
                gts.append('.')
                continue
            a = int(rng.choice(n_alt + 1, p=freqs))
            counts[a] += 1
            gts.append(str(a))
            continue
        sep = '|' if rng.random() < 0.88 else '/'
        if u < 0.03:
            gts.append('.' + sep + '.')
            continue
        a = int(rng.choice(n_alt + 1, p=freqs))
        b = int(rng.choice(n_alt + 1, p=freqs))
        if u < 0.05:  # half-missing
            counts[a] += 1
            gts.append(f'{a}{sep}.' if rng.random() < 0.5 else f'.{sep}{a}')
            continue
        counts[a] += 1
        counts[b] += 1
        gts.append(f'{a}{sep}{b}')
    return gts, counts


def _make_record(rng, kind):
    """Return (REF, [ALT...], VT) for a record kind."""
    if kind == 'snv':
        ref = _rand_seq(rng, 1)
        alt = rng.choice([b for b in BASES4 if b != ref])
        return ref, [str(alt)], 'SNP'
    if kind == 'multi':
        ref = _rand_seq(rng, 1)
        others = [b for b in BASES4 if b != ref]
        k = int(rng.integers(2, 4))
        alts = list(rng.permutation(others)[:k])
        if rng.random() < 0.3:  # mixed SNV + indel multiallelic
            alts[-1] = ref + _rand_seq(rng, int(rng.integers(1, 4)))
        return ref, [str(a) for a in alts], 'SNP' if rng.random() < 0.7 else 'SNP,INDEL'
    if kind == 'ins':
        ref = _rand_seq(rng, 1)
        return ref, [ref + _rand_seq(rng, int(rng.integers(1, 12)))], 'INDEL'
    if kind == 'del':
        n = int(rng.integers(2, 14))
        ref = _rand_seq(rng, n)
        return ref, [ref[0]], 'INDEL'
    if kind == 'mnp':
        n = int(rng.integers(2, 4))
        ref = _rand_seq(rng, n)
        return ref, [_rand_seq(rng, n)], 'SNP'
    if kind == 'repeat':
        n = int(rng.integers(1, 4))
        unit = _rand_seq(rng, n)
        reps = [int(x) for x in rng.integers(0, 5, int(rng.integers(1, 3)))]
        alts = []
        for k in reps:
            alts.append(unit * k if k > 0 else '.')
        # dedupe but keep order
        seen, out = set(), []
        for a in alts:
            if a not in seen:
                seen.add(a)
                out.append(a)
        return unit, out, 'INDEL'
    if kind == 'sym':
        ref = _rand_seq(rng, 1)
        k = 1 if rng.random() < 0.8 else 2
        alts = [str(a) for a in rng.choice(SYMBOLIC, k, replace=False)]
        return ref, alts, 'SV'
    if kind == 'mono':
        return _rand_seq(rng, 1), ['.'], 'SNP'
    if kind == 'star':
        ref = _rand_seq(rng, 1)
        alt = [b for b in BASES4 if b != ref][0]
        return ref, [alt, '*'], 'SNP'
    if kind == 'nref':
        n = int(rng.integers(1, 3))
        ref = ''.join('N' if rng.random() < 0.5 else b for b in _rand_seq(rng, n))
        return ref, [_rand_seq(rng, 1)], 'SNP'
    raise ValueError(kind)


KINDS = ['snv', 'multi', 'ins', 'del', 'mnp', 'repeat', 'sym', 'mono', 'star', 'nref']
KIND_P = [0.62, 0.07, 0.07, 0.07, 0.03, 0.05, 0.04, 0.02, 0.015, 0.015]


def generate_records(*, contig='22', n_records=2000, n_samples=16, seed=1,
                     start=16050075, quirks=False):
    """Generate VCF data records as lists of the 10 + n_samples VCF columns."""
    rng = np.random.default_rng(seed)
    haploid = np.zeros(n_samples, dtype=bool)
    if n_samples >= 4:
        haploid[rng.choice(n_samples, max(1, n_samples // 8), replace=False)] = True
    pos = start
    rows = []
    for r in range(n_records):
        if r:
            if rng.random() < 0.03:
                gap = 0
            else:
                gap = int(rng.geometric(1 / 32.0))
            pos += gap
        kind = str(rng.choice(KINDS, p=KIND_P))
        ref, alts, vt = _make_record(rng, kind)
        if rng.random() < 0.04:
            ref = ref.lower()
        if rng.random() < 0.03:
            alts = [a.lower() if not a.startswith('<') else a for a in alts]
        gts, counts = _genotypes(rng, n_samples, len(alts), haploid)
        if alts == ['.']:
            ac_vals = [0]
        else:
            ac_vals = [int(c) for c in counts[1:]]
        an = int(counts.sum())
        info = []
        if rng.random() < 0.05:
            info.append('AC_AFR=' + ','.join(str(int(rng.integers(0, 5))) for _ in alts))
        info.append('AC=' + ','.join(str(v) for v in ac_vals))
        af = [f'{(v / an) if an else 0:.4g}' for v in ac_vals]
        info.append('AF=' + ','.join(af))
        info.append(f'AN={an}')
        info.append(f'NS={n_samples}')
        info.append(f'DP={int(rng.integers(1000, 30000))}')
        for pop in ('EAS_AF', 'AMR_AF', 'AFR_AF', 'EUR_AF', 'SAS_AF'):
            info.append(pop + '=' + ','.join(f'{rng.random() * 0.1:.2f}' for _ in alts))
        if kind == 'sym':
            info.append(f'END={pos + int(rng.integers(50, 5000))}')
            info.append('SVTYPE=' + alts[0].strip('<>').split(':')[0])
        info.append('AA=.|||')
        if rng.random() < 0.95:
            info.append(f'VT={vt}')
        if quirks:
            u = rng.random()
            if u < 0.15:   # drop AC -> genotype fallback at search_variants.py:215-226
                info = [f for f in info if not f.startswith('AC=')]
            elif u < 0.25:  # drop AN -> genotype fallback at :244-250
                info = [f for f in info if not f.startswith('AN=')]
            elif u < 0.32:  # drop both
                info = [f for f in info if not (f.startswith('AC=') or f.startswith('AN='))]
            elif u < 0.36:  # duplicate AC (last wins)
                info.append('AC=' + ','.join(str(v + 1) for v in ac_vals))
            elif u < 0.40:
                info = []
        info_s = ';'.join(info) if info else '.'
        rid = f'rs{int(rng.integers(1, 10**9))}' if rng.random() < 0.7 else '.'
        rows.append([contig, str(pos), rid, ref, ','.join(alts), '100', 'PASS', info_s, 'GT'] + gts)
    return rows


def write_vcf(path, rows, n_samples, contig='22', contig_length=50818468):
    names = sample_names(n_samples)
    with open(path, 'w') as f:
        f.write('##fileformat=VCFv4.2\n')
        f.write(f'##contig=<ID={contig},length={contig_length}>\n')
        f.write('##INFO=<ID=AC,Number=A,Type=Integer,Description="Allele count">\n')
        f.write('##INFO=<ID=AN,Number=1,Type=Integer,Description="Total alleles">\n')
        f.write('##INFO=<ID=VT,Number=.,Type=String,Description="Variant type">\n')
        f.write('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n')
        f.write('#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t' + '\t'.join(names) + '\n')
        for row in rows:
            f.write('\t'.join(row) + '\n')


def make_fixture(path, *, contig='22', n_records=2000, n_samples=16, seed=1, quirks=False,
                 start=16050075):
    rows = generate_records(contig=contig, n_records=n_records, n_samples=n_samples,
                            seed=seed, quirks=quirks, start=start)
    write_vcf(path, rows, n_samples, contig=contig)
    return rows
