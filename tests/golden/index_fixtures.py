"""Deterministic BGZF VCF fixtures for the CSI / TBI goldens (test data only).

Each fixture is VCF text from a seeded generator, BGZF-compressed by the
synthetic-data library (sbs_bgzf_compress, zlib level 6, 0xff00-byte blocks)
so the virtual offsets are the same wherever the tests run.  Shapes cover
what the index has to get right: several contigs, records dense enough to
fill many BGZF blocks, long REF alleles and INFO END= spans that land in
upper-level bins, a contig whose records all fit one block, a sites-only
header (no FORMAT: the reference's sample count is -1), and POS past 2^29
(CSI only: TBI cannot address it)."""
from __future__ import annotations

import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

# name -> (seed, [(contig, n_records, first_pos, mean_gap)], n_samples (None = sites-only), formats)
FIXTURES = {
    'multi3': (11, [('1', 40000, 10000, 450), ('2', 25000, 5000, 900), ('X', 300, 2_000_000, 40)], 3,
               ('csi', 'tbi')),
    'sv_sites': (12, [('chr7', 30000, 100, 2500)], None, ('csi', 'tbi')),
    'far_csi': (13, [('5', 8000, 536_000_000, 300), ('6', 2000, 1000, 100)], 2, ('csi',)),
}


def vcf_text(name: str) -> bytes:
    seed, contigs, n_samples, _ = FIXTURES[name]
    rng = random.Random(seed)
    head = ['##fileformat=VCFv4.2', '##INFO=<ID=END,Number=1,Type=Integer,Description="End">',
            '##INFO=<ID=AC,Number=A,Type=Integer,Description="AC">']
    head += [f'##contig=<ID={c}>' for c, *_ in contigs]
    cols = '#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO'
    if n_samples is not None:
        cols += '\tFORMAT' + ''.join(f'\tS{i}' for i in range(n_samples))
    lines = head + [cols]
    for contig, n, pos, gap in contigs:
        for _ in range(n):
            pos += rng.randint(1, 2 * gap)
            r = rng.random()
            if r < 0.03:
                ref = ''.join(rng.choice('ACGT') for _ in range(rng.randint(20, 3000)))
            else:
                ref = rng.choice('ACGT')
            alt = rng.choice('ACGT')
            info = f'AC={rng.randint(0, 5)};AN=10'
            if r > 0.985:  # a structural variant: END far past POS (upper-level bins)
                alt = '<DEL>'
                info += f';END={pos + rng.randint(1000, 3_000_000)}'
            elif r > 0.98:  # END= not past POS: ignored by the tabix VCF preset
                info = f'END={pos - 5};' + info
            info += ';DP=5'  # INFO does not end in AC/AN: a sites-only line would read on into the next one
            line = f'{contig}\t{pos}\t.\t{ref}\t{alt}\t50\tPASS\t{info}'
            if n_samples is not None:
                line += '\tGT' + ''.join(f'\t{rng.randint(0, 1)}|{rng.randint(0, 1)}' for _ in range(n_samples))
            lines.append(line)
    return ('\n'.join(lines) + '\n').encode()


def write_fixture(name: str, directory: str) -> str:
    from sbeacon.workload import write_bgzf
    path = os.path.join(directory, f'{name}.vcf.gz')
    write_bgzf(path, [vcf_text(name)])
    return path
