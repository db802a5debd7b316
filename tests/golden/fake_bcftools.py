#!/usr/bin/env python3
"""Stand-in for ``bcftools query`` used ONLY to generate golden vectors.

TEST INFRASTRUCTURE — never imported by the product path.

The reference performQuery shells out to ``bcftools query --regions R --format F
[--samples S] vcf`` (``lambda/performQuery/search_variants.py:42-50``,
``search_variants_in_samples.py:36-42``).  bcftools/htslib is third-party, not
vendored, built from an unpinned ``develop`` branch (``init.sh:73-91``) and absent
from this image, so this script restates the slice of its behaviour the
reference consumes:

* ``--regions chrom:a-b`` emits every record of ``chrom`` that overlaps
  ``[a, b]`` (POS <= b and POS + rlen - 1 >= a, rlen from REF or INFO/END), in
  file order.  The reference keeps only ``a <= POS <= b`` afterwards, so any
  superset of those records gives identical answers;
* ``%POS %REF %ALT %INFO`` print the raw VCF columns;
* ``[%GT,]`` / ``[%SAMPLE,]`` print each (subset) sample's GT text / name
  followed by ``,``;
* ``--samples a,b`` keeps the named samples in VCF *header* order; an unknown
  name is a fatal error with no output (bcftools without ``--force-samples``).

Parity at this boundary is therefore "unpinned" (SURVEY.md §8c).
"""
import os
import sys


def parse_args(argv):
    assert argv[0] == 'query', argv
    opts = {'--samples': None}
    i = 1
    while i < len(argv) - 1:
        opts[argv[i]] = argv[i + 1]
        i += 2
    opts['vcf'] = argv[-1]
    return opts


def tokenize(fmt):
    """Split a bcftools format string into literal / field / per-sample tokens."""
    toks = []
    i = 0
    while i < len(fmt):
        c = fmt[i]
        if c == '[':
            j = fmt.index(']', i)
            toks.append(('sample', tokenize(fmt[i + 1:j])))
            i = j + 1
        elif c == '%':
            j = i + 1
            while j < len(fmt) and (fmt[j].isalnum() or fmt[j] == '_'):
                j += 1
            toks.append(('field', fmt[i + 1:j]))
            i = j
        elif c == '\\' and i + 1 < len(fmt):
            toks.append(('lit', {'t': '\t', 'n': '\n'}[fmt[i + 1]]))
            i += 2
        else:
            toks.append(('lit', c))
            i += 1
    return toks


def render(toks, cols, sample_idx, names, out):
    for kind, val in toks:
        if kind == 'lit':
            out.append(val)
        elif kind == 'field':
            if val == 'POS':
                out.append(cols[1])
            elif val == 'REF':
                out.append(cols[3])
            elif val == 'ALT':
                out.append(cols[4])
            elif val == 'INFO':
                out.append(cols[7])
            elif val == 'CHROM':
                out.append(cols[0])
            else:
                raise SystemExit(f'unsupported field {val}')
        else:
            for s in sample_idx:
                for k2, v2 in val:
                    if k2 == 'lit':
                        out.append(v2)
                    elif v2 == 'GT':
                        out.append(cols[9 + s])
                    elif v2 == 'SAMPLE':
                        out.append(names[s])
                    else:
                        raise SystemExit(f'unsupported sample field {v2}')


def main(argv):
    opts = parse_args(argv)
    region = opts['--regions']
    chrom = region[:region.rfind(':')]
    a, b = region[region.rfind(':') + 1:].split('-')
    a, b = int(a), int(b)
    toks = tokenize(opts['--format'])
    names = None
    out = []
    with open(opts['vcf']) as f:
        for line in f:
            if line.startswith('##'):
                continue
            if line.startswith('#CHROM'):
                names = line.rstrip('\n').split('\t')[9:]
                if opts['--samples'] is not None:
                    want = opts['--samples'].split(',')
                    for w in want:
                        if w not in names:
                            sys.stderr.write(f'Error: subset called for sample that does not exist in header: "{w}"\n')
                            return 1
                    wanted = set(want)
                    sample_idx = [i for i, n in enumerate(names) if n in wanted]
                else:
                    sample_idx = list(range(len(names)))
                continue
            cols = line.rstrip('\n').split('\t')
            if cols[0] != chrom:
                continue
            pos = int(cols[1])
            rlen = len(cols[3])
            for kv in cols[7].split(';'):
                if kv.startswith('END='):
                    try:
                        rlen = max(rlen, int(kv[4:]) - pos + 1)
                    except ValueError:
                        pass
            if pos > b or pos + rlen - 1 < a:
                continue
            render(toks, cols, sample_idx, names, out)
    try:
        sys.stdout.write(''.join(out))
        sys.stdout.flush()
    except BrokenPipeError:  # the reference stops reading early (break at :232/:254)
        os.dup2(os.open(os.devnull, os.O_WRONLY), sys.stdout.fileno())
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
