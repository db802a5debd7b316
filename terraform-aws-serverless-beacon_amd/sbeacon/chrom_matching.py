"""Canonical chromosome matching (``shared_resources/utils/chrom_matching.py:1-79``).

A VCF contig name matches ``referenceName`` when some suffix of it is one of
the canonical names ``1..22, X, Y, MT`` (aliases ``M -> MT``, ``x -> X``,
``y -> Y``) and that canonical name equals ``referenceName`` exactly.
"""
from __future__ import annotations

CHROMOSOME_ALIASES = {'M': 'MT', 'x': 'X', 'y': 'Y'}

CHROMOSOME_LENGTHS = {
    '1': 248956422, '2': 242193529, '3': 198295559, '4': 190214555, '5': 181538259,
    '6': 170805979, '7': 159345973, '8': 145138636, '9': 138394717, '10': 133797422,
    '11': 135086622, '12': 133275309, '13': 114364328, '14': 107043718, '15': 101991189,
    '16': 90338345, '17': 83257441, '18': 80373285, '19': 58617616, '20': 64444167,
    '21': 46709983, '22': 50818468, 'X': 156040895, 'Y': 57227415, 'MT': 16569,
}
CHROMOSOMES = CHROMOSOME_LENGTHS.keys()


def match_chromosome_name(chromosome_name):
    for i in range(len(chromosome_name)):
        chrom = chromosome_name[i:]
        if chrom in CHROMOSOMES:
            return chrom
        if chrom in CHROMOSOME_ALIASES:
            return CHROMOSOME_ALIASES[chrom]
    return None


def get_matching_chromosome(vcf_chromosomes, target_chromosome):
    for vcf_chrom in vcf_chromosomes:
        if match_chromosome_name(vcf_chrom) == target_chromosome:
            return vcf_chrom
    return None
