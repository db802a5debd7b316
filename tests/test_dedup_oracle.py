"""duplicateVariantSearch oracle (oracle/summarise_oracle.c orc_dedup_count)
and the host side of the handler, on hand-derived cases.

The reference C++ (lambda/duplicateVariantSearch/source, summariseSlice's
write_data_to_s3.h) needs AWS SDK C++ and cannot be built here, so these
cases pin the restatement to values worked out by hand from
write_data_to_s3.h:103-228, generalutils.hpp:19-45 and readVcfData.cpp:3-38
(parity unpinned against reference output)."""
import pytest


def rec(pos, ref, alt, chrom='22'):
    return f'{chrom}\t{pos}\t.\t{ref}\t{alt}\t.\tPASS\tAC=1;AN=2\tGT\t0|1\n'.encode()


def count(texts, lo=0, hi=10**9, contig='22'):
    from oracle.oracle import dedup_count
    return dedup_count(texts, contig, lo, hi)


def test_key_is_pos_text_plus_packed_alleles():
    # "12" + GAC'=0x31('1') 0x02 + '_' + G'=0x03 == "121" + C'=0x02 + '_' + 0x03
    t = rec(12, 'GAC', 'G') + rec(121, 'C', 'G')
    assert count([t]) == 1
    assert count([rec(12, 'GAC', 'G') + rec(121, 'C', 'T')]) == 2


def test_one_key_per_alt_and_case_folding():
    t = rec(5, 'A', 'G,T') + rec(5, 'a', 'g')  # a/A and g/G share a code
    assert count([t]) == 2
    assert count([rec(5, 'A', 'G,G')]) == 1


def test_empty_alt_parts_are_skipped():
    # readPastChars yields an empty field; recordHeader ignores it
    assert count([rec(5, 'A', 'G,,T')]) == 2
    assert count([rec(5, 'A', ',T')]) == 1


def test_symbolic_star_and_dot():
    t = rec(7, 'A', '<DEL>') + rec(7, 'A', '<DUP>') + rec(7, 'A', '*') + rec(7, 'A', '.')
    assert count([t]) == 4
    # '<DEL>' is stored as its inner text "DEL", not packed
    assert count([rec(7, 'A', '<DEL>') + rec(7, 'A', '<DEL>')]) == 1


def test_range_is_inclusive_and_per_contig():
    t = rec(10, 'A', 'G') + rec(20, 'A', 'G') + rec(30, 'A', 'G') + rec(20, 'A', 'C', chrom='X')
    assert count([t], 10, 30) == 3
    assert count([t], 11, 29) == 1
    assert count([t], 20, 20, contig='X') == 1


def test_union_of_vcfs():
    a = rec(10, 'A', 'G') + rec(20, 'A', 'G')
    b = rec(20, 'A', 'G') + rec(30, 'A', 'G')
    assert count([a, b]) == 3
    assert count([a, a]) == 2


def test_iupac_code_in_range_is_an_error():
    t = rec(10, 'A', 'G') + rec(20, 'R', 'G')
    with pytest.raises(ValueError):
        count([t], 0, 100)
    assert count([t], 0, 15) == 1  # outside the range it is never read


def test_bucket_key_and_region_paths():
    from sbeacon.dedup import bucket_key, region_path_bucket_key
    loc = 's3://bucket/dir/a.vcf.gz'
    assert bucket_key(loc) == 'bucket%dir%a'
    assert region_path_bucket_key('vcf-summaries/contig/22/bucket%dir%a/regions/100-200') == 'bucket%dir%a'
    with pytest.raises(ValueError):
        region_path_bucket_key('elsewhere/x')


def test_duplicate_tally_reports_once_all_ranges_done():
    from sbeacon.dedup import DuplicateTally
    t = DuplicateTally()
    t.expect('22', 'ds', [(1, 100), (101, 200)])
    assert t.update_duplicates('22', 'ds', 1, 100, 5) == -1
    assert t.update_duplicates('22', 'ds', 1, 100, 5) == -1  # condition fails: range already removed
    assert t.update_duplicates('22', 'ds', 101, 200, 7) == 12
