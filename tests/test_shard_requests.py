"""shard_requests (sbeacon/genome.py) against its definition, request by
request: rank r answers the splitQuery slices of a request whose first base
lies in its core [cuts[r], cuts[r + 1]) (lexicographic (contig, POS)), as the
sub-request [start_min + 10000 k0, min(start_max, start_min + 10000 k1 - 1)];
rows run from the first to the last request with a slice there, and a row
inside that range without one has start_max < start_min.  The vectorised
form only touches the two cut contigs' rows, so the cut positions are where
it can go wrong: every world size 1..6 is checked on every rank."""
import numpy as np
import pytest

from conftest import PKG  # noqa: F401

SPLIT = 10000


def _definition(shape, reqs, world, rank):
    cuts = shape.cuts(world)
    lo_cut, hi_cut = cuts[rank], cuts[rank + 1]
    out = []
    for i in range(len(reqs)):
        ci = int(reqs.ci[i])
        smin = int(reqs.start[i]) + 1
        smax = smin + int(reqs.width[i])
        ks = [k for k in range((smax - smin) // SPLIT + 1)
              if lo_cut <= (ci, smin + SPLIT * k) < hi_cut]
        out.append((ci, smin, smax, ks))
    return out


@pytest.mark.parametrize('world', [1, 2, 3, 4, 6])
def test_shard_requests_match_definition(world):
    from sbeacon.genome import GenomeShape, config3_requests, shard_requests
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    reqs = config3_requests(shape, n=3000, seed=17)
    covered = np.zeros(len(reqs), dtype=np.int64)
    for rank in range(world):
        sr = shard_requests(shape, reqs, world, rank)
        want = _definition(shape, reqs, world, rank)
        rows = [i for i, w in enumerate(want) if w[3]]
        if not rows:
            assert sr.n_rows == 0
            continue
        assert (sr.row_lo, sr.n_rows) == (rows[0], rows[-1] + 1 - rows[0])
        for w in range(sr.n_rows):
            i = sr.row_lo + w
            ci, smin, smax, ks = want[i]
            assert int(sr.ci[w]) == ci and int(sr.end_min[w]) == smin and int(sr.end_max[w]) == smax
            assert int(sr.vt[w]) == int(reqs.vt[i])
            if ks:
                assert ks == list(range(ks[0], ks[-1] + 1))  # one run of slices
                assert int(sr.start_min[w]) == smin + SPLIT * ks[0]
                assert int(sr.start_max[w]) == min(smax, smin + SPLIT * (ks[-1] + 1) - 1)
                covered[i] += len(ks)
            else:
                assert int(sr.start_max[w]) < int(sr.start_min[w])
    # every slice of every request on exactly one rank
    assert np.array_equal(covered, (reqs.width // SPLIT + 1).astype(np.int64))
