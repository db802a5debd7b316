"""Multi-GPU request answering over a contig-sharded store.

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL on ROCm,
``gloo`` for CPU tests).  Each rank holds one shard of the genome
(:mod:`sbeacon.genome`) and answers the performQuery slices whose first base
lies in its core.  Per step:

1. ``sb_batch_run``: the rank's slice queries on its GPU;
2. ``sb_batch_reduce_requests``: the route-level aggregation
   (``route_g_variants.py:144-171``) of those slices into one row per request
   of the rank's contiguous request window — exists (as a count of slices),
   n_variants, call_count, all_alleles_count, errors;
3. one collective: every rank's window rows go to rank 0 (``gather``; over
   xGMI with RCCL), which sums them into the global request table.  Requests
   whose slices straddle a shard cut get one row from each rank; the sum is
   the route's combination (exists OR = count > 0).

The per-slice semantics never cross GPUs (halo, see genome.py), so the only
exchange is this gather of per-request rows: 40 B x the rank's requests.
"""
from __future__ import annotations

import numpy as np

FIELDS = ('exists', 'n_variants', 'call_count', 'all_alleles_count', 'errors')
NF = len(FIELDS)


class RequestGather:
    """Fixed-shape gather of per-rank request windows to rank 0."""

    def __init__(self, dist, rank: int, world: int, row_lo: int, n_rows: int, n_requests: int, device):
        import torch
        self.dist, self.rank, self.world = dist, rank, world
        self.n_requests = n_requests
        meta = torch.tensor([row_lo, n_rows], dtype=torch.int64, device=device)
        if world > 1:
            metas = [torch.zeros_like(meta) for _ in range(world)]
            dist.all_gather(metas, meta)
            self.windows = [tuple(int(x) for x in m.tolist()) for m in metas]
        else:
            self.windows = [(row_lo, n_rows)]
        self.cap = max(1, max(n for _, n in self.windows))
        self.part = torch.zeros((self.cap, NF), dtype=torch.int64, device=device)  # this rank's rows
        self.recv = [torch.zeros_like(self.part) for _ in range(world)] if rank == 0 else None
        self.total = torch.zeros((n_requests, NF), dtype=torch.int64, device=device) if rank == 0 else None

    @property
    def part_ptr(self) -> int:
        return self.part.data_ptr()

    def exchange(self):
        """Gather the rows to rank 0 and sum them into ``total`` (rank 0)."""
        if self.world > 1:
            self.dist.gather(self.part, self.recv if self.rank == 0 else None, dst=0)
            parts = self.recv
        else:
            parts = [self.part]
        if self.rank == 0:
            self.total.zero_()
            for (lo, n), p in zip(self.windows, parts):
                if n:
                    self.total[lo:lo + n] += p[:n]
        return self.total


def combine_host(windows, parts, n_requests):
    """numpy restatement of RequestGather's combine (tests)."""
    tot = np.zeros((n_requests, NF), dtype=np.int64)
    for (lo, n), p in zip(windows, parts):
        if n:
            tot[lo:lo + n] += np.asarray(p)[:n]
    return tot


def request_rows_from_responses(owner, responses, n_rows):
    """Per-request rows from per-slice PerformQueryResponse dicts (or
    exception markers): the host statement of sb_batch_reduce_requests."""
    out = np.zeros((n_rows, NF), dtype=np.int64)
    for o, r in zip(owner, responses):
        if r is None or isinstance(r, (type, Exception)) or (isinstance(r, dict) and 'errorType' in r):
            out[o, 4] += 1
            continue
        d = r if isinstance(r, dict) else r.dump()
        out[o, 0] += 1 if d['exists'] else 0
        out[o, 1] += len(d['variants'])
        out[o, 2] += d['call_count']
        out[o, 3] += d['all_alleles_count']
    return out
