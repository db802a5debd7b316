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

:class:`ResultExchange` delivers rows AND hit lists (the ``variants`` of the
responses) to each request's host-facing rank: 'first' = the rank holding the
request's first slice (only requests that straddle a shard cut move, so the
exchange stays a few KB whatever N), 'rank0' = one host-facing rank for all.
Per step: an all_gather of every rank's per-destination (row, hit) counts,
then point-to-point sends of those row / hit ranges (a gatherv; RCCL
send / recv over xGMI, gloo on CPU), then the receiver sums the rows.
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


MODES = ('first', 'rank0')


class ResultExchange:
    """Per-step delivery of request rows + dense hit lists (sb_batch_compact_hits
    layout) to their host-facing ranks.

    ``owners``: owner rank of each of this rank's window rows (non-decreasing;
    ``owner_ranks`` builds them).  After :meth:`exchange`, :attr:`rows` holds
    the combined rows of the requests this rank owns (global request rows
    ``[own_lo, own_lo + n_own)``) and :meth:`hit_lists` yields each owned
    request's hits: its own slices' first, then each sender's in rank order
    (= position order: shards are cut in (contig, POS) order)."""

    def __init__(self, dist, rank: int, world: int, row_lo: int, n_rows: int, owners, device, row_fields: int = NF,
                 row_dtype=None):
        """``row_fields`` / ``row_dtype``: the rows' layout -- NF int64
        fields (sb_request_partial), or 4 int32 fields holding u32 sums
        (sb_request_row32, sb_requests_set_compact): received rows are then
        added modulo 2^32 with a device-side carry check (row_overflow)."""
        import torch
        row_dtype = torch.int64 if row_dtype is None else row_dtype
        self.dist, self.rank, self.world, self.device = dist, rank, world, device
        owners = np.asarray(owners, dtype=np.int64)
        assert len(owners) == n_rows and (np.diff(owners) >= 0).all()
        self.row_lo, self.n_rows = row_lo, n_rows
        # my rows per destination: [a, b) window rows
        self.sends = []
        for d in range(world):
            idx = np.flatnonzero(owners == d)
            if len(idx):
                assert idx[-1] - idx[0] + 1 == len(idx)
                self.sends.append((d, int(idx[0]), int(idx[-1]) + 1))
        own = [(a, b) for d, a, b in self.sends if d == rank]
        self.own_a, self.own_b = own[0] if own else (0, 0)
        self.sends = [x for x in self.sends if x[0] != rank]
        # everyone's plan: plan[s, d] = (global first row, rows) s sends to d
        plan = torch.zeros((world, 2), dtype=torch.int64)
        for d, a, b in self.sends:
            plan[d] = torch.tensor([row_lo + a, b - a])
        if world > 1:
            allp = [torch.zeros_like(plan) for _ in range(world)]
            dist.all_gather(allp, plan.to(device))
            allp = [x.cpu() for x in allp]
        else:
            allp = [plan]
        self.recvs = [(s_, int(allp[s_][rank, 0]), int(allp[s_][rank, 1])) for s_ in range(world)
                      if s_ != rank and int(allp[s_][rank, 1]) > 0]
        # owned global rows: my own window rows plus every received range
        lo = [row_lo + self.own_a] if self.own_b > self.own_a else []
        hi = [row_lo + self.own_b] if self.own_b > self.own_a else []
        for _, g, n in self.recvs:
            lo.append(g)
            hi.append(g + n)
        self.own_lo = min(lo) if lo else 0
        self.n_own = (max(hi) - self.own_lo) if hi else 0
        # 'first' mode: what a rank owns lies in its own window (a request's
        # first slice is on its owner), so the received rows are added into
        # `part` in place and the owned rows are a view of it
        self.inplace = self.n_own == 0 or (row_lo + self.own_a <= self.own_lo and
                                           self.own_lo + self.n_own <= row_lo + self.own_b)
        self.rows = None if self.inplace else torch.zeros((max(self.n_own, 1), row_fields), dtype=row_dtype,
                                                          device=device)
        self.recv_rows = [torch.zeros((n, row_fields), dtype=row_dtype, device=device) for _, _, n in self.recvs]
        self._ovf = torch.zeros((), dtype=torch.bool, device=device) if row_dtype == torch.int32 else None
        self.recv_hits = [None] * len(self.recvs)
        self.recv_hits_n = {}
        self._my_hits = None
        self._merge = None  # merge plan (dest indices), fixed per batch (merge)
        self._allc = None  # hit ranges [src, dst, (start, n)], fixed per batch (exchange)
        self._ops, self._ops_key, self._nccl = [], None, False

    def exchange(self, part, hits, row_off):
        """part: [n_rows, 5] rows; hits / row_off: sb_batch_compact_hits /
        sb_requests_run output (int64 tensors on the device, ``row_off``
        n_rows + 1) of ONE batch (its hit counts are fixed: see below)."""
        import torch
        dist = self.dist
        if self.world > 1:
            # hit range per destination: (first dense hit, count).  A batch's
            # rows and hit counts are the same on every pass, so the sizes are
            # gathered once (one host sync, first exchange) and reused: later
            # steps enqueue RCCL send/recv only, with no host round trip
            if self._allc is None:
                cnt = torch.zeros((self.world, 2), dtype=torch.int64, device=self.device)
                for d, a, b in self.sends:
                    cnt[d, 0] = row_off[a]
                    cnt[d, 1] = row_off[b] - row_off[a]
                allc = [torch.zeros_like(cnt) for _ in range(self.world)]
                dist.all_gather(allc, cnt)
                self._allc = torch.stack(allc).cpu()  # [src, dst, (start, n)]
            # the P2P op list is built once per (part, hits) pair -- a batch's
            # buffers -- and re-issued as is on every later step
            key = (part.data_ptr(), hits.data_ptr())
            if self._ops_key != key:
                allc = self._allc
                ops = []
                for d, a, b in self.sends:
                    st, n = int(allc[self.rank, d, 0]), int(allc[self.rank, d, 1])
                    ops.append((dist.isend, part[a:b], d))
                    if n:
                        ops.append((dist.isend, hits[st:st + n], d))
                for k, (s_, g, n) in enumerate(self.recvs):
                    nh = int(allc[s_, self.rank, 1])
                    if self.recv_hits[k] is None or self.recv_hits[k].numel() < nh:
                        self.recv_hits[k] = torch.zeros(nh + nh // 4 + 64, dtype=hits.dtype, device=self.device)
                    self.recv_hits_n[k] = nh
                    ops.append((dist.irecv, self.recv_rows[k], s_))
                    if nh:
                        ops.append((dist.irecv, self.recv_hits[k][:nh], s_))
                self._nccl = dist.get_backend() == 'nccl'
                self._ops = [dist.P2POp(f, t, p) for f, t, p in ops] if self._nccl else ops
                self._ops_key = key
            if self._ops:
                if self._nccl:  # one RCCL group: sends and receives together
                    works = dist.batch_isend_irecv(self._ops)
                else:
                    works = [f(t, p) for f, t, p in self._ops]
                for w in works:
                    w.wait()
        # combine: my own rows, then each received range added in
        self._my_hits = (hits, row_off)
        if self.inplace:
            for k, (_, g, n) in enumerate(self.recvs):
                self._add(part[g - self.row_lo:g - self.row_lo + n], self.recv_rows[k])
            return part[self.own_a:self.own_b] if self.n_own else part[:0]
        self.rows.zero_()
        if self.own_b > self.own_a:
            o = self.row_lo + self.own_a - self.own_lo
            self._add(self.rows[o:o + self.own_b - self.own_a], part[self.own_a:self.own_b])
        for k, (_, g, n) in enumerate(self.recvs):
            self._add(self.rows[g - self.own_lo:g - self.own_lo + n], self.recv_rows[k])
        return self.rows

    def _add(self, dst, src):
        """dst += src in place; u32 rows (int32 tensors) modulo 2^32, a sum
        past 32 bits flagged on the device (row_overflow), no host sync."""
        import torch
        if self._ovf is None:
            dst += src
            return
        t = (dst.to(torch.int64) & 0xffffffff) + (src.to(torch.int64) & 0xffffffff)
        self._ovf |= (t >> 32).any()
        dst.copy_(t.to(torch.int32))

    def row_overflow(self) -> bool:
        """True when a u32 row sum of some exchange left 32 bits (host sync):
        those rows are not exact and the caller must not use them."""
        return bool(self._ovf.item()) if self._ovf is not None else False

    def merge(self):
        """The owned requests' hit lists, merged densely on the device: each
        owned request's own slices' hits, then every sender's (rank order =
        position order), in request order.  Returns (hits, offs): request
        ``own_lo + i`` has ``hits[offs[i]:offs[i + 1]]``.  In 'first' mode
        the received rows are the last rows of the window (requests whose
        window crosses the next cut), so only the hits from the first such
        row on move: the rest of the window's dense output stays where the
        pass wrote it, and the merged lists are written into the pass's
        ``hits`` / ``row_off`` in place when the hit buffer has the room
        (else into new buffers).  The destination of every moved hit is
        planned once per batch (a batch's hit counts are fixed); a step is
        then one gather and one scatter, with no host round trip."""
        import torch
        hits, row_off = self._my_hits
        key = (hits.data_ptr(), row_off.data_ptr())
        if self._merge is None or self._merge['key'] != key:
            self._merge = self._merge_plan(hits, row_off, key)
        m = self._merge
        if m['trivial']:
            return hits, row_off[self.own_a:self.own_b + 1]
        vals = [hits[m['own_lo']:m['own_hi']].clone()] if m['own_hi'] > m['own_lo'] else []
        for k, nh in m['recv']:
            if nh:
                vals.append(self.recv_hits[k][:nh])
        if m['prefix'] is not None:  # new buffers: the unmoved prefix, one block
            a, n = m['prefix']
            m['out'][:n] = hits[a:a + n]
        if vals:
            m['out'][m['dest']] = torch.cat(vals) if len(vals) > 1 else vals[0]
        if m['off_tail'] is not None:  # in place: the moved rows' offsets (the pass rewrote them)
            m['off'][m['t'] + 1:] = m['off_tail']
        return m['out'], m['off']

    def _merge_plan(self, hits, row_off, key):
        import torch
        dev = hits.device
        ro = row_off.cpu().numpy().astype(np.int64)
        n = self.n_own
        recv = [(k, int(self.recv_hits_n.get(k, 0))) for k in range(len(self.recvs))]
        if self.inplace and not any(nh for _, nh in recv):
            return {'key': key, 'trivial': True}
        o = self.row_lo + self.own_a - self.own_lo  # first own row, relative to own_lo
        n_o = self.own_b - self.own_a               # own rows
        own_cnt = np.zeros(n, dtype=np.int64)
        if n_o:
            own_cnt[o:o + n_o] = np.diff(ro[self.own_a:self.own_b + 1])
        rcnt = []
        for k, (_, g, nr) in enumerate(self.recvs):
            c = np.zeros(n, dtype=np.int64)
            c[g - self.own_lo:g - self.own_lo + nr] = self.recv_rows[k][:, 1].cpu().numpy()
            rcnt.append(c)
        rsum = sum(rcnt) if rcnt else np.zeros(n, dtype=np.int64)
        off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(own_cnt + rsum, out=off[1:])
        # rows before t receive nothing: their hits keep their places (the
        # own rows start at 0 then, so their positions are the merged ones)
        got = np.flatnonzero(rsum)
        t = int(got[0]) if len(got) else n
        own_lo = int(ro[self.own_a + min(max(t - o, 0), n_o)]) if n_o else 0
        own_hi = int(ro[self.own_b]) if n_o else own_lo
        rows_t = np.arange(t, n)
        dest = []
        c = own_cnt[t:]
        first = np.repeat(np.cumsum(c) - c, c)
        dest.append(np.repeat(off[t:n], c) + (np.arange(int(c.sum())) - first))
        filled = own_cnt.copy()
        for ck_all in rcnt:
            ck = ck_all[t:]
            first = np.repeat(np.cumsum(ck) - ck, ck)
            dest.append(np.repeat(off[t:n] + filled[t:n], ck) + (np.arange(int(ck.sum())) - first))
            filled += ck_all
        dest = np.concatenate(dest).astype(np.int64)
        total = int(off[-1])
        base = int(ro[self.own_a]) if n_o else 0
        off_tail = None
        if self.inplace and hits.numel() >= base + total:
            out = hits
            m_off = row_off[self.own_a:self.own_a + n + 1]
            off_tail = torch.from_numpy(off[t + 1:] + base).to(dev)
            dest += base
            prefix = None
        else:
            out = torch.zeros(max(total, 1), dtype=hits.dtype, device=dev)
            m_off = torch.from_numpy(off).to(dev)
            prefix = (base, int(off[t])) if t > 0 and n_o else None
        return {'key': key, 'trivial': False, 'dest': torch.from_numpy(dest).to(dev), 'out': out, 'off': m_off,
                'off_tail': off_tail, 't': t, 'own_lo': own_lo, 'own_hi': own_hi, 'recv': recv, 'prefix': prefix}

    def hit_lists(self):
        """{global request row: [hit, ...]} of the owned requests (host; tests)."""
        hits, row_off = self._my_hits
        ro = row_off.cpu().numpy()
        h = hits[:int(ro[-1])].cpu().numpy().astype(np.uint64)
        out = {}
        for w in range(self.own_a, self.own_b):
            out[self.row_lo + w] = list(h[ro[w]:ro[w + 1]])
        for k, (s_, g, n) in enumerate(self.recvs):
            rows = self.recv_rows[k].cpu().numpy()
            nh = self.recv_hits_n.get(k, 0)
            rh = self.recv_hits[k][:nh].cpu().numpy().astype(np.uint64) if nh else np.zeros(0, np.uint64)
            at = 0
            for j in range(n):
                c = int(rows[j, 1])
                out.setdefault(g + j, []).extend(rh[at:at + c])
                at += c
        return out


def owner_ranks(first_rank_of_rows, mode: str, rank: int):
    """Owner rank of each window row: 'first' = the rank of the request's
    first slice, 'rank0' = 0."""
    if mode not in MODES:
        raise ValueError(f'delivery mode {mode!r} not in {MODES}')
    f = np.asarray(first_rank_of_rows, dtype=np.int64)
    return np.zeros_like(f) if mode == 'rank0' else f
