"""BGZF helpers for tests: block table and record virtual offsets."""
import random
import zlib


def blocks(path):
    """[(coffset, ustart, isize)] of every BGZF block (EOF block included)."""
    data = open(path, 'rb').read()
    out, p, u = [], 0, 0
    while p < len(data):
        assert data[p:p + 4] == b'\x1f\x8b\x08\x04', p
        xlen = data[p + 10] | (data[p + 11] << 8)
        bsize = None
        x = p + 12
        while x < p + 12 + xlen:
            slen = data[x + 2] | (data[x + 3] << 8)
            if data[x:x + 2] == b'BC' and slen == 2:
                bsize = (data[x + 4] | (data[x + 5] << 8)) + 1
            x += 4 + slen
        isize = int.from_bytes(data[p + bsize - 4:p + bsize], 'little')
        out.append((p, u, isize))
        u += isize
        p += bsize
    return out


def text(path):
    data = open(path, 'rb').read()
    out = []
    for c, u, n in blocks(path):
        xlen = data[c + 10] | (data[c + 11] << 8)
        d = zlib.decompressobj(-15)
        out.append(d.decompress(data[c + 12 + xlen:])[:n])
    return b''.join(out)


def voff(blk, u, prefer_end=False):
    """Virtual offset of stream offset u.  A u on a block boundary has two
    spellings: (next block, 0) or, with prefer_end, (this block, isize)."""
    for i, (c, us, n) in enumerate(blk):
        if us <= u < us + n or (prefer_end and u == us + n and n):
            return (c << 16) | (u - us)
    c, us, n = blk[-1]
    return (c << 16) | (u - us)


def record_starts(txt):
    """Stream offsets of the record lines (after the header)."""
    starts, p = [], 0
    while p < len(txt):
        nl = txt.find(b'\n', p)
        if nl < 0:
            nl = len(txt)
        if txt[p:p + 1] != b'#':
            starts.append(p)
        p = nl + 1
    return starts


def random_slices(txt, blk, rng: random.Random, n, max_records=400):
    """n record-aligned slices (both voff spellings for boundaries)."""
    starts = record_starts(txt)
    ends = starts[1:] + [len(txt)]
    out = []
    for _ in range(n):
        a = rng.randrange(len(starts))
        b = min(len(starts), a + rng.randrange(0, max_records))
        u0 = starts[a]
        u1 = ends[b - 1] if b > a else u0
        out.append((voff(blk, u0), voff(blk, u1, prefer_end=rng.random() < 0.5)))
    return out
