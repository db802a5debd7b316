#!/usr/bin/env python3
"""Probe: does a D2H copy into pinned host memory run on a CU blit kernel
(contending with a concurrent kernel) or on a copy engine?  Times a
memory-bound torch kernel alone and with a 64 MB D2H copy on a second stream,
and the copy alone.  Run under rocprofv3 --kernel-trace to see the copy's
kernel name (if any)."""
import json
import os
import sys
import time

import torch


def main():
    dev = torch.device('cuda', 0)
    x = torch.ones(512 * 2**20 // 4, dtype=torch.float32, device=dev)  # 512 MB
    src = torch.ones(64 * 2**20 // 8, dtype=torch.int64, device=dev)
    dst = torch.empty(src.shape, dtype=torch.int64, pin_memory=True)
    s_cmp, s_cp = torch.cuda.Stream(), torch.cuda.Stream()

    def compute(n=8):
        with torch.cuda.stream(s_cmp):
            for _ in range(n):
                x.mul_(1.0000001)

    def timed(fn):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s_cmp)
        fn()
        b.record(s_cmp)
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    for _ in range(3):
        compute()
        with torch.cuda.stream(s_cp):
            dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    alone = min(timed(compute) for _ in range(5))
    cp = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s_cp):
            dst.copy_(src, non_blocking=True)
        s_cp.synchronize()
        cp.append((time.perf_counter() - t) * 1e3)

    def both():
        with torch.cuda.stream(s_cp):
            for _ in range(4):
                dst.copy_(src, non_blocking=True)
        compute()
    conc = min(timed(both) for _ in range(5))
    out = {'env': {k: os.environ.get(k) for k in ('HSA_ENABLE_SDMA', 'GPU_BLIT_ENGINE_TYPE', 'GPU_FORCE_BLIT_COPY_SIZE',
                                                   'HSA_ENABLE_PEER_SDMA')},
           'compute_alone_ms': round(alone, 3), 'compute_with_copies_ms': round(conc, 3),
           'copy_64MB_ms': round(min(cp), 3), 'copy_GBps': round(64 * 2**20 / (min(cp) * 1e-3) / 1e9, 1)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
