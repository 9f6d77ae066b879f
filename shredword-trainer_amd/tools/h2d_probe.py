"""Host -> HBM rates on this box (round 5 load study): one large pinned copy, 32 MiB chunk copies
round-robin over streams, and the same with the chunks read from a page-cached file first by
reader threads (the streamed load's pattern).  python h2d_probe.py [FILE]"""
import os
import sys
import threading
import time

import torch

n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for rep in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
print(f"H2D one 1 GiB copy: {n / dt / 1e9:.1f} GB/s", flush=True)
chunk = 32 << 20
for ns in (1, 2, 8):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for c in range(n // chunk):
        with torch.cuda.stream(streams[c % ns]):
            d[c * chunk:(c + 1) * chunk].copy_(h[c * chunk:(c + 1) * chunk], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"H2D 32 MiB chunks over {ns} streams: {n / dt / 1e9:.1f} GB/s", flush=True)
path = sys.argv[1] if len(sys.argv) > 1 else None
if path and os.path.exists(path):
    size = min(os.path.getsize(path), 8 << 30)
    for T in (1, 4, 8, 16):
        fd = os.open(path, os.O_RDONLY)
        bufs = [torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(T)]
        t = time.perf_counter()
        tot = [0] * T

        def rd(i):
            mv = memoryview(bufs[i].numpy())
            for c in range(i, size // chunk, T):
                tot[i] += os.preadv(fd, [mv], c * chunk)
        th = [threading.Thread(target=rd, args=(i,)) for i in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t
        os.close(fd)
        print(f"pread page cache -> pinned, {T} threads: {sum(tot) / dt / 1e9:.1f} GB/s", flush=True)
