"""Diagnostic: which HIP/HSA runtime files a process maps after loading libtrainer.so without
torch, then importing torch (one copy of each is the goal)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "..", "shredword", "libtrainer.so"), mode=ctypes.RTLD_GLOBAL)
print("devices", lib.shred_device_count(), flush=True)


def maps(tag):
    seen = set()
    for line in open("/proc/self/maps"):
        f = line.split()[-1] if len(line.split()) >= 6 else ""
        if f.endswith(".so") or ".so." in f:
            seen.add(os.path.realpath(f))
    stems = {}
    for f in seen:
        stems.setdefault(os.path.basename(f).split(".so")[0], []).append(f)
    dup = {k: v for k, v in stems.items() if len(v) > 1}
    rocm = sorted(f for f in seen if "rocm" in f or "torch/lib" in f)
    print(tag, "duplicated:", dup, flush=True)
    if len(sys.argv) > 2:
        print(tag, "rocm/torch libs:", rocm, flush=True)


maps("before torch:")
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    maps("after import torch:")
    print(torch.arange(10, device="cuda").sum().item(), flush=True)
    maps("after cuda op:")
print("done", flush=True)
