"""Root cause of round 5's first MemPool crash (gpurun_out/r05_a: SIGSEGV at the pool's first allocation, VERDICT
r05 #1), reproduced in child processes: a torch.cuda.MemPool built on a CUDAPluggableAllocator whose Python object
is then dropped -- torch._C._MemPool keeps only a raw pointer to the allocator -- against the same pool with the
allocator held (what _engine.pool_allocator does).  Each case runs in its own child process; this parent never
touches the GPU and prints each child's exit status.  A child killed by SIGSEGV is the expected outcome of the
"dropped" case, so run this as the LAST GPU step of a call.

    python tools/mempool_dangling.py
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import gc, sys, weakref
sys.path.insert(0, {root!r})
import torch
from ray_trace_pb_amd import _capi as C
C.lib()
alloc = torch.cuda.memory.CUDAPluggableAllocator(C.LIB_PATH, "rtpb_torch_alloc", "rtpb_torch_free")
inner = alloc.allocator()
refs_before = sys.getrefcount(inner)
pool = torch.cuda.MemPool(inner, use_on_oom=True)
print("pool built; references to the allocator object before / after MemPool():", refs_before, sys.getrefcount(inner),
      flush=True)
if {drop!r}:
    del alloc, inner
    gc.collect()
    print("allocator dropped (the pool still holds its raw pointer)", flush=True)
with torch.cuda.use_mem_pool(pool):
    t = torch.empty(1 << 20, device="cuda:0")
t.fill_(1.0)
torch.cuda.synchronize()
print("allocation OK:", float(t.sum()), flush=True)
'''


def main():
    for name, drop in (("held", False), ("dropped", True)):
        print(f"== case {name}", flush=True)
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, drop=drop)], capture_output=True,
                           text=True, timeout=240)
        sys.stdout.write(r.stdout)
        tail = [ln for ln in r.stderr.splitlines() if ln.strip() and "amdgpu.ids" not in ln][-3:]
        for ln in tail:
            print("  stderr:", ln)
        print(f"   exit status {r.returncode}" + ("  (SIGSEGV)" if r.returncode == -11 else ""), flush=True)
        if r.returncode != 0:
            break              # nothing more on the GPU after a crashed child
    return 0


if __name__ == "__main__":
    sys.exit(main())
