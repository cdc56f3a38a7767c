"""Does a hipMemsetAsync captured into a HIP graph re-run on every replay?

Round 1 saw accumulators cleared with hipMemsetAsync inside the captured
training step come out wrong from the second replay on and
switched to a zero-fill kernel.  This isolates the pattern: capture
[memset(acc) -> acc += 1 (kernel)] and replay it; after every replay acc must
be exactly 1.  Several sizes and both a buffer allocated before the capture
and one allocated inside it (the graph's private pool)."""
import ctypes
import sys

import torch

hip = ctypes.CDLL('libamdhip64.so.7' if sys.platform != 'win32' else 'amdhip64.dll')
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int
hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetD32Async.restype = ctypes.c_int


def check(nbytes, inside, fn_name):
    s = torch.cuda.Stream()
    outside = torch.zeros(nbytes // 4, dtype=torch.float32, device='cuda')
    g = torch.cuda.CUDAGraph()
    holder = {}
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        acc = torch.empty(nbytes // 4, dtype=torch.float32, device='cuda') if inside else outside
        st = torch.cuda.current_stream().cuda_stream
        if fn_name == 'memset':
            rc = hip.hipMemsetAsync(ctypes.c_void_p(acc.data_ptr()), 0, nbytes, ctypes.c_void_p(st))
        else:
            rc = hip.hipMemsetD32Async(ctypes.c_void_p(acc.data_ptr()), 0, nbytes // 4, ctypes.c_void_p(st))
        assert rc == 0, rc
        acc += 1.0
        holder['acc'] = acc
    bad = []
    for r in range(5):
        holder['acc'].fill_(7.0)          # garbage between replays: the memset must clear it
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        a = holder['acc']
        if not bool((a == 1.0).all()):
            bad.append((r, float(a.min()), float(a.max())))
    return bad


for fn in ('memset', 'memsetD32'):
    for inside in (False, True):
        for nbytes in (4, 64, 4096, 1 << 20, 5 * 1024 * 1024 + 12, 64 << 20):
            nbytes -= nbytes % 4
            bad = check(nbytes, inside, fn)
            print(f'{fn:9s} {"pool" if inside else "outside":8s} {nbytes:>10d} B: ' +
                  ('ok' if not bad else f'WRONG at replays {bad}'), flush=True)
