"""grk_gemm on the C2 step's dense-layer shapes, device time per call (HIP graph of
50 calls between events): run once with the default backend (grk's MFMA GEMM) and
once with GRK_GEMM_BACKEND=hipblaslt (tuned hipBLASLt plans), each in its own process.

    python scripts/microbench/mgemm.py            # both backends, one line per shape
"""
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

M = 14336
SHAPES = [('uvqk fwd', M, 2048, 512, 0), ('uvqk dX', M, 512, 2048, 1), ('out fwd', M, 512, 512, 0),
          ('out dX', M, 512, 512, 1), ('itemdnn fwd', M, 512, 552, 0), ('itemdnn dX', M, 552, 512, 1),
          ('pair itemdnn fwd', 2 * M, 512, 552, 0)]


def timed(fn, reps=50):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def run():
    from tencent_recommendation_2025_amd import kernels as K
    out = {}
    for name, m, n, k, layout in SHAPES:
        g = torch.Generator(device='cuda').manual_seed(0)
        a = torch.randn(m, k, device='cuda', generator=g).bfloat16()
        b = (torch.randn(n, k, device='cuda', generator=g) if layout == 0 else
             torch.randn(k, n, device='cuda', generator=g)).bfloat16()
        bias = torch.randn(n, device='cuda', generator=g)
        c = torch.empty(m, n, device='cuda').bfloat16()
        relu = 'dnn' in name and 'fwd' in name
        us = timed(lambda: K.gemm(a, b, trans_b=layout == 0, out=c, bias=bias if layout == 0 else None, relu=relu))
        out[name] = us
    print(json.dumps(out))


def run_eager(reps=5):
    """Each shape `reps` times, eagerly (for rocprofv3 counter passes)."""
    from tencent_recommendation_2025_amd import kernels as K
    for name, m, n, k, layout in SHAPES:
        g = torch.Generator(device='cuda').manual_seed(0)
        a = torch.randn(m, k, device='cuda', generator=g).bfloat16()
        b = (torch.randn(n, k, device='cuda', generator=g) if layout == 0 else
             torch.randn(k, n, device='cuda', generator=g)).bfloat16()
        c = torch.empty(m, n, device='cuda').bfloat16()
        for _ in range(reps):
            K.gemm(a, b, trans_b=layout == 0, out=c)
        torch.cuda.synchronize()
        print(name, flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'one':
        run()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'eager':
        run_eager()
        sys.exit(0)
    res = {}
    mf = {'GRK_GEMM_BACKEND': 'mfma'}
    variants = {'routed': {}, 'c1_bk64': {**mf, 'GRK_MGEMM_CFG': '1'}, 'c2_256x128': {**mf, 'GRK_MGEMM_CFG': '2'},
                'c3_256x256': {**mf, 'GRK_MGEMM_CFG': '3'}, 'c4_128x128': {**mf, 'GRK_MGEMM_CFG': '4'},
                'c5_256x256w8': {**mf, 'GRK_MGEMM_CFG': '5'}, 'hipblaslt': {'GRK_GEMM_BACKEND': 'hipblaslt'}}
    for name, extra in variants.items():
        env = dict(os.environ, **extra)
        r = subprocess.run([sys.executable, __file__, 'one'], env=env, capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
    print(f'{"shape":18s} {"M":>6s} {"N":>5s} {"K":>5s}' + ''.join(f' {v:>10s} {"TF/s":>5s}' for v in variants))
    for name, m, n, k, _ in SHAPES:
        f = 2.0 * m * n * k
        print(f'{name:18s} {m:6d} {n:5d} {k:5d}' + ''.join(f' {res[v][name]:10.1f} {f / res[v][name] / 1e6:5.0f}'
                                                        for v in variants))
