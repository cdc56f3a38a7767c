"""grk_wgrad at the jagged C2 step's weight-gradient shapes (bench.py's recorded trace):
the ring kernels (default), with thinner K slices (GRK_WGRAD_SLICE) and on grk_mgemm's
K-major mode (GRK_WGRAD_MGEMM=1), each in its own process, device time per call (HIP graph of 30
calls between events; k_wgrad* + the slice reduction, bias gradient included).

    python scripts/microbench/wgrad_ab.py
"""
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [(13824, 2048, 512, 4), (27648, 512, 552, 1), (13824, 512, 552, 1), (13824, 512, 520, 1),
          (13824, 512, 512, 4)]


def timed(fn, reps=30):
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
    out, ref = {}, {}
    for k, m, n, _ in SHAPES:
        g = torch.Generator(device='cuda').manual_seed(k + m + n)
        dy = torch.randn(k, m, device='cuda', generator=g).bfloat16()
        x = torch.randn(k, n, device='cuda', generator=g).bfloat16()
        out[f'{k}x{m}x{n}'] = timed(lambda: K.wgrad(dy, x, want_db=True))
        dw, db = K.wgrad(dy, x, want_db=True)
        want = dy.float().t() @ x.float()
        ref[f'{k}x{m}x{n}'] = (float((dw - want).norm() / want.norm()),
                               float((db - dy.float().sum(0)).norm() / dy.float().sum(0).norm()))
    print(json.dumps({'us': out, 'err': ref}))


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'one':
        run()
        sys.exit(0)
    res = {}
    for name, extra in (('default', {}), ('slice256', {'GRK_WGRAD_SLICE': '256'}),
                        ('slice128', {'GRK_WGRAD_SLICE': '128'}), ('mgemm', {'GRK_WGRAD_MGEMM': '1'})):
        r = subprocess.run([sys.executable, __file__, 'one'], env=dict(os.environ, **extra), capture_output=True,
                           text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
    tot = {v: 0.0 for v in res}
    for k, m, n, calls in SHAPES:
        key = f'{k}x{m}x{n}'
        f = 2.0 * k * m * n
        line = f'K={k:6d} M={m:5d} N={n:4d} x{calls}'
        for v in res:
            us = res[v]['us'][key]
            tot[v] += us * calls
            line += f'  {v}: {us:7.1f} us {f / us / 1e6:5.0f} TF/s err {res[v]["err"][key][0]:.1e}/{res[v]["err"][key][1]:.1e}'
        print(line)
    print('per step (ms):', {v: round(t / 1e3, 4) for v, t in tot.items()})
