"""The process's own HIP streams (grk_stream_create), wrapped as torch streams.

torch.cuda.Stream() hands out pooled streams round-robin, so it can return the
very stream a process group records its collectives' events on; a HIP graph
captured on that stream makes the NCCL watchdog's query of those events fail
(hipErrorCapturedEvent: "event last recorded in a capturing stream"), which it
treats as fatal.  Every stream the trainer captures or
forks work onto is one of these instead: created once per (device, index),
never destroyed (they live as long as the process)."""
from __future__ import annotations

import contextlib
import ctypes

import torch

_STREAMS = {}


def private_stream(device, index=0, priority=None):
    """Private stream number ``index`` of ``device`` (``priority``: a HIP stream priority
    for its creation, lower = more urgent; None = the default)."""
    from . import _lib as L
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _STREAMS.get((idx, index))
    if s is None:
        with torch.cuda.device(idx):
            raw = ctypes.c_void_p()
            if priority is None:
                L.check(L.lib().grk_stream_create(ctypes.byref(raw)), 'grk_stream_create')
            else:
                L.check(L.lib().grk_stream_create_priority(ctypes.byref(raw), int(priority)),
                        'grk_stream_create_priority')
            s = _STREAMS[(idx, index)] = torch.cuda.ExternalStream(raw.value, device=torch.device('cuda', idx))
    return s


def run_branches(fns, device, first_index=1):
    """Run independent pieces of device work concurrently: fns[i] on private stream
    first_index + i, each forked from and joined back into the current stream (in
    a HIP graph capture: parallel branches of the graph).  Chains of small kernels
    (table-group reductions and updates) then overlap their launch latencies
    instead of adding them up.  The fns must not synchronize with the host."""
    fns = [f for f in fns if f is not None]
    if len(fns) <= 1 or torch.device(device).type != 'cuda':
        for f in fns:
            f()
        return
    cur = torch.cuda.current_stream(device)
    used = []
    for i, f in enumerate(fns):
        s = private_stream(device, first_index + i)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            f()
        used.append(s)
    for s in used:
        cur.wait_stream(s)
