"""The process's own HIP streams (grk_stream_create), wrapped as torch streams.

torch.cuda.Stream() hands out pooled streams round-robin, so it can return the
very stream a process group records its collectives' events on; a HIP graph
captured on that stream makes the NCCL watchdog's query of those events fail
(hipErrorCapturedEvent: "event last recorded in a capturing stream"), which it
treats as fatal.  Every stream the trainer captures or
forks work onto is one of these instead: created once per (device, index),
never destroyed (they live as long as the process)."""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import os
import sys
import time

import torch

_STREAMS = {}

# GRK_HOST_TIMES=1: host issue time of the eager phases of a row-sharded replayed
# step (host_lap), printed per step at exit -- where the device waits on the host.
HOST_TIMES = os.environ.get('GRK_HOST_TIMES') == '1'
_HOST_T = {}
_HOST_LAST = [0.0]
_HOST_ON = [False]


def host_lap(key=None, step=False):
    """Add the host time since the previous lap to ``key`` (None: (re)start the clock and
    the recording -- laps outside a recorded step, e.g. warm-up, are not counted);
    step=True counts one step and stops the recording.  No-op unless GRK_HOST_TIMES=1."""
    if not HOST_TIMES:
        return
    t = time.perf_counter()
    if key is None:
        _HOST_ON[0] = True
    elif _HOST_ON[0]:
        _HOST_T[key] = _HOST_T.get(key, 0.0) + t - _HOST_LAST[0]
    if step and _HOST_ON[0]:
        _HOST_T['#steps'] = _HOST_T.get('#steps', 0) + 1
        _HOST_ON[0] = False
    _HOST_LAST[0] = t


_HOST_EV = {}


def host_mark(name):
    """Record a device event ``name`` on the current stream (GRK_HOST_TIMES=1)."""
    if HOST_TIMES and _HOST_ON[0]:
        e = torch.cuda.Event()
        e.record()
        _HOST_EV[name] = e


def host_check(name, key):
    """Count (under ``key``, per step) whether event ``name`` has completed: the device
    has drained up to that point when the host gets here."""
    if HOST_TIMES and _HOST_ON[0] and name in _HOST_EV:
        _HOST_T[key] = _HOST_T.get(key, 0) + (1 if _HOST_EV[name].query() else 0)


@atexit.register
def _report_host_times():
    n = _HOST_T.get('#steps')
    if n:
        print('host issue us/step: ' + ', '.join(f'{k} {1e6 * v / n:.0f}' for k, v in _HOST_T.items()
                                                 if k != '#steps' and not k.startswith('n:')), file=sys.stderr)
        print('fraction of steps: ' + ', '.join(f'{k[2:]} {v / n:.2f}' for k, v in _HOST_T.items()
                                                if k.startswith('n:')), file=sys.stderr)


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
