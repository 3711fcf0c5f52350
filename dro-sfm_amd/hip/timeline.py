"""In-graph step timeline (diagnostics; tools/step_timeline.py).

rocprofv3's kernel trace serialises the streams of a replayed step, so its
per-kernel sums do not say where the 16-17 ms of a graph replay go.  Here the
step itself records the device's constant-rate real-time counter
(csrc/dro_capi.hip `dro_timestamp`, 100 MHz, common to all XCDs) at named
points, on the stream that reaches them: forward phases via stamp(), backward
phases via stamp_grad() (an identity whose backward stamps when the gradient
reaches that tensor, on the stream autograd runs that node on).  The stamps
are captured into the hipGraph like any launch; every replay overwrites the
same slots.  Inactive (the default) both calls cost one Python check.
"""
import ctypes

import torch

from . import _lib


class Timeline:
    """Context manager: while active, stamp()/stamp_grad() record into slots."""

    _active = None

    def __init__(self, device, capacity=1024):
        self.buf = torch.zeros(capacity, dtype=torch.int64, device=device)
        self.names = []            # slot -> (name, stream id)
        self.capacity = capacity
        hz = ctypes.c_longlong(0)
        _lib.check(_lib.load().dro_wall_clock_hz(ctypes.byref(hz)), "dro_wall_clock_hz")
        self.hz = hz.value

    def __enter__(self):
        Timeline._active = self
        return self

    def __exit__(self, *exc):
        Timeline._active = None

    def record(self, name):
        if len(self.names) >= self.capacity:
            raise RuntimeError("timeline: out of slots")
        st = torch.cuda.current_stream(self.buf.device)
        slot = len(self.names)
        self.names.append((name, st.stream_id))
        _lib.check(_lib.load().dro_timestamp(ctypes.c_void_p(self.buf.data_ptr()), slot,
                                             ctypes.c_void_p(st.cuda_stream)), "dro_timestamp")

    def read(self, first=0):
        """[(name, stream id, microseconds since slot `first`)] of slots >= first."""
        t = self.buf.cpu().tolist()
        t0 = t[first]
        return [(n, s, (t[i] - t0) * 1e6 / self.hz) for i, (n, s) in enumerate(self.names) if i >= first]


def stamp(name):
    tl = Timeline._active
    if tl is not None:
        tl.record(name)


class _StampGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, name):
        ctx.name = name
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        stamp(ctx.name)
        return g, None


def stamp_grad(x, name):
    """x itself; while a timeline is active, a stamp when x's gradient arrives."""
    if Timeline._active is None or not torch.is_tensor(x) or not x.requires_grad:
        return x
    return _StampGrad.apply(x, name)
