"""Data-parallel training over RCCL (replaces the reference's Horovod path).

Reference: HorovodTrainer (dro_sfm/trainers/horovod_trainer.py:14-127) with
hvd.DistributedOptimizer commented out (:67-69) and world_size pinned to 1
(:40-50) -- data parallelism is dormant there.  This module
provides it MI355X-first:

  * one process per GPU (torchrun), backend "nccl" == RCCL over xGMI;
  * every gradient lives in ONE flat fp32 buffer (param.grad are views into
    it), cut into ~bucket_mb buckets in reverse registration order -- the order
    backward produces them;
  * a post-accumulate hook per parameter counts arrivals per bucket; a full
    bucket's all-reduce is issued (async) as soon as every bucket before it in
    one rank-independent order has been issued, so communication of late
    layers overlaps backward of early ones and every rank issues the same
    sequence of collectives even when its buckets complete in another order
    or a gradient does not arrive on some step;
  * from the second step on, parameters whose gradient autograd produces
    (everything but the conv-engine weights written in place) start the
    backward with .grad = None, so AccumulateGrad adopts the produced tensor
    instead of launching an add into the zeroed flat buffer; a complete
    bucket's adopted gradients are copied into the flat buffer with one
    multi-tensor launch (torch._foreach_copy_) -- ~160 add launches per step
    become a handful;
  * the conv-engine weights whose gradients are written in place (batched
    over all uses of a weight) get their weight-gradient launch from their own
    post-accumulate hook, i.e. as soon as autograd has back-propagated their
    last use, so the update blocks' buckets are reduced while the encoders'
    backward still runs;
  * parameters that never receive a gradient (DepthPoseNet.cnet, dead in the
    reference forward) are discovered on the first step and left out;
  * initial parameters and buffers are broadcast from rank 0 (BatchNorm keeps
    per-replica batch statistics, as the reference: no SyncBN).

The step order matches HorovodTrainer.train: zero_grad -> forward -> loss ->
backward -> (all-reduce) -> Adam step.
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def graph_safe_nccl_env():
    """Environment for RCCL collectives captured in hipGraphs, set before the
    process group is created (explicit settings win): no flight recorder and
    no event cache (event objects recycled between eager and captured
    collectives).  Neither hides an error: a HIP error the watchdog sees still
    aborts the process, as by default.  The capture abort of round 5 was the
    watchdog polling the warm-up steps' eager collectives inside the capture
    (drain_watchdog)."""
    os.environ.setdefault("TORCH_NCCL_TRACE_BUFFER_SIZE", "0")
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


# ProcessGroupNCCL's watchdog retires completed works once per poll (every
# 100 ms in this torch); waiting three polls covers a late one
_WATCHDOG_DRAIN_S = float(os.environ.get("DRO_WATCHDOG_DRAIN_S", "0.3"))


def drain_watchdog():
    """Block until the RCCL watchdog can no longer hold an eager collective.

    Cause of the round-5 abort (hipErrorCapturedEvent thrown by the watchdog
    thread, `WorkNCCL::finishedGPUExecutionInternal`, while GraphedTrainStep
    captured with collectives inside): the watchdog tracks every EAGER
    collective until a poll finds it complete -- up to one poll interval after
    it finished.  The warm-up steps' last all-reduces were still tracked when
    the capture began; their end events were recorded on RCCL's internal
    stream, which the first captured collective pulls into the capture; a
    poll landing after that queried an event whose stream was capturing and
    got hipErrorCapturedEvent (timing-dependent: "1 run in 7";
    tools/rccl_watchdog_probe.py makes the window deterministic).  Captured
    collectives are never tracked, so after this wait the capture has nothing
    for the watchdog to query."""
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    time.sleep(_WATCHDOG_DRAIN_S)


def init_distributed(backend=None):
    """Initialise the default process group from torchrun's env (no-op for 1 rank).
    Returns (rank, world_size, local_rank)."""
    graph_safe_nccl_env()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            # DRO_DIST_BACKEND=gloo: rehearse the N > 1 path with several ranks
            # on one GPU (RCCL refuses two ranks on one device)
            backend = os.environ.get("DRO_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


class GradBuckets:
    """Flat gradient storage + bucketed, backward-overlapped all-reduce.

    Gradients come in two kinds:
      * adopted: autograd produces the tensor (.grad is None at the start of a
        step); a complete bucket copies them into the flat buffer;
      * direct: the hip conv engine accumulates them in place into the flat
        .grad views (hip/conv.py, `_dro_direct_used`), batched per weight.
    Autograd runs every parameter's post-accumulate hook once per backward,
    after the last use of that parameter has been back-propagated (for a
    direct one the hook sees the None the conv returned).  For a direct
    parameter the hook first launches its queued weight-gradient kernel
    (`direct_flush`, hip.conv.flush_param_grads on the GPU) and records the
    stream it went to; then it counts down like any other.  A bucket is
    complete when all its parameters' hooks have run: the current stream waits
    for every stream that wrote into it, the adopted gradients are gathered,
    and an event marks the gathered state -- the all-reduce, issued later
    from whichever stream runs that hook, waits for that event first.
    """

    def __init__(self, params, bucket_mb=25.0, group=None, groups=(), direct_flush=None,
                 always_reduce=False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # always_reduce: issue the collectives even at world size 1 (tests of the
        # RCCL path inside a captured graph on a single-GPU box)
        self.reduce = self.world > 1 or (always_reduce and dist.is_initialized())
        # suspend: no collectives from the hooks or finish(); reduce_now() runs
        # them after the step's backward (GraphedTrainStep keeps RCCL out of
        # the captured graph, see there)
        self.suspend = False
        self.params = _adjacent_order([p for p in params if p.requires_grad], groups)
        if any(p.dtype != torch.float32 for p in self.params):
            raise RuntimeError("GradBuckets: fp32 parameters only")
        self.flat = torch.zeros(sum(p.numel() for p in self.params), device=self.params[0].device)
        self.offsets, off = {}, 0
        for p in self.params:
            self.offsets[p] = off
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        if direct_flush is None and self.flat.is_cuda:
            from ..hip.conv import flush_param_grads as direct_flush
        self.direct_flush = direct_flush
        self.bucket_bytes = int(bucket_mb * 1024 * 1024)
        self.active = None            # params that receive gradients (learned on step 1)
        self.buckets, self._pending, self._seen = [], [], set()
        self.issued = []              # bucket indices in issue order (last step; tests)
        self.issued_in_backward = 0   # of those, issued from backward hooks (tests)
        # GraphedTrainStep sets this to the capture's origin stream while it
        # captures with collectives inside; each collective's issuing stream
        # must then be part of the capture (issue_capturing, one flag per
        # collective of the last step): a collective issued from a stream
        # outside the capture is tracked by RCCL's watchdog as eager while its
        # kernel and end event land in the capture through RCCL's own stream
        self.capture_origin = None
        self.issue_capturing = []
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        # the stream every bucket's collective is issued from: created here, never
        # during a graph capture (a stream first created inside a capture was
        # the common factor of round 3's capture_end crashes)
        self._comm = torch.cuda.Stream(device=self.flat.device) if self.flat.is_cuda else None
        for p in self.params:
            # hip convs may accumulate this gradient in place (hip/conv.py, direct path)
            p._dro_direct = True

    def _build(self, active):
        self.active = [p for p in self.params if p in active]
        self.buckets, cur, nbytes = [], [], 0
        for p in reversed(self.active):                     # the order backward finishes them
            cur.append(p)
            nbytes += p.numel() * 4
            if nbytes >= self.bucket_bytes:
                self.buckets.append(cur)
                cur, nbytes = [], 0
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {p: i for i, b in enumerate(self.buckets) for p in b}
        # gradients adopted from autograd (.grad = None at the start of a step);
        # the direct ones stay flat views and are written in place
        self._adopt = [[p for p in b if not _direct_used(p)] for b in self.buckets]
        # maximal contiguous flat ranges of active parameters (reduce_now skips
        # the never-used ones, e.g. DepthPoseNet.cnet: 3.5 M of 16.1 M floats)
        self._runs = []
        for p in self.active:
            lo, hi = self.offsets[p], self.offsets[p] + p.numel()
            if self._runs and self._runs[-1][1] == lo:
                self._runs[-1][1] = hi
            else:
                self._runs.append([lo, hi])
        self._need = [len(b) for b in self.buckets]
        # ONE all-reduce order, identical on every rank: backward order.  A bucket
        # is issued only after every bucket before it in this order, so ranks
        # whose buckets complete in different orders -- or not at all on some
        # step (a gradient that never arrives) -- still pair their collectives
        # one for one (as DDP's in-order bucket launch does).
        self._order = list(range(len(self.buckets)))

    def _slice(self, bucket):
        """One contiguous flat slice covering a bucket (slots of inactive params
        inside it are zeros and reduce harmlessly)."""
        lo = min(self.offsets[p] for p in bucket)
        hi = max(self.offsets[p] + p.numel() for p in bucket)
        return self.flat[lo:hi]

    def _on_grad(self, p):
        direct = _direct_used(p)
        wrote = None
        if direct and self.direct_flush is not None:
            # every use of p is back-propagated: launch its queued weight gradient
            wrote = self.direct_flush(p)
        if self.active is None:
            self._seen.add(p)
            return
        b = self._bucket_of.get(p)
        if b is None or self._ready[b]:
            return
        if self.flat.is_cuda:
            # the hook runs on the stream that produced this gradient (the context
            # encoders' backward runs on side streams), the in-place weight
            # gradient went to `wrote`: remember both for the bucket.  A `wrote`
            # other than the hook's stream (the weight-gradient flush stream)
            # must not be waited for here: that would put the data-gradient
            # chain behind the weight gradients again; the collective waits for
            # it instead, and the step's end joins it
            cur = torch.cuda.current_stream()
            self._bstreams[b].add(cur)
            if wrote is not None:
                (self._bstreams[b] if wrote == cur else self._bside[b]).add(wrote)
        self._left[b] -= 1
        if self._left[b] == 0:
            self._complete(b)
            self._issue_ready()

    def _complete(self, b):
        """Bucket b's gradients are final: order the current stream after every
        stream that produced or wrote one of them, gather the adopted ones into
        the flat buffer, and mark that point with an event."""
        if self.flat.is_cuda:
            cur = torch.cuda.current_stream()
            for st in self._bstreams[b]:
                if st != cur:
                    cur.wait_stream(st)
        self._gather(b)
        if self.flat.is_cuda:
            self._events[b] = torch.cuda.Event()
            self._events[b].record(torch.cuda.current_stream())
        self._ready[b] = True

    def _issue_ready(self):
        """Issue the all-reduce of every ready bucket at the head of the order.
        The issuing stream first waits for the bucket's completion event: the
        bucket may have been gathered on another stream."""
        while self._next < len(self._order) and self._ready[self._order[self._next]]:
            b = self._order[self._next]
            self._next += 1
            self.issued.append(b)
            if self.reduce and not self.suspend:
                if self._comm is None:                       # CPU (gloo tests)
                    self._pending.append(dist.all_reduce(self._slice(self.buckets[b]), op=dist.ReduceOp.SUM,
                                                         group=self.group, async_op=True))
                    continue
                # from the comm stream, after the bucket's gather (its event) and
                # any in-place weight gradients written on another stream: the
                # backward's next kernels on the compute streams do not wait for it
                comm = self._comm
                comm.wait_event(self._events[b])
                for st in self._bside[b]:
                    comm.wait_stream(st)
                with torch.cuda.stream(comm):
                    if self.capture_origin is not None:
                        self.issue_capturing.append(torch.cuda.is_current_stream_capturing())
                    self._pending.append(dist.all_reduce(self._slice(self.buckets[b]), op=dist.ReduceOp.SUM,
                                                         group=self.group, async_op=True))

    def _gather(self, b):
        """Copy bucket b's adopted gradients into the flat buffer (one launch).
        A gradient that never arrived this step keeps its zeroed slot, which
        becomes its .grad (the all-reduced average may still be non-zero)."""
        ps = [p for p in self._adopt[b] if p.grad is not None and not self._is_view(p)]
        if ps:
            torch._foreach_copy_([self._view(p) for p in ps], [p.grad for p in ps])
            for p in ps:
                p.grad = self._view(p)
        for p in self._adopt[b]:
            if p.grad is None:
                p.grad = self._view(p)

    def _view(self, p):
        off = self.offsets[p]
        return self.flat[off:off + p.numel()].view_as(p)

    def _is_view(self, p):
        g = p.grad
        return (g.untyped_storage().data_ptr() == self.flat.untyped_storage().data_ptr()
                and g.storage_offset() == self.offsets[p])

    def zero(self):
        self.flat.zero_()
        self._pending = []
        self.issued = []
        self.issue_capturing = []
        if self.active is not None:
            self._left = list(self._need)
            self._ready = [False] * len(self.buckets)
            self._events = [None] * len(self.buckets)
            self._next = 0
            self._bstreams = [set() for _ in self.buckets]
            self._bside = [set() for _ in self.buckets]
            for ps in self._adopt:
                for p in ps:
                    p.grad = None

    def finish(self):
        """Complete every bucket's all-reduce and average over ranks."""
        self.issued_in_backward = len(self.issued)
        if self.active is None:
            seen = self._seen | {p for p in self.params if _direct_used(p)}
            if self.world > 1:
                flags = torch.tensor([float(p in seen) for p in self.params], device=self.flat.device)
                dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.group)
                seen = {p for p, f in zip(self.params, flags.tolist()) if f > 0}
            self._build(seen)
            if self.reduce:                                  # step 1: reduce synchronously
                for b in self.buckets:
                    dist.all_reduce(self._slice(b), op=dist.ReduceOp.SUM, group=self.group)
        else:
            # buckets some of whose gradients never arrived this step (their
            # missing slots are the zeros of zero()): complete them, then issue
            # everything not issued yet, in the common order
            for b in range(len(self.buckets)):
                if not self._ready[b]:
                    self._complete(b)
            self._issue_ready()
            for work in self._pending:
                work.wait()
            self._pending = []
            if self._comm is not None and self.reduce and not self.suspend:
                torch.cuda.current_stream().wait_stream(self._comm)
        if self.world > 1 and not self.suspend:
            self.flat.div_(self.world)

    def reduce_now(self):
        """All-reduce the flat gradient and average: the exchange of a step
        whose backward ran with `suspend` set.  One collective per contiguous
        run of active parameters (two for DepthPoseNet: its unused cnet sits
        between the update blocks and the context encoders); the never-used
        slots stay zero."""
        if not self.reduce:
            return
        runs = getattr(self, "_runs", None) or [[0, self.flat.numel()]]
        for lo, hi in runs:
            dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
        if self.world > 1:
            self.flat.div_(self.world)


def agree_all(ok, group=None, device=None):
    """True iff `ok` holds on every rank: one MIN all-reduce, issued outside any
    graph capture.  Ranks that must take the same branch (GraphedTrainStep's
    choice of exchange path) decide on the agreed value, never on their own."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def capture_with_agreement(try_in_graph, fallback, group=None, device=None, sync=None, log=None):
    """Run `try_in_graph()` (a capture with the collectives inside); every rank
    then learns whether it succeeded on ALL ranks and, if not, every rank runs
    `fallback()` (the capture without collectives, exchange after replay).
    A rank deciding alone could leave it reducing after replay while its peers
    run collectives inside their graphs: a deadlock.  Capturing a
    collective does not communicate, so a rank that fails mid-capture cannot
    block one that succeeded before both reach the agreement.  Returns True
    when the in-graph path was kept."""
    ok, err = True, None
    try:
        try_in_graph()
    except RuntimeError as e:
        ok, err = False, e
    if sync is not None:
        sync()
    if agree_all(ok, group, device):
        return True
    if log is not None:
        log(f"capture with in-graph all-reduces failed on {'this rank' if not ok else 'another rank'}"
            + (f" ({err})" if err is not None else "") + "; every rank falls back to the exchange after each replay")
    fallback()
    return False


def collective_signature(grads):
    """The sequence of collectives the last backward issued: (bucket, flat
    offset, length) per all-reduce, in issue order."""
    out = []
    for b in grads.issued:
        s = grads._slice(grads.buckets[b])
        out.append((int(b), int(s.storage_offset()), int(s.numel())))
    return tuple(out)


def check_same_across_ranks(sig, group=None, device=None, what="collective sequence"):
    """Raise unless `sig` (any repr-able value) is identical on every rank: a
    CRC of its repr, MIN- and MAX-reduced."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    import zlib
    h = zlib.crc32(repr(sig).encode())
    t = torch.tensor([h, -h], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    if int(t[0]) != h or -int(t[1]) != h:
        raise RuntimeError(f"{what} differs between ranks (rank {dist.get_rank(group)}: crc {h}, "
                           f"min {int(t[0])}, max {-int(t[1])})")


def _direct_used(p):
    return getattr(p, "_dro_direct_used", False)


def _adjacent_order(params, groups):
    """params in registration order, except that each group (a list of
    parameters read as one fused tensor, e.g. SepConvGRU's z|r weights) is
    placed back to back at its first member's position."""
    if not groups:
        return list(params)
    present = set(params)
    lead = {}
    for g in groups:
        g = [p for p in g if p in present]
        if len(g) > 1:
            for p in g:
                lead[p] = g
    out, done = [], set()
    for p in params:
        if p in done:
            continue
        for q in lead.get(p, [p]):
            if q not in done:
                out.append(q)
                done.add(q)
    return out


def param_groups(model):
    """Fused-parameter groups declared by modules (`dro_param_groups()`)."""
    groups = []
    for m in model.modules():
        fn = getattr(m, "dro_param_groups", None)
        if callable(fn):
            groups.extend(fn())
    return groups


def broadcast_module(module, src=0, group=None):
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad off) over ONE flat parameter buffer: a single
    fused HIP launch per step (csrc/optim.hip) instead of per-tensor kernels.

    A torch.optim.Optimizer, so torch.optim.lr_scheduler wraps it (the
    reference builds StepLR, model_wrapper.py:192-193).  The step counter AND
    the hyper-parameters {lr, beta1, beta2, eps, weight_decay} live in device
    memory and the kernel reads them at run time: a captured hipGraph follows
    a schedule.  Eager step() syncs param_groups into the device copy;
    GraphedTrainStep.step() calls sync_hyper() before each replay.

    state_dict() / load_state_dict() use torch.optim.Adam's per-parameter
    layout ({'state': {i: {'step', 'exp_avg', 'exp_avg_sq'}}, 'param_groups':
    [{..., 'params': [0..n-1]}]}), indexed in the order of `params` -- the
    reference saves its Adam state that way under 'optimizer'
    (model_checkpoint.py:76), so checkpoints interchange in both directions.
    `params` is the module's whole parameter list, as the reference's Adam
    group over depth_net.parameters() (model_wrapper.py:173): frozen
    parameters (absent from `offsets`) keep their index and never get state.
    The saved group says capturable=False (a torch.optim.Adam loading it keeps
    its default code path); this optimizer's own capture safety does not
    depend on that flag.  One step counter is shared by every parameter: a
    parameter that first receives a gradient after step 1 is saved with the
    global step (torch.optim.Adam would count its own)."""

    def __init__(self, params, flat_param, flat_grad, lr=2e-4, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, offsets=None):
        from ..hip import _lib
        self._lib = _lib
        _lib.load()
        params = list(params)
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        amsgrad=False, maximize=False, foreach=None, capturable=False,
                        differentiable=False, fused=None)
        super().__init__(params if params else [flat_param], defaults)
        self.params, self.flat_param, self.flat_grad = params, flat_param, flat_grad
        if offsets is None:
            offsets, off = {}, 0
            for p in params:
                offsets[p] = off
                off += p.numel()
        self.offsets = offsets
        self.active = None               # params that ever receive a gradient (None: all)
        self.exp_avg = torch.zeros_like(flat_param)
        self.exp_avg_sq = torch.zeros_like(flat_param)
        self.step_t = torch.zeros((), device=flat_param.device, dtype=torch.float32)
        # the flat moments + step are this optimizer's whole state (restored in
        # place by callers that snapshot optimizer.state, e.g. test_graph_step)
        self.state["flat"] = {"step": self.step_t, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}
        self.hyper_t = torch.zeros(5, device=flat_param.device, dtype=torch.float32)
        self._hyper_host = None
        self.sync_hyper()

    def _hyper(self):
        g = self.param_groups[0]
        return (float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]),
                float(g["weight_decay"]))

    def sync_hyper(self):
        """Write param_groups' hyper-parameters to the device copy the kernel
        reads (only when they changed; never during graph capture -- the write
        would be baked into the graph)."""
        h = self._hyper()
        if h == self._hyper_host:
            return
        if self.hyper_t.is_cuda and torch.cuda.is_current_stream_capturing():
            return
        self.hyper_t.copy_(torch.tensor(h, dtype=torch.float32), non_blocking=False)
        self._hyper_host = h

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise RuntimeError("FlatAdam.step: closures are not supported")
        self.sync_hyper()
        self.step_t += 1
        lib = self._lib
        lib.check(lib.load().dro_adam_step(lib.ptr(self.flat_param), lib.ptr(self.flat_grad),
                                           lib.ptr(self.exp_avg), lib.ptr(self.exp_avg_sq),
                                           self.flat_param.numel(), lib.ptr(self.step_t),
                                           lib.ptr(self.hyper_t), lib.stream_of(self.flat_param)),
                  "dro_adam_step")

    def zero_grad(self, set_to_none=False):
        self.flat_grad.zero_()

    def _slot(self, buf, p):
        off = self.offsets[p]
        return buf[off:off + p.numel()].view_as(p)

    def state_dict(self):
        g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        g["params"] = list(range(len(self.params)))
        state = {}
        if float(self.step_t) > 0:               # torch.optim.Adam has no state before its first step
            for i, p in enumerate(self.params):
                if p not in self.offsets or (self.active is not None and p not in self.active):
                    continue                 # torch.optim.Adam keeps no state without a grad
                # a CPU step tensor, as torch.optim.Adam(capturable=False) saves it
                state[i] = {"step": torch.tensor(float(self.step_t), dtype=torch.float32),
                            "exp_avg": self._slot(self.exp_avg, p).detach().clone(),
                            "exp_avg_sq": self._slot(self.exp_avg_sq, p).detach().clone()}
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd):
        """In place (a captured graph holds these buffers' addresses).  Accepts
        torch.optim.Adam state dicts over the same parameter list."""
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.params):
            raise ValueError("FlatAdam.load_state_dict: expected one group over "
                             f"{len(self.params)} parameters")
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            steps = set()
            for slot, i in enumerate(groups[0]["params"]):
                st = sd["state"].get(i)
                p = self.params[slot]
                if st is None or p not in self.offsets:
                    continue                 # no state, or a parameter frozen here
                self._slot(self.exp_avg, p).copy_(st["exp_avg"])
                self._slot(self.exp_avg_sq, p).copy_(st["exp_avg_sq"])
                steps.add(float(st["step"]))
            if len(steps) > 1:
                raise ValueError(f"FlatAdam.load_state_dict: per-parameter steps differ {sorted(steps)}")
            self.step_t.fill_(steps.pop() if steps else 0.0)
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = tuple(v) if k == "betas" else v
        self.sync_hyper()


def flatten_parameters(params, offsets, total, device):
    """Move the parameters into one contiguous buffer (same layout as the flat
    gradient buffer); each parameter becomes a view of it."""
    flat = torch.empty(total, device=device, dtype=torch.float32)
    with torch.no_grad():
        for p in params:
            off = offsets[p]
            flat[off:off + p.numel()].copy_(p.data.reshape(-1))
            p.data = flat[off:off + p.numel()].view_as(p)
    return flat


class DataParallelTrainer:
    """fit()-less step driver: `loss, metrics = trainer.step(batch)`.

    `model(batch)` must return a dict with a 'loss' tensor (the SfmModelMF
    family does).  Adam with the reference's lr (configs/*.yaml: 2e-4).
    `capturable=True` keeps Adam's step counters on the device so the whole
    step can be replayed from a hipGraph (GraphedTrainStep)."""

    def __init__(self, model, lr=2e-4, bucket_mb=25.0, group=None, betas=(0.9, 0.999), eps=1e-8,
                 capturable=False, always_reduce=False):
        self.model = model
        broadcast_module(model, 0, group)
        self.grads = GradBuckets(model.parameters(), bucket_mb=bucket_mb, group=group,
                                 groups=param_groups(model), always_reduce=always_reduce)
        dev = self.grads.flat.device
        if dev.type == "cuda":
            # fused Adam over flat buffers (the product path on the GPU)
            self.flat_params = flatten_parameters(self.grads.params, self.grads.offsets,
                                                  self.grads.flat.numel(), dev)
            # indexed in registration order over ALL parameters, like the
            # reference's Adam over depth_net.parameters() (model_wrapper.py:168-187)
            order = list(model.parameters())
            self.optimizer = FlatAdam(order, self.flat_params, self.grads.flat, lr=lr,
                                      betas=betas, eps=eps, offsets=self.grads.offsets)
        else:
            # CPU (gloo tests of the data-parallel host logic): PyTorch's Adam
            self.optimizer = torch.optim.Adam(self.grads.params, lr=lr, betas=betas, eps=eps,
                                              foreach=True, capturable=capturable)

    def _forward_backward(self, batch, **fwd_kw):
        from ..hip.timeline import stamp, stamp_grad
        stamp("step:begin")
        self.grads.zero()
        out = self.model(batch, **fwd_kw)
        loss = out["loss"]
        stamp("fwd:loss")
        stamp_grad(loss, "bwd:begin").sum().backward()
        stamp("bwd:end")
        self.grads.finish()
        if isinstance(self.optimizer, FlatAdam) and self.optimizer.active is None \
                and self.grads.active is not None:
            self.optimizer.active = set(self.grads.active)
        return loss.detach(), out.get("metrics", {})

    def _step_inner(self, batch, **fwd_kw):
        from ..hip.timeline import stamp
        res = self._forward_backward(batch, **fwd_kw)
        self.optimizer.step()
        stamp("step:end")
        return res

    def step(self, batch, **fwd_kw):
        self.model.train()
        return self._step_inner(batch, **fwd_kw)


def _clone_batch(batch):
    out = {}
    for k, v in batch.items():
        if torch.is_tensor(v):
            out[k] = v.clone()
        elif isinstance(v, (list, tuple)) and v and torch.is_tensor(v[0]):
            out[k] = [t.clone() for t in v]
        else:
            out[k] = v
    return out


def _copy_batch(dst, src):
    for k, v in src.items():
        if k not in dst:
            continue
        if torch.is_tensor(v):
            dst[k].copy_(v, non_blocking=True)
        elif isinstance(v, (list, tuple)) and v and torch.is_tensor(v[0]):
            for d, s_ in zip(dst[k], v):
                d.copy_(s_, non_blocking=True)


class GraphedTrainStep:
    """The whole training step -- zero -> forward -> loss -> backward -> RCCL
    all-reduce -> Adam -- captured once into a hipGraph per branch of the
    random left-right flip (SfmModelMF.py:110), then replayed: no Python
    dispatch and no launch gaps in the steady state.

    The batch is copied into static device buffers before each replay; the
    intrinsics are restored from `intrinsics_ref` INSIDE the graph because the
    flip branch mutates them in place (as the reference does).
    The first eager steps (bucket discovery, MIOpen algorithm selection) run
    before capture on a side stream and are real training steps.

    With a gradient exchange over RCCL (world > 1, backend "nccl"), the
    bucketed all-reduces are captured IN the graph (reduce_in_graph, the
    default): each bucket's collective is issued from the backward hook that
    completes it, on the comm stream, so the replayed graph runs it beside the
    rest of the backward (horovod_trainer.py:66-69's DistributedOptimizer
    hooks, done as graph branches).  With any other backend (gloo: the CPU
    tests and the one-GPU rehearsal), or reduce_in_graph=False, the graph
    holds zero -> forward -> loss -> backward and each step() all-reduces the
    flat gradient after the replay, then runs Adam.

    The graphs hold the ADDRESSES of the parameters, gradients and Adam state:
    restore checkpoints in place (tensor.copy_), or build a new GraphedTrainStep
    after optimizer.load_state_dict (which replaces the state tensors).
    """

    def __init__(self, trainer, example_batch, warmup=3, flips=(False, True), share_pool=True,
                 reduce_in_graph=None):
        self.tr = trainer
        if reduce_in_graph is None:
            reduce_in_graph = (os.environ.get("DRO_REDUCE_IN_GRAPH", "1") != "0" and dist.is_initialized()
                               and dist.get_backend(trainer.grads.group) == "nccl")
        self.in_graph = trainer.grads.reduce and bool(reduce_in_graph)
        # collectives outside the graph when there is an exchange that is not captured
        self.outside = trainer.grads.reduce and not reduce_in_graph
        self.model = trainer.model
        self.static = _clone_batch(example_batch)
        self.static["intrinsics_ref"] = example_batch["intrinsics"].clone()
        self.model.train()
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for i in range(max(warmup, len(flips))):
                self._body(flips[i % len(flips)])
        cur.wait_stream(side)
        torch.cuda.synchronize()
        if self.in_graph:
            # the warm-up's eager collectives must be retired by the RCCL watchdog
            # before any collective is captured (drain_watchdog)
            drain_watchdog()
        self.pool = torch.cuda.graph_pool_handle() if share_pool else None
        group, dev = trainer.grads.group, trainer.grads.flat.device
        if not self.in_graph:
            self._capture_all(flips)
        else:
            def fallback():
                self.graphs = {}
                torch.cuda.synchronize()
                self.in_graph, self.outside = False, True
                self.pool = torch.cuda.graph_pool_handle() if share_pool else None
                self._capture_all(flips)

            # every rank falls back together or none does (capture_with_agreement)
            capture_with_agreement(lambda: self._capture_all(flips), fallback, group, dev,
                                   sync=torch.cuda.synchronize,
                                   log=lambda m: print(f"[GraphedTrainStep] {m}", file=sys.stderr, flush=True))
        # each rank replays the flip graph its own draw picks (as the reference
        # flips per rank, SfmModelMF.py:110): every graph must issue the same
        # collectives in the same order, on every rank
        seqs = set(self.issue_seq.values())
        if len(seqs) != 1:
            raise RuntimeError(f"GraphedTrainStep: the flip graphs issue different collective sequences: "
                               f"{self.issue_seq}")
        check_same_across_ranks(next(iter(seqs)), group, dev, "captured collective sequence")

    def _capture_all(self, flips):
        self.graphs, self.issue_seq, self.issue_capturing = {}, {}, {}
        for f in flips:
            g = torch.cuda.CUDAGraph()
            # thread_local: the RCCL watchdog thread queries the events of the
            # warm-up steps' collectives; under the default (global) mode that
            # query from another thread invalidated the capture (measured:
            # hipErrorStreamCaptureUnsupported in the watchdog, then an abort)
            grads = self.tr.grads
            with torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):
                grads.capture_origin = torch.cuda.current_stream() if self.in_graph else None
                try:
                    out = self._captured(f)
                finally:
                    grads.capture_origin = None
            if self.in_graph and not all(grads.issue_capturing):
                # such a collective would run in the graph AND be polled by the
                # watchdog as an eager one (its end event inside the capture)
                raise RuntimeError(f"GraphedTrainStep: {grads.issue_capturing.count(False)} collective(s) "
                                   "issued from a stream outside the capture")
            self.issue_capturing[f] = list(grads.issue_capturing)
            self.graphs[f] = (g, out)
            # in-graph: the buckets the hooks issued inside this capture; after
            # replay: reduce_now's fixed runs (the same for every graph)
            self.issue_seq[f] = (collective_signature(self.tr.grads) if not self.outside
                                 else ("after-replay", tuple(map(tuple, getattr(self.tr.grads, "_runs", [])))))
        torch.cuda.synchronize()

    def _body(self, flip):
        self.static["intrinsics"].copy_(self.static["intrinsics_ref"])
        return self.tr._step_inner(self.static, flip=flip)

    def _captured(self, flip):
        if not self.outside:
            return self._body(flip)
        self.static["intrinsics"].copy_(self.static["intrinsics_ref"])
        self.tr.grads.suspend = True
        try:
            return self.tr._forward_backward(self.static, flip=flip)
        finally:
            self.tr.grads.suspend = False

    def step(self, batch, flip=None):
        sync = getattr(self.tr.optimizer, "sync_hyper", None)
        if sync is not None:
            sync()                       # a scheduler's lr reaches the captured Adam
        _copy_batch(self.static, {k: v for k, v in batch.items() if k != "intrinsics"})
        self.static["intrinsics_ref"].copy_(batch["intrinsics"], non_blocking=True)
        if flip is None:
            flip = self.model._rng.random() < self.model.flip_lr_prob
        g, out = self.graphs[bool(flip)]
        g.replay()
        if self.outside:
            self.tr.grads.reduce_now()
            self.tr.optimizer.step()
        return out
