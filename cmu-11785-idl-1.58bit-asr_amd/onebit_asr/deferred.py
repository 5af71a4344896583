"""Deferred gradient finishes: every BitLinear weight-gradient finish and every LayerNorm
dgamma / dbeta reduction (and every depthwise-conv weight-gradient finish) of a backward runs
in ONE launch per kind, at the end of the backward.

In the reference step (train.py:104-111: loss.backward(), clip_grad_norm_, AdamW) a parameter
gradient is read only after the backward ends. On the HIP library each BitLinear dW is a
split-M partial GEMM plus a small finish launch (chunk sum, STE mask, db, dalpha;
csrc/dw.hip) and each LayerNorm backward is a row kernel plus a small parameter-reduce launch
(csrc/layernorm.hip); at Conformer-S that is ~230 launches of 5-7 us each, mostly launch
floor. Inside a ``scope()`` (the training step's forward + backward) the backward entries
instead write their finish descriptors into device tables (``*_defer`` entry points: the
producing launch writes its own entry) and one table launch per kind runs them all, from an
autograd final callback on the backward's stream -- captured into the HIP graph like the
rest of the backward.

A gradient is deferred only when nothing can read it before the flush:
* the tensor is a leaf (a parameter, not a view or copy of one) whose ``.grad`` is None
  (AccumulateGrad then installs the returned tensor
  without a kernel; an existing ``.grad`` -- gradient accumulation, the N > 1 flat buffer --
  would be added to on the spot), and
* the parameter was used by exactly one deferrable op in this scope's forward (several uses
  -- the literal three-pass step -- make autograd add the contributions as they arrive;
  the model ties no weights, so every use of these parameters goes through a counted op).
* no hook can observe the gradient as it is produced: ``scope(enabled=False)`` for a step
  module wrapped in DistributedDataParallel (its reducer copies each gradient into a bucket
  and starts the all-reduce from a hook right after AccumulateGrad, before the flush), and
  no deferral for a parameter carrying a post-accumulate-grad hook.
The workspaces holding the partials are kept referenced until the flush. A slot is counted
only once its producing launch returned OB_OK; a scope left by an exception drops the
pending entries instead of launching them.

Streams: the step may run branches of its backward on several streams (train_step.py: the
decoder branch on a side stream beside the CTC branch). The flush runs on the stream that
was current when the scope opened (the step's own stream, the one the optimizer then uses),
after an event wait on every other stream that produced an entry; the tensors kept for the
flush are recorded on the flush stream (record_stream), so the allocator does not hand them
to their producing stream's next allocation while the flush still reads them.
"""
from __future__ import annotations

import ctypes
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch

from . import _lib

__all__ = ["scope", "note", "can_defer", "dw_slot", "ln_slot", "ln_done", "cm_slot", "keep",
           "add_grad_after_flush", "active", "dwg_take"]

_ON = True  # parity-test hook (tests/test_stacked_step_gpu.py: False = finish on the spot)
_DWG = True  # grouped dW launch (ob_dw_grouped); tests flip it to compare with per-layer dW
_CAP = 512  # table entries per kind
_TICKETS = 1 << 16  # ob_dw_grouped ticket words per device (zeroed once, left zero by every launch)
# (N, K, M, P, bitlinear, index of the first gemm with the same X) of every gemm of the latest
# grouped launch (bench.py's roofline times a launch of the same composition)
LAST_DWG: List[tuple] = []


class DwgGemm(ctypes.Structure):
    """ob_dwg_gemm (include/onebit_hip.h)."""
    _fields_ = [("dY", ctypes.c_void_p), ("X", ctypes.c_void_p), ("W", ctypes.c_void_p),
                ("alpha", ctypes.c_void_p), ("pass_bits", ctypes.c_void_p),
                ("dW", ctypes.c_void_p), ("db", ctypes.c_void_p), ("dalpha", ctypes.c_void_p),
                ("N", ctypes.c_int64), ("K", ctypes.c_int64), ("M", ctypes.c_int64),
                ("P", ctypes.c_int64), ("alpha_raw", ctypes.c_int32), ("bits", ctypes.c_int32)]


class _State:
    def __init__(self):
        self.active = False
        self.uses: Dict[int, int] = {}
        self.tables: Dict[int, tuple] = {}  # device index -> (dw, ln, cm tables)
        self.home: Optional[int] = None  # the stream current when the scope opened
        self.home_dev: Optional[int] = None  # ... and the device it belongs to
        self.reset()

    def reset(self):
        self.dw_n = 0
        self.dw_blocks = 0
        self.ln_n = 0
        self.ln_dmax = 0
        self.cm_n = 0
        self.cm_nmax = 0
        self.refs: List[torch.Tensor] = []
        self.dwg: List[DwgGemm] = []  # weight gradients for the grouped launch
        self.post: List[tuple] = []  # (param, src): param.grad += src after the tables
        self.stream: Optional[int] = None
        self.streams = set()  # every stream that produced an entry
        self.dev: Optional[int] = None
        self.queued = False


_S = _State()


def active() -> bool:
    return _ON and _S.active


# The N > 1 exchange's flat gradient buffer (graph_step, exchange "deferred"): id(param) ->
# (flat, element offset, shape). A backward site that allocates a parameter's gradient takes
# it from grad_buf(): a fresh view of the flat buffer, which AccumulateGrad adopts as .grad
# (the gradient is written in place, no pack copy before the all-reduce).
_ARENA: Dict[int, tuple] = {}


def set_arena(entries) -> None:
    """entries: [(param, flat, offset)] or None (no arena)."""
    _ARENA.clear()
    for p, flat, off in entries or ():
        _ARENA[id(p)] = (flat, off, tuple(p.shape))


def grad_buf(param, shape=None, device=None) -> torch.Tensor:
    """The tensor a backward writes ``param``'s gradient into: its view of the registered flat
    buffer when autograd will adopt it (inside an active scope, ``param.grad`` None, and the
    parameter has exactly ONE producing site in this scope), else a new fp32 tensor of
    ``shape`` (default: the parameter's). A NEW view object every call: an extra reference
    held here would make AccumulateGrad copy instead of adopt.

    The single-producer rule matters for the literal three-pass step: with several uses,
    ``param.grad`` stays None until autograd has SUMMED every incoming gradient, so each
    site would otherwise write the same flat slice and clobber the previous pass's
    contribution before autograd's input buffer adds them. Such parameters get
    fresh tensors; the exchange copies their summed ``.grad`` into the flat buffer."""
    if param is not None and _S.active and _ARENA:
        e = _ARENA.get(id(param))
        if e is not None and param.grad is None and _S.uses.get(id(param), 0) == 1:
            flat, off, shp = e
            n = 1
            for d in shp:
                n *= d
            return flat[off:off + n].view(shp)
    if shape is None:
        shape = param.shape
    return torch.empty(shape, dtype=torch.float32,
                       device=device if device is not None else param.device)


@contextmanager
def scope(enabled: bool = True):
    """Forward + backward of one training step: deferrable gradients are finished by one
    launch per kind at the end of the backward. ``enabled=False``: everything finishes on the
    spot (e.g. under DistributedDataParallel, whose hooks read each gradient as it lands)."""
    prev = _S.active
    _S.active = bool(enabled)
    _S.uses = {}
    on = enabled and torch.cuda.is_available() and torch.cuda.is_initialized()
    _S.home = torch.cuda.current_stream().cuda_stream if on else None
    _S.home_dev = torch.cuda.current_device() if on else None
    ok = False
    try:
        yield
        ok = True
    finally:
        if ok:
            _flush()  # (a no-op when the backward's final callback already ran)
        else:
            _S.reset()  # an entry point failed: its slot may hold a stale descriptor
        _S.active = prev
        _S.uses = {}


def note(*params) -> None:
    """A deferrable op's forward uses these parameters (counted per scope)."""
    if not _S.active:
        return
    for p in params:
        if p is not None:
            _S.uses[id(p)] = _S.uses.get(id(p), 0) + 1


def can_defer(*params) -> bool:
    if not (_ON and _S.active):
        return False
    for p in params:
        if p is None:
            continue
        # a leaf: a derived tensor (a permuted view of a weight, e.g. the subsampling output
        # layer's) passes its gradient on through autograd ops that would read it at once
        if (not p.is_leaf or not p.is_cuda or p.grad is not None
                or _S.uses.get(id(p), 0) != 1):
            return False
        if getattr(p, "_post_accumulate_grad_hooks", None):  # a hook reads it on arrival
            return False
    return True


def _tables(dev: torch.device):
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _S.tables.get(idx)
    if t is None:
        lib = _lib.load()
        dw = torch.zeros((_CAP * lib.ob_dw_finish_entry_bytes(),), dtype=torch.uint8, device=dev)
        ln = torch.zeros((_CAP * lib.ob_ln_param_entry_bytes(),), dtype=torch.uint8, device=dev)
        cm = torch.zeros((_CAP * lib.ob_cm_wgrad_entry_bytes(),), dtype=torch.uint8, device=dev)
        tk = torch.zeros((_TICKETS,), dtype=torch.int32, device=dev)
        t = (dw, ln, cm, tk)
        _S.tables[idx] = t
    return idx, t


def _begin(dev: torch.device, stream: int) -> None:
    if _S.stream is None:
        # the flush stream: the scope's own (home) stream when it is on this device
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        # (compared with the device the home stream was taken on, not the engine thread's)
        home_ok = _S.home is not None and _S.home_dev == idx
        _S.stream = _S.home if home_ok else stream
        _S.dev = idx
    _S.streams.add(stream)
    if not _S.queued:
        torch.autograd.Variable._execution_engine.queue_callback(_flush)
        _S.queued = True


def dw_slot(dev: torch.device, stream: int, n: int = 1):
    """(table pointer, first slot, start block) for n dW finish entries, or None when the
    table is full (finish immediately)."""
    if _S.dw_n + n > _CAP:
        return None
    _begin(dev, stream)
    _, (dw, _, _, _) = _tables(dev)
    return dw.data_ptr(), _S.dw_n, _S.dw_blocks


def dw_done(n: int, blocks: int) -> None:
    if blocks > 0:
        _S.dw_n += n
        _S.dw_blocks += blocks


def ln_slot(dev: torch.device, stream: int, d: int, n: int = 1):
    """(table pointer, first slot) for n LayerNorm parameter entries, or None when the table
    is full; the caller reports the slots with ln_done once the producing launch succeeded."""
    if _S.ln_n + n > _CAP:
        return None
    _begin(dev, stream)
    _, (_, ln, _, _) = _tables(dev)
    return ln.data_ptr(), _S.ln_n


def ln_done(n: int, d: int) -> None:
    _S.ln_n += n
    _S.ln_dmax = max(_S.ln_dmax, d)


def cm_slot(dev: torch.device, stream: int):
    """(table pointer, slot) for one depthwise weight-gradient finish (ob_convmod_bwd_defer),
    or None when the table is full."""
    if _S.cm_n + 1 > _CAP:
        return None
    _begin(dev, stream)
    _, (_, _, cm, _) = _tables(dev)
    return cm.data_ptr(), _S.cm_n


def cm_done(n_out: int) -> None:
    """The slot handed out by cm_slot was taken (n_out = C * (K + 1) outputs)."""
    _S.cm_n += 1
    _S.cm_nmax = max(_S.cm_nmax, n_out)


def dwg_take(dy, x, P, m, n, k, gw, gb, stream, weight, bias, alpha=None, ga=None,
             pass_bits=None, bits=2) -> bool:
    """Queue one weight gradient for the grouped launch at the end of the backward
    (ob_dw_grouped: every queued dW of the backward in ONE persistent launch). A BitLinear's
    when ``alpha`` is given (dW with the STE mask, dalpha at pass_bits[p] -- or ``bits`` -- for
    the rows p*m .. p*m+m-1, db), else a dense linear's (dW, db). False: not taken (the
    parameters cannot be deferred, or the shape is off the grouped kernel): finish here."""
    if not (_DWG and _ON and _S.active):
        return False
    params = (weight, alpha, bias) if alpha is not None else (weight, bias)
    if not can_defer(*params) or not all(p.requires_grad for p in params if p is not None):
        return False  # (a gradient autograd drops would be freed before the launch writes it)
    lib = _lib.load()
    if (not lib.ob_dw_grouped_supported(n, k) or m < 1 or not 1 <= P <= 4
            or dy.data_ptr() % 16 or x.data_ptr() % 16
            or not dy.is_contiguous() or not x.is_contiguous()):
        return False
    # the grouped launch's 32-bit index limits (dwg_plan in csrc/dw.hip rejects the whole
    # table otherwise): such a gemm finishes on the per-layer path instead
    if m * P >= 1 << 30 or m * max(n, k) * 4 >= 1 << 31 or n * k * 4 >= 1 << 31:
        return False
    _begin(dy.device, stream)
    _tables(dy.device)
    _S.dwg.append(DwgGemm(dy.data_ptr(), x.data_ptr(),
                          weight.data_ptr() if alpha is not None else None,
                          _lib.ptr(alpha), _lib.ptr(pass_bits), gw.data_ptr(), _lib.ptr(gb),
                          _lib.ptr(ga), n, k, m, P, 1, bits))
    # the inputs stay allocated until the launch; the outputs are NOT referenced here: an extra
    # reference would make AccumulateGrad install a copy (unwritten) instead of the tensor
    keep(dy, x, pass_bits)
    return True


def dense_dw(g2, x2d, m, n, k, gw, gb, ws, wsb, stream, weight, bias) -> None:
    """ob_dense_dw (full-precision weight gradient on the dW kernels), its finish deferred
    when the parameters qualify; queued for the grouped launch when its shape allows."""
    if dwg_take(g2, x2d, 1, m, n, k, gw, gb, stream, weight, bias):
        return
    lib = _lib.load()
    slot = dw_slot(g2.device, stream) if can_defer(weight, bias) else None
    if slot is not None:
        nb = ctypes.c_int64(0)
        _lib.check(lib.ob_dense_dw_defer(g2.data_ptr(), x2d.data_ptr(), m, n, k, gw.data_ptr(),
                                         _lib.ptr(gb), ws.data_ptr(), wsb, slot[0], slot[1],
                                         slot[2], ctypes.addressof(nb), stream),
                   "ob_dense_dw_defer")
        dw_done(1, nb.value)
        keep(ws)
        return
    _lib.check(lib.ob_dense_dw(g2.data_ptr(), x2d.data_ptr(), m, n, k, gw.data_ptr(),
                               _lib.ptr(gb), ws.data_ptr(), wsb, stream), "ob_dense_dw")


def keep(*tensors) -> None:
    _S.refs.extend(t for t in tensors if t is not None)


def add_grad_after_flush(param: torch.Tensor, src: torch.Tensor) -> None:
    """param.grad += src on the flush stream right after the table launches: a correction to
    a deferred gradient the tables are still to write. Keyed by the parameter, not the
    pending gradient tensor: an extra reference to that tensor would make AccumulateGrad
    copy it (unwritten) instead of adopting it."""
    _S.post.append((param, src))


def _grouped(lib, gemms, tk) -> None:
    """ONE ob_dw_grouped launch of ``gemms`` on the flush stream."""
    n = len(gemms)
    arr = (DwgGemm * n)(*gemms)
    ad = ctypes.addressof(arr)
    wsb = lib.ob_dw_grouped_workspace(ad, n)
    need = lib.ob_dw_grouped_tickets(ad, n)
    if not wsb or need > tk.numel():
        raise _lib.OneBitHipError(f"ob_dw_grouped: {n} gradients do not fit "
                                  f"(workspace {wsb}, tickets {need} > {tk.numel()})")
    ws = torch.empty((wsb,), dtype=torch.uint8, device=tk.device)
    _lib.check(lib.ob_dw_grouped(ad, n, ws.data_ptr(), wsb, tk.data_ptr(), tk.numel(),
                                 _S.stream), "ob_dw_grouped")
    keep(ws)


# The N > 1 deferred exchange's overlap (graph_step._ChunkedExchange; None: one grouped launch,
# the exchange after the backward). When set, the flush runs the finish tables first, hands
# the gradients formed outside the flat buffer to ``copy_in()``, then splits the grouped launch
# into ``chunks`` launches of whole gemms in DESCENDING flat-buffer order and calls
# ``start(lo, hi)`` (element offsets) after each: that bucket is complete, so its all-reduce
# runs on the exchange's stream under the next chunk's weight gradients; ``start(0, rest)``
# covers the buffer's head (no grouped gradient left in it).
_XCHG = None
PLAN_NOTE = ""  # why the latest flush with an exchange set ran one launch (diagnostics)


def set_exchange(x) -> None:
    global _XCHG
    _XCHG = x


def _chunk_plan(x):
    """([(gemms, lo, hi)] in launch order, rest) or None (an output outside the flat buffer:
    no overlap, one launch)."""
    global PLAN_NOTE
    base, n = x.flat.data_ptr(), x.flat.numel()
    items = []
    for g in _S.dwg:
        outs = [(g.dW, g.N * g.K)] + ([(g.db, g.N)] if g.db else []) + \
               ([(g.dalpha, 1)] if g.dalpha else [])
        lo, hi = n, 0
        for ptr, size in outs:
            off = (ptr - base) // 4
            if ptr < base or (ptr - base) % 4 or off + size > n:
                PLAN_NOTE = f"output outside the flat buffer (N {g.N} K {g.K} M {g.M})"
                return None
            lo, hi = min(lo, off), max(hi, off + size)
        items.append((lo, hi, g.M * g.P * g.N * g.K, [g]))
    # gemms whose output ranges overlap (the row halves of one packed weight and its bias,
    # linear.linear_rows_split) are one unit: a chunk boundary never separates them
    items.sort(key=lambda t: t[0])
    units = []
    for t in items:
        if units and t[0] < units[-1][1]:
            lo, hi, w, gs = units[-1]
            units[-1] = (lo, max(hi, t[1]), w + t[2], gs + t[3])
        else:
            units.append(t)
    items = units[::-1]  # descending flat offset: launch order
    k = max(1, min(int(x.chunks), len(items)))
    total = sum(t[2] for t in items)
    chunks, cur, acc = [], [], 0
    for t in items:
        cur.append(t)
        acc += t[2]
        if len(chunks) < k - 1 and acc * k >= total * (len(chunks) + 1):
            chunks.append(cur)
            cur = []
    if cur:
        chunks.append(cur)
    out, upper = [], n
    for ch in chunks:
        lo = min(t[0] for t in ch)
        out.append(([g for t in ch for g in t[3]], lo, upper))
        upper = lo
    return out, upper


def _flush() -> None:
    if _S.stream is None:
        _S.reset()
        return
    # (the final callback runs on the engine's thread, whose current stream is whatever the
    # last node used: allocations and torch ops of the flush belong to the flush stream)
    with torch.cuda.stream(torch.cuda.ExternalStream(_S.stream,
                                                     device=torch.device("cuda", _S.dev))):
        _flush_tables()


_SIDE_TABLES = True  # finish tables beside the grouped launch (tests flip it)
_SIDES: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """One side stream per device for the finish tables (created once: a captured graph keeps
    the stream it forked to)."""
    st = _SIDES.get(dev.index)
    if st is None:
        st = _SIDES[dev.index] = torch.cuda.Stream(device=dev)
    return st


def _flush_tables() -> None:
    lib = _lib.load()
    dw, ln, cm, tk = _S.tables[_S.dev]
    others = sorted(x for x in _S.streams if x != _S.stream)
    if others:  # entries produced on other streams: the flush waits for them (module docstring)
        dev = torch.device("cuda", _S.dev)
        home = torch.cuda.ExternalStream(_S.stream, device=dev)
        for x in others:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(x, device=dev))
            home.wait_event(ev)
        for t in _S.refs:
            if t.is_cuda:
                t.record_stream(home)
    plan = _chunk_plan(_XCHG) if (_XCHG is not None and _S.dwg) else None

    def tables(stream: int) -> None:
        if _S.dw_n:
            _lib.check(lib.ob_dw_finish_table(dw.data_ptr(), _S.dw_n, _S.dw_blocks, stream),
                       "ob_dw_finish_table")
        if _S.ln_n:
            _lib.check(lib.ob_ln_param_table(ln.data_ptr(), _S.ln_n, _S.ln_dmax, stream),
                       "ob_ln_param_table")
        if _S.cm_n:
            _lib.check(lib.ob_cm_wgrad_table(cm.data_ptr(), _S.cm_n, _S.cm_nmax, stream),
                       "ob_cm_wgrad_table")

    if _S.dwg:
        xs = [g.X for g in _S.dwg]  # (q / k / v of one LN output share X)
        LAST_DWG[:] = [(g.N, g.K, g.M, g.P, bool(g.W), xs.index(g.X)) for g in _S.dwg]
    if _S.dwg and plan is None and _SIDE_TABLES and (_S.dw_n or _S.ln_n or _S.cm_n):
        # The finish tables (memory-bound, every input produced before the flush, outputs
        # disjoint from the grouped launch's) on a side stream forked from the flush stream,
        # joined before the post ops: they run beside the MFMA-bound grouped launch instead
        # of after it (a fork / join in the captured step graph).
        dev = torch.device("cuda", _S.dev)
        home = torch.cuda.ExternalStream(_S.stream, device=dev)
        side = _side_stream(dev)
        fork = torch.cuda.Event()
        fork.record(home)
        side.wait_event(fork)
        tables(side.cuda_stream)
        _grouped(lib, _S.dwg, tk)
        join = torch.cuda.Event()
        join.record(side)
        home.wait_event(join)
    else:
        if _S.dwg and plan is None:
            _grouped(lib, _S.dwg, tk)
        tables(_S.stream)
    if _S.post:
        dev = torch.device("cuda", _S.dev)
        with torch.cuda.stream(torch.cuda.ExternalStream(_S.stream, device=dev)):
            for param, src in _S.post:
                param.grad.add_(src)
    if plan is not None:
        # every gradient outside the grouped launch is final here: into the flat buffer, then
        # the grouped weight gradients chunk by chunk, each chunk's bucket all-reduced on the
        # exchange's stream while the next chunk runs (the flat buffer's tail first)
        chunks, rest = plan
        dev = torch.device("cuda", _S.dev)
        with torch.cuda.stream(torch.cuda.ExternalStream(_S.stream, device=dev)):
            _XCHG.copy_in()
            for gemms, lo, hi in chunks:
                _grouped(lib, gemms, tk)
                _XCHG.start(lo, hi)
            if rest > 0:
                _XCHG.start(0, rest)
    _S.reset()
