"""The optimizer tail of the training step on the HIP library: clip_grad_norm_ + AdamW.

Reference: onebit_asr/train.py:116-118 (``clip_grad_norm_(model.parameters(), 5.0)``,
``optimizer.step()``) with ``AdamW(lr, betas=(0.9, 0.98), weight_decay=1e-2)``
(train.py:259). ``FusedAdamW.step()`` is three launches (``ob_adamw_clip_step``) over a
device table of (param, grad, exp_avg, exp_avg_sq) pointers instead of torch's per-tensor
norm / scale / update kernels for every parameter tensor. lr and the step counter are
device scalars, so a captured step replays with the schedule's current lr
(``WarmupCosine`` fills ``param_groups[0]["lr"]``).

Semantics follow torch: parameters without a gradient are skipped (they are left out of
the table, which is re-planned when the set changes); the global norm covers exactly the
parameters in the table; gradients are clipped in registers (``p.grad`` is not rescaled
in place, unlike ``clip_grad_norm_``). There is no CPU path.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List

import torch

from . import _lib

__all__ = ["FusedAdamW"]


class FusedAdamW:
    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 5e-4,
                 betas=(0.9, 0.98), eps: float = 1e-8, weight_decay: float = 1e-2,
                 max_norm: float = 5.0):
        self.params: List[torch.nn.Parameter] = list(params)
        if not self.params:
            raise ValueError("FusedAdamW got an empty parameter list")
        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedAdamW runs only on a ROCm device (HIP kernels, no CPU fallback)")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise TypeError("FusedAdamW needs contiguous fp32 parameters")
        self.device = dev
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        self.max_norm = float(max_norm)
        self.grad_scale = 1.0
        self.lr = torch.tensor(float(lr), dtype=torch.float32, device=dev)
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.total_norm = torch.zeros((), dtype=torch.float32, device=dev)
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in self.params]
        # torch.optim-like surface for WarmupCosine
        self.param_groups = [{"lr": self.lr, "initial_lr": float(lr), "params": self.params}]
        self._members = None
        self._ptrs = None
        # Pinned staging for the table's H2D copy, allocated here because pinning host
        # memory is not allowed while a stream is being captured. A buffer used during
        # capture is never written again (the graph's copy node re-reads it on replay).
        rows = len(self.params)
        self._ring = [torch.empty((rows, 5), dtype=torch.int64).pin_memory() for _ in range(2)]
        self._ring_ev = [None, None]
        self._rr = 0
        self._capture_bufs = [torch.empty((rows, 5), dtype=torch.int64).pin_memory()
                              for _ in range(2)]
        self._frozen = []

    # ------------------------------------------------------------------ table
    def _plan(self, members):
        lib = _lib.load()
        numels = (ctypes.c_int64 * len(members))(*[self.params[i].numel() for i in members])
        nb = lib.ob_adamw_plan(ctypes.addressof(numels), len(members), None)
        _lib.check(0 if nb > 0 else int(nb), "ob_adamw_plan")
        cmap = (ctypes.c_int64 * (2 * nb))()
        lib.ob_adamw_plan(ctypes.addressof(numels), len(members), ctypes.addressof(cmap))
        self.map = torch.tensor(list(cmap), dtype=torch.int64).to(self.device)
        self.n_blocks = int(nb)
        self.ws_bytes = lib.ob_adamw_workspace(nb)
        self.ws = torch.empty((self.ws_bytes,), dtype=torch.uint8, device=self.device)
        self.table = torch.empty((len(members), 5), dtype=torch.int64, device=self.device)
        self._members = members
        self._ptrs = None

    def _refresh(self):
        members = tuple(i for i, p in enumerate(self.params) if p.grad is not None)
        if not members:
            return False
        if members != self._members:
            self._plan(members)
        ptrs = []
        for i in members:
            p = self.params[i]
            g = p.grad
            if g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
                raise TypeError("FusedAdamW needs contiguous fp32 gradients shaped like the parameter")
            ptrs.append((p.data_ptr(), g.data_ptr(), self.exp_avg[i].data_ptr(),
                         self.exp_avg_sq[i].data_ptr(), p.numel()))
        if ptrs != self._ptrs:
            self._stage(ptrs)
            self._ptrs = ptrs
        return True

    def _stage(self, ptrs):
        n = len(ptrs)
        src = torch.tensor(ptrs, dtype=torch.int64)
        if torch.cuda.is_current_stream_capturing():
            if not self._capture_bufs:
                raise RuntimeError("FusedAdamW: no pinned staging buffer left for capture")
            buf = self._capture_bufs.pop()
            self._frozen.append(buf)
            buf[:n].copy_(src)
            self.table.copy_(buf[:n], non_blocking=True)
            return
        i = self._rr % len(self._ring)
        self._rr += 1
        if self._ring_ev[i] is not None:
            self._ring_ev[i].synchronize()  # its previous copy has been consumed
        buf = self._ring[i]
        buf[:n].copy_(src)
        self.table.copy_(buf[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._ring_ev[i] = ev

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self):
        if not self._refresh():
            return
        lib = _lib.load()
        st = lib.ob_adamw_clip_step(
            self.table.data_ptr(), len(self._members), self.map.data_ptr(), self.n_blocks,
            self.lr.data_ptr(), self.step_t.data_ptr(), self.grad_scale, self.betas[0],
            self.betas[1], self.eps, self.weight_decay, self.max_norm, self.total_norm.data_ptr(),
            self.ws.data_ptr(), self.ws_bytes, torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(st, "ob_adamw_clip_step")
        self.mark_updated()

    def mark_updated(self):
        """Tell autograd the parameters changed in place (the kernel writes them through raw
        pointers): bumps their version counters, which also invalidates version-keyed
        caches such as QuantizedLinear's packed codes."""
        for i in self._members:
            torch.autograd.graph.increment_version(self.params[i])

    @torch.no_grad()
    def reset_state(self):
        """Back to a fresh optimizer (zero moments, step 0) in place: captured graphs keep
        their addresses."""
        for t in self.exp_avg + self.exp_avg_sq:
            t.zero_()
        self.step_t.zero_()
        self.total_norm.zero_()

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()
