"""The training step (reference onebit_asr/train.py:82-120) captured as HIP graphs.

An eager step of the 3-pass Conformer-S body issues ~4000 kernel launches from Python;
at B=32 x 1000 frames the GPU work is short enough that host launch overhead is a large
part of the step. Once nothing in the step synchronises with the host (bitwidths as Python
ints or device values, the HIP CTC with device-side lengths, the decoder's causal hint,
AdamW with a device lr) the whole body is captured once and replayed:

* graph A: zero the flat gradient buffer, the three passes, their losses, backward;
* N > 1: the gradient exchange, bucketed and overlapped with the backward (below);
* clip_grad_norm_(5.0) + AdamW as the three-launch ``FusedAdamW`` (the 1/world average is
  folded into its gradient scale) -- all of it one graph.

Both step bodies capture: the stacked one (``OneBitStep(stacked=True)``) and the
reference's literal three forwards. Nothing inside the captured region may rely on a
captured ``hipMemsetAsync`` (not replayed correctly on this ROCm build, see
onebit_asr/linear.py): torch's bias-gradient reductions are replaced by fixed-order HIP
column sums, and the library zeroes its counters with kernels. ``tests/
test_graph_step_gpu.py`` checks that every replay reproduces the eager gradients.

What changes per step without re-capture:
* the stochastic-precision mask: ``StackedBits.set`` / ``DeviceBits.set`` copies the new
  per-block bitwidths into the device slots the captured BitLinear kernels read;
* the learning rate: ``WarmupCosine`` fills the device lr tensor AdamW reads
  (capturable=True);
* the batch: copied into the captured input tensors (same shapes; a different padded
  shape needs another ``GraphedTrainStep``);
* dropout masks: torch's philox offsets advance per replay.

N > 1 (reference train.py:116-118 is single-device: loss.backward(), clip, step), the
``exchange``:

* ``"deferred"`` (default): the backward runs exactly as at N == 1 -- every weight
  gradient in the grouped launch, the other finishes deferred to one table launch per kind
  at the end (deferred.py) -- but the gradient sites write IN PLACE into their views of one
  flat fp32 buffer (``deferred.grad_buf`` over the ``arena``; autograd adopts the views).
  Only a parameter with a single producing site in the step gets its view (with several --
  the literal three-pass step -- autograd sums the contributions before ``.grad`` exists,
  so each site gets a fresh tensor); the gradients formed elsewhere (that case, and sites
  that do not take a view) are copied into the buffer with one ``foreach`` copy, the buffer
  is all-reduced (SUM), and those gradients are copied back out -- all inside the step
  graph with RCCL. Over RCCL the all-reduce is overlapped (round 6, ``overlap_chunks``,
  ``_ChunkedExchange``): the end-of-backward flush runs the finish tables, copies the
  gradients formed elsewhere into the buffer, then launches the grouped weight gradients in
  ``overlap_chunks`` launches of whole gemms, highest flat offsets first, and all-reduces
  each finished bucket on a communication stream while the next launch runs (the buffer's
  head, which holds no grouped gradient, last). Measured per rank on one GPU (world size 1
  through the test hook below, ``tools/multi_path_bench.py``); the bucketed path's
  on-the-spot finishes cost ~2.3 ms/step more than the exchange they would overlap (47 MB:
  a few hundred us on a ring over xGMI).
* ``"bucketed"``: gradients are views of the flat buffer (parameter order), cut into
  ``bucket_mb`` buckets (default 12 MB: 4 for Conformer-S's 47 MB) of contiguous parameters
  taken in REVERSE order (the backward produces the decoder / CTC-head and last-block
  gradients first). A post-accumulate-grad hook counts each bucket's parameters; when a
  bucket's last gradient has landed its slice is all-reduced on a communication stream
  while the backward goes on (``BucketedAllReduce``); the update waits for it. Deferral
  cannot apply (a hook needs its finished gradient): ~230 more small launches per step.
* ``"flat"``: the gradient views of the flat buffer, one all-reduce after the backward.

With RCCL the whole step (forward, backward, the exchange, update) is captured as one
graph; with gloo (host staging, not capturable) the exchange runs eagerly between graph A
and the update graph. A failed RCCL capture raises: the communicator's state after a broken
capture is not something to build on.

The captured collectives run on a process group of their own (``capture_group``: the same
ranks, a second RCCL communicator connected eagerly, before capture, by
``eager_connect_single_device`` -- no collective). ProcessGroupNCCL's watchdog thread polls
the completion event of every eager collective it is handed, and HIP refuses that query
(hipErrorCapturedEvent, "operation not permitted on an event last recorded in a capturing
stream") once the communicator's stream has joined a capture: an eager collective still on
the watchdog's list when the capture starts (the warm-up steps' exchanges, the barrier)
aborted the process in round 4. The capture group never runs an eager collective, so its
watchdog never holds an event to query; the warm-up and the barrier use the caller's group.
Captured collectives are not handed to the watchdog (torch skips ``workEnqueue`` while the
stream captures). Capture also runs in ``thread_local`` error mode, so no other thread's
call can invalidate it. With N == 1 autograd's own gradient buffers are used as they
are (``p.grad = None`` before backward, so no accumulate kernels). Parameters that receive
no gradient in the step are excluded from the optimizer exactly like the reference (AdamW
skips grad=None).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import deferred
from .optim import FusedAdamW
from .quant import DeviceBits, QuantizedLinear
from .train_step import WarmupCosine

__all__ = ["GraphedTrainStep", "BucketedAllReduce"]


class BucketedAllReduce:
    """SUM all-reduce of a flat gradient buffer in buckets, each started from a
    post-accumulate-grad hook as soon as its last parameter's gradient has landed. ``params``
    are laid out in ``flat`` in order; buckets are contiguous runs of them taken from the end
    (the backward's order). CUDA: the bucket is reduced on ``comm`` after an event on the
    producing stream; ``finish`` makes the current stream wait. CPU (gloo): async works,
    waited in ``finish``."""

    def __init__(self, params, flat: torch.Tensor, pg, bucket_bytes: int, offs=None):
        self.flat = flat
        self.pg = pg
        self.enabled = False
        if offs is None:
            offs = flat_offsets(params)
        off = flat.numel()
        self.buckets = []  # (lo, hi, n_params)
        self.bucket_of = {}
        hi, lo, n = off, off, 0
        for i in range(len(params) - 1, -1, -1):
            p = params[i]
            lo = offs[i]
            self.bucket_of[id(p)] = len(self.buckets)
            n += 1
            if (hi - lo) * 4 >= bucket_bytes or i == 0:
                self.buckets.append((lo, hi, n))
                hi, n = lo, 0
        self.count = [0] * len(self.buckets)
        self.works = []
        self.cuda = flat.is_cuda
        self.comm = torch.cuda.Stream(flat.device) if self.cuda else None
        self.handles = [p.register_post_accumulate_grad_hook(self._hook) for p in params]

    def begin(self):
        self.count = [0] * len(self.buckets)
        self.works = []

    def _hook(self, p):
        if not self.enabled:
            return
        k = self.bucket_of[id(p)]
        self.count[k] += 1
        if self.count[k] == self.buckets[k][2]:
            self._launch(k)

    def _launch(self, k):
        lo, hi, _ = self.buckets[k]
        view = self.flat[lo:hi]
        if self.cuda:
            self.comm.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self.comm):
                dist.all_reduce(view, group=self.pg)
        else:
            self.works.append(dist.all_reduce(view, group=self.pg, async_op=True))

    def finish(self):
        """Every bucket has been started (each parameter's hook fired once); make the
        update wait for the exchange."""
        if any(c != b[2] for c, b in zip(self.count, self.buckets)):
            raise RuntimeError("bucketed all-reduce: a bucket did not complete "
                               f"({self.count} of {[b[2] for b in self.buckets]})")
        if self.cuda:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.comm)
        for w in self.works:
            w.wait()
        self.works = []


class _ChunkedExchange:
    """The deferred exchange overlapped with the grouped weight gradients (deferred.set_exchange,
    RCCL only): the flush splits the grouped dW launch into ``chunks`` launches in descending
    flat-buffer order and starts each finished bucket's SUM all-reduce on ``comm`` while the
    next chunk runs; ``finish`` makes the current stream wait and copies the reduced buffer
    back into the gradients that live outside it."""

    def __init__(self, gs: "GraphedTrainStep", chunks: int):
        self.gs = gs
        self.flat = gs.flat
        self.chunks = chunks
        self.comm = torch.cuda.Stream(gs.device)
        self.out = []
        self.started = False

    def reset(self):
        self.out = []
        self.started = False

    def copy_in(self):
        """The gradients formed outside the flat buffer, into it (one foreach copy)."""
        gs = self.gs
        self.out = [(p.grad, v) for p, v in zip(gs.params, gs.flat_views)
                    if p.grad.data_ptr() != v.data_ptr()]
        if self.out:
            torch._foreach_copy_([v for _, v in self.out], [g for g, _ in self.out])

    def start(self, lo: int, hi: int):
        self.comm.wait_stream(torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(self.comm):
            dist.all_reduce(self.flat[lo:hi], group=self.gs.xpg)
        self.started = True

    def finish(self):
        torch.cuda.current_stream(self.flat.device).wait_stream(self.comm)
        gs = self.gs
        if not gs.fused:
            self.flat.div_(gs.world)
        if self.out:
            torch._foreach_copy_([g for g, _ in self.out], [v for _, v in self.out])
        gs.copied = len(self.out)


def flat_offsets(params, align: int = 4):
    """Element offset of every parameter in the flat gradient buffer: each one starts on a
    16-byte boundary (the HIP kernels that write gradients in place store dwordx4), the gaps
    stay zero."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += -(-p.numel() // align) * align
    return offs


# Test hook: run the multi-rank exchange path (flat buffer, buckets, the all-reduce captured
# into the step graph) at world size 1, so a single-GPU test can capture RCCL collectives
# (tests/test_rccl_capture_gpu.py). Not read from the environment.
_MULTI_RANK_PATH_AT_WORLD_1 = False


_CAPTURE_GROUPS: Dict[tuple, dist.ProcessGroup] = {}


def capture_group(pg: dist.ProcessGroup, device: torch.device) -> dist.ProcessGroup:
    """A second RCCL process group over ``pg``'s ranks for the collectives captured into the
    step graph, its communicator connected now (no collective, so its watchdog never tracks
    an eager event; module docstring). Every rank of ``pg`` calls this in the same order.
    Cached per (group, device): every GraphedTrainStep of a process (one per padded batch
    shape) shares one communicator instead of leaking one each. Only captured collectives
    ever run on it, so sharing it keeps its watchdog free of eager events."""
    key = (id(pg), device.index)
    g = _CAPTURE_GROUPS.get(key)
    if g is not None:
        return g
    ranks = dist.get_process_group_ranks(pg)
    g = dist.new_group(ranks=ranks, backend="nccl", use_local_synchronization=True)
    g._get_backend(device).eager_connect_single_device(device)
    _CAPTURE_GROUPS[key] = g
    return g


class GraphedTrainStep:
    def __init__(self, step_module, n_layers: int, lr: float = 5e-4, warmup_steps: int = 4000,
                 total_steps: int = 100000, max_norm: float = 5.0,
                 process_group: Optional[dist.ProcessGroup] = None, warmup_iters: int = 2,
                 use_graph: bool = True, fused_optimizer: bool = True,
                 bucket_mb: Optional[float] = 12.0, exchange: str = "deferred",
                 overlap_chunks: int = 3):
        if exchange not in ("deferred", "bucketed", "flat"):
            raise ValueError(f"exchange must be 'deferred', 'bucketed' or 'flat', got {exchange!r}")
        self.step_module = step_module
        self.n_layers = n_layers
        self.lr0 = lr
        self.warmup_steps = warmup_steps
        self.total_steps = total_steps
        self.max_norm = max_norm
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if process_group is not None else 1
        # the multi-rank path: flat gradient buffer + the exchange (world > 1, or the test hook)
        self.multi = self.world > 1 or (_MULTI_RANK_PATH_AT_WORLD_1 and process_group is not None)
        self.warmup_iters = warmup_iters
        self.use_graph = use_graph
        self.fused_optimizer = fused_optimizer
        self.device = next(step_module.parameters()).device
        make_bits = getattr(step_module, "make_bits", None)
        self.bits = make_bits(self.device) if make_bits else DeviceBits(n_layers, self.device)
        self.batch: Optional[Dict[str, torch.Tensor]] = None
        self.params: List[torch.nn.Parameter] = []
        self.flat: Optional[torch.Tensor] = None
        self.opt = None
        self.fused = False
        self.sched = None
        self.graph_a = self.graph_b = None
        self.loss = self.parts = None
        self.steps_done = 0
        self.exchange = exchange
        self.bucket_bytes = int(bucket_mb * 2**20) if (bucket_mb and exchange == "bucketed") else 0
        self.flat_views: List[torch.Tensor] = []
        self.arena = None  # [(param, flat, offset)]: the deferred exchange's in-place gradients
        self.copied = 0    # gradients the deferred exchange copies in and out (last exchange)
        self.buckets: Optional[BucketedAllReduce] = None
        self.comm_in_graph = False
        self.xpg = process_group  # the group the exchange's collectives run on
        # deferred exchange over RCCL: the grouped dW in this many launches, each finished
        # bucket all-reduced under the next (_ChunkedExchange); 1 = one launch, then exchange
        self.overlap_chunks = overlap_chunks
        self.xchg: Optional[_ChunkedExchange] = None

    # ------------------------------------------------------------------ setup
    def _set_batch(self, batch):
        if self.batch is None:
            self.batch = {k: v.clone() for k, v in batch.items()}
            return
        for k, v in batch.items():
            dst = self.batch[k]
            if dst.shape != v.shape:
                raise ValueError(f"batch[{k!r}] shape {tuple(v.shape)} != captured {tuple(dst.shape)}")
            if dst.data_ptr() != v.data_ptr():
                dst.copy_(v, non_blocking=True)

    def _discover_params(self):
        """One forward+backward (no update) to find the parameters the step differentiates."""
        for p in self.step_module.parameters():
            p.grad = None
        with deferred.scope():
            loss, _ = self.step_module(self.batch, self.bits)
            loss.backward()
        self.params = [p for p in self.step_module.parameters() if p.grad is not None]
        for p in self.step_module.parameters():
            p.grad = None
        if self.multi:
            # one flat gradient buffer: the exchange's all-reduce(s) run on it
            offs = flat_offsets(self.params)
            last = self.params[-1].numel() if self.params else 0
            total = (offs[-1] + -(-last // 4) * 4) if self.params else 0
            self.flat = torch.zeros(total, dtype=torch.float32, device=self.device)
            for p, off in zip(self.params, offs):
                self.flat_views.append(self.flat[off:off + p.numel()].view_as(p))
            if self.exchange != "deferred":  # the gradients ARE the flat buffer's views
                for p, v in zip(self.params, self.flat_views):
                    p.grad = v
            elif self.device.type == "cuda":
                # the backward's gradient sites write into the flat buffer's views
                # (deferred.grad_buf): only the gradients formed elsewhere are copied in
                self.arena = [(p, self.flat, off) for p, off in zip(self.params, offs)]
                if (self.overlap_chunks > 1 and self.pg is not None
                        and dist.get_backend(self.pg) == dist.Backend.NCCL):
                    self.xchg = _ChunkedExchange(self, self.overlap_chunks)
            if self.bucket_bytes:
                self.buckets = BucketedAllReduce(self.params, self.flat, self.pg, self.bucket_bytes,
                                                 offs)
        if self.device.type == "cuda" and self.fused_optimizer:
            self.fused = True
            self.opt = FusedAdamW(self.params, lr=self.lr0, betas=(0.9, 0.98), eps=1e-8,
                                  weight_decay=1e-2, max_norm=self.max_norm)
            self.opt.grad_scale = 1.0 / self.world
        else:  # torch AdamW + clip (host path of the gloo tests; A/B checks on the GPU)
            self.fused = False
            cap = self.device.type == "cuda"
            lr = torch.tensor(self.lr0, dtype=torch.float32, device=self.device) if cap else self.lr0
            self.opt = torch.optim.AdamW(self.params, lr=lr, betas=(0.9, 0.98),
                                         weight_decay=1e-2, foreach=True, capturable=cap)
            if not self.multi and cap:  # N == 1 torch path needs stable grads for capture
                total = sum(p.numel() for p in self.params)
                self.flat = torch.zeros(total, dtype=torch.float32, device=self.device)
                off = 0
                for p in self.params:
                    n = p.numel()
                    p.grad = self.flat[off:off + n].view_as(p)
                    off += n
        self.sched = WarmupCosine(self.opt, self.warmup_steps, self.total_steps)

    def _fwd_bwd(self, overlap: bool = False):
        """Forward + backward; ``overlap``: the buckets' all-reduces start from the backward
        (finished by ``_allreduce``)."""
        if self.flat is not None and (not self.multi or self.exchange != "deferred"):
            self.flat.zero_()
        else:  # autograd hands its gradient buffers over (no accumulate kernels)
            for p in self.params:
                p.grad = None
        if self.buckets is not None:
            self.buckets.begin()
            self.buckets.enabled = overlap
        deferred.set_arena(self.arena)
        if self.xchg is not None:
            self.xchg.reset()
            deferred.set_exchange(self.xchg)
        try:
            with deferred.scope():  # one finish launch per kind at the end of the backward
                loss, parts = self.step_module(self.batch, self.bits)
                loss.backward()
        finally:
            deferred.set_arena(None)
            deferred.set_exchange(None)
            if self.buckets is not None:
                self.buckets.enabled = False
        return loss.detach(), parts

    def _update(self):
        if self.fused:  # clip + AdamW in three launches (grad_scale = 1/world)
            self.opt.step()
            return
        if self.multi and self.exchange != "deferred":
            self.flat.div_(self.world)
        torch.nn.utils.clip_grad_norm_(self.params, max_norm=self.max_norm, foreach=True)
        self.opt.step()

    def _allreduce(self, overlapped: bool = False):
        if not self.multi:
            return
        if self.exchange == "deferred" and self.xchg is not None and self.xchg.started:
            self.xchg.finish()  # the buckets were reduced under the grouped dW chunks
        elif self.exchange == "deferred":
            # the gradients the backward wrote into the flat buffer (deferred.grad_buf) are in
            # place; the rest are copied in (one foreach copy), one all-reduce, and copied back
            # out; the non-fused update takes the average here (the fused one scales by 1/world)
            out = [(p.grad, v) for p, v in zip(self.params, self.flat_views)
                   if p.grad.data_ptr() != v.data_ptr()]
            self.copied = len(out)
            if out:
                torch._foreach_copy_([v for _, v in out], [g for g, _ in out])
            dist.all_reduce(self.flat, group=self.xpg)
            if not self.fused:
                self.flat.div_(self.world)
            if out:
                torch._foreach_copy_([g for g, _ in out], [v for _, v in out])
        elif overlapped:
            self.buckets.finish()
        else:
            dist.all_reduce(self.flat, group=self.xpg)

    def _eager(self):
        ov = self.buckets is not None
        loss, parts = self._fwd_bwd(overlap=ov)
        self._allreduce(overlapped=ov)
        self._update()
        return loss, parts

    def _warm(self):
        for _ in range(self.warmup_iters):
            self.loss, self.parts = self._eager()

    def _rng_snapshot(self):
        from .fused import rng_snapshot

        cuda = self.device.type == "cuda"
        return (rng_snapshot(self.device),
                torch.cuda.get_rng_state(self.device) if cuda else torch.get_rng_state())

    def _snapshot(self, rng):
        return [p.detach().clone() for p in self.params], rng

    @torch.no_grad()
    def _restore(self, snap):
        """Undo the warm-up: parameters back to their values, optimizer state and schedule
        back to a fresh start (AdamW's state starts at zero with step 0), so that the
        first ``step()`` performs exactly one update (train.py:114-120); the dropout
        streams (the fused call sites' hash counter and host offsets, torch's generator)
        back to where they were, so the first real step draws the masks an un-warmed run
        would. In-place writes keep every address the captured graph will use and bump the
        parameters' versions (which invalidates version-keyed code caches)."""
        from .fused import rng_restore

        params, (rng, torch_rng) = snap
        for p, s in zip(self.params, params):
            p.copy_(s)
        rng_restore(self.device, rng)
        if self.device.type == "cuda":
            torch.cuda.set_rng_state(torch_rng, self.device)
        else:
            torch.set_rng_state(torch_rng)
        if self.fused:
            self.opt.reset_state()
        else:
            for st in self.opt.state.values():
                for v in st.values():
                    if isinstance(v, torch.Tensor):
                        v.zero_()
        self.sched.reset()

    @staticmethod
    def _drop_code_caches(module):
        for m in module.modules():
            if isinstance(m, QuantizedLinear):
                m._codes_cache = {}

    def prime(self, batch, sp_mask):
        """Static inputs, flat grads, optimizer; ``warmup_iters`` eager steps on a side stream
        (library heuristics, allocator) whose effects are then undone; then capture. The
        warm-up leaves no trace: the model, optimizer, schedule and dropout streams are
        restored."""
        self._set_batch(batch)
        self.bits.set(sp_mask)
        if self.device.type != "cuda":  # host path (gloo tests of the exchange logic)
            self.use_graph = False
            self._discover_params()
            return
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            rng = self._rng_snapshot()  # before the discovery pass draws any mask
            self._discover_params()
            snap = self._snapshot(rng)
            self._warm()
            self._restore(snap)
        torch.cuda.current_stream(self.device).wait_stream(side)
        if not self.use_graph:
            return
        torch.cuda.synchronize(self.device)
        self._drop_code_caches(self.step_module)
        pool = torch.cuda.graph_pool_handle()
        if self.multi and dist.get_backend(self.pg) == dist.Backend.NCCL:
            # the whole step in one graph with its exchange (bucketed: the all-reduces overlap
            # the backward); RCCL collectives capture into a graph, gloo's host staging does not
            # the captured collectives go to a group that has never run an eager one (module
            # docstring: its watchdog holds no event HIP would refuse to query mid-capture)
            self.xpg = capture_group(self.pg, self.device)
            if self.buckets is not None:
                self.buckets.pg = self.xpg
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.pg, device_ids=[self.device.index])
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            ov = self.buckets is not None
            try:
                with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                    self.loss, self.parts = self._fwd_bwd(overlap=ov)
                    self._allreduce(overlapped=ov)
                    self._update()
            except Exception as e:
                raise RuntimeError("capturing the step with its RCCL exchange failed; the "
                                   "communicator is not reused after a broken capture") from e
            self.graph_a, self.comm_in_graph = g, True
        else:
            self.xpg = self.pg
        if not self.comm_in_graph:
            self.graph_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_a, pool=pool):
                self.loss, self.parts = self._fwd_bwd()
                if not self.multi:
                    self._update()
            if self.multi:
                self.graph_b = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_b, pool=pool):
                    self._update()
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ step
    def step(self, batch, sp_mask):
        """One training step (train.py:82-120): exactly one optimizer update per call.
        Returns device (loss, parts); no host sync. The first call also primes and
        captures."""
        if self.opt is None:
            self.prime(batch, sp_mask)
        else:
            self._set_batch(batch)
            self.bits.set(sp_mask)
        if self.graph_a is None:
            self.loss, self.parts = self._eager()
        else:
            self.graph_a.replay()
            if self.multi and not self.comm_in_graph:
                self._allreduce()
                self.graph_b.replay()
            if self.fused:  # the replayed update wrote the parameters in place
                self.opt.mark_updated()
        self.sched.step()
        self.steps_done += 1
        return self.loss, self.parts
