"""Deferred gradient finishes (onebit_asr/deferred.py) where something reads a gradient before
the end-of-backward flush:

* DistributedDataParallel: the reducer's hooks copy each gradient into its bucket right after
  AccumulateGrad. ``train_step`` therefore disables deferral for a DDP-wrapped step module;
  one eager step under DDP (gloo, world size 1, the gradients as bucket views) must update
  every parameter exactly like the plain step with deferral on.
* A LayerNorm pair (ob_layernorm_bwd_pair) whose first LN's output has a second consumer:
  the first LN's backward is completed with the LN backward of that consumer's gradient
  (its dgamma / dbeta after the deferred tables ran) and every gradient matches the
  unpaired launches.
Reference: onebit_asr/train.py:114-118 (backward, clip, step), conformer.py:19-24.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("grouped", [False, True])
def test_ddp_step_equals_plain_step(gpu, tmp_path, grouped, monkeypatch):
    """grouped: the plain step's weight gradients from the grouped stream-K dW launch
    (deferred._DWG, the default), whose fixed row partition sums in another order than the
    per-layer split-M kernel DDP's on-the-spot finishes use. Then the gradients agree to 1e-5
    of their max (the updated parameters are not compared: AdamW's first step divides by
    |g| + eps and turns a last-bit difference of a near-zero gradient into an lr-sized one).
    With the per-layer kernel on both sides the updated parameters agree to 1e-6."""
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from onebit_asr import deferred

    monkeypatch.setattr(deferred, "_DWG", grouped)
    bar = 1e-5 if grouped else 1e-6

    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep, make_optimizer, train_step

    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    init = f"file://{tmp_path / 'store'}"
    dist.init_process_group("gloo", init_method=init, rank=0, world_size=1)
    try:
        out = {}
        for wrap in (False, True):
            torch.manual_seed(0)
            m = ConformerASR(80, 5004, **cfg).to(gpu)
            step = OneBitStep(m, n_layers=2, stacked=True)
            if wrap:
                step = DDP(step, device_ids=[gpu.index or 0], broadcast_buffers=False,
                           gradient_as_bucket_view=True)
            opt = make_optimizer(m.parameters())
            loss, _ = train_step(step, opt, None, batch, [1, 0])
            torch.cuda.synchronize()
            src = ({k: p.grad.detach().clone() for k, p in m.named_parameters()
                    if p.grad is not None} if grouped else
                   {k: p.detach().clone() for k, p in m.named_parameters()})
            out[wrap] = (loss.item(), src)
    finally:
        dist.destroy_process_group()
    assert out[False][0] == out[True][0]
    assert out[False][1].keys() == out[True][1].keys()
    for k, p in out[False][1].items():
        q = out[True][1][k]
        assert torch.isfinite(q).all(), k
        assert (p - q).abs().max().item() <= bar * p.abs().max().item() + 1e-9, k


@pytest.mark.parametrize("other_scale", [1.0, 1e-4])
def test_layernorm_pair_with_second_consumer(gpu, monkeypatch, other_scale):
    """The pair's first output with a consumer besides the next LN (layernorm._pair_correction):
    every gradient within 1e-5 of the unpaired path's max -- also when the other consumer's
    gradient is 1e-4 of the pair's (the correction's subtraction resolves it only to the
    rounding of the total, which is what the bar is relative to)."""
    from onebit_asr import deferred, layernorm

    d, rows = 144, 333
    g = torch.Generator().manual_seed(5)
    x = torch.randn(rows, d, generator=g).to(gpu)
    gy2, gres, gy1 = (torch.randn(rows, d, generator=g).to(gpu) for _ in range(3))
    gy1 = gy1 * other_scale
    params = [torch.nn.Parameter((1 + 0.1 * torch.randn(d, generator=g)).to(gpu))
              for _ in range(4)]
    w1, b1, w2, b2 = params
    res = {}
    for on in (False, True):
        monkeypatch.setattr(layernorm, "_PAIR", on)
        for p in params:
            p.grad = None
        xi = x.clone().requires_grad_()
        with deferred.scope():
            y1 = layernorm.layer_norm_pair(xi, w1, b1, 1e-5, w2, b2, 1e-5)
            y2, r = layernorm.layer_norm_fork(y1, w2, b2, 1e-5)
            # y1's second consumer (besides the fork's LN and residual)
            loss = (y2 * gy2).sum() + (r * gres).sum() + (y1 * gy1).sum()
            loss.backward()
        torch.cuda.synchronize()
        res[on] = [xi.grad.clone()] + [p.grad.clone() for p in params]
    for a, b in zip(res[True], res[False]):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item(), (a - b).abs().max()
