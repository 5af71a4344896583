"""The stacked three-pass step (OneBitStep(stacked=True)) against the reference's literal
three forwards (stacked=False) on cfg1, dropout 0: same loss and loss parts (rel <= 1e-5,
parts atol 2e-6 for the small KL parts),
same gradients for every parameter (max|err| <= 2e-4 * max|g| + 1e-7, scalar alpha
gradients 1e-3; only the order in which the passes' contributions are summed differs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# parameters whose gradient is mathematically zero (softmax shift / BatchNorm follows):
# what the two step forms produce there is rounding noise of different summation orders
NOISE_ONLY = ("k_proj.bias", "conv.dw.bias", "in_proj_bias")


def _model(gpu):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1

    torch.manual_seed(0)
    return ConformerASR(80, 5004, **CFG1).to(gpu)


@pytest.mark.parametrize("sp_mask", [[1, 0], [0, 1], [1, 1]])
def test_stacked_equals_literal(gpu, sp_mask):
    from onebit_asr.data import synthetic_batch
    from onebit_asr.train_step import OneBitStep

    batch = synthetic_batch([734, 349], [27, 12], seed=0, device=gpu)
    res = {}
    for stacked in (False, True):
        m = _model(gpu)
        loss, parts = OneBitStep(m, n_layers=2, stacked=stacked)(batch, sp_mask)
        loss.backward()
        res[stacked] = (loss.item(), parts.cpu(), {k: p.grad.detach().cpu() for k, p in m.named_parameters()
                                                  if p.grad is not None})
    (l0, p0, g0), (l1, p1, g1) = res[False], res[True]
    assert abs(l1 - l0) <= 1e-5 * abs(l0), (l1, l0)
    # atol: a KL part (~0.04 here) carries the fp32 rounding of log-probabilities of size
    # log V ~ 8.5 (ulp 9.5e-7) in torch's literal form; the stacked kernel rounds O(1)
    # differences instead (csrc/seqloss.hip), so the two differ by up to ~1e-6 (seen 7.5e-7)
    torch.testing.assert_close(p1, p0, rtol=1e-5, atol=2e-6)
    assert g0.keys() == g1.keys()
    scale = max(g.abs().max().item() for g in g0.values())
    for k in g0:
        err = (g1[k] - g0[k]).abs().max().item()
        if any(n in k for n in NOISE_ONLY):  # exact gradient 0: rounding noise only
            assert err <= 1e-6 * scale, (k, err)
            continue
        # scalar alpha gradients are cancellation-prone sums over N*K products
        rel = 1e-3 if k.endswith(".alpha") else 2e-4
        assert err <= rel * g0[k].abs().max().item() + 1e-7, (k, err)


def test_stacked_graph_step_runs(gpu):
    """GraphedTrainStep over the stacked step captures and replays with changing masks."""
    from onebit_asr.data import synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.quant import StackedBits
    from onebit_asr.train_step import OneBitStep

    m = _model(gpu)
    gs = GraphedTrainStep(OneBitStep(m, n_layers=2), n_layers=2, warmup_iters=1)
    assert isinstance(gs.bits, StackedBits)
    batch = synthetic_batch([734, 349], [27, 12], seed=0, device=gpu)
    losses = [gs.step(batch, mk)[0].item() for mk in ([1, 0], [0, 1], [1, 1], [0, 0])]
    assert gs.graph_a is not None
    assert all(torch.isfinite(torch.tensor(losses)))


def test_deferred_finishes_equal_immediate(gpu, monkeypatch):
    """Inside deferred.scope() every BitLinear dW finish and LayerNorm parameter reduction of
    the stacked step runs as one table launch per kind at the end of the backward: every
    gradient is bit-identical to finishing each layer on the spot (OB_DEFER=0), and the
    tables were actually used (the launch count drops)."""
    from onebit_asr import deferred
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    # d_model 144 / d_ff 576 (Conformer-S widths: the dW shapes that take the LDS path),
    # two blocks, short utterances
    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    res = {}
    used = {}
    monkeypatch.setattr(deferred, "_DWG", False)  # the per-layer dW GEMMs, finishes deferred
    for on in (False, True):
        monkeypatch.setattr(deferred, "_ON", on)
        torch.manual_seed(0)
        m = ConformerASR(80, 5004, **cfg).to(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True)
        counts = []

        def spy(orig=deferred._flush, counts=counts):
            counts.append((deferred._S.dw_n, deferred._S.ln_n))
            orig()

        monkeypatch.setattr(deferred, "_flush", spy)
        with deferred.scope():
            loss, _ = step(batch, [1, 0])
            loss.backward()
        torch.cuda.synchronize()
        used[on] = max((c for c in counts), default=(0, 0))
        res[on] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    assert used[False] == (0, 0)
    assert used[True][0] >= 2 * 9 and used[True][1] >= 2 * 5, used[True]
    assert res[False].keys() == res[True].keys()
    for k in res[False]:
        assert torch.equal(res[False][k], res[True][k]), k


def test_layernorm_pairs_equal_single_launches(gpu, monkeypatch):
    """A block's final LN and the next LN (next block's ff1.ln, the encoder's ln_out) formed
    in one launch (ob_layernorm_fwd_pair) == every LN its own launch: loss and every gradient
    of the stacked step bit for bit, and the pair path was taken."""
    from onebit_asr import layernorm
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    from onebit_asr import fused

    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    res, losses, taken = {}, {}, {}
    # (the FFN epilogue would form these LNs too: left to the pair / single launches here)
    monkeypatch.setattr(fused, "_LN_EPI", False)
    for on in (False, True):
        monkeypatch.setattr(layernorm, "_PAIR", on)
        calls = []
        orig = layernorm._take_pre

        def spy(*a, orig=orig, calls=calls):
            r = orig(*a)
            calls.append(r is not None)
            return r

        monkeypatch.setattr(layernorm, "_take_pre", spy)
        torch.manual_seed(0)
        m = ConformerASR(80, 5004, **cfg).to(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True)
        loss, _ = step(batch, [1, 0])
        loss.backward()
        torch.cuda.synchronize()
        losses[on] = loss.detach().clone()
        taken[on] = sum(calls)
        res[on] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    assert taken[False] == 0 and taken[True] >= 2, taken
    assert torch.equal(losses[False], losses[True])
    assert res[False].keys() == res[True].keys()
    for k in res[False]:
        assert torch.equal(res[False][k], res[True][k]), k


def test_ffn_layernorm_epilogue_equals_separate(gpu, monkeypatch):
    """The LayerNorms after each FFN (ff1 -> mhsa.ln; ff2 -> the block's final LN and the next
    LN) formed in the FFN's second-GEMM epilogue (ob_bitlinear_fwd_residual_ln) == their own
    launches (ob_layernorm_fwd / ob_layernorm_fwd_pair): loss and every gradient of the
    stacked step bit for bit, and both epilogue forms (one LN, two LNs) were taken."""
    from onebit_asr import fused, layernorm
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    res, losses, taken = {}, {}, {}
    for on in (False, True):
        monkeypatch.setattr(fused, "_LN_EPI", on)
        calls = {"pre": 0, "pre2": 0}

        def spy(*a, orig=layernorm._take_pre, calls=calls):
            r = orig(*a)
            calls["pre"] += int(r is not None and len(r) == 3)  # (not a pair launch's)
            return r

        def spy2(*a, orig=layernorm._take_pre2, calls=calls):
            r = orig(*a)
            calls["pre2"] += int(r is not None)
            return r

        monkeypatch.setattr(layernorm, "_take_pre", spy)
        monkeypatch.setattr(layernorm, "_take_pre2", spy2)
        torch.manual_seed(0)
        m = ConformerASR(80, 5004, **cfg).to(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True)
        loss, _ = step(batch, [1, 0])
        loss.backward()
        torch.cuda.synchronize()
        losses[on] = loss.detach().clone()
        taken[on] = dict(calls)
        res[on] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    n_blocks = len(m.encoder.blocks)
    assert taken[False] == {"pre": 0, "pre2": 0}, taken
    # every block: mhsa.ln from ff1, the final LN from ff2 (+ its pair partner)
    assert taken[True]["pre"] >= 2 * n_blocks and taken[True]["pre2"] >= n_blocks, taken
    assert torch.equal(losses[False], losses[True])
    assert res[False].keys() == res[True].keys()
    for k in res[False]:
        assert torch.equal(res[False][k], res[True][k]), k


def test_layernorm_pair_backward_matches_separate(gpu, monkeypatch):
    """The pair's two LN backwards in one launch (ob_layernorm_bwd_pair) vs one launch each:
    every gradient of the stacked step within 1e-6 of max (the kernels' row arithmetic is the
    same; hipcc may contract it differently), loss identical (the forward is unchanged)."""
    from onebit_asr import layernorm
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    res, losses, used = {}, {}, {}
    for on in (False, True):
        monkeypatch.setattr(layernorm, "_PAIR_BWD", on)
        calls = []
        orig = layernorm._pair_backward

        def spy(*a, orig=orig, calls=calls):
            calls.append(1)
            return orig(*a)

        monkeypatch.setattr(layernorm, "_pair_backward", spy)
        torch.manual_seed(0)
        m = ConformerASR(80, 5004, **cfg).to(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True)
        loss, _ = step(batch, [1, 0])
        loss.backward()
        torch.cuda.synchronize()
        losses[on] = loss.detach().clone()
        used[on] = len(calls)
        res[on] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    assert used[False] == 0 and used[True] >= 1, used
    assert torch.equal(losses[False], losses[True])
    assert res[False].keys() == res[True].keys()
    exact = 0
    for k in res[False]:
        a, b = res[True][k], res[False][k]
        exact += int(torch.equal(a, b))
        assert (a - b).abs().max().item() <= 1e-6 * b.abs().max().item() + 1e-12, k
    print(f"bit-identical gradients: {exact} / {len(res[False])}")


def test_grouped_dw_matches_immediate(gpu, monkeypatch):
    """With the grouped launch (deferred._DWG, ob_dw_grouped) every qualifying weight gradient
    of the stacked step -- the BitLinears and the 144-multiple dense linears -- is computed by
    one launch at the end of the backward: the same products as the per-layer dW kernels in
    another summation order, so every gradient equals the on-the-spot path within 2e-6 of
    its max (alpha: 1e-4, biases 1e-5), the loss is identical, and the grouped launch took the gradients."""
    from onebit_asr import deferred
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    cfg = dict(CFG1, enc_d_model=144, enc_d_ff=576)
    batch = synthetic_batch([400, 233], [17, 9], seed=0, device=gpu)
    res, losses, taken = {}, {}, {}
    for on in (False, True):
        monkeypatch.setattr(deferred, "_ON", on)
        torch.manual_seed(0)
        m = ConformerASR(80, 5004, **cfg).to(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True)
        counts = []

        def spy(orig=deferred._flush, counts=counts):
            counts.append(len(deferred._S.dwg))
            orig()

        monkeypatch.setattr(deferred, "_flush", spy)
        with deferred.scope():
            loss, _ = step(batch, [1, 1])
            loss.backward()
        torch.cuda.synchronize()
        taken[on] = max(counts, default=0)
        losses[on] = loss.detach().clone()
        res[on] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    assert taken[False] == 0 and taken[True] >= 2 * 9, taken
    assert torch.equal(losses[False], losses[True])
    assert res[False].keys() == res[True].keys()
    scale = max(g.abs().max().item() for g in res[False].values())
    for k in res[False]:
        a, b = res[True][k], res[False][k]
        if any(n in k for n in NOISE_ONLY):  # exact gradient 0: rounding noise only
            assert (a - b).abs().max().item() <= 1e-6 * scale, k
            continue
        # alpha and bias gradients are cancellation-prone sums (over N*K products / rows)
        bar = 1e-4 if k.endswith(".alpha") else 1e-5 if k.endswith("bias") else 2e-6
        assert (a - b).abs().max().item() <= bar * b.abs().max().item() + 1e-12, k


@pytest.mark.parametrize("graphed", [False, True])
def test_branch_streams_equal_single_stream(gpu, graphed):
    """OneBitStep(branch_streams=True), opt-in: the decoder branch on a side stream beside
    the CTC branch (forward and backward), deferred finishes joined across the two streams.
    Same kernels, same per-node arithmetic: the loss, its parts and every gradient equal the
    single-stream step bit for bit, eagerly (with the deferred finishes) and as the captured
    graph replayed twice (the fork / join as graph edges)."""
    from onebit_asr import deferred
    from onebit_asr.data import synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep

    batch = synthetic_batch([734, 349], [27, 12], seed=3, device=gpu)
    res = {}
    for branch in (False, True):
        m = _model(gpu)
        step = OneBitStep(m, n_layers=2, stacked=True, branch_streams=branch)
        if graphed:
            gs = GraphedTrainStep(step, 2, warmup_iters=1)
            outs = [gs.step(batch, [1, 0]) for _ in range(2)]
            torch.cuda.synchronize()
            res[branch] = ([(lo.item(), pa.cpu()) for lo, pa in outs],
                           {k: p.detach().cpu().clone() for k, p in m.named_parameters()})
        else:
            with deferred.scope():
                loss, parts = step(batch, [1, 0])
                loss.backward()
            torch.cuda.synchronize()
            res[branch] = ([(loss.item(), parts.cpu())],
                           {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()
                            if p.grad is not None})
    (o0, t0), (o1, t1) = res[False], res[True]
    for (l0, p0), (l1, p1) in zip(o0, o1):
        assert l0 == l1 and torch.equal(p0, p1)
    assert t0.keys() == t1.keys()
    for k in t0:
        assert torch.equal(t0[k], t1[k]), k
