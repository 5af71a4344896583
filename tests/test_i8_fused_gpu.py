"""int8-activation inference call sites (act_quant="absmax_int8", eval, no autograd):
the fused path -- LayerNorm emitting the per-tensor absmax (ob_layernorm_fwd_amax), lin1 on
the int8 matrix cores with swish and the next absmax in its epilogue, lin2 / out_proj with
the residual (and padded-frame zeroing) in theirs (ob_bitlinear_fwd_i8_epi) -- equals the
unfused module path (separate absmax passes, torch silu / add) bit for bit, and the
absmaxes equal the oracle's max|x|."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_layernorm_amax(gpu):
    from onebit_asr.layernorm import layer_norm, layer_norm_amax

    torch.manual_seed(0)
    for rows, d in [(1, 144), (1000, 144), (3 * 7968, 144), (37, 64)]:
        x = torch.randn(rows, d, device=gpu) * 3
        w, b = torch.randn(d, device=gpu), torch.randn(d, device=gpu)
        y = layer_norm_amax(x, w, b)
        ref = layer_norm(x, w, b)
        assert torch.equal(y, ref)
        assert y._ob_amax.item() == ref.abs().max().item()


@pytest.mark.parametrize("bits", [2, 1])
def test_ffn_i8_fused_equals_unfused(gpu, bits, monkeypatch):
    from onebit_asr.conformer import FeedForwardModule
    from onebit_asr.quant import set_act_quant

    torch.manual_seed(1)
    m = FeedForwardModule(144, 576, 0.1).to(gpu).eval()
    with torch.no_grad():
        for lin in (m.lin1, m.lin2):
            lin.bias.uniform_(-0.1, 0.1)
    set_act_quant(m, "absmax_int8")
    x = torch.randn(4, 249, 144, device=gpu)
    with torch.no_grad():
        monkeypatch.setenv("OB_FUSED", "1")
        y1 = m(x, bits)
        monkeypatch.setenv("OB_FUSED", "0")
        m.ln.emit_amax = False
        y0 = m(x, bits)
        # the fused swish is silu through v_exp / a fast reciprocal (tgemm_i8.hip), torch's
        # is expf + IEEE division: a few ulp apart, so an element of lin2's int8 operand can
        # round one step differently; each such step moves an output by 0.5 * osc (lin2's
        # output scale, a * g / 127) at most
        hid = torch.nn.functional.silu(m.lin1(m.ln(x), bits))
        osc = (m.lin2.alpha.abs() + 1e-8).item() * hid.abs().max().item() / 127.0
    diff = (y1 - y0).abs()
    assert diff.max().item() <= 4 * 0.5 * osc * (1 + 1e-3), (diff.max().item(), osc)
    assert (diff > 0).float().mean().item() < 0.05


def test_mhsa_i8_out_proj_residual(gpu, monkeypatch):
    """linear_residual_i8 with ragged lengths == out_proj (int8) + padded-row zeroing + x."""
    from onebit_asr.fused import linear_residual_i8
    from onebit_asr.quant import QuantizedLinear

    torch.manual_seed(2)
    lin = QuantizedLinear(144, 144, act_quant="absmax_int8").to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    B, T = 3, 50
    lens = torch.tensor([50, 17, 1], dtype=torch.int32, device=gpu)
    ctx = torch.randn(B, T, 144, device=gpu)
    x = torch.randn(B, T, 144, device=gpu)
    with torch.no_grad():
        y = linear_residual_i8(ctx, x, lin, 2, 1.0, lens, T)
        valid = (torch.arange(T, device=gpu)[None, :] < lens[:, None]).float()
        ref = x + lin(ctx, 2) * valid[..., None]
    assert torch.equal(y, ref)


# ---- int8 activations in HBM (ob_layernorm_fwd_i8 / ob_bitlinear_fwd_i8q) ---------------

def _np_quant(y: np.ndarray, amax: float) -> np.ndarray:
    """oracle/quant_oracle.py::np_act_quant_i8 at a given absmax (the producer's)."""
    gam = np.float32(max(np.float32(amax), np.float32(1e-5)))
    sx = np.float32(np.float32(127.0) / gam)
    return np.clip(np.rint((y.astype(np.float32) * sx).astype(np.float32)), -127, 127).astype(np.int8)


@pytest.mark.parametrize("rows,d", [(1, 144), (3 * 7968, 144), (37, 64), (5, 36)])
def test_layernorm_i8_is_quantised_layernorm(gpu, rows, d):
    """The int8 LN == the oracle quantisation of the fp32 LN at its absmax, bit for bit."""
    from onebit_asr.layernorm import layer_norm, layer_norm_i8

    torch.manual_seed(3)
    x = torch.randn(rows, d, device=gpu) * 2 + 0.3
    w, b = torch.randn(d, device=gpu), torch.randn(d, device=gpu)
    h = layer_norm_i8(x, w, b)
    ref = layer_norm(x, w, b)
    assert h.q.dtype == torch.int8 and tuple(h.q.shape) == (rows, d)
    amax = ref.abs().max().item()
    assert h.amax.item() == amax
    assert np.array_equal(h.q.cpu().numpy(), _np_quant(ref.cpu().numpy(), amax))


@pytest.mark.parametrize("K,N", [(144, 576), (576, 144), (144, 144), (64, 256)])
@pytest.mark.parametrize("bits", [2, 1])
def test_i8q_gemm_equals_fp32_operand_path(gpu, K, N, bits):
    """ob_bitlinear_fwd_i8q on the int8 image == ob_bitlinear_fwd_i8(_epi) on the fp32
    operand (mode 0: plain; mode 2: residual; mode 3: int8 swish at its own absmax), and mode
    0 == the oracle's np_bitlinear_fwd_i8."""
    from onebit_asr.fused import _i8_epi, _i8q
    from onebit_asr.quant import QuantizedLinear, act_absmax
    from oracle import quant_oracle as qo

    torch.manual_seed(4)
    M = 1000
    lin = QuantizedLinear(K, N, act_quant="absmax_int8").to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    x = torch.randn(M, K, device=gpu) * 1.5
    amax = act_absmax(x, 1)
    xq = torch.from_numpy(_np_quant(x.cpu().numpy(), amax.item())).to(gpu)
    with torch.no_grad():
        y0, _ = _i8q(xq, amax, lin, bits, 0)
        ref = lin(x, bits)  # module path: fp32 operand quantised in registers
        assert torch.equal(y0, ref)
        W, alpha = lin.weight.cpu().numpy(), float(lin.alpha.item())
        o = qo.np_bitlinear_fwd_i8(x.cpu().numpy(), W, alpha, lin.bias.cpu().numpy(), bits)
        assert np.array_equal(y0.cpu().numpy(), o)
        R = torch.randn(M, N, device=gpu)
        y2, _ = _i8q(xq, amax, lin, bits, 2, R=R, rscale=0.5)
        r2, _ = _i8_epi(x, amax, lin, bits, 2, R=R, rscale=0.5)
        assert torch.equal(y2, r2)
        y3, a3 = _i8q(xq, amax, lin, bits, 3)
        s1, a1 = _i8_epi(x, amax, lin, bits, 1)
        assert a3.item() == a1.item() == s1.abs().max().item()
        assert y3.dtype == torch.int8
        assert np.array_equal(y3.cpu().numpy(), _np_quant(s1.cpu().numpy(), a1.item()))


def test_mhsa_i8_int8_operands_equal_unfused(gpu, monkeypatch):
    """MHSA in the int8 mode: LN as int8, q/k/v on the int8 operand, the fused attention core,
    out_proj + residual == the module path with fp32 operands quantised in registers."""
    from onebit_asr.conformer import MHSA, RelPositionalEncoding
    from onebit_asr.quant import set_act_quant

    torch.manual_seed(5)
    m = MHSA(144, 4, 0.1).to(gpu).eval()
    set_act_quant(m, "absmax_int8")
    x = torch.randn(3, 61, 144, device=gpu)
    _, pos = RelPositionalEncoding(144).to(gpu)(x)
    with torch.no_grad():
        monkeypatch.setenv("OB_FUSED", "1")
        y1 = m(x, None, 2, pos)
        monkeypatch.setenv("OB_FUSED", "0")
        y0 = m(x, None, 2, pos)
    assert torch.equal(y1, y0), (y1 - y0).abs().max().item()


def test_fast_silu_monotone_on_nonnegatives(gpu):
    """The int8 absmax launch (I8_SWISH_AMAX, csrc/tgemm_i8.hip) takes a lane's max|silu| as
    silu(max y): exact only if fast_silu is non-decreasing on y >= 0. Checked here over EVERY
    fp32 in [0, 128] on the device (past 128, exp(-y) is 0 in fp32 and silu(y) = y)."""
    from onebit_asr import _lib

    lib = _lib.load()
    bad = torch.zeros(1, dtype=torch.int32, device=gpu)
    lo, hi = 0, int(np.float32(128.0).view(np.uint32))
    _lib.check(lib.ob_silu_fast_monotone_check(lo, hi, bad.data_ptr(), _lib.stream_of(bad)),
               "ob_silu_fast_monotone_check")
    torch.cuda.synchronize()
    assert bad.item() == 0
    assert lib.ob_silu_fast_monotone_check(hi, lo, bad.data_ptr(), None) == -2


@pytest.mark.parametrize("scale", [1e-4, 0.05])
def test_i8_swish_amax_small_outputs(gpu, scale):
    """Outputs too small for the one-silu-a-lane max (silu(max y) < 0.28, or every y < 0 in a
    lane): the exact fallback gives the same absmax as the every-element epilogue."""
    from onebit_asr.fused import _i8_epi, _i8q
    from onebit_asr.quant import QuantizedLinear, act_absmax

    torch.manual_seed(5)
    M, K, N = 700, 144, 576
    lin = QuantizedLinear(K, N, act_quant="absmax_int8").to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-scale, 0.0)
    x = torch.randn(M, K, device=gpu) * scale
    amax = act_absmax(x, 1)
    xq = torch.from_numpy(_np_quant(x.cpu().numpy(), amax.item())).to(gpu)
    with torch.no_grad():
        y3, a3 = _i8q(xq, amax, lin, 2, 3)
        s1, a1 = _i8_epi(x, amax, lin, 2, 1)
    assert a3.item() == a1.item() == s1.abs().max().item()
    assert np.array_equal(y3.cpu().numpy(), _np_quant(s1.cpu().numpy(), a1.item()))
