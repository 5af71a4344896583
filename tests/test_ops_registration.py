"""CPU: the torch.library registration of the BitLinear boundary (onebit_asr/ops.py) --
every operator exists under torch.ops.onebit and traces with fake tensors (the shapes a
compiler sees), and the real implementation refuses a CPU tensor (no CPU fallback)."""
import pytest
import torch


def test_ops_registered_and_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    import onebit_asr.ops  # noqa: F401  (registers torch.ops.onebit.*)

    for name in ("bitlinear", "pack_codes", "bitlinear_fwd", "bitlinear_dx", "bitlinear_dw"):
        assert hasattr(torch.ops.onebit, name), name
    with FakeTensorMode():
        x = torch.empty(3, 5, 144)
        w = torch.empty(576, 144)
        a = torch.empty(())
        b = torch.empty(576)
        y = torch.ops.onebit.bitlinear(x, w, a, b, 2)
        assert y.shape == (3, 5, 576)
        c, ct = torch.ops.onebit.pack_codes(w, a, 1)
        assert c.shape == (576, 9) and ct.shape == (144, 36) and c.dtype == torch.int32
        gx = torch.ops.onebit.bitlinear_dx(torch.empty(15, 576), ct, a, 144)
        assert gx.shape == (15, 144)
        gw, ga, gb = torch.ops.onebit.bitlinear_dw(torch.empty(15, 576), torch.empty(15, 144),
                                                   w, a, 2, True)
        assert gw.shape == w.shape and ga.shape == () and gb.shape == (576,)


def test_op_refuses_cpu():
    from onebit_asr.ops import bitlinear

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        bitlinear(torch.randn(2, 16), torch.randn(8, 16), torch.tensor(0.1), None, 2)
