"""Decoder embedding backward (ob_embedding_bwd) against torch's nn.Embedding backward on
the CPU (padding_idx row zero, repeated tokens summed in index order): max|err| <=
1e-6 * max|ref|; deterministic."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,v,c,pad", [(3936, 5004, 144, 0), (10, 7, 3, None), (0, 5, 4, 0),
                                       (500, 40, 1024, 3)])
def test_embedding_bwd_matches_torch(gpu, n, v, c, pad):
    from onebit_asr.embedding import embedding

    g = torch.Generator().manual_seed(n + v)
    idx = torch.randint(0, v, (n,), generator=g)
    if n:
        idx[::7] = 0 if pad is None else pad
    w = torch.randn(v, c, generator=g)
    gout = torch.randn(n, c, generator=g)
    wr = w.clone().requires_grad_()
    torch.nn.functional.embedding(idx, wr, pad).backward(gout)
    wd = w.to(gpu).requires_grad_()
    out = embedding(idx.to(gpu), wd, pad)
    assert torch.equal(out.detach().cpu(), torch.nn.functional.embedding(idx, w, pad))
    out.backward(gout.to(gpu))
    err = (wd.grad.cpu() - wr.grad).abs().max().item() if n else wd.grad.abs().max().item()
    assert err <= 1e-6 * max(wr.grad.abs().max().item(), 1.0)
    g1 = wd.grad.clone()
    wd.grad = None
    embedding(idx.to(gpu), wd, pad).backward(gout.to(gpu))
    assert torch.equal(g1, wd.grad)
