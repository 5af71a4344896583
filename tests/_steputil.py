"""Helpers shared by the GPU step tests: one forward+backward of the training step
(``OneBitStep``), eager or captured in a HIP graph and replayed, with every gradient."""
import torch


def build(cfg: dict, device, dropout: float = 0.0, seed: int = 1234):
    from onebit_asr.conformer import ConformerASR

    cfg = dict(cfg)
    cfg.update(enc_dropout=dropout, dec_dropout=dropout)
    torch.manual_seed(seed)
    return ConformerASR(80, 5004, **cfg).to(device)


def grads(model):
    return {k: (p.grad.detach().clone() if p.grad is not None else None)
            for k, p in model.named_parameters()}


def rel_errors(a: dict, b: dict):
    """{name: rel-L2 of a vs b} for every parameter with a gradient on both sides; a
    parameter with a gradient on one side only is an error (inf)."""
    out = {}
    for k in b:
        x, y = a.get(k), b[k]
        if x is None and y is None:
            continue
        if x is None or y is None:
            out[k] = float("inf")
            continue
        d = (x.double() - y.double()).norm().item()
        n = y.double().norm().item()
        if not torch.isfinite(x).all():
            out[k] = float("inf")
        elif n == 0.0:
            out[k] = 0.0 if d == 0.0 else float("inf")
        else:
            out[k] = d / n
    return out


class StepRunner:
    """fwd+bwd of ``OneBitStep`` on a fixed batch / SP mask, no optimizer."""

    def __init__(self, model, n_layers, batch, sp_mask, stacked):
        from onebit_asr.train_step import OneBitStep

        self.model = model
        self.step = OneBitStep(model, n_layers=n_layers, stacked=stacked)
        self.batch = batch
        self.bits = self.step.make_bits(batch["feats"].device)
        self.bits.set(sp_mask)
        self.graph = None

    def fwd_bwd(self):
        for p in self.model.parameters():
            p.grad = None
        loss, parts = self.step(self.batch, self.bits)
        loss.backward()
        return loss.detach(), parts

    def eager(self):
        loss, parts = self.fwd_bwd()
        torch.cuda.synchronize()
        return loss.clone(), parts.clone(), grads(self.model)

    def capture(self, warm: int = 2):
        from onebit_asr.quant import QuantizedLinear

        dev = self.batch["feats"].device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warm):
                self.fwd_bwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        for m in self.model.modules():
            if isinstance(m, QuantizedLinear):
                m._codes_cache = {}
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self.fwd_bwd()

    def replay(self):
        self.graph.replay()
        torch.cuda.synchronize()
        loss, parts = self.out
        return loss.clone(), parts.clone(), grads(self.model)
