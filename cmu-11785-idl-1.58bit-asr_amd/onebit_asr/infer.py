"""Inference path (BASELINE configs[4]): packed-ternary weights, optional int8 activations,
batched greedy CTC decode -- the encoder + CTC head forward of the reference's eval loop
(eval.py:91-124: ``model(batch, precision)``, valid lengths from the mask) followed by
metrics.py:51-60's greedy decode, for a whole padded batch at once.

* weights: each QuantizedLinear's 2-bit codes are packed once and cached (they are only
  repacked when a weight or alpha changes), so a forward streams 2-bit codes, never W;
* activations: ``act_quant="absmax_int8"`` runs the BitLinear GEMMs on the int8 matrix
  cores (the north-star mode, csrc/tgemm_i8.hip); ``None`` keeps the reference's fp32;
* decode: ``ob_ctc_greedy_decode`` (csrc/decode.hip), argmax + collapse on the device;
* ``GraphedInference`` captures forward + decode as one HIP graph for a fixed padded shape.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from .quant import set_act_quant

__all__ = ["ctc_greedy_decode_batch", "ctc_greedy_decode", "GraphedInference", "encode_and_decode"]


def ctc_greedy_decode_batch(logits: torch.Tensor, lens: torch.Tensor, blank_id: int = 3
                            ) -> Tuple[torch.Tensor, torch.Tensor]:
    """logits [B, T, V] fp32 (device), lens [B] valid frames -> (tokens int32 [B, T], padded
    with -1; counts int32 [B]). No host synchronisation."""
    if not logits.is_cuda:
        raise RuntimeError("ctc_greedy_decode_batch runs on the HIP library (no CPU fallback)")
    b, t, v = logits.shape
    x = logits.contiguous().float()
    ln = lens.to(device=x.device, dtype=torch.int64).contiguous()
    ids = torch.empty((b, t), dtype=torch.int32, device=x.device)
    out = torch.empty((b, t), dtype=torch.int32, device=x.device)
    cnt = torch.empty((b,), dtype=torch.int32, device=x.device)
    lib = _lib.load()
    _lib.check(lib.ob_ctc_greedy_decode(x.data_ptr(), ln.data_ptr(), b, t, v, blank_id,
                                        ids.data_ptr(), out.data_ptr(), cnt.data_ptr(),
                                        _lib.stream_of(x)), "ob_ctc_greedy_decode")
    return out, cnt


def ctc_greedy_decode(logits: torch.Tensor, blank_id: int = 3) -> List[int]:
    """metrics.py:51-60 signature: one utterance's logits [T, V] -> token list."""
    t = logits.size(0)
    out, cnt = ctc_greedy_decode_batch(logits.unsqueeze(0),
                                       torch.tensor([t], device=logits.device), blank_id)
    n = int(cnt.item())
    return out[0, :n].tolist()


@torch.no_grad()
def encode_and_decode(model, batch: Dict[str, torch.Tensor], precision: int = 2,
                      blank_id: int = 3):
    """Encoder + CTC head + greedy decode of one padded batch (eval.py:118-124 for one
    precision, with greedy instead of beam search). Returns (tokens, counts, logits)."""
    _, mask, logits = model(batch, precision=precision)
    lens = mask.sum(dim=1)
    out, cnt = ctc_greedy_decode_batch(logits, lens, blank_id)
    return out, cnt, logits


class GraphedInference:
    """Forward + decode for a fixed padded batch shape, captured once as a HIP graph.
    ``run(batch)`` copies the batch into the captured inputs and replays."""

    def __init__(self, model, precision: int = 2, act_quant: Optional[str] = "absmax_int8",
                 blank_id: int = 3, use_graph: bool = True):
        self.model = model.eval()
        set_act_quant(self.model, act_quant)
        self.precision = precision
        self.blank_id = blank_id
        self.use_graph = use_graph
        self.graph = None
        self.inputs = None
        self.outputs = None

    def _body(self):
        return encode_and_decode(self.model, self.inputs, self.precision, self.blank_id)

    def run(self, batch: Dict[str, torch.Tensor]):
        if self.inputs is None:
            self.inputs = {k: v.clone() for k, v in batch.items()}
            if not self.use_graph:
                return self._body()
            side = torch.cuda.Stream(batch["feats"].device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):  # warm-up: packs codes, picks kernels, allocates
                    self._body()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.outputs = self._body()
        else:
            for k, v in batch.items():
                if self.inputs[k].shape != v.shape:
                    raise ValueError(f"batch[{k!r}] shape {tuple(v.shape)} != captured "
                                     f"{tuple(self.inputs[k].shape)}")
                if self.inputs[k].data_ptr() != v.data_ptr():
                    self.inputs[k].copy_(v, non_blocking=True)
            if not self.use_graph:
                return self._body()
        self.graph.replay()
        return self.outputs
