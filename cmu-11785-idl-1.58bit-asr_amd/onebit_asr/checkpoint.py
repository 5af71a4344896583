"""Packed-ternary checkpoints: 2-bit codes + alpha + bias per BitLinear, everything else fp32.

The reference saves and reloads whole fp32 state dicts (train.py:307-317,
``torch.save({'model': model.state_dict(), ...})``; eval.py:228,282
``model.load_state_dict(checkpoint['model'])``) and re-quantizes every QuantizedLinear
inside each forward (quant.py:123-126). For 1.58-bit / 1-bit inference the fp32 weight is
only ever used through Q(W / |alpha|_eps), so a deployable checkpoint needs just the codes:

  <layer>.codes2 / <layer>.codes1   int32 [N, ceil(K/16)]  (uint32 code words, 16 x 2 bits,
                                    0 -> 0, 1 -> +1, 3 -> -1; include/onebit_hip.h)
  <layer>.alpha                     fp32 scalar, the raw parameter (|alpha| + 1e-8 at use)
  <layer>.bias                      fp32 [N] (when the layer has one)
  every other state-dict entry      as saved by model.state_dict() (the reference's keys)

in a safetensors file (a loader that executes nothing from the file), with the layer table
in its metadata. 16x smaller than fp32 for the BitLinear weights. Loading installs the codes
into each layer's code cache and marks it packed: forwards at bitwidth 1 / 2 (and the
stacked PassBits step, inference only) use them as they are -- bit-identical outputs to
the model that was saved; bitwidth 32 and training raise (the fp32 weights are not in the
file).

Codes are produced by the product's HIP pack kernel (ob_quant_pack), so exporting needs the
GPU, like every BitLinear forward; the file format itself is host-side.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Iterable, Optional

import numpy as np
import torch
import torch.nn as nn

from .quant import QuantizedLinear, pack_codes

FORMAT = "onebit-packed-ternary/1"


def _transpose_codes(codes: np.ndarray, n: int, k: int) -> np.ndarray:
    """codes [N][ceil(K/16)] -> codes_t [K][ceil(N/16)] (same 2-bit fields, transposed)."""
    words = codes.astype(np.uint32).astype(np.uint64)
    shifts = (2 * np.arange(16, dtype=np.uint64))[None, None, :]
    fields = ((words[:, :, None] >> shifts) & np.uint64(3)).reshape(n, -1)[:, :k]  # [N][K]
    ft = np.ascontiguousarray(fields.T)  # [K][N]
    nw = (n + 15) // 16
    pad = np.zeros((k, nw * 16), np.uint64)
    pad[:, :n] = ft
    packed = (pad.reshape(k, nw, 16) << shifts).sum(-1).astype(np.uint32)
    return packed.view(np.int32)


def _quant_layers(model: nn.Module) -> Dict[str, QuantizedLinear]:
    return {name: m for name, m in model.named_modules()
            if isinstance(m, QuantizedLinear) and m.quant_off is None}


def packed_state(model: nn.Module, bits: Iterable[int] = (2, 1)):
    """(tensors, metadata) of the packed checkpoint of ``model`` (its BitLinear weights,
    alpha and bias on the GPU)."""
    bits = tuple(int(b) for b in bits)
    if not bits or any(b not in (1, 2) for b in bits):
        raise ValueError(f"packed bitwidths must be 1 and/or 2, got {bits}")
    layers = _quant_layers(model)
    skip = {f"{n}.weight" for n in layers}
    tensors: Dict[str, torch.Tensor] = {}
    for key, t in model.state_dict().items():
        if key not in skip:
            tensors[key] = t.detach().to("cpu").contiguous()
    table = {}
    with torch.no_grad():
        for name, m in layers.items():
            if getattr(m, "_packed", None):
                raise ValueError(f"{name} is already packed: re-export the file it came from")
            n, k = m.weight.shape
            for b in bits:
                codes, _ = pack_codes(m.weight, m.alpha, b, alpha_raw=True)
                tensors[f"{name}.codes{b}"] = codes.to("cpu").contiguous()
            table[name] = [int(n), int(k), m.bias is not None]
    meta = {"format": FORMAT, "bits": ",".join(str(b) for b in bits),
            "layers": json.dumps(table, sort_keys=True)}
    return tensors, meta


def save_packed(model: nn.Module, path, bits: Iterable[int] = (2, 1),
                extra: Optional[Dict[str, str]] = None) -> None:
    """Write the packed checkpoint of ``model`` to ``path`` (safetensors)."""
    from safetensors.torch import save_file

    tensors, meta = packed_state(model, bits)
    if extra:
        meta.update({str(k): str(v) for k, v in extra.items()})
    save_file(tensors, str(path), metadata=meta)


def read_packed(path):
    """(tensors on the CPU, metadata) of a packed checkpoint; refuses other files."""
    from safetensors import safe_open

    with safe_open(str(path), framework="pt", device="cpu") as f:
        meta = f.metadata() or {}
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a packed-ternary checkpoint ({meta.get('format')!r})")
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    return tensors, meta


def load_packed(model: nn.Module, path, device=None) -> nn.Module:
    """Load a packed checkpoint into ``model`` (built with the same architecture): the
    non-BitLinear state by load_state_dict, each BitLinear's alpha / bias, and its codes
    into the layer's code cache. Returns ``model`` (on ``device`` if given)."""
    tensors, meta = read_packed(path)
    table = json.loads(meta["layers"])
    bits = [int(b) for b in meta["bits"].split(",")]
    layers = _quant_layers(model)
    if set(table) != set(layers):
        missing, extra = sorted(set(layers) - set(table)), sorted(set(table) - set(layers))
        raise ValueError(f"BitLinear layers differ from the checkpoint: model-only {missing[:4]}, "
                         f"file-only {extra[:4]}")
    if device is not None:
        model.to(device)
    plain = {k: v for k, v in tensors.items() if ".codes" not in k}
    result = model.load_state_dict(plain, strict=False)
    expected_missing = {f"{n}.weight" for n in layers}
    if set(result.missing_keys) != expected_missing or result.unexpected_keys:
        raise ValueError(f"state mismatch: missing {sorted(set(result.missing_keys) - expected_missing)[:4]}, "
                         f"unexpected {result.unexpected_keys[:4]}")
    for name, m in layers.items():
        n, k, has_bias = table[name]
        if tuple(m.weight.shape) != (n, k) or (m.bias is not None) != has_bias:
            raise ValueError(f"{name}: shape / bias differ from the checkpoint")
        dev = m.weight.device
        packed = {}
        for b in bits:
            c = tensors[f"{name}.codes{b}"]
            ct = torch.from_numpy(_transpose_codes(c.numpy(), n, k))
            packed[b] = (c.to(dev), ct.to(dev))
        m.install_packed(packed)
    return model
