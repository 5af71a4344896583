"""Synthetic padded-utterance batches in the reference's batch-dict contract.

dataloader_stub.py:13-19: ``feats [B,T,F] f32``, ``feat_lens [B] i64``, ``tokens [B,U] i64``
(pad 0, no BOS/EOS), ``token_lens [B] i64``; collate pads features with 0.0
(src/data/dataset.py:245-249). Token ids are drawn from [4, vocab) (SPM ids offset by +4,
dataloader_stub.py:255). No LibriSpeech audio exists offline: features are
N(0,1), which matches CMVN-normalised fbank statistics.
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch

__all__ = ["synthetic_batch", "CONFORMER_S", "CFG1"]

# Conformer-S training config and the 2-block parity config.
CONFORMER_S = dict(enc_d_model=144, enc_layers=16, enc_heads=4, enc_d_ff=576, enc_conv_kernel=31,
                   enc_dropout=0.1, dec_layers=2, dec_heads=4, dec_d_ff=1024, dec_dropout=0.1)
CFG1 = dict(enc_d_model=64, enc_layers=2, enc_heads=4, enc_d_ff=256, enc_conv_kernel=31,
            enc_dropout=0.0, dec_layers=2, dec_heads=4, dec_d_ff=1024, dec_dropout=0.0)


def synthetic_batch(feat_lens: Sequence[int], token_lens: Sequence[int], n_mels: int = 80,
                    vocab: int = 5004, seed: int = 0, device="cpu") -> Dict[str, torch.Tensor]:
    """Padded batch: utterance b has feat_lens[b] frames (padded to the max with 0.0) and
    token_lens[b] tokens (padded with 0)."""
    g = torch.Generator().manual_seed(seed)
    bsz, tmax, umax = len(feat_lens), max(feat_lens), max(token_lens)
    feats = torch.zeros(bsz, tmax, n_mels)
    tokens = torch.zeros(bsz, umax, dtype=torch.long)
    for b, (t, u) in enumerate(zip(feat_lens, token_lens)):
        feats[b, :t] = torch.randn(t, n_mels, generator=g)
        tokens[b, :u] = torch.randint(4, vocab, (u,), generator=g)
    batch = {
        "feats": feats,
        "feat_lens": torch.tensor(list(feat_lens), dtype=torch.long),
        "tokens": tokens,
        "token_lens": torch.tensor(list(token_lens), dtype=torch.long),
    }
    return {k: v.to(device) for k, v in batch.items()}
