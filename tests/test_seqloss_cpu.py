"""CPU: the stacked step's torch decoder-loss expressions (OneBitStep._att_kl_torch, the path
when csrc/seqloss.hip does not apply) equal the per-pass reference losses -- att_ce_loss
(losses.py:22-35, label smoothing and its scalar-mean quirk, or plain CE with ignore_index)
and kl_logits (losses.py:50-59) against pass 0 -- as train.py:82-111 evaluates them."""
from types import SimpleNamespace

import pytest
import torch

PAD = 0


@pytest.mark.parametrize("ls", [0.1, 0.0])
def test_att_kl_torch_equals_per_pass_losses(ls):
    from onebit_asr.losses import att_ce_loss, kl_logits
    from onebit_asr.train_step import OneBitStep

    g = torch.Generator().manual_seed(7)
    P, B, U, V = 3, 3, 6, 20
    logits = torch.randn(P * B, U, V, generator=g, dtype=torch.float64)
    t_out = torch.randint(1, V, (B, U), generator=g)
    t_out[0, 4:] = PAD
    t_out[2, 2:] = PAD
    t_pad = torch.zeros(B, U, dtype=torch.bool)
    t_pad[0, 5:] = True
    t_pad[2, 3:] = True
    me = SimpleNamespace(special={"pad_id": PAD}, label_smoothing=ls)
    l_att, l_kl = OneBitStep._att_kl_torch(me, logits, t_out, t_pad, P)
    per = logits.view(P, B, U, V)
    for p in range(P):
        ref = att_ce_loss(per[p], t_out, PAD, label_smoothing=ls)
        # the reference's float mask makes its result fp32 (a 0-dim float64 loss times an fp32
        # mask promotes to fp32), hence the fp32-level bar
        torch.testing.assert_close(l_att[p], ref, rtol=1e-6, atol=1e-7, check_dtype=False)
    for p in range(1, P):
        ref = kl_logits(per[p], per[0], t_pad)
        torch.testing.assert_close(l_kl[p - 1], ref, rtol=1e-12, atol=1e-12)
