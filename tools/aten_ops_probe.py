import sys, collections
from pathlib import Path
ROOT = Path('/root/repo') if Path('/root/repo').exists() else Path('.')
import os
R = os.environ.get('GRAFT_REPO_ROOT', '.')
sys.path[:0] = [R, R + '/cmu-11785-idl-1.58bit-asr_amd']
import torch
from torch.profiler import profile, ProfilerActivity
from onebit_asr.conformer import ConformerASR
from onebit_asr.data import CONFORMER_S, synthetic_batch
from onebit_asr.train_step import OneBitStep, sample_sp_mask
from onebit_asr.graph_step import GraphedTrainStep
dev = torch.device('cuda', 0)
torch.manual_seed(1234)
model = ConformerASR(80, 5004, **CONFORMER_S).to(dev)
n_layers = CONFORMER_S['enc_layers']
batch = synthetic_batch([1000] * 32, [40] * 32, seed=1234, device=dev)
gs = GraphedTrainStep(OneBitStep(model, n_layers=n_layers), n_layers, use_graph=False, warmup_iters=1)
gen = torch.Generator().manual_seed(4321)
for _ in range(2):
    gs.step(batch, sample_sp_mask(n_layers, generator=gen))
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    gs.step(batch, sample_sp_mask(n_layers, generator=gen))
    torch.cuda.synchronize()
ev = prof.events()
cnt = collections.Counter()
for e in ev:
    name = e.name
    if not name.startswith('aten::') or name in ('aten::empty', 'aten::empty_strided', 'aten::view', 'aten::as_strided', 'aten::reshape', 'aten::_reshape_alias', 'aten::t', 'aten::transpose', 'aten::detach', 'aten::slice', 'aten::select', 'aten::unsqueeze', 'aten::squeeze', 'aten::expand', 'aten::permute', 'aten::contiguous', 'aten::alias', 'aten::lift_fresh', 'aten::resolve_conj', 'aten::resolve_neg', 'aten::result_type', 'aten::is_nonzero', 'aten::item', 'aten::_local_scalar_dense', 'aten::split', 'aten::chunk', 'aten::narrow', 'aten::unbind', 'aten::flatten', 'aten::unflatten', 'aten::view_as', 'aten::empty_like', 'aten::set_', 'aten::record_stream'):
        continue
    st = [s for s in (e.stack or []) if 'onebit_asr' in s or 'graph_step' in s]
    where = st[0] if st else '?'
    cnt[(name, str(e.input_shapes)[:60], where[-90:])] += 1
for (n, sh, w), c in cnt.most_common(60):
    print(f"{c:4d} {n:28s} {sh:60s} {w}")
