"""CPU, world_size 2 (gloo): the product's DDP step wiring -- one OneBitStep forward per
backward, identical SP masks on every rank, gradient all-reduce = mean of per-shard
gradients, replicas identical after the optimizer step. The model is the CPU oracle (the
product BitLinear has no CPU path); the step module and train_step are the product's."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

TINY = dict(enc_d_model=32, enc_layers=2, enc_heads=2, enc_d_ff=64, enc_conv_kernel=7,
            enc_dropout=0.0, dec_layers=1, dec_heads=2, dec_d_ff=64, dec_dropout=0.0)
TINY_ORACLE = dict(input_dim=40, vocab_size=48, d_model=32, n_layers=2, n_heads=2, d_ff=64,
                   conv_kernel=7, dec_layers=1, dec_heads=2, dec_d_ff=64, dropout=0.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model():
    from onebit_asr.conformer import ConformerASR
    from oracle.conformer_oracle import OracleConformer

    torch.manual_seed(0)
    prod = ConformerASR(40, 48, **TINY)
    return OracleConformer(prod.state_dict(), **TINY_ORACLE)


def _batch(rank):
    from onebit_asr.data import synthetic_batch

    return synthetic_batch([120, 97], [5, 3], n_mels=40, vocab=48, seed=100 + rank)


def _worker(rank, world, port, out_dir):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "cmu-11785-idl-1.58bit-asr_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torch.nn.parallel import DistributedDataParallel as DDP

    from onebit_asr.train_step import OneBitStep, make_optimizer, sample_sp_mask, train_step

    model = _model()
    step = DDP(OneBitStep(model, n_layers=2), broadcast_buffers=False)
    gen = torch.Generator().manual_seed(7)
    sp_mask = sample_sp_mask(2, generator=gen)
    loss, _ = step(_batch(rank), sp_mask)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    # one full product train_step (clip + AdamW) on top, to check replicas stay identical
    opt = make_optimizer(model.parameters())
    train_step(step, opt, None, _batch(rank), sp_mask)
    params = {k: p.detach().clone() for k, p in model.named_parameters()}
    torch.save({"sp_mask": sp_mask, "grads": grads, "params": params, "loss": loss.item()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_ddp_two_ranks_gloo(tmp_path):
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert res[0]["sp_mask"] == res[1]["sp_mask"]
    # reference: mean over shards of single-process gradients
    sp_mask = sample_sp_mask(2, generator=torch.Generator().manual_seed(7))
    assert sp_mask == res[0]["sp_mask"]
    per_rank = []
    for r in range(world):
        m = _model()
        loss, _ = OneBitStep(m, n_layers=2)(_batch(r), sp_mask)
        loss.backward()
        per_rank.append({k: p.grad for k, p in m.named_parameters()})
    for k in per_rank[0]:
        ref = (per_rank[0][k] + per_rank[1][k]) / 2
        # shard gradients can cancel in the mean: bound the error by the shards' magnitude
        scale = max(per_rank[0][k].abs().max().item(), per_rank[1][k].abs().max().item())
        for r in range(world):
            err = (res[r]["grads"][k] - ref).abs().max().item()
            assert err <= 1e-5 * scale + 1e-6, (k, err, scale)  # dw.bias grad is ~0 (BN follows)
    for k in res[0]["params"]:
        assert torch.equal(res[0]["params"][k], res[1]["params"][k]), k


class _HostBitsStep(torch.nn.Module):
    """OneBitStep over the CPU oracle, reading the DeviceBits slots back as the reference's
    per-block list (the oracle has no device-bits path)."""

    def __init__(self, model):
        super().__init__()
        from onebit_asr.train_step import OneBitStep

        self.inner = OneBitStep(model, n_layers=2)

    def forward(self, batch, bits):
        return self.inner(batch, [1 if v == 1 else 0 for v in bits.tensor.tolist()])


def _graph_step_worker(rank, world, port, out_dir, bucket_mb=12.0, tag="g", exchange="deferred"):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "cmu-11785-idl-1.58bit-asr_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from onebit_asr.graph_step import GraphedTrainStep

    model = _model()
    gs = GraphedTrainStep(_HostBitsStep(model), n_layers=2, process_group=dist.group.WORLD,
                          warmup_iters=1, warmup_steps=4, total_steps=10, bucket_mb=bucket_mb,
                          exchange=exchange)
    losses = []
    for mask in ([1, 0], [0, 1], [1, 1]):
        loss, _ = gs.step(_batch(rank), mask)
        losses.append(loss.item())
    params = {k: p.detach().clone() for k, p in model.named_parameters()}
    nb = len(gs.buckets.buckets) if gs.buckets is not None else 0
    torch.save({"params": params, "losses": losses, "buckets": nb},
               os.path.join(out_dir, f"{tag}{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_graph_step_flat_allreduce_gloo(tmp_path):
    """GraphedTrainStep's N>1 exchange (flat-buffer SUM all-reduce, /world, clip, AdamW,
    warmup-cosine) equals single-process training on the mean of the shard gradients."""
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer

    world = 2
    mp.spawn(_graph_step_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"g{r}.pt", weights_only=True) for r in range(world)]
    model = _model()
    step = OneBitStep(model, n_layers=2)
    opt = make_optimizer(model.parameters())
    sched = WarmupCosine(opt, 4, 10)
    for mask in ([1, 0], [0, 1], [1, 1]):
        shard = []
        for r in range(world):
            model.zero_grad(set_to_none=True)
            loss, _ = step(_batch(r), mask)
            loss.backward()
            shard.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
        for k, p in model.named_parameters():
            p.grad = (shard[0][k] + shard[1][k]) / 2 if k in shard[0] else None
        torch.nn.utils.clip_grad_norm_([p for p in model.parameters() if p.grad is not None], 5.0)
        opt.step()
        sched.step()
    # k_proj.bias (softmax shift; also inside the decoder in_proj_bias) and the depthwise-conv bias (BatchNorm follows) have a
    # mathematically zero gradient: Adam turns its rounding noise into +-lr steps, so those
    # two only get a bound of the summed learning rates.
    noise_only = ("k_proj__bias", "dw__bias", "in_proj_bias")  # in_proj_bias holds the k bias
    for k, p in model.named_parameters():
        for r in range(world):
            err = (res[r]["params"][k] - p.detach()).abs().max().item()
            if any(n in k for n in noise_only):
                assert err <= 1e-3, (k, r, err)
            else:
                assert err <= 1e-5 * p.detach().abs().max().item() + 1e-7, (k, r, err)
    for k in res[0]["params"]:
        assert torch.equal(res[0]["params"][k], res[1]["params"][k]), k


@pytest.mark.slow
def test_bucketed_overlapped_allreduce_equals_flat_gloo(tmp_path):
    """The three exchanges train the replicas to exactly the same parameters (SUM over two
    ranks does not depend on how the buffer is cut or packed): the bucketed one started
    bucket by bucket from the backward's post-accumulate hooks (BucketedAllReduce, tiny
    buckets: one per few parameters), the single flat all-reduce over the gradient views,
    and the default deferred one (autograd's gradient buffers packed into the flat buffer,
    one all-reduce, copied back)."""
    world = 2
    runs = ((None, "flat", "flat"), (0.002, "bkt", "bucketed"), (None, "dfr", "deferred"))
    for bucket_mb, tag, exchange in runs:
        mp.spawn(_graph_step_worker,
                 args=(world, _free_port(), str(tmp_path), bucket_mb, tag, exchange),
                 nprocs=world, join=True)
    res = {tag: [torch.load(tmp_path / f"{tag}{r}.pt", weights_only=True) for r in range(world)]
           for _, tag, _ in runs}
    flat, bkt, dfr = res["flat"], res["bkt"], res["dfr"]
    assert flat[0]["buckets"] == 0 and dfr[0]["buckets"] == 0 and bkt[0]["buckets"] > 8, bkt[0]["buckets"]
    for r in range(world):
        for other in (bkt, dfr):
            assert flat[r]["losses"] == other[r]["losses"]
            for k, p in flat[r]["params"].items():
                assert torch.equal(p, other[r]["params"][k]), k
