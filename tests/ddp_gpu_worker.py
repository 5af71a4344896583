"""Worker of tests/test_ddp_gpu.py (launched by torch.distributed.run, 2 ranks): the
multi-rank path of GraphedTrainStep on the GPU -- flat gradient buffer, graph A (forward +
backward), the eager all-reduce between the replays, graph B (clip + FusedAdamW with the
1/world gradient scale). Both ranks share the box's one GPU, so the exchange runs over gloo
(CUDA tensors); the bench's 8-GPU runs use RCCL for the same all_reduce call.

Each rank first computes its shard's single-process gradient (eager OneBitStep forward +
backward on a replica of the same init) for the reference, then runs 2 graphed steps.
Writes rank{r}.pt: local grads, the flat (summed) gradients after step 1, params after 2."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir = sys.argv[1]
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    batch = synthetic_batch([400, 333], [20, 13], seed=100 + rank, device=dev)
    sp_mask = sample_sp_mask(CFG1["enc_layers"], generator=torch.Generator().manual_seed(9))

    def fresh():
        torch.manual_seed(0)
        return ConformerASR(80, 5004, **CFG1).to(dev)

    ref_model = fresh()
    loss, _ = OneBitStep(ref_model, n_layers=CFG1["enc_layers"])(batch, sp_mask)
    loss.backward()
    local = {k: p.grad.detach().clone().cpu() for k, p in ref_model.named_parameters()
             if p.grad is not None}
    del ref_model

    model = fresh()
    names = {id(p): k for k, p in model.named_parameters()}
    gs = GraphedTrainStep(OneBitStep(model, n_layers=CFG1["enc_layers"]), CFG1["enc_layers"],
                          process_group=dist.group.WORLD, warmup_iters=1)
    gs.step(batch, sp_mask)
    torch.cuda.synchronize()
    summed = {names[id(p)]: p.grad.detach().clone().cpu() for p in gs.params}
    gs.step(batch, sp_mask)
    torch.cuda.synchronize()
    params = {k: p.detach().clone().cpu() for k, p in model.named_parameters()}
    torch.save({"local": local, "summed": summed, "params": params,
                "graphed": gs.graph_a is not None and gs.graph_b is not None},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
