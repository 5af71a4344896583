"""Worker of tests/test_rccl_capture_gpu.py (a child process on the box's one GPU): the
multi-rank step path over RCCL at world size 1 (graph_step._MULTI_RANK_PATH_AT_WORLD_1),
both exchanges captured into the same graph as the forward, backward and update: the
bucketed all-reduce started from the backward's gradient hooks, and the default deferred
one (gradients written in place into the flat buffer, one all-reduce), the latter also with
the literal three-pass step body (OneBitStep(stacked=False)). With one rank the all-reduce is an identity, so two
steps must give the parameters of the single-GPU path.
Writes result.pt: whether the collectives were captured, bucket count, the parameters of
both runs."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir, port = sys.argv[1], sys.argv[2]
    mode = sys.argv[3] if len(sys.argv) > 3 else ""
    if "nocache" in mode:
        os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)

    from onebit_asr import graph_step
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    batch = synthetic_batch([400, 333], [20, 13], seed=100, device=dev)
    sp_mask = sample_sp_mask(CFG1["enc_layers"], generator=torch.Generator().manual_seed(9))

    def run(multi, exchange="deferred", stacked=None):
        graph_step._MULTI_RANK_PATH_AT_WORLD_1 = multi
        torch.manual_seed(0)
        model = ConformerASR(80, 5004, **CFG1).to(dev)
        # small buckets: several captured collectives (Conformer cfg1 has ~2 MB of gradients)
        gs = GraphedTrainStep(OneBitStep(model, n_layers=CFG1["enc_layers"], stacked=stacked),
                              CFG1["enc_layers"],
                              process_group=dist.group.WORLD, warmup_iters=1, bucket_mb=0.25,
                              exchange=exchange)
        for _ in range(2):
            gs.step(batch, sp_mask)
        torch.cuda.synchronize()
        nb = len(gs.buckets.buckets) if gs.buckets is not None else 0
        params = {k: p.detach().clone().cpu() for k, p in model.named_parameters()}
        return gs.comm_in_graph, nb, gs.multi, params

    cap, nb, multi, p_multi = run(True, "bucketed")
    cap_d, nb_d, multi_d, p_dfr = run(True, "deferred")
    _, _, plain_multi, p_plain = run(False)
    # the reference's literal three forwards (several producing sites per parameter: ADVICE r5,
    # no site may write the shared flat slice) through the deferred exchange
    cap_l, _, multi_l, p_lit = run(True, "deferred", stacked=False)
    _, _, _, p_lit_plain = run(False, stacked=False)
    torch.save({"captured": cap, "buckets": nb, "multi": multi, "plain_multi": plain_multi,
                "p_multi": p_multi, "p_plain": p_plain, "captured_deferred": cap_d,
                "buckets_deferred": nb_d, "multi_deferred": multi_d, "p_deferred": p_dfr,
                "captured_literal": cap_l, "multi_literal": multi_l, "p_literal": p_lit,
                "p_literal_plain": p_lit_plain},
               os.path.join(out_dir, "result.pt"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
