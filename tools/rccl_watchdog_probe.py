"""Root cause of the round-4 RCCL-capture abort (VERDICT r4 Next #2), one child process per
mode, world size 1 over RCCL:

  sep      eager all-reduce + barrier on the default group, then capture an all-reduce on a
           second group connected eagerly (graph_step.capture_group) -- the product path
  same_tl  the same, but the captured all-reduce on the default group, thread_local mode
  same     the same, but the captured all-reduce on the default group, global mode

Inside the capture the process sleeps 1.5 s (> ProcessGroupNCCL's watchdog poll interval),
so an eager collective still on the watchdog's list is polled while the stream captures.
Prints one line per mode: rc and the tail of stderr. Run `same*` modes last in a GPU call:
they are expected to abort.

usage: python tools/rccl_watchdog_probe.py MODE [MODE ...]
"""
import os
import socket
import subprocess
import sys
import time


def child(mode: str, port: int) -> None:
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cmu-11785-idl-1.58bit-asr_amd"))
    from onebit_asr.graph_step import capture_group

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=dev)
    pg = dist.group.WORLD
    x = torch.ones(1 << 20, device=dev)
    cg = capture_group(pg, dev) if mode == "sep" else pg
    for _ in range(3):  # eager collectives: handed to the default group's watchdog
        dist.all_reduce(x, group=pg)
    dist.barrier(group=pg, device_ids=[0])
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    mode_err = "global" if mode == "same" else "thread_local"
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode=mode_err):
            y = x * 2
            dist.all_reduce(y, group=cg)
            time.sleep(1.5)
            z = y + 1
    g.replay()
    torch.cuda.synchronize()
    ok = bool((z == 3).all().item())
    print(f"child {mode}: replay ok={ok}", flush=True)
    time.sleep(1.0)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        return
    for mode in sys.argv[1:]:
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
        so.close()
        r = subprocess.run([sys.executable, __file__, "--child", mode, str(port)],
                           capture_output=True, text=True, timeout=120)
        tail = (r.stdout + r.stderr).strip().splitlines()[-6:]
        print(f"=== {mode}: rc={r.returncode}", flush=True)
        for ln in tail:
            print("   ", ln[:400], flush=True)
        if r.returncode != 0:
            break  # nothing more on the GPU after an abort


if __name__ == "__main__":
    main()
