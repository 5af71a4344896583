#!/usr/bin/env python3
"""Per-phase cycles of one attention kernel from a diagnostic build (-DOB_ATTN_STAMPS=K:
s_memtime stamps per wave, written to a device buffer of their own). K = 1 flash-style
backward, 2 query-side backward, 3 forward, 4 key-side backward.
Build:  make -C cmu-11785-idl-1.58bit-asr_amd/csrc OUT=$PWD/exp/libstampK.so BUILD=$PWD/exp/stampK \
        HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DOB_ATTN_STAMPS=K"
Run:    ONEBIT_HIP_LIB=exp/libstampK.so python tools/attn_stamps.py K [waves] [blocks per (b,h)]"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402

PHASES = {
    1: ["p3 work", "top wait", "0a stage", "0a wait", "X", "X wait", "S/dP/dK/dV", "wait",
        "band", "band wait"],
    2: ["dO/delta", "dPd", "band row0", "dQu", "band sync", "dQv", "dq+sums", "red sync",
        "dS' out", "-"],
    3: ["q", "X", "row64", "sync1", "anchors+scores", "softmax", "sync2", "v stage", "sync3",
        "ctx"],
    4: ["first fetch", "sync a", "stage", "sync b", "mfma", "store", "-", "-", "-", "-"],
}
# (waves per block, blocks per (b, h)) at T = 249
GRID = {1: (8, 2), 2: (4, 4), 3: (4, 4), 4: (4, 4)}


def main():
    kern = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    if kern == 1:
        os.environ["OB_ATTN_BWD"] = "flash"
    lib = _lib.load()
    dev = torch.device("cuda:0")
    Bt, P, T, H, d = 96, 3, 249, 4, 36
    C = H * d
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v, do = (torch.randn(Bt, T, C, device=dev, generator=g) for _ in range(4))
    pos = torch.randn(P, T, C, device=dev, generator=g)
    u, vb = torch.randn(H, d, device=dev) * 0.01, torch.randn(H, d, device=dev) * 0.01
    lens = torch.full((Bt,), T, dtype=torch.int32, device=dev)
    rng = torch.tensor([1234, 1], dtype=torch.int64, device=dev)
    saved = torch.empty(lib.ob_relattn_saved_elems(Bt, T, H, d), device=dev)
    ctx = torch.empty_like(q)
    outs = [torch.empty_like(x) for x in (q, k, v, pos, u, vb)]
    wsb = lib.ob_relattn_bwd_workspace(Bt, T, H, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.ob_relattn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(),
                                  u.data_ptr(), vb.data_ptr(), lens.data_ptr(), Bt, P, T, H, d,
                                  0.1, rng.data_ptr(), 0, saved.data_ptr(), None, ctx.data_ptr(),
                                  s), "fwd")
    for _ in range(3):
        _lib.check(lib.ob_relattn_bwd(do.data_ptr(), ctx.data_ptr(), q.data_ptr(), k.data_ptr(),
                                      v.data_ptr(), pos.data_ptr(), u.data_ptr(), vb.data_ptr(),
                                      lens.data_ptr(), Bt, P, T, H, d, 0.1, rng.data_ptr(), 0,
                                      saved.data_ptr(), saved.numel(), *(o.data_ptr() for o in outs),
                                      ws.data_ptr(), wsb, s), "bwd")
    torch.cuda.synchronize()
    buf = np.zeros(65536, dtype=np.uint64)
    fn = lib.ob_attn_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else GRID[kern][0]
    nblk = Bt * H * (int(sys.argv[3]) if len(sys.argv) > 3 else GRID[kern][1])
    st = buf[: nblk * nw * 10].reshape(nblk, nw, 10).astype(np.float64)
    tot = st.sum(axis=2)
    print(f"block cycles: median {np.median(tot):.0f} (wave-summed over phases)")
    # block concurrency and the shader clock from s_memrealtime (100 MHz) at wave start / end
    rt = np.zeros(16384, dtype=np.uint64)
    fr = lib.ob_attn_rt
    fr.restype = ctypes.c_int
    fr.argtypes = [ctypes.c_void_p]
    assert fr(rt.ctypes.data) == 0
    rt = rt[: nblk * nw * 2].reshape(nblk, nw, 2).astype(np.float64)
    b0, b1 = rt[:, :, 0].min(axis=1), rt[:, :, 1].max(axis=1)
    span_us = (b1.max() - b0.min()) / 100.0
    dur_us = (b1 - b0) / 100.0
    clk = np.median(tot / np.maximum((rt[:, :, 1] - rt[:, :, 0]) / 100.0, 1e-9))  # cycles / us
    print(f"kernel span {span_us:.1f} us; block duration median {np.median(dur_us):.1f} us, "
          f"max {dur_us.max():.1f}; blocks in flight on average {dur_us.sum() / span_us:.1f}; "
          f"shader clock ~{clk / 1e3:.2f} GHz")
    starts = np.sort(b0 - b0.min()) / 100.0
    print("block start offsets (us) at quantiles 0/25/50/75/100 %:",
          " ".join(f"{np.quantile(starts, q):.1f}" for q in (0, 0.25, 0.5, 0.75, 1)))
    for wv in range(nw):
        med = np.median(st[:, wv, :], axis=0)
        print(f"wave {wv}: " + "  ".join(f"{n} {m:.0f}" for n, m in zip(PHASES[kern], med)))


if __name__ == "__main__":
    main()
