#!/usr/bin/env python3
"""Per-phase cycles of the flash-style attention backward from a diagnostic build
(-DOB_ATTN_STAMPS: s_memtime stamps per wave, written to a device buffer of their own).
Build:  make -C cmu-11785-idl-1.58bit-asr_amd/csrc OUT=$PWD/exp/libstamp.so BUILD=$PWD/exp/stamp \
        HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DOB_ATTN_STAMPS"
Run:    ONEBIT_HIP_LIB=exp/libstamp.so python tools/attn_stamps.py"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402

PHASES = ["p3 work", "top wait", "0a stage", "0a wait", "X", "X wait", "S/dP/dK/dV", "wait",
          "band", "band wait"]


def main():
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
                                      saved.data_ptr(), *(o.data_ptr() for o in outs),
                                      ws.data_ptr(), wsb, s), "bwd")
    torch.cuda.synchronize()
    buf = np.zeros(65536, dtype=np.uint64)
    fn = lib.ob_attn_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nblk = Bt * H * (int(sys.argv[2]) if len(sys.argv) > 2 else 2)
    st = buf[: nblk * nw * 10].reshape(nblk, nw, 10).astype(np.float64)
    tot = st.sum(axis=2)
    print(f"block cycles: median {np.median(tot):.0f} (wave-summed over phases)")
    for wv in range(nw):
        med = np.median(st[:, wv, :], axis=0)
        print(f"wave {wv}: " + "  ".join(f"{n} {m:.0f}" for n, m in zip(PHASES, med)))


if __name__ == "__main__":
    main()
