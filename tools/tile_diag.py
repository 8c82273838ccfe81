#!/usr/bin/env python3
"""Where a k_gemm3g tile form goes wrong: NaN / error pattern of one dense x3 GEMM per (tile, MFMA
shape, K), repeated, against fp64. python tools/tile_diag.py [tiles] [ks] [reps]"""
import importlib
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")


def main():
    tiles = [int(t) for t in (sys.argv[1] if len(sys.argv) > 1 else "9,10").split(",")]
    ks = [int(k) for k in (sys.argv[2] if len(sys.argv) > 2 else "642,640,96").split(",")]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    lib = FU._setup()
    m, n = 81920, 512
    for k in ks:
        ldx = (k + 3) // 4 * 4
        torch.manual_seed(m + n + k)
        buf = torch.randn(m, ldx, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        wp, ldw = FU._pad_cols(w)
        x3 = FU.X3(wp, ldw, n, k)
        ref = F.linear(buf[:, :k].double(), w.double(), b.double())
        for tile in tiles:
            for mf in (0, 1):
                lib.gm_gemm_set_tile(tile)
                FU.L.check(lib.gm_gemm_set_mfma(mf))
                for r in range(reps):
                    y = torch.full((m, n), 7.0, device="cuda")
                    FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 0,
                            y.data_ptr(), n, x3=x3)
                    torch.cuda.synchronize()
                    err = (y.double() - ref).abs()
                    bad = ~(err < 1e-4)
                    nb = int(bad.sum())
                    msg = f"k={k} tile={tile} mfma={mf} rep={r}: bad={nb} max_err={err[~bad].max().item() if nb < err.numel() else -1:.2e}"
                    if nb:
                        rr, cc = bad.nonzero(as_tuple=True)
                        msg += (f" nan={int(torch.isnan(y).sum())} rows {rr.min().item()}..{rr.max().item()}"
                                f" (tiles {sorted(set((rr // 128).tolist()))[:8]}) cols {cc.min().item()}..{cc.max().item()}"
                                f" rows%128 {sorted(set((rr % 128).tolist()))[:16]} cols%256 {sorted(set((cc % 256).tolist()))[:16]}")
                    print(msg, flush=True)
    lib.gm_gemm_set_tile(-1)
    FU.L.check(lib.gm_gemm_set_mfma(2))


if __name__ == "__main__":
    main()
