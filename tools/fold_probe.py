"""Lab A/B for the algebraic BN-backward fold.

The fold replaces a BatchNorm backward's apply pass, dt = k0*du - k1*xhat - k2
(read du, t; write dt), by GEMMs that read [du | t] directly:
  dX = du (k0 o W) - t (k1/sigma o W) + c W   -> K doubles (512 -> 1024)
  dW = k0 o (du^T X) - k1/sigma o (t^T X) + c (x) colsum(X) -> two products
Per fold site this times, on the library's own kernels at the bench shape
(B = 131072, H = 512, bf16): the dX GEMM at K = 512 (weight-stationary
gemm_ws) and K = 1024 (outside gemm_ws's 512-deep register-resident weight:
the generic MFMA GEMM, and torch/hipBLASLt for reference), and the weight
gradient of 512 vs 1024 output rows, against the apply pass it removes.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
from dcnr import _lib  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main(M=131072, H=512):
    dev = torch.device("cuda")
    lib = _lib.load()
    s = _lib.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    for K in (H, 2 * H):
        X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        W = (torch.randn(H, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(H, device=dev)
        C = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
        out[f"dx_K{K}_ours"] = timed(lambda: _lib.check(lib.dcnr_linear_bf16(
            X.data_ptr(), K, M, K, W.data_ptr(), K, H, b.data_ptr(), C.data_ptr(), H, 0, s), "linear"))
        Wt = W.t()
        out[f"dx_K{K}_hipblaslt"] = timed(lambda: torch.mm(X, Wt))
    for N in (H, 2 * H):
        dY = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        X = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
        dW = torch.empty(N, H, device=dev)
        ws = torch.empty(lib.dcnr_linear_wgrad_workspace_size(N, H, M), dtype=torch.uint8, device=dev)
        out[f"dw_N{N}_ours"] = timed(lambda: _lib.check(lib.dcnr_linear_wgrad_bf16(
            dY.data_ptr(), N, X.data_ptr(), H, M, N, H, dW.data_ptr(), 0, ws.data_ptr(), ws.numel(), s),
            "wgrad"))
    for k, v in out.items():
        print(f"{k:24s} {v:8.1f} us", flush=True)
    dx = out[f"dx_K{2*H}_ours"] - out[f"dx_K{H}_ours"]
    dxb = out[f"dx_K{2*H}_hipblaslt"] - out[f"dx_K{H}_ours"]
    dw = out[f"dw_N{2*H}_ours"] - out[f"dw_N{H}_ours"]
    print(f"per fold site: dX +{dx:.1f} us (ours) / +{dxb:.1f} us (hipBLASLt at K=1024 vs ours at 512), "
          f"dW +{dw:.1f} us, against one apply pass of ~70 us alone (DESIGN.md section 8: 402 MB at 5.9 TB/s)")


if __name__ == "__main__":
    main()
