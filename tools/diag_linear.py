"""Sweep dcnr_linear_bf16 shapes vs torch (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import torch
from dcnr import _lib
dev = torch.device("cuda:0")
lib = _lib.load()
for M in (1000, 1024, 4096):
    for K in (456, 512, 64):
        for N in (512, 96):
            for f32 in (0, 1):
                g = torch.Generator(device=dev).manual_seed(1)
                X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
                W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
                b = torch.randn(N, device=dev, generator=g)
                C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
                _lib.check(lib.dcnr_linear_bf16(X.data_ptr(), K, M, K, W.data_ptr(), K, N, b.data_ptr(),
                                                C.data_ptr(), N, f32, _lib.stream_ptr(dev)), "lin")
                ref = X.float() @ W.float().T + b
                e = (C.float() - ref).abs()
                bad = (e > 0.05 * ref.abs().max()).nonzero()
                print(M, K, N, f32, "maxerr %.4f" % e.max().item(), "bad", bad.shape[0],
                      "rows", bad[:, 0].unique()[:8].tolist() if bad.numel() else [],
                      "cols", bad[:, 1].unique()[:8].tolist() if bad.numel() else [], flush=True)
