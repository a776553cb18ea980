"""Round-5 debug: dcnr_linear_bf16 (gemm_wsp at 256 < K <= 512) repeated on
fixed data with the output pre-filled with NaN: unwritten or nondeterministic
elements, by row / column pattern."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import torch
from dcnr import _lib

dev = torch.device("cuda")
lib = _lib.load()
for (M, K, N) in [(16384, 456, 256), (32768, 456, 256), (131072, 512, 512), (16384, 512, 512), (1000, 456, 512)]:
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g)
    ref = None
    bad = 0
    for it in range(12):
        C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        _lib.check(lib.dcnr_linear_bf16(X.data_ptr(), K, M, K, W.data_ptr(), K, N, b.data_ptr(),
                                        C.data_ptr(), N, 0, _lib.stream_ptr(dev)), "linear")
        torch.cuda.synchronize()
        nan = torch.isnan(C.float())
        if ref is None:
            ref = C.clone()
            r = torch.addmm(b, X.float(), W.float().t())
            err = ((C.float() - r).norm() / r.norm()).item()
            print(f"M={M} K={K} N={N}: rel err vs torch {err:.3e}, NaN {int(nan.sum())}")
        diff = (C != ref) & ~(torch.isnan(C.float()) & torch.isnan(ref.float()))
        nd = int(diff.sum())
        if nd or int(nan.sum()):
            bad += 1
            rows = torch.nonzero(diff.any(1)).flatten()
            cols = torch.nonzero(diff.any(0)).flatten()
            print(f"  it {it}: {nd} differ, NaN {int(nan.sum())}; rows {rows[:8].tolist()}.. ({rows.numel()}),"
                  f" cols {cols[:8].tolist()}.. ({cols.numel()}); row%32 {sorted(set((rows % 32).tolist()))[:12]}")
    print(f"  {bad} of 12 runs differ")
