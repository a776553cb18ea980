"""Check that oracle/torch_cpu.py (the CPU baseline bench.py reports) costs
what the reference's own training step costs on the same host cores.

Build container only (imports /root/reference/train.py the way
tests/golden/make_golden.py does, optuna stubbed).  Times, at the bench's
model (1M x 32 users, 100k x 32 items, 12 x 1000 cat, 8 dense, 3 cross,
4 x 512, dropout 0.6) and batch B, the reference step of train.py:219-226
(zero_grad, forward, BCEWithLogitsLoss, backward, AdamW.step) with the
reference DCN_RecSys, and the same step with the restatement; prints both.

    python tools/validate_cpu_baseline.py [--batch 32768 --steps 3 --threads 8]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch_cpu as tc  # noqa: E402

CAT = [1000] * 12


def load_reference():
    sys.modules.setdefault("optuna", types.ModuleType("optuna"))
    spec = importlib.util.spec_from_file_location("ref_train", "/root/reference/train.py")
    mod = importlib.util.module_from_spec(spec)
    cwd = os.getcwd()
    os.chdir("/tmp")
    try:
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--rounds", type=int, default=2,
                    help="alternate reference / restatement this many times (order effects)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    B = args.batch
    batches = [tc.make_cpu_batch(1_000_000, 100_000, CAT, 8, B, s) for s in range(args.steps + 1)]

    ref = load_reference()
    params = dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4, dropout=0.6)
    loss_fn = torch.nn.BCEWithLogitsLoss()

    def time_reference():
        torch.manual_seed(42)
        m = ref.DCN_RecSys(1_000_000, 100_000, {f"c{k}": 1000 for k in range(12)}, 8, params)
        m.train()
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)

        def ref_step(u, i, c, n, y):   # train.py:219-226
            opt.zero_grad()
            loss = loss_fn(m(u, i, c, n), y.float())
            loss.backward()
            opt.step()
        return tc.time_steps(ref_step, batches)

    def time_port():
        port = tc.TorchCPUStep(1_000_000, 100_000, CAT, 8, 32, 512, 3, 4, 0.6)
        return tc.time_steps(port.step, batches)

    t_ref, t_port = [], []
    for r in range(args.rounds):
        if r % 2 == 0:
            t_ref.append(time_reference())
            t_port.append(time_port())
        else:
            t_port.append(time_port())
            t_ref.append(time_reference())
    t_ref, t_port = min(t_ref), min(t_port)
    print(f"threads={args.threads} batch={B} steps={args.steps} rounds={args.rounds} (best of)")
    print(f"reference train.py step : {t_ref * 1e3:9.1f} ms  {B / t_ref:10.0f} samples/s")
    print(f"oracle/torch_cpu.py step: {t_port * 1e3:9.1f} ms  {B / t_port:10.0f} samples/s")
    print(f"ratio restatement/reference time: {t_port / t_ref:.3f}")


if __name__ == "__main__":
    main()
