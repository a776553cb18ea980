"""TEST / MEASUREMENT INFRASTRUCTURE ONLY -- never imported by the product
package.  bench.py's ``cpu_baseline`` leg times it on the GPU box's host
cores; tools/validate_cpu_baseline.py checks here that its step time is
within 10 % of the imported reference module's on the same workload.

A functional torch-CPU restatement of the reference's training step, op for
op in the reference's order (fp32, autograd, aten CPU kernels):

  forward   train.py:155-170   embeddings -> cat -> initial Linear ->
                               ResBlock x R (train.py:111-122: Linear, BN
                               (batch stats, momentum 0.1), ReLU, Dropout,
                               Linear, BN, += identity, ReLU) -> CrossLayer x L
                               (train.py:96-99: x + (x[:, :, None] @
                               w(x[:, None, :])) + b, the reference's batched
                               matmul form) -> cat -> final Linear -> squeeze
  loss      train.py:206, 224  BCEWithLogitsLoss (mean)
  backward  train.py:225       loss.backward() (dense embedding grads)
  optimizer train.py:201-202   torch.optim.AdamW(lr, weight_decay), zero_grad
                               (train.py:222) before the forward

Parameters are freshly initialised with the reference's module shapes
(nn.Embedding N(0,1), nn.Linear U(+-1/sqrt(fan_in)), BN gamma=1/beta=0);
values do not change the CPU cost of these dense ops.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List

import torch
import torch.nn.functional as F


def cat_width(n: int) -> int:
    """train.py:139: int(np.sqrt(n_cat)) + 1."""
    w = int(math.isqrt(n)) + 1
    return w


class TorchCPUStep:
    def __init__(self, n_users, n_items, cat_dims: List[int], n_num, emb_dim, hidden, n_cross,
                 n_res, dropout, lr=1e-3, weight_decay=1e-4, seed=0):
        g = torch.Generator().manual_seed(seed)
        D = 2 * emb_dim + sum(cat_width(n) for n in cat_dims) + n_num
        self.dropout = dropout
        self.n_res, self.n_cross = n_res, n_cross

        def lin(o, i, bias=True):
            b = 1.0 / math.sqrt(i)
            w = (torch.rand((o, i), generator=g) * 2 - 1) * b
            return [w.requires_grad_(), ((torch.rand(o, generator=g) * 2 - 1) * b).requires_grad_()] \
                if bias else [w.requires_grad_()]

        p: Dict[str, torch.Tensor] = {}
        p["user"] = torch.randn((n_users, emb_dim), generator=g).requires_grad_()
        p["item"] = torch.randn((n_items, emb_dim), generator=g).requires_grad_()
        self.cats = []
        for k, n in enumerate(cat_dims):
            p[f"cat{k}"] = torch.randn((n, cat_width(n)), generator=g).requires_grad_()
            self.cats.append(f"cat{k}")
        p["W0"], p["b0"] = lin(hidden, D)
        self.bn = []
        for j in range(n_res):
            for l in (1, 2):
                p[f"W{j}_{l}"], p[f"b{j}_{l}"] = lin(hidden, hidden)
                p[f"g{j}_{l}"] = torch.ones(hidden).requires_grad_()
                p[f"be{j}_{l}"] = torch.zeros(hidden).requires_grad_()
                self.bn.append([torch.zeros(hidden), torch.ones(hidden)])
        for l in range(n_cross):
            (p[f"cw{l}"],) = lin(1, D, bias=False)
            p[f"cb{l}"] = torch.zeros(D).requires_grad_()
        p["Wf"], p["bf"] = lin(1, hidden + D)
        self.p = p
        self.opt = torch.optim.AdamW(list(p.values()), lr=lr, weight_decay=weight_decay)

    def forward(self, user, item, cat, num, train=True):
        """train.py:155-170; train=False: eval semantics (running-stat BN,
        no dropout), the scoring call of main.py:319-322."""
        p = self.p
        embs = [F.embedding(user, p["user"]), F.embedding(item, p["item"])]
        embs += [F.embedding(cat[:, k], p[name]) for k, name in enumerate(self.cats)]
        x0 = torch.cat(embs + [num], dim=1)
        h = F.linear(x0, p["W0"], p["b0"])
        for j in range(self.n_res):
            rm1, rv1 = self.bn[2 * j]
            rm2, rv2 = self.bn[2 * j + 1]
            out = F.linear(h, p[f"W{j}_1"], p[f"b{j}_1"])
            out = F.batch_norm(out, rm1, rv1, p[f"g{j}_1"], p[f"be{j}_1"], train, 0.1, 1e-5)
            out = F.relu(out)
            out = F.dropout(out, self.dropout, train)
            out = F.linear(out, p[f"W{j}_2"], p[f"b{j}_2"])
            out = F.batch_norm(out, rm2, rv2, p[f"g{j}_2"], p[f"be{j}_2"], train, 0.1, 1e-5)
            out = out + h
            h = F.relu(out)
        x = x0
        for l in range(self.n_cross):
            xa, xt = x.unsqueeze(2), x.unsqueeze(1)
            x = xa.squeeze(2) + torch.matmul(xa, F.linear(xt, p[f"cw{l}"])).squeeze(2) + p[f"cb{l}"]
        return F.linear(torch.cat([h, x], dim=1), p["Wf"], p["bf"]).squeeze()

    def score(self, user, item, cat, num):
        """Eval-mode logits under no_grad (main.py:319-322)."""
        with torch.no_grad():
            return self.forward(user, item, cat, num, train=False)

    def step(self, user, item, cat, num, y):
        self.opt.zero_grad()
        z = self.forward(user, item, cat, num)
        loss = F.binary_cross_entropy_with_logits(z, y)
        loss.backward()
        self.opt.step()
        return float(loss.detach())


def make_cpu_batch(n_users, n_items, cat_dims, n_num, B, seed):
    g = torch.Generator().manual_seed(seed)
    user = torch.randint(0, n_users, (B,), generator=g)
    item = torch.randint(0, n_items, (B,), generator=g)
    cat = torch.stack([torch.randint(0, n, (B,), generator=g) for n in cat_dims], 1)
    num = torch.rand((B, n_num), generator=g)
    y = (torch.rand(B, generator=g) < 0.5).float()
    return user, item, cat, num, y


def time_steps(step_fn, batches, warmup=1):
    """Seconds per step over ``batches`` after ``warmup`` untimed steps."""
    for b in batches[:warmup]:
        step_fn(*b)
    t0 = time.perf_counter()
    for b in batches[warmup:]:
        step_fn(*b)
    return (time.perf_counter() - t0) / max(1, len(batches) - warmup)
