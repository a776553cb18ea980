"""Data-parallel step on the device (a world-2 DP step with
SyncBN equals the single-process step at the global batch).

Two ranks share cuda:0 over gloo (RCCL refuses two ranks on one device; the
exchange code is backend-agnostic: FusedTrainer pre-scales the BCE gradient
by 1/world and SUM-reduces the flat gradient, SyncBN sums each BatchNorm's
fp64 statistics buffer across ranks inside the native forward/backward).
Rank r trains on rows [r*B/2, (r+1)*B/2) of the batch the single process
trains on whole.  After one step the summed gradient, the logits, the BN
running statistics and the updated parameters must match the single-process
step (fp32 mode, dropout 0: the counter-based dropout mask is a function of
the local row index).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import golden_common as gc

pytestmark = pytest.mark.gpu

CFG = dict(n_users=3000, n_items=700, cat_dims={"a": 50, "b": 1000, "c": 7}, n_num=5,
           params=dict(emb_dim=16, hidden_dim=128, n_cross_layers=2, n_res_blocks=2,
                       dropout=0.0))
B = 2048


def _model(dev):
    import dcnr
    torch.manual_seed(5)
    m = dcnr.DCN_RecSys(CFG["n_users"], CFG["n_items"], CFG["cat_dims"], CFG["n_num"],
                        dict(CFG["params"]), precision="fp32")
    gc.perturb_state(m, 6)
    return m.to(dev)


def _batch(dev):
    u, i, c, n, y = gc.make_inputs(CFG, B, 123)
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (u, i, c, n, y)]


def _worker(rank, world, port, path, shard):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcnr
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        m = _model(dev)
        tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, sync_bn=True,
                               shard_optimizer=shard)
        seen = []
        hook = tr._on_grads_ready

        def spy(ctx, group, stream):   # the backward's gradient-group hook fired, in order
            seen.append(group)
            return hook(ctx, group, stream)
        tr._on_grads_ready = spy
        tr._grad_ready_cb = dcnr._lib.GRAD_READY_FN(spy)
        m.grad_ready = tr._grad_ready_cb
        lo, hi = rank * B // world, (rank + 1) * B // world
        batch = [t[lo:hi] for t in _batch(dev)]
        loss, z = tr.step(*batch, return_logits=True)
        torch.cuda.synchronize()
        assert seen == [dcnr._lib.GRADS_DENSE, dcnr._lib.GRADS_EMBEDDING], seen
        zs = [torch.empty_like(z) for _ in range(world)]
        dist.all_gather(zs, z.contiguous())
        if rank == 0:
            ref = torch.load(path, weights_only=True)
            zz = torch.cat(zs).cpu().double()
            assert (zz - ref["z"]).abs().max().item() <= 1e-5 * max(1.0, ref["z"].abs().max().item())
            names = [k for k, _ in m.named_parameters()]
            bad = []
            for k, p in m.named_parameters():   # the exchanged (summed) gradients
                a, b = p.grad.cpu().double().reshape(-1), ref["grads"][k].reshape(-1)
                if ".layer" in k and k.endswith(".bias"):    # BN-invariant: ~0
                    continue
                if shard and "embedding" in k:   # reduce-scattered into tr.gshard, not
                    continue                     # into p.grad: the params check covers it
                e = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
                if e > 1e-4:
                    bad.append((k, e))
            assert not bad, bad
            for k, v in m.state_dict().items():
                if k in ref["params"] and not (".layer" in k and k.endswith(".bias")):
                    # the AdamW step on the exchanged gradient: its first update is
                    # ~lr * sign(g), so an element whose summed gradient is pure
                    # rounding noise may move the other way -- allow 0.1 % of them
                    d = (v.cpu().double() - ref["params"][k].double()).abs()
                    frac = (d > 1e-6).double().mean().item()
                    assert frac <= 1e-3 and d.max().item() <= 2.5e-3, (k, frac)
                if "running" in k:
                    np.testing.assert_allclose(v.cpu().numpy(), ref["sd"][k].numpy(),
                                               rtol=1e-5, atol=1e-6, err_msg=k)
                if "num_batches_tracked" in k:
                    assert int(v) == int(ref["sd"][k]) == 1
            assert len(names) > 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shard", [False, True])
def test_dp_world2_syncbn_equals_single_process(dev, shard):
    """shard=True: the embedding segment goes through reduce-scatter -> shard
    AdamW -> all-gather, the dense segment's all-reduce is started by the
    backward's DCNR_GRADS_DENSE hook; shard=False: all-reduce of both."""
    import dcnr
    m = _model(dev)
    tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4)
    batch = _batch(dev)
    loss, z = tr.step(*batch, return_logits=True)
    torch.cuda.synchronize()
    ref = {"z": z.detach().cpu().double(),
           "grads": {k: p.grad.detach().cpu().double().clone() for k, p in m.named_parameters()},
           "params": {k: p.detach().cpu().clone() for k, p in m.named_parameters()},
           "sd": {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}}
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ref.pt")
        torch.save(ref, path)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.spawn(_worker, args=(2, port, path, shard), nprocs=2, join=True)
