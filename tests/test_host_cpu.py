"""CPU-only tests of the host side: the C-ABI library loads and exports every
symbol include/dcnr.h declares (no compute calls), shape/workspace queries,
module construction parity with the reference (state_dict keys, shapes and
initial weights), and loud failure without a HIP device."""
import os
import re

import numpy as np
import pytest
import torch

import golden_common as gc
from conftest import ROOT, golden
from helpers import check_checksums, our_model


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "dcnr.h")).read()
    return sorted(set(re.findall(r"\b(dcnr_[a-z0-9_]+)\s*\(", txt)) - {"dcnr_allreduce_fn"})


def test_library_exports_header_symbols():
    from dcnr import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f"libdcnr.so does not export {s}"
    assert sorted(_lib.exported_symbols()) == syms
    assert lib.dcnr_abi_version() == _lib.ABI_VERSION == 4


def test_input_dim_and_workspace_queries():
    import dcnr
    m = our_model(gc.CFG3R)
    lib = dcnr._lib.load()
    import ctypes
    desc = m.desc()
    assert lib.dcnr_input_dim(ctypes.byref(desc)) == 456
    ev = m.workspace_bytes(131072, 0)
    tr = m.workspace_bytes(131072, 1)
    assert 0 < ev < tr
    # train workspace holds >= 3 activations per res block + x0 (bf16 halves it)
    mb = our_model(gc.CFG3R, precision="bf16")
    assert mb.workspace_bytes(131072, 1) < tr
    assert m.workspace_bytes(0, 0) >= 0 and m.workspace_bytes(1, 1) > 0


def test_size_queries_take_empty_shapes():
    """The host-only size queries at zero / tiny shapes (no queries, no rows,
    a table of k rows) return instead of dividing by zero."""
    from dcnr import _lib
    lib = _lib.load()
    for N, Q, k in [(11, 0, 11), (0, 5, 11), (0, 0, 1), (11, 2, 11), (1, 1, 1), (65537, 33, 64)]:
        assert lib.dcnr_cosine_topk_workspace_size(N, Q, k) >= 0
    assert lib.dcnr_cosine_topk_workspace_size(1_000_000, 256, 11) > lib.dcnr_cosine_topk_workspace_size(
        1_000_000, 1, 11)
    for N, K, B in [(0, 64, 100), (64, 0, 100), (64, 64, 0), (256, 256, 131072)]:
        assert lib.dcnr_linear_wgrad_workspace_size(N, K, B) >= 0
    assert lib.dcnr_linear_wgrad_workspace_size(256, 256, 131072) > 0


@pytest.mark.parametrize("fname,cfg", [("f1_cfg1_eval.npz", gc.CFG1), ("f3_cfg3r_train.npz", gc.CFG3R),
                                       ("f3b_odd_train.npz", gc.CFG_ODD)])
def test_same_init_and_state_dict_as_reference(fname, cfg):
    check_checksums(our_model(cfg), golden(fname))


def test_width_rule_matches_reference():
    import dcnr
    fx = golden("f5_width_rule.npz")
    for n, w in zip(fx["n"], fx["width"]):
        m = dcnr.DCN_RecSys(3, 3, {"a": int(n)}, 1, dict(emb_dim=4, hidden_dim=8, n_cross_layers=1,
                                                          n_res_blocks=1, dropout=0.0))
        assert m.cat_embeddings[0].weight.shape[1] == w
        import ctypes
        desc = m.desc()
        assert m._dims["input_dim"] == 8 + w + 1
        assert dcnr._lib.load().dcnr_input_dim(ctypes.byref(desc)) == 8 + w + 1


def test_cpu_model_raises():
    import dcnr
    cfg = gc.CFG_ODD
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]))
    u, i, c, n, _ = gc.make_inputs(cfg, 4, 3)
    with pytest.raises(RuntimeError):
        m(*[torch.from_numpy(a) for a in (u, i, c, n)])


def test_bad_precision_rejected():
    import dcnr
    with pytest.raises(ValueError):
        dcnr.DCN_RecSys(3, 3, {}, 1, dict(emb_dim=4, hidden_dim=8, n_cross_layers=1, dropout=0.0),
                        precision="fp8")


def test_state_dict_file_roundtrip_and_flat_views(tmp_path):
    """On-disk compatibility: the reference saves
    ``model.state_dict()`` with torch.save (train.py:391) and main.py loads it
    with load_state_dict (main.py:264); item_embeddings.npy is the item table
    (train.py:393-394).  Our module round-trips the same file format, also
    after FusedTrainer moved the parameters into its flat buffer."""
    import numpy as np
    import torch
    import dcnr
    cfg = gc.CFG1
    a = our_model(cfg)
    path = tmp_path / "final_dcn_model.pth"
    torch.save(a.state_dict(), path)
    b = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]))
    tr = dcnr.FusedTrainer(b, lr=1e-3)          # parameters now views of tr.flat
    b.load_state_dict(torch.load(path, weights_only=True))
    for (k, x), (k2, y) in zip(a.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(x, y), k
    # the loaded values live in the trainer's flat buffer
    w = b.final_linear.weight
    off = (w.data_ptr() - tr.flat.data_ptr()) // 4
    assert torch.equal(tr.flat[off:off + w.numel()], w.reshape(-1))
    np.save(tmp_path / "item_embeddings.npy", b.item_embedding.weight.detach().numpy())
    emb = np.load(tmp_path / "item_embeddings.npy")
    assert emb.shape == (cfg["n_items"], cfg["params"]["emb_dim"]) and emb.dtype == np.float32


def test_device_loader_permutation_is_dataloaders():
    """DeviceLoader's epoch order is the reference DataLoader(shuffle=True)'s
    (train.py:195-196) for the same global seed state."""
    import torch
    from torch.utils.data import DataLoader, TensorDataset
    from dcnr.data import randomsampler_permutation
    n = 1000
    for seed in (0, 7):
        torch.manual_seed(seed)
        ref = torch.cat([b[0] for b in DataLoader(TensorDataset(torch.arange(n)), batch_size=64,
                                                  shuffle=True)])
        torch.manual_seed(seed)
        assert torch.equal(randomsampler_permutation(n), ref)


def test_reference_artifacts_load_cpu():
    """F9 (written by the reference's own DCN_RecSys + train.py:391-394's
    torch.save/np.save): a weights-only load fills our model's state_dict
    exactly (same keys, shapes, values), and item_embeddings.npy is the item
    table; save_artifacts writes files the same loaders read back."""
    import os
    import tempfile
    import golden_common as gc
    import dcnr
    d = os.path.join(os.path.dirname(__file__), "golden", "f9_artifacts")
    sd = torch.load(os.path.join(d, "final_dcn_model.pth"), map_location="cpu", weights_only=True)
    torch.manual_seed(0)
    m = dcnr.DCN_RecSys(gc.CFG1["n_users"], gc.CFG1["n_items"], gc.CFG1["cat_dims"],
                        gc.CFG1["n_num"], dict(gc.CFG1["params"]))
    assert list(sd.keys()) == list(m.state_dict().keys())
    m.load_state_dict(sd)
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "f1_cfg1_eval.npz"))
    ck = gc.state_checksums(m)
    np.testing.assert_allclose(np.stack([ck[k] for k in fx["ck_names"]]), fx["ck"], rtol=1e-12,
                               atol=1e-9)
    emb = np.load(os.path.join(d, "item_embeddings.npy"), allow_pickle=False)
    assert np.array_equal(emb, m.item_embedding.weight.detach().numpy())
    with tempfile.TemporaryDirectory() as t:
        dcnr.artifacts.save_artifacts(m, t)
        sd2 = torch.load(os.path.join(t, "final_dcn_model.pth"), weights_only=True)
        assert all(torch.equal(sd2[k], v) for k, v in sd.items())
        assert np.array_equal(np.load(os.path.join(t, "item_embeddings.npy")), emb)


def test_model_copies_and_pickles():
    """deepcopy / pickle of the module (the reference's torch.save-of-model
    and copy idioms): the copy has its own (empty) id-check watch and equal
    parameters."""
    import copy
    import pickle
    m = our_model(gc.CFG1)
    for c in (copy.deepcopy(m), pickle.loads(pickle.dumps(m))):
        assert c._index_watch is not m._index_watch and c._index_watch.pending == []
        for (k, a), (_, b) in zip(m.state_dict().items(), c.state_dict().items()):
            assert torch.equal(a, b), k


def test_workspace_query_huge_table():
    """A table of more than 2^24 rows sizes its workspace for the radix-sort
    path (embed_bwd.hip) instead of failing."""
    import dcnr
    cfg = dict(gc.CFG1, n_users=(1 << 24) + 3)
    m = our_model(cfg, precision="bf16")
    assert m.workspace_bytes(4096, 1) > m.workspace_bytes(4096, 0) > 0


def test_index_error_watch_ring():
    """The deferred id-check ring (dcnr.model.IndexErrorWatch): a reserved
    slot reads PENDING (-1) until the device stores the call's word; a
    completed 0 frees the slot, a nonzero word raises IndexError on the next
    poll, and at DEPTH calls in flight the oldest is waited for.  (The ring
    is pinned host memory on a GPU box; a plain host tensor here, written by
    the test where the forward's last kernel would.)"""
    from dcnr.model import IndexErrorWatch
    w = IndexErrorWatch()
    w.ring = torch.zeros(IndexErrorWatch.RING, dtype=torch.int32)
    w.view = w.ring.numpy()
    slots = []
    for _ in range(3):
        s, ptr = w.reserve()
        assert w.view[s] == IndexErrorWatch.PENDING and ptr == w.ring.data_ptr() + 4 * s
        w.commit(s)
        slots.append(s)
    assert len(set(slots)) == 3
    w.poll()                                   # nothing finished: all kept
    assert w.pending == slots
    w.view[slots[0]] = 0
    w.view[slots[1]] = 0
    w.poll()
    assert w.pending == [slots[2]] and slots[0] in w.free
    w.view[slots[2]] = 1                       # an out-of-range id in that call
    with pytest.raises(IndexError):
        w.poll()
    assert w.pending == []
    # a failed call gives its slot back
    s, _ = w.reserve()
    w.cancel(s)
    assert s in w.free
    # DEPTH calls in flight: the next reserve waits for the oldest
    held = []
    for _ in range(IndexErrorWatch.DEPTH):
        s, _ = w.reserve()
        w.view[s] = 0                          # (already finished)
        w.commit(s)
        held.append(s)
    s, _ = w.reserve()
    assert held[0] not in w.pending and s is not None


def test_index_error_watch_orphans_and_dead_writer():
    """(1) a slot whose call drained its stream without storing
    the word (the writer never ran: a sticky error, a failed launch after
    commit) raises RuntimeError instead of spinning forever, and the slot
    returns to the ring; a stream error raised by the query propagates.
    (2) Slots still PENDING when an IndexError drops the pending list become
    orphans and return to the ring once their word lands, so repeated bad ids
    never exhaust the 64-slot ring."""
    from dcnr.model import IndexErrorWatch

    class FakeStream:
        def __init__(self, idle=True, err=None):
            self.idle, self.err = idle, err

        def query(self):
            if self.err:
                raise RuntimeError(self.err)
            return self.idle

    w = IndexErrorWatch()
    w.SPIN_S = 1e-4
    w.ring = torch.zeros(IndexErrorWatch.RING, dtype=torch.int32)
    w.view = w.ring.numpy()
    n_free = len(w.free)
    s, _ = w.reserve()
    w.commit(s, FakeStream(idle=True))         # drained, word never stored
    with pytest.raises(RuntimeError, match="never stored"):
        w.poll(all_=True)
    assert w.pending == [] and s in w.free and len(w.free) == n_free
    s, _ = w.reserve()
    w.commit(s, FakeStream(err="hipErrorLaunchFailure"))
    with pytest.raises(RuntimeError, match="LaunchFailure"):
        w.poll(all_=True)
    w.cancel(w.pending.pop())                  # (the caller's cleanup)
    # orphans: a bad word drops two later calls still in flight
    a, _ = w.reserve(); w.commit(a, FakeStream(idle=False))
    b, _ = w.reserve(); w.commit(b, FakeStream(idle=False))
    c, _ = w.reserve(); w.commit(c, FakeStream(idle=False))
    w.view[a] = 1
    with pytest.raises(IndexError):
        w.poll()
    assert w.pending == [] and sorted(w.orphans) == sorted([b, c])
    assert b not in w.free and c not in w.free
    w.view[b] = 0                              # b's late store lands
    w.poll()
    assert b in w.free and w.orphans == [c]
    w.view[c] = 0
    w.poll()
    assert w.orphans == [] and c in w.free
    # many bad calls never leak slots
    for _ in range(3 * IndexErrorWatch.RING):
        x, _ = w.reserve(); w.commit(x, FakeStream(idle=False))
        y, _ = w.reserve(); w.commit(y, FakeStream(idle=False))
        w.view[x] = 1
        with pytest.raises(IndexError):
            w.poll()
        w.view[y] = 0
    w.poll()
    assert len(w.free) + len(w.orphans) + len(w.pending) == IndexErrorWatch.RING
    assert w.orphans == []


def test_row_map_workspace_is_last():
    """DCNR_FLAG_ROW_MAP (ABI 4) appends a byte per table row to the train
    workspace and moves nothing else: every other stored tensor keeps its
    offset; eval and flag-less train workspaces have no map."""
    from dcnr import _lib
    m = our_model(gc.CFG3R, precision="bf16")
    B = 1024
    F = _lib.FLAG_ROW_MAP
    rows = gc.CFG3R["n_users"] + gc.CFG3R["n_items"] + sum(gc.CFG3R["cat_dims"].values())
    assert m.workspace_offset(B, _lib.TRAIN, "row_map") == -1
    assert m.workspace_offset(B, _lib.EVAL, "row_map", extra_flags=F) == -1
    off = m.workspace_offset(B, _lib.TRAIN, "row_map", extra_flags=F)
    assert off > 0
    assert m.workspace_bytes(B, _lib.TRAIN, F) >= off + rows
    assert m.workspace_bytes(B, _lib.TRAIN, F) - m.workspace_bytes(B, _lib.TRAIN) >= rows
    for kind in _lib.WS_KINDS[:-1]:
        for idx in (0, 1):
            assert m.workspace_offset(B, _lib.TRAIN, kind, idx) == \
                m.workspace_offset(B, _lib.TRAIN, kind, idx, extra_flags=F), kind
