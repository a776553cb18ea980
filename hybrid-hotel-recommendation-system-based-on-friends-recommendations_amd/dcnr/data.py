"""Device-resident replacement for the reference's training input pipeline
(train.py:195-196)::

    train_ds = TensorDataset(X_train_collab, X_train_cat, X_train_num, y_train)
    train_dl = DataLoader(train_ds, batch_size=params['batch_size'], shuffle=True)

``DeviceLoader`` keeps the four tensors in HBM and assembles each batch with
one launch (dcnr_gather_rows) instead of ``default_collate`` stacking rows on
the host and copying every batch over PCIe.  Batch composition is the
reference's: every epoch draws the permutation exactly as torch's
``RandomSampler`` does (a seed from the default CPU generator, then
``torch.randperm`` with it), batches of ``batch_size`` in permutation order,
the last one partial (``drop_last=False``); ``shuffle=False`` is the
sequential order.  Iterating yields the same ``(collab, cat, num, y)`` tuples
the reference's loop unpacks (train.py:219).
"""
from __future__ import annotations

import ctypes
from typing import Iterator, Optional, Tuple

import torch

from . import _lib


def randomsampler_permutation(n: int, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """The index order a DataLoader(shuffle=True) epoch yields: its iterator
    first draws the workers' base seed from ``generator`` (default: the global
    CPU generator), then RandomSampler (replacement=False) seeds a fresh CPU
    generator from the default one (when none is given) and takes
    torch.randperm(n)."""
    torch.empty((), dtype=torch.int64).random_(generator=generator)   # _base_seed
    if generator is None:
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        generator = torch.Generator()
        generator.manual_seed(seed)
    return torch.randperm(n, generator=generator)


class DeviceLoader:
    def __init__(self, collab, cat, num, y, batch_size: int = 1, shuffle: bool = False,
                 generator: Optional[torch.Generator] = None, device='cuda'):
        dev = torch.device(device)
        if dev.type != 'cuda':
            raise RuntimeError("DeviceLoader keeps the dataset on the HIP device")
        self.tensors = [torch.as_tensor(t).to(dev).contiguous() for t in (collab, cat, num, y)]
        n = self.tensors[0].shape[0]
        if any(t.shape[0] != n for t in self.tensors):
            raise ValueError("Size mismatch between tensors")
        if batch_size < 1:
            raise ValueError("batch_size should be a positive integer")
        self.n, self.batch_size, self.shuffle, self.generator = n, batch_size, shuffle, generator
        self.device = dev
        self._row_bytes = (ctypes.c_int64 * 4)(*[
            t.element_size() * (t[0].numel() if t.dim() > 1 else 1) for t in self.tensors])

    def __len__(self):
        return (self.n + self.batch_size - 1) // self.batch_size

    def _gather(self, idx: torch.Tensor):
        lib = _lib.load()
        B = idx.numel()
        out = [torch.empty((B,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
               for t in self.tensors]
        if B:
            _lib.check(lib.dcnr_gather_rows(idx.data_ptr(), B, self.n, 4,
                                            _lib.ptr_array(self.tensors), _lib.ptr_array(out),
                                            self._row_bytes, _lib.stream_ptr(self.device)),
                       "dcnr_gather_rows")
        return tuple(out)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, ...]]:
        if self.shuffle:
            perm = randomsampler_permutation(self.n, self.generator).to(self.device)
        else:   # the DataLoader iterator still draws its base seed
            torch.empty((), dtype=torch.int64).random_(generator=self.generator)
            perm = torch.arange(self.n, device=self.device)
        for s in range(0, self.n, self.batch_size):
            yield self._gather(perm[s:s + self.batch_size])
