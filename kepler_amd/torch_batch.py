"""Device-resident batches via PyTorch (plumbing only: device memory + streams).

The engine's C ABI takes raw device pointers; torch tensors provide the HBM
allocations and the stream the kernel is launched on.  Unsigned arrays are
moved as same-width signed views (only the bytes matter).
"""

from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .accel import KaccInterval, make_interval

_VIEW = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}


def to_device(arrays: Dict[str, np.ndarray], device: str = "cuda") -> Dict[str, torch.Tensor]:
    out = {}
    for name, a in arrays.items():
        if a is None:
            continue
        a = np.ascontiguousarray(a)
        v = a.view(_VIEW.get(a.dtype, a.dtype))
        out[name] = torch.from_numpy(v).to(device, non_blocking=False)
    return out


def interval_from_tensors(tensors: Dict[str, torch.Tensor], sizes: dict, flags: int = 0) -> KaccInterval:
    return make_interval(tensors, sizes, flags, ptr=lambda t: t.data_ptr())


def current_stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream
