"""Device-buffer helpers for the -m gpu tests (torch is only the allocator here)."""
import numpy as np


def torch_mod():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def to_dev(x, pad_elems=0, offset_elems=0):
    """Copy numpy array x to a fresh device buffer; returns (tensor, ptr of x's first element).

    offset_elems shifts the data inside the allocation (to test unaligned pointers)."""
    torch = torch_mod()
    x = np.ascontiguousarray(x)
    esz = x.dtype.itemsize
    total = (x.size + pad_elems + offset_elems) * esz
    t = torch.empty(max(1, total), dtype=torch.uint8, device="cuda")
    if x.size:
        t[offset_elems * esz: offset_elems * esz + x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
    return t, t.data_ptr() + offset_elems * esz


def from_dev(t, dtype, n, offset_elems=0):
    esz = np.dtype(dtype).itemsize
    torch_mod().cuda.synchronize()
    raw = t[offset_elems * esz: offset_elems * esz + n * esz].cpu().numpy()
    return raw.view(dtype)


def filled_dev(nbytes, byte=0xA5):
    torch = torch_mod()
    t = torch.full((max(1, nbytes),), byte, dtype=torch.uint8, device="cuda")
    return t, t.data_ptr()
