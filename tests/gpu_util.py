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


def hip_runtime():
    """The HIP runtime this process already uses (torch's, which libftar binds to: ftar/__init__.py)."""
    import ctypes

    import ftar  # noqa: F401  (loads torch first, then libftar)
    return ctypes.CDLL("libamdhip64.so.7")


def poison_exchange(comm, byte=0xFF):
    """Fill this rank's own exchange buffer with `byte` (0xFF: NaN in fp32 and bf16) and wait for it.  The
    caller makes sure no peer reads it meanwhile (a barrier on each side)."""
    import ctypes
    ptr, nbytes = comm.exchange_buffer(comm.rank)
    if not ptr:
        return 0
    hip = hip_runtime()
    assert hip.hipMemset(ctypes.c_void_p(ptr), ctypes.c_int(byte), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0
    return nbytes


def exchange_fingerprints(comm, page=2 << 20, chunk=256 << 20):
    """Per rank q, the sums (int64, wrapping) of every `page` bytes of q's exchange buffer as THIS process
    maps it: rank r's list for q equals rank q's list for itself exactly when r's mapping of q's buffer shows
    q's memory page for page (at the time both read it, with no writer in between)."""
    import ctypes

    import torch
    hip = hip_runtime()
    out = []
    buf = None
    for q in range(comm.nranks):
        ptr, nbytes = comm.exchange_buffer(q)
        sums = []
        for lo in range(0, nbytes, chunk):
            n = min(chunk, nbytes - lo)
            if buf is None:
                buf = torch.empty(chunk, dtype=torch.uint8, device="cuda")
            assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ptr + lo), ctypes.c_size_t(n), 3) == 0
            whole = n // page * page
            if whole:
                sums += buf[:whole].view(torch.int64).view(-1, page // 8).sum(1).cpu().tolist()
            if n > whole:
                tail = buf[whole:n]
                sums.append(int(tail[:len(tail) // 8 * 8].view(torch.int64).sum().item()) ^ int(tail.sum().item()))
        out.append(sums)
    return out
