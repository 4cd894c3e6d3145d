"""numpy model of the gather wire format (csrc/wire.hip), for the CPU tests: the same
exact rebuild test, no fast filter.  Test infrastructure only: the product's pack and
unpack are the HIP kernels (engine.wire_pack / wire_unpack)."""
import numpy as np


def pack(mz, it, cmax):
    """(M f32, I f32, C int64): the smallest c <= cmax whose f32(x * c) divides back to
    exactly x for both values (C = 0: none)."""
    n = len(mz)
    M = np.zeros(n, np.float32)
    I = np.full(n, np.nan, np.float32)
    C = np.zeros(n, np.int64)
    mnan = np.isnan(mz)
    for c in range(1, cmax + 1):
        todo = C == 0
        if not todo.any():
            break
        with np.errstate(over="ignore", invalid="ignore"):
            Mc = np.where(mnan, 0.0, mz * c).astype(np.float32)
            Ic = (it * c).astype(np.float32)
            okm = mnan | ((Mc != 0) & (Mc.astype(np.float64) / c == mz))
            oki = Ic.astype(np.float64) / c == it
        ok = todo & okm & oki
        M[ok], I[ok], C[ok] = Mc[ok], Ic[ok], c
    return M, I, C


def unpack(M, I, C):
    c = np.maximum(C, 1).astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(M == 0, np.nan, M.astype(np.float64) / c), I.astype(np.float64) / c


def torch_ops():
    """(pack, unpack) with engine.wire_pack / wire_unpack's signatures on CPU tensors."""
    import torch

    def wpack(mz, it, max_count, stream=None, mi=None, cnt=None, n_fail=None):
        M, I, C = pack(mz.numpy(), it.numpy(), max_count)
        if n_fail is None:
            n_fail = torch.zeros(1, dtype=torch.int32)
        n_fail += int((C == 0).sum())
        dt = np.uint8 if max_count <= 255 else np.int16
        return (torch.from_numpy(np.stack([M, I], 1).ravel().copy()), torch.from_numpy(C.astype(dt)), n_fail)

    def wunpack(mi, cnt, mz, inten, stream=None):
        a = mi.numpy()
        c = cnt.numpy().astype(np.uint16).astype(np.int64)
        m, i = unpack(a[0::2], a[1::2], c)
        mz[:len(m)] = torch.from_numpy(m)
        inten[:len(i)] = torch.from_numpy(i)
        return mz, inten

    return wpack, wunpack
