"""The stable key sort behind every order the ops define (csrc/primitives.hpp
radix_sort_pairs, o3dml_sort_pairs): (key, index) pairs vs numpy's stable
argsort of the masked keys, bit-exact, for the one-workgroup sorts (LSD radix
and bitonic, n <= 8,192) and the multi-workgroup passes; keys with a few
varying bits per field (the SparseConvUnet grid keys), heavy duplicates, full
64-bit keys, masked end bits and payloads."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sort(keys, vals, end_bit, kind):
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle, workspace
    dev = keys.device
    lib = _lib.load()
    kb = keys.element_size()
    n = keys.shape[0]
    ko = torch.empty_like(keys)
    vo = torch.empty(n, dtype=torch.int32, device=dev)
    ws = workspace(lib.o3dml_sort_pairs_workspace_size(n, kb), dev)
    _lib.call("o3dml_sort_pairs", ptr(keys), ptr(vals), ptr(ko), ptr(vo), n, kb, end_bit, kind, ptr(ws), ws.numel(),
              stream_handle(dev))
    return ko, vo


def _keys(kind, n, rng, bits):
    if kind == "grid":  # three 20-bit fields, ~8 varying bits each (calculate_grid keys)
        x, y, z = (rng.integers(100, 360, n) for _ in range(3))
        return (x.astype(np.uint64) << 40) | (y.astype(np.uint64) << 20) | z.astype(np.uint64)
    if kind == "dup":  # heavy duplicates
        return rng.integers(0, 7, n).astype(np.uint64) << np.uint64(bits - 3)
    if kind == "const":
        return np.full(n, 12345, np.uint64)
    return rng.integers(0, 2 ** 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)


@pytest.mark.parametrize("n", [1, 2, 63, 1000, 1024, 1025, 3000, 4097, 8192, 8193, 30000])
@pytest.mark.parametrize("kb", [4, 8])
@pytest.mark.parametrize("kind", ["grid", "dup", "const", "full"])
def test_sort_pairs_matches_stable_argsort(cuda, n, kb, kind):
    rng = np.random.default_rng(n * 31 + kb * 7 + len(kind))
    bits = 8 * kb
    k = _keys(kind, n, rng, bits)
    if kb == 4:
        k = (k ^ (k >> np.uint64(32))) & np.uint64(0xFFFFFFFF) if kind in ("full", "grid") else k & np.uint64(0xFFFFFFFF)
        k = k.astype(np.uint32)
    end_bits = [bits, bits - 5] if kind == "full" else [bits]
    payload = torch.from_numpy(rng.permutation(n).astype(np.int32)).to(cuda)
    k0 = k
    for end_bit in end_bits:  # keys < 2^end_bit (the ABI's contract)
        mask = np.uint64((1 << end_bit) - 1) if kb == 8 else np.uint32((1 << end_bit) - 1)
        k = k0 & mask
        kt = torch.from_numpy(k.view(np.int64 if kb == 8 else np.int32)).to(cuda)
        order = np.argsort(k, kind="stable")
        for small in (0, 1):
            for vals in (None, payload):
                ko, vo = _sort(kt, vals, end_bit, small)
                got_k = ko.cpu().numpy().view(k.dtype)
                assert np.array_equal(got_k, k[order]), (end_bit, small)
                want_v = order.astype(np.int32) if vals is None else payload.cpu().numpy()[order]
                assert np.array_equal(vo.cpu().numpy(), want_v), (end_bit, small)
