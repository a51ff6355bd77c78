"""CPU checks of the C ABI: the library exists, loads, and exports every symbol
include/o3dml_amd.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "o3dml_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(o3dml_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding():
    from o3dml_amd import _lib
    assert sorted(_lib.exported_symbols()) == declared_symbols()


def test_library_loads_and_exports_all():
    from o3dml_amd import _lib
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.o3dml_version() >= 1


def test_hash_table_splits_host_helper():
    import numpy as np
    from o3dml_amd import _lib
    import oracle as O
    rs = np.array([0, 10, 10, 5000, 70000], np.int64)
    a = np.zeros(5, np.uint32)
    t = _lib.load().o3dml_hash_table_splits(4, rs.ctypes.data, 1 / 64, 33554432, a.ctypes.data)
    b = np.zeros(5, np.uint32)
    t2 = O.lib().orc_hash_table_splits(ctypes.c_int64(4), rs.ctypes.data_as(ctypes.c_void_p),
                                       ctypes.c_double(1 / 64), ctypes.c_int64(33554432),
                                       b.ctypes.data_as(ctypes.c_void_p))
    assert t == t2 and np.array_equal(a, b)


def test_ops_fail_loudly_without_gpu():
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from o3dml_amd import ops
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        ops.fixed_radius_search(torch.zeros(4, 3), torch.zeros(4, 3), 0.1)


def test_layer_paths_fail_loudly_without_gpu():
    """The one-call layer path and the collate's dense path have no CPU
    fallback either."""
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from o3dml_amd import layers
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        layers.FixedRadiusSearch()(torch.zeros(4, 3), torch.zeros(4, 3), 0.1)


def test_layer_workspace_sizes():
    """o3dml_fixed_radius_search_layer_workspace_size covers the count
    workspace and the table build's scratch (host-only helper)."""
    from o3dml_amd import _lib
    lib = _lib.load()
    for n, m, b in ((65536, 65536, 1), (4194304, 4194304, 64), (1000, 10, 3)):
        t = max(b, n // 64)
        lay = lib.o3dml_fixed_radius_search_layer_workspace_size(n, m, b, t)
        assert lay >= lib.o3dml_fixed_radius_search_workspace_size(n, m, b)
        assert lay >= lib.o3dml_build_spatial_hash_table_workspace_size(n, t)


def test_workspace_size_caches_are_bounded():
    """The per-shape workspace-size memos (BN, Linear+BN, rigid KPConv,
    sparse conv) are LRUs of bounded size: KPFCNN's per-step point counts
    would otherwise grow them for the whole run."""
    from o3dml_amd import batchnorm, kpconv, sparse_conv
    from o3dml_amd._util import SizeCache
    for c in (batchnorm._WS, batchnorm._LWS, kpconv._KWS, sparse_conv._FWS):
        assert isinstance(c, SizeCache) and c.cap <= 4096
    for n in range(1, 3000):
        batchnorm._WS(n, 64)
    assert len(batchnorm._WS) <= batchnorm._WS.cap
    assert batchnorm._WS(5, 64) == max(int(__import__("o3dml_amd")._lib.load().o3dml_batch_norm_workspace_size(5, 64)), 1)
