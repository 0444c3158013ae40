"""The C-ABI library loads on a GPU-less host and exports every symbol include/ergm_hip.h declares."""
import ctypes
import os
import re

from ergm_amd import _lib as L

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ergm_hip.h")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ergm_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _declared() == L.EXPORTED


def test_library_loads_and_exports_everything():
    lib = L.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.ergm_version() == L.ABI_VERSION


def test_errors_are_reported_without_a_gpu():
    lib = L.load()
    d = L.GemmDesc(M=64, N=64, K=60, lda=60, ldb=60, ldc=64)
    rc = lib.ergm_gemm(ctypes.byref(d), None, None, None, None, 0, None)
    assert rc == L.ERGM_EINVAL
    assert "null" in L.last_error()


def test_workspace_queries_are_host_only():
    lib = L.load()
    dims = L.ModelDims(vocab=50260, vocab_pad=50304, n_embd=768, n_layer=12, n_head=12, n_inner=3072,
                       n_positions=1024, batch=16, seq=128, eps=1e-5, has_features=1, ld_vis=768)
    ws = lib.ergm_model_workspace_size(ctypes.byref(dims))
    # activations of GPT-2-small at B=16,S=128 fit comfortably in HBM (< 4 GB)
    assert 5e8 < ws < 4e9
    assert lib.ergm_embed_bwd_workspace_size(2048) >= 3 * 2048 * 8
