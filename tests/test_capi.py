"""The C-ABI library: it loads (no GPU needed) and exports every symbol include/sqr.h declares."""
import os
import re

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sqr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sqr_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("sqr_implicit_loss_fwd_bwd", "sqr_explicit_loss_fwd_bwd", "sqr_iou_counts", "sqr_conv2d_fwd",
              "sqr_conv2d_bwd_data", "sqr_conv2d_bwd_weight", "sqr_last_error_string"):
        assert s in syms


def test_library_loads_and_exports_all_symbols():
    from sqr import _lib
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert set(declared_symbols()) == set(_lib.SIGNATURES)
    assert L.sqr_version() >= 1


def test_argument_validation_without_gpu():
    # invalid arguments are rejected on the host before any HIP call
    from sqr import _lib
    L = _lib.lib()
    rc = L.sqr_implicit_loss_fwd_bwd(None, None, 0, 256, 256, 32, 1.0, 100.0, 1, None, None, None, 0, None)
    assert rc == -1
    assert b"B=0" in L.sqr_last_error_string()
    assert L.sqr_implicit_loss_workspace_bytes(4, 32) == 4 * 4 * 18 * 4
    # fused stem geometry: conv1 output tiles by 8 x 32 and the input rows are read as 4-pixel vectors
    assert L.sqr_stem_fused_supported(2, 256, 256) == 1
    assert L.sqr_stem_fused_supported(2, 512, 512) == 1
    assert L.sqr_stem_fused_supported(2, 64, 63) == 0  # conv1 width 32, but W % 4 != 0
    assert L.sqr_stem_fused_supported(2, 64, 96) == 0  # conv1 width 48


def test_comm_binds_torch_rccl_without_gpu():
    """sqr_comm_load binds the RCCL torch maps (no GPU needed for the version / unique id); the
    collective entry points reject a null communicator on the host."""
    import ctypes
    from sqr import _lib, dist
    L = _lib.lib()
    ver = ctypes.c_int(0)
    path = dist._torch_rccl_path()
    assert L.sqr_comm_load(path.encode() if path else None, ctypes.byref(ver)) == 0, L.sqr_last_error_string()
    assert ver.value >= 20000  # NCCL-style version code, e.g. 22606
    uid = (ctypes.c_ubyte * 128)()
    assert L.sqr_comm_unique_id(uid) == 0, L.sqr_last_error_string()
    assert any(bytes(uid))
    assert L.sqr_comm_allreduce_sum_f32(None, None, 0, None) == -1
    assert b"null communicator" in L.sqr_last_error_string()
    assert L.sqr_comm_destroy(None) == 0
