"""ctypes binding of libsqr.so (the C ABI declared in include/sqr.h).

The library is built in-tree (``make -C sq-recovery_amd/csrc`` or ``__graft_entry__.build()``)
into this directory.  There is no fallback: if the library is missing, ``lib()`` raises, so a
GPU run can never silently take another code path.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (loads torch's libamdhip64 first; libsqr binds to that runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SQR_LIB", os.path.join(_HERE, "libsqr.so"))

_lock = threading.Lock()
_lib = None

c_int, c_float, c_double, c_size_t, c_void_p = (ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                                ctypes.c_size_t, ctypes.c_void_p)


class SqrConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("N", "C", "H", "W", "K", "R", "S", "stride", "pad", "dtype")]


class SqrPackJob(ctypes.Structure):
    _fields_ = [("w_kcrs", c_void_p), ("desc", SqrConvDesc), ("w_krsc", c_void_p), ("w_crsk", c_void_p)]


class SqrBnOperand(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("stats", c_void_p), ("stats_rows", c_int), ("gamma", c_void_p), ("beta", c_void_p),
                ("running_mean", c_void_p), ("running_var", c_void_p), ("momentum", c_float), ("eps", c_float),
                ("save_mean", c_void_p), ("save_invstd", c_void_p)]


class SqrBnBwdFin(ctypes.Structure):
    _fields_ = [("stats", c_void_p), ("stats_rows", c_int), ("M", ctypes.c_longlong), ("C", c_int),
                ("gamma", c_void_p), ("save_mean", c_void_p), ("save_invstd", c_void_p), ("dgamma", c_void_p),
                ("dbeta", c_void_p), ("coef", c_void_p)]


class SqrBnBwdRed(ctypes.Structure):
    _fields_ = [("kind", c_int), ("dy", c_void_p), ("relu_mask", c_void_p), ("x_a", c_void_p), ("mean_a", c_void_p),
                ("x_b", c_void_p), ("mean_b", c_void_p), ("M", ctypes.c_longlong), ("C", c_int), ("part", c_void_p),
                ("part_rows", ctypes.POINTER(c_int))]


class SqrTailDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("B", "P", "C0", "F1", "F2", "dtype")] + \
        [("w0", c_void_p), ("b0", c_void_p), ("w1", c_void_p), ("b1", c_void_p),
         ("wh", c_void_p * 4), ("bh", c_void_p * 4)]


class SqrTailGrads(ctypes.Structure):
    _fields_ = [("g_out", c_void_p * 4), ("ld", c_int * 4), ("dx", c_void_p), ("dw0", c_void_p),
                ("db0", c_void_p), ("dw1", c_void_p), ("db1", c_void_p), ("dwh", c_void_p * 4),
                ("dbh", c_void_p * 4)]


class SqrAdamParam(ctypes.Structure):
    _fields_ = [("p", c_void_p), ("g", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("step", c_void_p), ("n", ctypes.c_longlong), ("desc", SqrConvDesc), ("w_krsc", c_void_p),
                ("w_crsk", c_void_p)]


# name -> (restype, argtypes); must mirror include/sqr.h exactly
SIGNATURES = {
    "sqr_version": (c_int, []),
    "sqr_last_error_string": (ctypes.c_char_p, []),
    "sqr_probe_arm": (c_int, [c_void_p, c_void_p]),
    "sqr_probe_arm_clock": (c_int, [c_void_p]),
    "sqr_wall_clock_khz": (c_int, [ctypes.POINTER(c_int)]),
    "sqr_implicit_loss_workspace_bytes": (c_size_t, [c_int, c_int]),
    "sqr_implicit_loss_fwd_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float,
                                          c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_implicit_loss_fwd_bwd_mean": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float,
                                               c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_loss_grad_scale": (c_int, [c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_void_p]),
    "sqr_implicit_render": (c_int, [c_void_p, c_int, c_int, c_float, c_float, c_void_p, c_void_p]),
    "sqr_explicit_loss_workspace_bytes": (c_size_t, [c_int, c_int]),
    "sqr_explicit_loss_fwd_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                          c_void_p, c_size_t, c_void_p]),
    "sqr_explicit_loss_fwd_bwd_mean": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                               c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_iou_counts": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sqr_iou_counts_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sqr_conv2d_out_hw": (c_int, [ctypes.POINTER(SqrConvDesc), ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "sqr_conv2d_workspace_bytes": (c_size_t, [ctypes.POINTER(SqrConvDesc), c_int]),
    "sqr_conv2d_pack_weight": (c_int, [c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p, c_void_p, c_void_p]),
    "sqr_conv2d_pack_weights": (c_int, [ctypes.POINTER(SqrPackJob), c_int, c_void_p]),
    "sqr_conv2d_fwd": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p, c_size_t,
                               c_void_p]),
    "sqr_conv_set_direct": (c_int, [c_int]),
    "sqr_conv_set_deep_ring": (c_int, [c_int]),
    "sqr_conv2d_stats_floats": (c_size_t, [ctypes.POINTER(SqrConvDesc)]),
    "sqr_conv2d_fwd_stats": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p,
                                     ctypes.POINTER(c_int), c_void_p, c_size_t, c_void_p]),
    "sqr_conv2d_fwd_stats_bnin": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          ctypes.POINTER(SqrConvDesc), c_void_p, ctypes.POINTER(c_int), c_void_p]),
    "sqr_conv2d_bnin_nso_supported": (c_int, [ctypes.POINTER(SqrConvDesc)]),
    "sqr_bn_fwd_finalize": (c_int, [c_void_p, c_int, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sqr_bn_apply": (c_int, [c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                             c_void_p]),
    "sqr_conv2d_bwd_data": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p,
                                    c_size_t, c_void_p]),
    "sqr_conv2d_bwd_data_acc": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc),
                                        c_void_p, c_size_t, c_void_p]),
    "sqr_conv2d_bwd_data_acc_masked": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                ctypes.POINTER(SqrConvDesc), c_void_p, c_size_t, c_void_p]),
    "sqr_conv2d_bwd_data_acc_s2": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc),
                                           c_void_p, c_size_t, c_void_p]),
    "sqr_conv2d_bwd_data_bn_stats_floats": (c_size_t, [ctypes.POINTER(SqrConvDesc)]),
    "sqr_conv2d_bwd_data_bn": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       ctypes.POINTER(c_int), ctypes.POINTER(SqrConvDesc), c_void_p, c_size_t,
                                       c_void_p]),
    "sqr_conv2d_bwd_data_bn_act": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(SqrConvDesc), c_void_p]),
    "sqr_bn_bwd_stats": (c_int, [c_void_p, c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_int, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_conv2d_bwd_weight": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p,
                                      c_size_t, c_void_p]),
    "sqr_conv2d_bwd_weight_bn": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc),
                                         ctypes.POINTER(SqrBnBwdFin), ctypes.POINTER(SqrBnBwdRed), c_void_p, c_size_t,
                                         c_void_p]),
    "sqr_bn_bwd_red_doubles": (c_size_t, [ctypes.c_longlong, c_int, c_int]),
    "sqr_bn_bwd_part": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_int,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "sqr_bn_add_bwd_part": (c_int, [ctypes.POINTER(SqrBnOperand), ctypes.POINTER(SqrBnOperand), c_void_p, c_void_p,
                                    ctypes.c_longlong, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_bn_bwd_apply": (c_int, [c_void_p, c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sqr_conv2d_bwd_weight_col": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(SqrConvDesc), c_void_p,
                                          c_size_t, c_void_p]),
    "sqr_bn_workspace_bytes": (c_size_t, [ctypes.c_longlong, c_int]),
    "sqr_bn_add_workspace_bytes": (c_size_t, [ctypes.c_longlong, c_int]),
    "sqr_bn_add_fwd": (c_int, [ctypes.POINTER(SqrBnOperand), ctypes.POINTER(SqrBnOperand), ctypes.c_longlong, c_int,
                               c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_bn_add_bwd": (c_int, [ctypes.POINTER(SqrBnOperand), ctypes.POINTER(SqrBnOperand), c_void_p, c_void_p,
                               ctypes.c_longlong, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_bn_fwd": (c_int, [c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_float, c_float, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_size_t, c_void_p]),
    "sqr_bn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_bn_fwd_stats": (c_int, [c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_float, c_float, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_stem_fwd_stats": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "sqr_stem_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "sqr_stem_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                             c_void_p]),
    "sqr_stem_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_stem_fused_supported": (c_int, [c_int, c_int, c_int]),
    "sqr_stem_fused_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "sqr_stem_fused_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "sqr_stem_fused_bwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                   c_void_p]),
    "sqr_adam_step": (c_int, [ctypes.POINTER(SqrAdamParam), c_int, c_double, c_double, c_double, c_double,
                              c_double, c_void_p]),
    "sqr_adam_step_amp": (c_int, [ctypes.POINTER(SqrAdamParam), c_int, c_double, c_double, c_double, c_double,
                                  c_double, c_void_p, c_void_p, c_void_p]),
    "sqr_amp_check_finite": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_longlong), c_int, c_void_p,
                                     c_void_p]),
    "sqr_amp_check_finite_scaled": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_longlong), c_int,
                                            c_void_p, c_double, c_void_p, c_void_p]),
    "sqr_amp_update_scale": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_float, c_int, c_void_p]),
    "sqr_tail_save_floats": (c_size_t, [ctypes.POINTER(SqrTailDesc)]),
    "sqr_tail_fwd": (c_int, [ctypes.POINTER(SqrTailDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p]),
    "sqr_tail_fwd_packed": (c_int, [ctypes.POINTER(SqrTailDesc), c_void_p, c_void_p, c_void_p, c_void_p]),
    "sqr_tail_workspace_bytes": (c_size_t, [ctypes.POINTER(SqrTailDesc)]),
    "sqr_tail_bwd": (c_int, [ctypes.POINTER(SqrTailDesc), c_void_p, ctypes.POINTER(SqrTailGrads), c_void_p,
                             c_size_t, c_void_p]),
    "sqr_comm_load": (c_int, [ctypes.c_char_p, ctypes.POINTER(c_int)]),
    "sqr_comm_unique_id": (c_int, [c_void_p]),
    "sqr_comm_init_rank": (c_int, [ctypes.POINTER(c_void_p), c_void_p, c_int, c_int]),
    "sqr_comm_allreduce_sum_f32": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "sqr_comm_broadcast": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "sqr_comm_async_error": (c_int, [c_void_p]),
    "sqr_comm_destroy": (c_int, [c_void_p]),
    "sqr_comm_abort": (c_int, [c_void_p]),
    "sqr_comm_proxy": (c_int, [c_void_p, c_void_p, c_size_t, c_int, ctypes.c_double, c_void_p]),
}


class SqrError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle; raises if libsqr.so is absent or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise SqrError("libsqr.so not found at %s — build it with `make -C sq-recovery_amd/csrc` "
                           "(or __graft_entry__.build()); there is no fallback path" % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)  # AttributeError = library/header mismatch: fail loudly
            fn.restype = res
            fn.argtypes = args
        if os.environ.get("SQR_D3_DEEP") in ("0", "1"):  # A/B switch (sqr_conv_set_deep_ring)
            h.sqr_conv_set_deep_ring(int(os.environ["SQR_D3_DEEP"]))
        _lib = h
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().sqr_last_error_string().decode(errors="replace")
        raise SqrError("%s failed (code %d): %s" % (what, rc, msg))


def stream_ptr(device=None):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else c_void_p(0)
