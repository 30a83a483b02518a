"""BatchNorm + ReLU applied on load by the persistent layer-1 conv (sqr_conv2d_fwd_stats_bnin:
bn1 -> relu -> conv2 of a BasicBlock, torch/models.py:181) against the two-pass path it replaces
(sqr_bn_apply, then sqr_conv2d_fwd_stats): the activation, its ReLU mask, the conv output and its
BatchNorm partials bitwise equal -- the same arithmetic on the same values, the zero padding left
alone -- at the config-2 (64 x 64 maps, B=64) and config-5 (128 x 128, B=16) shapes."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("N,H", [(64, 64), (16, 128), (2, 64), (1, 128)])
def test_conv_bnin_equals_apply_then_conv(N, H, dtype):
    from sqr import conv as sc
    from sqr._lib import check, lib, ptr, stream_ptr
    L = lib()
    g = torch.Generator(device=DEV).manual_seed(N * 7 + H)
    C = 64
    x_pre = (torch.randn(N, C, H, H, device=DEV, generator=g) * 2 + 0.3).to(dtype).contiguous(
        memory_format=torch.channels_last)
    coef = torch.cat([torch.randn(C, device=DEV, generator=g) * 0.8,      # scale (some negative)
                      torch.randn(C, device=DEV, generator=g) * 0.5])    # shift
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) / 24.0
    d = sc._desc(N, C, H, H, C, 3, 3, 1, 1, dtype)
    krsc, _ = sc.pack_weight(w, d, False)
    st = stream_ptr(torch.device(DEV))
    M = N * H * H
    # two passes: the BatchNorm apply, then the conv on its output
    a_ref = torch.empty_like(x_pre)
    m_ref = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    check(L.sqr_bn_apply(ptr(x_pre), ctypes.c_longlong(M), C, sc._DT[dtype], ptr(coef), None, 1, ptr(a_ref), ptr(m_ref),
                         st), "apply")
    y_ref, s_ref = sc.conv2d_fwd(a_ref, krsc, d, stats=True)
    # one pass: applied while staging
    a = torch.full_like(x_pre, float("nan"))
    m = torch.full((M * C // 8,), 0x5A, dtype=torch.uint8, device=DEV)
    y, s = sc.conv2d_fwd_bnin(x_pre, coef, a, m, krsc, d)
    torch.cuda.synchronize()
    assert torch.equal(a, a_ref)
    assert torch.equal(m, m_ref)
    assert torch.equal(y, y_ref)
    assert s.shape == s_ref.shape and torch.equal(s, s_ref)


def test_conv_bnin_declines_other_shapes():
    from sqr import conv as sc
    x = torch.zeros(2, 128, 32, 32, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d = sc._desc(2, 128, 32, 32, 128, 3, 3, 1, 1, torch.bfloat16)
    krsc, _ = sc.pack_weight(torch.zeros(128, 128, 3, 3, device=DEV), d, False)
    coef = torch.zeros(256, device=DEV)
    a = torch.empty_like(x)
    m = torch.empty(2 * 32 * 32 * 128 // 8, dtype=torch.uint8, device=DEV)
    assert sc.conv2d_fwd_bnin(x, coef, a, m, krsc, d) is None


@pytest.mark.parametrize("config", [2, 5])
def test_block_step_with_apply_on_load_equals_without(config):
    """The bench step (one eager forward + backward) with bn1 applied on load and with its separate
    apply pass: the same loss and every gradient bitwise (run in two child processes: the switch is
    read at import)."""
    import os
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as tmp:
        outs = []
        for on in ("1", "0"):
            out = os.path.join(tmp, "g%s.pt" % on)
            env = dict(os.environ, SQR_BN_DEFER=on)
            subprocess.run([sys.executable, os.path.join(root, "tools", "step_grads.py"), out, str(config)], env=env,
                           check=True, timeout=300)
            outs.append(torch.load(out, weights_only=True))
        a, b = outs
        assert a["loss"] == b["loss"]
        for n in a["grads"]:
            assert torch.equal(a["grads"][n], b["grads"][n]), n


# ---- apply-on-load without side outputs (the activation never written by the forward): the
# forward (persistent layer-1 and tiled layer 2-4 kernels) and the backward-data launch that rebuilds
# the activation and its mask (tiled layers 2-4; layer 1 keeps the forward's side outputs), against
# the two-pass path, bitwise -- ResNetSQ's bn1 -> conv2 shapes at 256^2 (B=64) and 512^2 input
NSO_SHAPES = [(64, 64, 64), (64, 128, 32), (64, 256, 16), (64, 512, 8), (16, 64, 128), (64, 128, 64), (64, 256, 32),
              (64, 512, 16)]


def _nso_operands(N, C, H, dtype, seed):
    from sqr import conv as sc
    g = torch.Generator(device=DEV).manual_seed(seed)
    x_pre = (torch.randn(N, C, H, H, device=DEV, generator=g) * 2 + 0.3).to(dtype).contiguous(
        memory_format=torch.channels_last)
    coef = torch.cat([torch.randn(C, device=DEV, generator=g) * 0.8, torch.randn(C, device=DEV, generator=g) * 0.5])
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) / (3.0 * C ** 0.5)
    d = sc._desc(N, C, H, H, C, 3, 3, 1, 1, dtype)
    krsc, crsk = sc.pack_weight(w, d, True)
    return g, x_pre, coef, d, krsc, crsk


def _apply(x_pre, coef, dtype):
    from sqr import conv as sc
    from sqr._lib import check, lib, ptr, stream_ptr
    N, C, H, W = x_pre.shape
    M = N * H * W
    a = torch.empty_like(x_pre)
    m = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    check(lib().sqr_bn_apply(ptr(x_pre), ctypes.c_longlong(M), C, sc._DT[dtype], ptr(coef), None, 1, ptr(a), ptr(m),
                             stream_ptr(torch.device(DEV))), "apply")
    return a, m


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("N,C,H", NSO_SHAPES)
def test_conv_bnin_no_side_outputs_equals_apply_then_conv(N, C, H, dtype):
    from sqr import conv as sc
    _, x_pre, coef, d, krsc, _ = _nso_operands(N, C, H, dtype, N * 13 + C + H)
    a_ref, _ = _apply(x_pre, coef, dtype)
    y_ref, s_ref = sc.conv2d_fwd(a_ref, krsc, d, stats=True)
    y, s = sc.conv2d_fwd_bnin(x_pre, coef, None, None, krsc, d)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert s.shape == s_ref.shape and torch.equal(s, s_ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("N,C,H", [s for s in NSO_SHAPES if s[1] != 64])
def test_bwd_data_bn_act_equals_mask_path(N, C, H, dtype):
    """The backward-data launch of the no-side-output path (mask recomputed from x and the
    coefficients, activation written) against the mask-reading one on the apply pass's mask: g, the
    BatchNorm backward partials and the activation bitwise."""
    from sqr import conv as sc
    g, x_pre, coef, d, _, crsk = _nso_operands(N, C, H, dtype, N * 17 + C + H)
    gy = torch.randn(N, C, H, H, device=DEV, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    mean = torch.randn(C, device=DEV, generator=g) * 0.3
    a_ref, m_ref = _apply(x_pre, coef, dtype)
    g_ref, s_ref = sc.conv2d_bwd_data_bn(gy, crsk, d, x_pre, m_ref, mean)
    act = torch.full_like(x_pre, float("nan"))
    g2, s2 = sc.conv2d_bwd_data_bn_act(gy, crsk, d, x_pre, coef, mean, act)
    torch.cuda.synchronize()
    assert torch.equal(act, a_ref)
    assert torch.equal(g2, g_ref)
    assert s2.shape == s_ref.shape and torch.equal(s2, s_ref)


def test_bnin_nso_query_picks_the_faster_path():
    """sqr_conv2d_bnin_nso_supported: the tiled 32/16-wide tiles take the no-side-output path, the
    persistent layer-1 kernel and the 8x8 layer-4 tiles keep theirs (BatchNorm)."""
    from sqr import conv as sc
    want = {(64, 64, 64): False, (64, 128, 32): True, (64, 256, 16): True, (64, 512, 8): False,
            (16, 64, 128): False, (64, 128, 64): True, (64, 256, 32): True, (64, 512, 16): True}
    for (N, C, H), on in want.items():
        d = sc._desc(N, C, H, H, C, 3, 3, 1, 1, torch.bfloat16)
        assert sc.bnin_nso_supported(d) == on, (N, C, H)


def test_bwd_data_bn_act_declines_layer1():
    """The persistent layer-1 shapes keep the forward's side outputs: the coefficient-mode
    backward-data is not offered there (SQR_E_UNSUPPORTED, nothing launched)."""
    from sqr import conv as sc
    from sqr._lib import SqrError
    _, x_pre, coef, d, _, crsk = _nso_operands(64, 64, 64, torch.bfloat16, 5)
    gy = torch.zeros_like(x_pre)
    with pytest.raises(SqrError):
        sc.conv2d_bwd_data_bn_act(gy, crsk, d, x_pre, coef, coef[:64], torch.empty_like(x_pre))
