"""HIP implicit-GEMM conv2d (libsqr) vs torch.nn.functional.conv2d in float64 on the CPU.

Floating-point kernel -> the reference is a plain PyTorch conv of the same op (float64, CPU).
Tolerances, relative to max|ref| of each output:
  f32 (exact-f32 MFMA, the parity mode): 1e-5 (sums of up to 4608 products, f32 accumulate;
      measured <= 2.7e-6)
  bf16 inputs (f32 accumulate): y/dx rounded to bf16 -> 8e-3; dw stays f32 -> 2e-4
  fp16 inputs (f32 accumulate): y/dx rounded to fp16 (2^-11 relative) -> 1e-3; dw -> 2e-4
  (the 16-bit reference is computed from the same rounded operands).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (N, C, H, K, R, stride, pad) — every conv of ResNetSQ at 256x256 input + GenericNetSQ
# shapes + odd edge cases
RESNET = [
    (2, 1, 256, 64, 7, 2, 3),      # conv1 (im2col path)
    (2, 64, 64, 64, 3, 1, 1),      # layer1.*
    (2, 64, 64, 128, 3, 2, 1),     # layer2.0.conv1
    (2, 64, 64, 128, 1, 2, 0),     # layer2.0.downsample
    (2, 128, 32, 128, 3, 1, 1),    # layer2.*
    (2, 128, 32, 256, 3, 2, 1),    # layer3.0.conv1
    (2, 128, 32, 256, 1, 2, 0),    # layer3.0.downsample
    (2, 256, 16, 256, 3, 1, 1),    # layer3.*
    (2, 256, 16, 512, 3, 2, 1),    # layer4.0.conv1
    (2, 256, 16, 512, 1, 2, 0),    # layer4.0.downsample
    (2, 512, 8, 512, 3, 1, 1),     # layer4.*
]
EXTRA = [
    (3, 32, 128, 32, 3, 1, 1),     # GenericNetSQ 32-channel convs (multi-tap k tiles)
    (3, 32, 128, 64, 3, 2, 1),
    (1, 8, 13, 16, 3, 1, 1),       # odd spatial size, tiny channels
    (3, 16, 9, 8, 5, 2, 2),
    (2, 3, 31, 64, 7, 2, 3),       # C=3 im2col
    (1, 64, 7, 128, 1, 1, 0),
]


def _ref(x, w, stride, pad, gy):
    xd = x.detach().double().cpu().requires_grad_(True)
    wd = w.detach().double().cpu().requires_grad_(True)
    y = F.conv2d(xd, wd, stride=stride, padding=pad)
    y.backward(gy.detach().double().cpu())
    return y.detach(), xd.grad, wd.grad


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _totals(st):
    """(sum, sum of squares) per channel from a conv's forward-statistics partials: Welford rows
    (mean_t, M2_t) and their pixel counts (sqr.bn.partial_counts) -> sum n_t mean_t and
    sum (M2_t + n_t mean_t^2), float64."""
    from sqr.bn import partial_counts
    n = partial_counts(st).double()[:, None]
    m, q = st[:, 0].double(), st[:, 1].double()
    return torch.stack([(n * m).sum(0), (q + n * m * m).sum(0)])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16], ids=["f32", "bf16", "f16"])
@pytest.mark.parametrize("shape", RESNET + EXTRA, ids=lambda s: "N%dC%dH%dK%dR%ds%dp%d" % s)
def test_conv_fwd_bwd(shape, dtype):
    from sqr import conv as sc
    N, C, H, K, R, st, pad = shape
    g = torch.Generator().manual_seed(N * 1000 + C * 10 + K)
    x = torch.randn(N, C, H, H, generator=g)
    w = torch.randn(K, C, R, R, generator=g) / (C * R * R) ** 0.5
    if dtype != torch.float32:
        x = x.to(dtype).float()
        w_used = w.to(dtype).float()
    else:
        w_used = w
    Ho = (H + 2 * pad - R) // st + 1
    gy = torch.randn(N, K, Ho, Ho, generator=g)
    if dtype != torch.float32:
        gy = gy.to(dtype).float()
    yr, dxr, dwr = _ref(x, w_used, st, pad, gy)

    xg = x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(C >= 8)
    wg = w.to(DEV).requires_grad_(True)
    y = sc.conv2d(xg, wg, None, st, pad)
    assert y.dtype == dtype and y.shape == (N, K, Ho, Ho)
    y.backward(gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    tol_y = {torch.float32: 1e-5, torch.bfloat16: 8e-3, torch.float16: 1e-3}[dtype]
    tol_w = 1e-5 if dtype == torch.float32 else 2e-4
    assert _rel(y, yr) <= tol_y
    assert wg.grad.dtype == torch.float32
    assert _rel(wg.grad, dwr) <= tol_w
    if C >= 8:
        assert _rel(xg.grad, dxr) <= tol_y


def test_conv_module_matches_nn_conv2d_state_dict():
    from sqr.conv import Conv2d
    a = torch.nn.Conv2d(64, 128, 3, 2, 1, bias=True)
    b = Conv2d(64, 128, 3, 2, 1, bias=True)
    b.load_state_dict(a.state_dict())
    assert list(a.state_dict()) == list(b.state_dict())
    x = torch.randn(2, 64, 20, 20)
    yr = a(x)
    b = b.to(DEV)
    y = b(x.to(DEV).contiguous(memory_format=torch.channels_last))
    assert _rel(y, yr) <= 2e-6


def test_conv_deterministic():
    from sqr import conv as sc
    x = torch.randn(4, 64, 32, 32, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w = torch.randn(64, 64, 3, 3, device=DEV, requires_grad=True)
    outs = []
    for _ in range(2):
        x.grad = None
        w.grad = None
        y = sc.conv2d(x, w, None, 1, 1)
        y.float().square().sum().backward()
        outs.append((y.clone(), x.grad.clone(), w.grad.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


# direct 3x3/s1/p1 kernel (sqr_conv3.hip): one shape per tile configuration (and multi-tile rows,
# Cin != Nout); forced on (mode 2) so the small test batches take it, and compared with the
# implicit-GEMM path (mode 0) and the float64 reference
DIRECT = [
    (2, 64, 64, 64),     # layer-1 persistent kernel (resident weights), one tile per workgroup
    (20, 64, 64, 64),    # persistent, several tiles per workgroup (640 tiles > CUs)
    (1, 64, 128, 64),    # cfg 0, two tiles per image row
    (2, 128, 32, 128),   # cfg 1 (TW 32 x TH 8, double-buffered window, 2 chunks)
    (1, 128, 64, 128),   # cfg 1, two tiles per row
    (2, 256, 16, 256),   # cfg 2 (TW 16 x TH 8)
    (2, 512, 8, 512),    # cfg 5 (two 8 x 8 images per tile, 8 chunks)
    (3, 512, 8, 512),    # cfg 3 (odd batch: one image per tile)
    (2, 128, 16, 256),   # Cin != Nout
    (2, 64, 32, 128),    # fwd direct (cfg 1, one chunk); dgrad falls back
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", DIRECT, ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3_direct(shape, dtype):
    from sqr import conv as sc
    from sqr._lib import lib
    N, C, H, K = shape
    g = torch.Generator().manual_seed(N + C + H + K)
    x = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H, H, generator=g).to(dtype).float()
    yr, dxr, dwr = _ref(x, w.to(dtype).float(), 1, 1, gy)
    res = {}
    old = lib().sqr_conv_set_direct(2)
    try:
        for mode in (2, 0):
            lib().sqr_conv_set_direct(mode)
            xg = x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            wg = w.to(DEV).requires_grad_(True)
            y, st = sc.conv2d(xg, wg, None, 1, 1, stats=True)
            y.backward(gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res[mode] = (y.float(), xg.grad.float(), _totals(st), wg.grad.clone())
    finally:
        lib().sqr_conv_set_direct(old)
    for mode in (2, 0):
        y, dx, st, dw = res[mode]
        assert _rel(y, yr) <= 8e-3
        assert _rel(dx, dxr) <= 8e-3
        assert _rel(dw, dwr) <= 2e-4
        yd = y.double()
        assert _rel(st[0], yd.sum((0, 2, 3))) <= 1e-5
        assert _rel(st[1], (yd * yd).sum((0, 2, 3))) <= 1e-5
    assert _rel(res[2][0], res[0][0]) <= 8e-3
    assert _rel(res[2][1], res[0][1]) <= 8e-3
    assert _rel(res[2][3], res[0][3]) <= 2e-4


@pytest.mark.parametrize("N,H", [(64, 64), (48, 64), (128, 64), (64, 128), (48, 128), (16, 128)])
def test_conv3_persistent_bands(N, H):
    """The layer-1 persistent kernel at benchmark-sized batches (64 x 64 maps in 2-row tiles: bands
    of 8 and 16 tiles per workgroup; 128 x 128 maps, config 5, in 1-row tiles: bands of 32 / 8; the
    row ring wrapping many times) against the implicit-GEMM kernel on the same bf16 inputs, plus its
    per-workgroup BatchNorm partials against the output itself."""
    from sqr import conv as sc
    from sqr._lib import lib
    g = torch.Generator(device=DEV).manual_seed(N + H)
    x = torch.randn(N, 64, H, H, device=DEV, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3, device=DEV, generator=g) / 24.0
    gy = torch.randn(N, 64, H, H, device=DEV, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    d = sc._desc(N, 64, H, H, 64, 3, 3, 1, 1, torch.bfloat16)
    krsc, crsk = sc.pack_weight(w, d, True)
    res = {}
    old = lib().sqr_conv_set_direct(1)
    try:
        for mode in (1, 0):
            lib().sqr_conv_set_direct(mode)
            y, st = sc.conv2d_fwd(x, krsc, d, stats=True)
            dx = sc.conv2d_bwd_data(gy, crsk, d)
            torch.cuda.synchronize()
            res[mode] = (y.float(), _totals(st), dx.float(), st.shape[0])
    finally:
        lib().sqr_conv_set_direct(old)
    y1, st1, dx1, rows1 = res[1]
    y0, _, dx0, _ = res[0]
    assert rows1 <= 256
    assert _rel(y1, y0) <= 4e-3 and _rel(dx1, dx0) <= 4e-3
    assert (y1 - y0).abs().max().item() <= 0.02 * y0.abs().max().item()
    yd = y1.double()
    assert _rel(st1[0], yd.sum((0, 2, 3))) <= 1e-5
    assert _rel(st1[1], (yd * yd).sum((0, 2, 3))) <= 1e-5


@pytest.mark.parametrize("shape", [(2, 64, 64, 128), (3, 128, 32, 256), (3, 256, 16, 512), (64, 64, 64, 128),
                                   (64, 128, 32, 256), (64, 256, 16, 512),
                                   (2, 64, 128, 128), (2, 128, 64, 256), (2, 256, 32, 512),  # 512x512 input
                                   (16, 64, 128, 128), (16, 128, 64, 256), (16, 256, 32, 512)],
                         ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3s2_dgrad_direct(shape):
    """Direct stride-2 backward-data kernel (layers 2-4 first convs: all four parity classes in one
    launch) against the float64 reference (small N) and the parity-class implicit GEMM (mode 0)."""
    from sqr import conv as sc
    from sqr._lib import lib
    N, C, H, K = shape
    g = torch.Generator().manual_seed(7 * N + C + K)
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H // 2, H // 2, generator=g).bfloat16().float()
    d = sc._desc(N, C, H, H, K, 3, 3, 2, 1, torch.bfloat16)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    gyg = gy.to(DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    res = {}
    old = lib().sqr_conv_set_direct(1)
    try:
        for mode in (1, 0):
            lib().sqr_conv_set_direct(mode)
            res[mode] = sc.conv2d_bwd_data(gyg, crsk, d).float()
            torch.cuda.synchronize()
    finally:
        lib().sqr_conv_set_direct(old)
    assert _rel(res[1], res[0]) <= 8e-3
    assert (res[1] - res[0]).abs().max().item() <= 0.02 * res[0].abs().max().item()
    if N <= 4:
        x = torch.zeros(N, C, H, H)
        _, dxr, _ = _ref(x, w.bfloat16().float(), 2, 1, gy)
        assert _rel(res[1], dxr) <= 8e-3


# ---------------------------------------------------------------------------- benchmark sizes
# The kernels the B=64 bench step runs, at exactly its shapes, against float64 CPU references on
# the same 16-bit-rounded operands (not only against another HIP kernel).

def _f64_fwd_dgrad_wgrad(x, w, gy, stride, pad):
    xd, wd, gd = x.double(), w.double(), gy.double()
    y = F.conv2d(xd, wd, stride=stride, padding=pad)
    dx = torch.nn.grad.conv2d_input(xd.shape, wd, gd, stride=stride, padding=pad)
    dw = torch.nn.grad.conv2d_weight(xd, wd.shape, gd, stride=stride, padding=pad)
    return y, dx, dw


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("N,H", [(64, 64), (48, 64), (16, 128)])
def test_conv3p_bench_size_vs_f64(N, H, dtype):
    """Layer-1 3x3 64->64 at the bench batch (config 5's 128 x 128 maps at batch 16): the
    persistent resident-weight kernel (bands of 8+ tiles per workgroup, the row ring wrapping) for
    forward and backward-data, the direct weight gradient, and the fused BatchNorm partials — all
    against float64."""
    from sqr import conv as sc
    g = torch.Generator().manual_seed(1000 + N + H)
    x = torch.randn(N, 64, H, H, generator=g).to(dtype).float()
    w = (torch.randn(64, 64, 3, 3, generator=g) / 24.0)
    gy = torch.randn(N, 64, H, H, generator=g).to(dtype).float()
    yr, dxr, dwr = _f64_fwd_dgrad_wgrad(x, w.to(dtype).float(), gy, 1, 1)
    d = sc._desc(N, 64, H, H, 64, 3, 3, 1, 1, dtype)
    krsc, crsk = sc.pack_weight(w.to(DEV), d, True)
    xg = x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    gyg = gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    y, st = sc.conv2d_fwd(xg, krsc, d, stats=True)
    dx = sc.conv2d_bwd_data(gyg, crsk, d)
    dw = sc.conv2d_bwd_weight(xg, gyg, d)
    torch.cuda.synchronize()
    assert st.shape[0] <= 256  # one partial row per persistent workgroup
    tol = 8e-3 if dtype == torch.bfloat16 else 1e-3
    assert _rel(y, yr) <= tol
    assert _rel(dx, dxr) <= tol
    assert _rel(dw, dwr) <= 2e-4
    yd = y.double().cpu()
    tot = _totals(st)
    assert _rel(tot[0], yd.sum((0, 2, 3))) <= 1e-5
    assert _rel(tot[1], (yd * yd).sum((0, 2, 3))) <= 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", [(64, 64, 64, 128), (64, 128, 32, 256), (64, 256, 16, 512)],
                         ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3s2_dgrad_bench_size_vs_f64(shape, dtype):
    """The direct stride-2 backward-data kernel of layers 2-4 at the bench batch vs float64."""
    from sqr import conv as sc
    N, C, H, K = shape
    g = torch.Generator().manual_seed(7 * N + C + K)
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H // 2, H // 2, generator=g).to(dtype).float()
    d = sc._desc(N, C, H, H, K, 3, 3, 2, 1, dtype)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    dx = sc.conv2d_bwd_data(gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last), crsk, d)
    torch.cuda.synchronize()
    dxr = torch.nn.grad.conv2d_input((N, C, H, H), w.to(dtype).double(), gy.double(), stride=2, padding=1)
    assert _rel(dx, dxr) <= (8e-3 if dtype == torch.bfloat16 else 1e-3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", [(64, 64, 64, 128), (64, 128, 32, 256), (64, 256, 16, 512), (2, 64, 64, 128),
                                   (3, 128, 32, 256), (1, 256, 16, 512), (2, 64, 128, 64)],
                         ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3s2_wgrad_vs_f64(shape, dtype):
    """The direct stride-2 weight gradient (four phase planes of the input window; layers 2-4's
    first conv) at the bench batch and at a few images (few chunks per split, several tiles per
    row at 128 input) vs float64."""
    from sqr import conv as sc
    N, C, H, K = shape
    g = torch.Generator().manual_seed(11 * N + C + K + H)
    x = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    gy = torch.randn(N, K, H // 2, H // 2, generator=g).to(dtype).float()
    d = sc._desc(N, C, H, H, K, 3, 3, 2, 1, dtype)
    dw = sc.conv2d_bwd_weight(x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last),
                              gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last), d)
    torch.cuda.synchronize()
    dwr = torch.nn.grad.conv2d_weight(x.double(), (K, C, 3, 3), gy.double(), stride=2, padding=1)
    assert _rel(dw, dwr) <= 2e-4


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", [(64, 64, 64, 128), (64, 128, 32, 256), (64, 256, 16, 512), (2, 64, 64, 128),
                                   (3, 128, 32, 256), (1, 256, 16, 512), (2, 64, 128, 128), (2, 128, 64, 256),
                                   (2, 256, 32, 512)],
                         ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3s2_fwd_vs_f64(shape, dtype):
    """The direct stride-2 forward (conv3_kernel's four-plane window; layers 2-4's first conv at 256
    and 512 input) at the bench batch and at a few images (direct forced) vs float64, and its
    BatchNorm statistics partials vs the stored output."""
    from sqr import conv as sc
    from sqr._lib import lib
    N, C, H, K = shape
    g = torch.Generator().manual_seed(13 * N + C + K + H)
    x = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    yr = F.conv2d(x.double(), w.to(dtype).double(), stride=2, padding=1)
    d = sc._desc(N, C, H, H, K, 3, 3, 2, 1, dtype)
    krsc, _ = sc.pack_weight(w.to(DEV), d, False)
    old = lib().sqr_conv_set_direct(2)
    try:
        y, st = sc.conv2d_fwd(x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last), krsc, d,
                              stats=True)
        torch.cuda.synchronize()
    finally:
        lib().sqr_conv_set_direct(old)
    assert _rel(y, yr) <= (8e-3 if dtype == torch.bfloat16 else 1e-3)
    from sqr.bn import partial_counts
    cnt = partial_counts(st).double()
    assert int(cnt.sum()) == N * (H // 2) ** 2
    yf = y.double().cpu()
    mean = (cnt[:, None] * st[:, 0].double()).sum(0).cpu() / cnt.sum().cpu()
    m2 = (st[:, 1].double() + cnt[:, None] * (st[:, 0].double() - mean.to(DEV)) ** 2).sum(0).cpu()
    assert _rel(mean, yf.mean((0, 2, 3))) <= 1e-5
    assert _rel(m2, ((yf - yf.mean((0, 2, 3), keepdim=True)) ** 2).sum((0, 2, 3))) <= 1e-5


@pytest.mark.parametrize("shape", [(64, 128, 32, 128), (64, 256, 16, 256), (64, 512, 8, 512)],
                         ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv3_tiled_bench_size_vs_f64(shape):
    """The tiled direct 3x3/s1 kernels of layers 2-4 (fwd + dgrad) and their weight gradient at
    the bench batch vs float64 (bf16 operands)."""
    from sqr import conv as sc
    N, C, H, K = shape
    g = torch.Generator().manual_seed(N + C + H)
    x = torch.randn(N, C, H, H, generator=g).bfloat16().float()
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H, H, generator=g).bfloat16().float()
    yr, dxr, dwr = _f64_fwd_dgrad_wgrad(x, w.bfloat16().float(), gy, 1, 1)
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, torch.bfloat16)
    krsc, crsk = sc.pack_weight(w.to(DEV), d, True)
    xg = x.to(DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    gyg = gy.to(DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    y = sc.conv2d_fwd(xg, krsc, d)
    dx = sc.conv2d_bwd_data(gyg, crsk, d)
    dw = sc.conv2d_bwd_weight(xg, gyg, d)
    torch.cuda.synchronize()
    assert _rel(y, yr) <= 8e-3 and _rel(dx, dxr) <= 8e-3 and _rel(dw, dwr) <= 2e-4


# every conv of ResNetSQ at 512x512 input (BASELINE config 5), N=2, direct kernels forced where the
# shape tiles (at N=2 the default routing would leave some to the implicit GEMM)
RESNET512 = [
    (2, 1, 512, 64, 7, 2, 3),
    (2, 64, 128, 64, 3, 1, 1),
    (2, 64, 128, 128, 3, 2, 1),
    (2, 64, 128, 128, 1, 2, 0),
    (2, 128, 64, 128, 3, 1, 1),
    (2, 128, 64, 256, 3, 2, 1),
    (2, 128, 64, 256, 1, 2, 0),
    (2, 256, 32, 256, 3, 1, 1),
    (2, 256, 32, 512, 3, 2, 1),
    (2, 256, 32, 512, 1, 2, 0),
    (2, 512, 16, 512, 3, 1, 1),
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("direct", [2, 0], ids=["direct", "gemm"])
@pytest.mark.parametrize("shape", RESNET512, ids=lambda s: "N%dC%dH%dK%dR%ds%dp%d" % s)
def test_conv_512(shape, direct, dtype):
    from sqr import conv as sc
    from sqr._lib import lib
    N, C, H, K, R, st, pad = shape
    g = torch.Generator().manual_seed(N * 1000 + C * 10 + K + H)
    x = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    w = torch.randn(K, C, R, R, generator=g) / (C * R * R) ** 0.5
    Ho = (H + 2 * pad - R) // st + 1
    gy = torch.randn(N, K, Ho, Ho, generator=g).to(dtype).float()
    yr, dxr, dwr = _f64_fwd_dgrad_wgrad(x, w.to(dtype).float(), gy, st, pad)
    old = lib().sqr_conv_set_direct(direct)
    try:
        xg = x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(C >= 8)
        wg = w.to(DEV).requires_grad_(True)
        y = sc.conv2d(xg, wg, None, st, pad)
        y.backward(gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        lib().sqr_conv_set_direct(old)
    tol = 8e-3 if dtype == torch.bfloat16 else 1e-3
    assert _rel(y, yr) <= tol
    assert _rel(wg.grad, dwr) <= 2e-4
    if C >= 8:
        assert _rel(xg.grad, dxr) <= tol


# ---------------------------------------------------------------------------- fused residual add
# sqr_conv2d_bwd_data_acc: dx = bwd_data(dy) + addend.  Each dgrad that feeds a residual block's
# input: layer-1 persistent kernel (N=4 and the bench batch: band / ring wrap, the ACC store
# order), the tiled kernels of layers 2-4, the direct stride-2 kernel, and the implicit-GEMM +
# add fallback (1x1 / fp32).  Reference: float64 dgrad of the same rounded operands + addend.
ACC_SHAPES = [
    (4, 64, 64, 64, 3, 1), (64, 64, 64, 64, 3, 1), (48, 64, 64, 64, 3, 1),
    (4, 128, 32, 128, 3, 1), (4, 256, 16, 256, 3, 1), (4, 512, 8, 512, 3, 1),
    (4, 64, 64, 128, 3, 2), (4, 128, 32, 256, 3, 2), (4, 256, 16, 512, 3, 2), (64, 64, 64, 128, 3, 2),
    (4, 64, 64, 128, 1, 2), (2, 64, 128, 64, 3, 1), (2, 64, 128, 128, 3, 2), (16, 64, 128, 64, 3, 1),
    # 512x512 input at batch 16 (config 5's step test): several tiles per image row in the tiled
    # 8-wave layer-2 kernel and the layer-3 stride-2 kernel
    (16, 128, 64, 128, 3, 1), (16, 128, 64, 256, 3, 2), (16, 256, 32, 512, 3, 2), (16, 256, 32, 256, 3, 1),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=["bf16", "f16", "f32"])
@pytest.mark.parametrize("shape", ACC_SHAPES, ids=lambda s: "N%dC%dH%dK%dR%ds%d" % s)
def test_conv_bwd_data_acc(shape, dtype):
    from sqr import conv as sc
    N, C, H, K, R, st = shape
    if dtype == torch.float32 and N > 8:
        pytest.skip("fp32 runs the implicit GEMM + add; the small batch covers it")
    pad = R // 2
    g = torch.Generator().manual_seed(11 * N + C + K + R)
    Ho = (H + 2 * pad - R) // st + 1
    w = torch.randn(K, C, R, R, generator=g) / (C * R * R) ** 0.5
    gy = torch.randn(N, K, Ho, Ho, generator=g).to(dtype).float()
    add = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    d = sc._desc(N, C, H, H, K, R, R, st, pad, dtype)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    gyg = gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    addg = add.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dx = sc.conv2d_bwd_data_acc(gyg, crsk, d, addg)
    plain = sc.conv2d_bwd_data(gyg, crsk, d)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.to(dtype).double(), gy.double(), stride=st, padding=pad)
    ref = ref + add.double()
    tol = {torch.bfloat16: 1.2e-2, torch.float16: 2e-3, torch.float32: 1e-5}[dtype]
    assert _rel(dx, ref) <= tol
    # the fused sum equals the separate sum up to one rounding of the 16-bit result
    assert _rel(dx, plain.double() + addg.double()) <= (1.0 if dtype == torch.float32 else 2.0) * tol
    assert torch.equal(addg.cpu().float(), add.to(dtype).float())  # the addend is not modified


# sqr_conv2d_bwd_data_acc_masked: the addend is an identity block's ReLU-masked gradient kept as
# (dy, mask) (sqr.conv.MaskedGrad); must equal the ACC launch on the materialised masked tensor
# bitwise (masked-out halves are +0 either way), and float64 within the 16-bit tolerance.
MASKED_SHAPES = [(4, 64, 64, 64), (64, 64, 64, 64), (4, 128, 32, 128), (4, 256, 16, 256), (4, 512, 8, 512),
                 (64, 128, 32, 128), (64, 512, 8, 512), (16, 64, 128, 64)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("shape", MASKED_SHAPES, ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv_bwd_data_acc_masked(shape, dtype):
    import ctypes
    from sqr import conv as sc
    from sqr._lib import lib, ptr, stream_ptr
    N, C, H, K = shape
    g = torch.Generator().manual_seed(7 * N + C + K)
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H, H, generator=g).to(dtype).float()
    dy = torch.randn(N, C, H, H, generator=g).to(dtype).float()
    keep = torch.rand(N, H, H, C, generator=g) > 0.4  # NHWC element order, as the ReLU mask
    bits = keep.reshape(-1, 8).to(torch.uint8)
    mask = (bits << torch.arange(8, dtype=torch.uint8)).sum(dim=1, dtype=torch.uint8)
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, dtype)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    gyg = gy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dyg = dy.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    mg = sc.MaskedGrad(dyg, mask.to(DEV))
    full = mg.full()
    dx = torch.empty((N, C, H, H), dtype=dtype, device=DEV, memory_format=torch.channels_last)
    ws, n = sc._ws(d, 1, gyg.device)
    rc = lib().sqr_conv2d_bwd_data_acc_masked(ptr(gyg), ptr(crsk), ptr(dx), ptr(dyg), ptr(mg.mask), ctypes.byref(d),
                                              ptr(ws), n, stream_ptr(gyg.device))
    ref_acc = sc.conv2d_bwd_data_acc(gyg, crsk, d, full)
    torch.cuda.synchronize()
    masked_ref = dy * keep.permute(0, 3, 1, 2).float()
    assert torch.equal(full.cpu().float(), masked_ref.to(dtype).float())
    if rc == -2:  # no direct kernel at this size (too few tiles): sqr.conv masks (full()) and adds
        assert b"masked addend" in lib().sqr_last_error_string()
        assert N < 64
        return
    assert rc == 0, lib().sqr_last_error_string()
    assert torch.equal(dx, ref_acc)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.to(dtype).double(), gy.double(), stride=1, padding=1)
    ref = ref + masked_ref.double()
    assert _rel(dx, ref) <= {torch.bfloat16: 1.2e-2, torch.float16: 2e-3}[dtype]


# ---------------------------------------------------------------- dgrad + BatchNorm-backward sums
# sqr_conv2d_bwd_data_bn (a BasicBlock's conv2 backward-data feeding bn1's backward): g = dgrad * mask
# and the per-channel sums (sum g, sum g*(x - mean)) — the persistent layer-1 kernel (ring wrap at
# the bench batch), the tiled kernels of layers 2-4, and the implicit-GEMM fallback (fp32, odd size).
# sqr_conv2d_bwd_data_acc_s2: a stride-2 conv's dgrad + a compact [N, C, H/2, W/2] addend on the
# (even, even) pixels (the stride-2 1x1 downsample branch of a BasicBlock's input gradient): the direct
# stride-2 kernel's copy-out (layers 2-4, 256 and 512 input) and the implicit GEMM + scatter-add fallback
# (fp32, and a 1x1 conv)
S2C_SHAPES = [(4, 64, 64, 128, 3), (64, 64, 64, 128, 3), (4, 128, 32, 256, 3), (64, 256, 16, 512, 3),
              (16, 128, 64, 256, 3), (2, 64, 128, 128, 3), (4, 64, 64, 128, 1)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=["bf16", "f16", "f32"])
@pytest.mark.parametrize("shape", S2C_SHAPES, ids=lambda s: "N%dC%dH%dK%dR%d" % s)
def test_conv_bwd_data_acc_s2(shape, dtype):
    from sqr import conv as sc
    N, C, H, K, R = shape
    if dtype == torch.float32 and N > 8:
        pytest.skip("fp32 runs the implicit GEMM + scatter-add; the small batch covers it")
    pad = R // 2
    g = torch.Generator().manual_seed(17 * N + C + K + R)
    w = torch.randn(K, C, R, R, generator=g) / (C * R * R) ** 0.5
    gy = torch.randn(N, K, H // 2, H // 2, generator=g).to(dtype).float()
    addc = torch.randn(N, C, H // 2, H // 2, generator=g).to(dtype).float()
    d = sc._desc(N, C, H, H, K, R, R, 2, pad, dtype)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    cl = dict(memory_format=torch.channels_last)
    dx = sc.conv2d_bwd_data_acc_s2(gy.to(DEV).to(dtype).contiguous(**cl), crsk, d,
                                   addc.to(DEV).to(dtype).contiguous(**cl))
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.to(dtype).double(), gy.double(), stride=2, padding=pad)
    ref[:, :, ::2, ::2] += addc.double()
    assert _rel(dx, ref) <= {torch.bfloat16: 1.2e-2, torch.float16: 2e-3, torch.float32: 1e-5}[dtype]


BNB_SHAPES = [(4, 64, 64, 64), (64, 64, 64, 64), (4, 128, 32, 128), (64, 128, 32, 128), (4, 256, 16, 256),
              (4, 512, 8, 512), (2, 64, 128, 64), (3, 32, 20, 32), (16, 128, 64, 128), (16, 256, 32, 256),
              (16, 64, 128, 64)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=["bf16", "f16", "f32"])
@pytest.mark.parametrize("shape", BNB_SHAPES, ids=lambda s: "N%dC%dH%dK%d" % s)
def test_conv_bwd_data_bn(shape, dtype):
    from sqr import conv as sc
    N, C, H, K = shape
    if dtype == torch.float32 and N > 8:
        pytest.skip("fp32 runs the implicit GEMM + mask/reduce fallback; small batches cover it")
    g = torch.Generator().manual_seed(5 * N + C + K + H)
    w = torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H, H, generator=g).to(dtype).float()
    x = (torch.randn(N, C, H, H, generator=g) * 1.5 + 0.3).to(dtype).float()
    keep = torch.rand(N, C, H, H, generator=g) > 0.4  # the BatchNorm's ReLU mask
    mean = torch.randn(C, generator=g) * 0.2
    # 1-bit mask in the NHWC element order, 8 channels per byte (bit i = channel 8v + i)
    bits = keep.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.int64)
    mask = (bits << torch.arange(8)).sum(1).to(torch.uint8)
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, dtype)
    _, crsk = sc.pack_weight(w.to(DEV), d, True)
    cl = dict(memory_format=torch.channels_last)
    gg, st = sc.conv2d_bwd_data_bn(gy.to(DEV).to(dtype).contiguous(**cl), crsk, d, x.to(DEV).to(dtype).contiguous(**cl),
                                   mask.to(DEV), mean.to(DEV))
    plain = sc.conv2d_bwd_data(gy.to(DEV).to(dtype).contiguous(**cl), crsk, d)
    torch.cuda.synchronize()
    # g is exactly the plain 16-bit dgrad with the masked elements zeroed
    assert torch.equal(gg.cpu(), (plain.cpu() * keep.to(plain.dtype)))
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.to(dtype).double(), gy.double(), stride=1, padding=1) * keep
    tol = {torch.bfloat16: 8e-3, torch.float16: 1e-3, torch.float32: 1e-5}[dtype]
    assert _rel(gg, ref) <= tol
    # the sums are those of the stored g (f64 over the rows)
    gd = gg.double().cpu()
    s1 = gd.sum((0, 2, 3))
    s2 = (gd * (x.double() - mean.double().view(1, C, 1, 1))).sum((0, 2, 3))
    tot = st.double().sum(0).cpu()
    assert st.shape[1:] == (2, C)
    assert _rel(tot[0], s1) <= 1e-5 and _rel(tot[1], s2) <= 1e-5

