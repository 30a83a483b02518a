"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Run in the survey/build container only (it needs /root/reference, which never
travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

The reference's torch/ modules import cv2, h5py, torchsummary and torchvision at
module level (classes.py:1-16, models.py:4) although none of them is used by
the functions pinned here.  None of those four is installed in this image, so
empty placeholder modules are put into ``sys.modules`` before the import; every
fixture below is produced by the reference's own Python code running on torch
CPU (float64 where the reference computes in float64).

What is pinned (reference file:line):
  * ImplicitLoss fwd (loss) + autograd bwd (d loss / d pred)  classes.py:203-295
  * ExplicitLoss fwd + bwd                                      classes.py:109-201
  * IoUAccuracy (reduce and per-sample)                         classes.py:374-447
  * mat_from_quaternion / conjugate / multiply                  quaternion.py:19-67
  * RotationHead/SizeHead/ShapeHead/PositionHead                models.py:7-99
  * GenericNetSQ forward with seeded weights                    models.py:125-169
  * parse_csv on the example labels (header row dropped)        helpers.py:188-218
  * the 10 example depth images (data/example_imgs/*.bmp, decoded here with a
    plain BMP reader; the images are data files of the reference, not code)

Outputs are numpy .npz files (no pickles).
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/torch"
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_placeholders():
    for name in ("cv2", "h5py", "torchsummary", "torchvision", "tqdm"):
        if name in sys.modules:
            continue
        try:
            __import__(name)
            continue
        except ImportError:
            pass
        m = types.ModuleType(name)
        if name == "torchsummary":
            m.summary = lambda *a, **k: None
        if name == "torchvision":
            m.models = types.ModuleType("torchvision.models")
        if name == "tqdm":
            m.tqdm = lambda x, *a, **k: x
        sys.modules[name] = m
    sys.path.insert(0, REF)


def read_bmp_gray(path):
    """24-bit bottom-up BMP -> uint8 [H,W] (what cv2.imread(path, 0) returns for gray BMPs)."""
    b = open(path, "rb").read()
    off = int.from_bytes(b[10:14], "little")
    w = int.from_bytes(b[18:22], "little", signed=True)
    h = int.from_bytes(b[22:26], "little", signed=True)
    bpp = int.from_bytes(b[28:30], "little")
    assert bpp == 24
    stride = (w * 3 + 3) & ~3
    rows = np.frombuffer(b[off:off + stride * abs(h)], np.uint8).reshape(abs(h), stride)[:, :w * 3]
    rgb = rows.reshape(abs(h), w, 3)
    assert (rgb[..., 0] == rgb[..., 1]).all() and (rgb[..., 1] == rgb[..., 2]).all()
    img = rgb[..., 0]
    if h > 0:
        img = img[::-1]
    return np.ascontiguousarray(img)


def sample_params(rng, n):
    """§8d synthetic distribution: gen_rand_rot.py:21-31 normalised as parse_csv does."""
    a = rng.uniform(25, 75, (n, 3)) / 255.0
    e = rng.uniform(0.1, 1.0, (n, 2))
    t = (128.0 + rng.uniform(-40, 40, (n, 3))) / 255.0
    u = rng.uniform(0, 1, (n, 3))
    q = np.stack([np.sqrt(1 - u[:, 0]) * np.sin(2 * np.pi * u[:, 1]),
                  np.sqrt(1 - u[:, 0]) * np.cos(2 * np.pi * u[:, 1]),
                  np.sqrt(u[:, 0]) * np.sin(2 * np.pi * u[:, 2]),
                  np.sqrt(u[:, 0]) * np.cos(2 * np.pi * u[:, 2])], 1)
    return np.concatenate([a, e, t, q], 1).astype(np.float32)


def main():
    _install_placeholders()
    import classes  # noqa: E402
    import quaternion  # noqa: E402
    import models  # noqa: E402
    import helpers  # noqa: E402

    torch.set_num_threads(8)
    cpu = torch.device("cpu")
    rng = np.random.default_rng(20260415)

    # ---------------- example images + labels ----------------
    ex_dir = "/root/reference/data/example_imgs"
    imgs = np.stack([read_bmp_gray(os.path.join(ex_dir, "%06d.bmp" % i)) for i in range(10)])
    lines = open(os.path.join(ex_dir, "labels.txt")).read().split("\n")
    tmp_csv = "/tmp/_sqr_labels_noheader.csv"
    with open(tmp_csv, "w") as f:
        f.write("\n".join(lines[1:]))
    labels = np.stack(helpers.parse_csv(tmp_csv))  # [10,12] f32
    raw21 = np.array([[float(v) for v in l.split(",")[1:]] for l in lines[1:] if l], np.float64)
    np.savez_compressed(os.path.join(HERE, "example_images.npz"), images=imgs, labels=labels,
                        raw_csv=raw21, csv_text=np.array("\n".join(lines[1:])))

    # ---------------- quaternion ----------------
    q = rng.normal(size=(16, 4))
    q[:8] /= np.linalg.norm(q[:8], axis=1, keepdims=True)  # half unit, half un-normalised
    mats = np.stack([quaternion.mat_from_quaternion(torch.tensor(qi))[0].numpy() for qi in q])
    conj = quaternion.conjugate(torch.tensor(q)).numpy()
    q2 = rng.normal(size=(16, 4))
    mul = quaternion.multiply(torch.tensor(q), torch.tensor(q2)).numpy()
    np.savez_compressed(os.path.join(HERE, "quaternion.npz"), q=q, q2=q2, mat=mats, conj=conj, mul=mul)

    # ---------------- ImplicitLoss ----------------
    cases = []

    def add_implicit(name, R, tau, s, true_img, pred):
        crit = classes.ImplicitLoss(R, cpu, tau, s)
        p = torch.tensor(pred, dtype=torch.float32, requires_grad=True)
        t = torch.tensor(true_img, dtype=torch.float32)
        loss = crit(t, p)
        loss.backward()
        depth = crit.depth_projection(p.detach()).numpy()
        cases.append(dict(name=name, R=R, tau=tau, s=s, true=true_img.astype(np.float32),
                          pred=pred.astype(np.float32), loss=loss.item(), grad=p.grad.numpy().copy(),
                          depth=depth, loss_dtype=str(loss.dtype)))

    ex = imgs.astype(np.float32)[:, None] / 255.0  # [10,1,256,256]
    # KATs: the 10 example images against their own labels (R=64, tau=1.5, s=260: train.py:64)
    add_implicit("kat10_R64", 64, 1.5, 260, ex, labels)
    # random predictions against example images, several (R, tau, s)
    add_implicit("rand_R16_t1_s100", 16, 1.0, 100, ex[:2], sample_params(rng, 2))
    add_implicit("rand_R32_t15_s260", 32, 1.5, 260, ex[2:6], sample_params(rng, 4))
    add_implicit("rand_R64_t1_s100", 64, 1.0, 100, ex[6:8], sample_params(rng, 2))
    # H=512 targets (nearest 512->32 / 512->64 sampling)
    big = np.kron(ex[:2], np.ones((1, 1, 2, 2), np.float32))
    cb = ((np.arange(512)[:, None] + np.arange(512)[None, :]) % 3).astype(np.float32)
    big = big + 0.004 * cb * (big > 0)  # odd pixels differ, so the nearest-index rule matters
    add_implicit("rand_H512_R32", 32, 1.5, 260, big, sample_params(rng, 2))
    add_implicit("rand_H512_R64", 64, 1.5, 260, big, sample_params(rng, 2))
    # non-integer ratio (256 -> 48) exercises the nearest-index rule
    add_implicit("rand_R48", 48, 1.5, 260, ex[:2], sample_params(rng, 2))
    # clamp boundaries and out-of-range values, un-normalised quaternion
    pe = sample_params(rng, 4)
    pe[0, 0] = 0.05; pe[0, 3] = 0.1; pe[0, 5] = 0.0          # exactly on the lower bounds
    pe[1, 1] = 1.0; pe[1, 4] = 1.0; pe[1, 7] = 1.0           # exactly on the upper bounds
    pe[2, 0] = 0.01; pe[2, 3] = 0.05; pe[2, 6] = -0.2        # below the lower bounds
    pe[2, 2] = 1.3; pe[2, 4] = 1.2                           # above the upper bounds
    pe[3, 8:] = pe[3, 8:] * 1.3                              # |q| != 1
    add_implicit("clamp_edges_R32", 32, 1.5, 260, ex[4:8], pe)
    # target in raw 0..255 units (what train.py feeds: classes.py:63,84 + train.py:92)
    add_implicit("raw255_R32", 32, 1.5, 260, ex[8:10] * 255.0, sample_params(rng, 2))
    # B=1 and a perfectly axis-aligned SQ centred on grid nodes (A1==0 zero-fix path)
    pz = np.array([[0.2, 0.25, 0.3, 0.5, 0.7, 16 / 31, 10 / 31, 20 / 31, 0, 0, 0, 1]], np.float32)
    add_implicit("axis_aligned_R32", 32, 1.5, 260, ex[:1], pz)

    out = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            out["c%d_%s" % (i, k)] = np.asarray(v)
    out["n"] = np.asarray(len(cases))
    np.savez_compressed(os.path.join(HERE, "implicit_loss.npz"), **out)

    # ---------------- ExplicitLoss ----------------
    ecases = []
    for (name, R, B) in (("R16_B3", 16, 3), ("R32_B4", 32, 4)):
        tp = sample_params(rng, B)
        pp = sample_params(rng, B)
        if name == "R16_B3":
            pp[0, 0] = 0.05; pp[0, 3] = 0.1; pp[1, 2] = 1.2; pp[2, 8:] *= 0.8
        crit = classes.ExplicitLoss(R, cpu)
        p = torch.tensor(pp, requires_grad=True)
        loss = crit(torch.tensor(tp), p)
        loss.backward()
        ecases.append(dict(name=name, R=R, true=tp, pred=pp, loss=loss.item(), grad=p.grad.numpy().copy()))
    out = {}
    for i, c in enumerate(ecases):
        for k, v in c.items():
            out["c%d_%s" % (i, k)] = np.asarray(v)
    out["n"] = np.asarray(len(ecases))
    np.savez_compressed(os.path.join(HERE, "explicit_loss.npz"), **out)

    # ---------------- IoUAccuracy ----------------
    icases = []
    for (name, R, B) in (("R32_B4", 32, 4), ("R64_B3", 64, 3)):
        tp = sample_params(rng, B)
        pp = tp.copy()
        pp[:, :8] += rng.normal(scale=0.03, size=(B, 8)).astype(np.float32)
        pp[0] = tp[0]  # identical pair -> IoU 1 (classes.py:453-474 smoke test)
        acc = classes.IoUAccuracy(R, cpu)
        red = acc(torch.tensor(tp), torch.tensor(pp)).item()
        acc_n = classes.IoUAccuracy(R, cpu, reduce=False)
        per = acc_n(torch.tensor(tp), torch.tensor(pp)).numpy()
        icases.append(dict(name=name, R=R, true=tp, pred=pp, iou=red, iou_per=per))
    out = {}
    for i, c in enumerate(icases):
        for k, v in c.items():
            out["c%d_%s" % (i, k)] = np.asarray(v)
    out["n"] = np.asarray(len(icases))
    np.savez_compressed(os.path.join(HERE, "iou.npz"), **out)

    # ---------------- heads + GenericNetSQ (seeded weights, regenerated on load) ----------------
    torch.manual_seed(1234)
    feats = torch.randn(5, 256)
    heads = {}
    for cls in ("SizeHead", "ShapeHead", "PositionHead", "RotationHead"):
        torch.manual_seed(99)
        h = getattr(models, cls)(256)
        heads[cls + "_w"] = h.out_layer[0].weight.detach().numpy()
        heads[cls + "_b"] = h.out_layer[0].bias.detach().numpy()
        heads[cls + "_y"] = h(feats).detach().numpy()
    heads["feats"] = feats.numpy()

    torch.manual_seed(4321)
    net = models.GenericNetSQ(4)
    net.eval()
    g = torch.Generator().manual_seed(777)
    x = torch.rand(2, 1, 256, 256, generator=g)
    with torch.no_grad():
        y = net(x).numpy()
    sd = net.state_dict()
    heads["gnet_keys"] = np.array(list(sd.keys()))
    heads["gnet_shapes"] = np.array([str(tuple(v.shape)) for v in sd.values()])
    heads["gnet_param_sums"] = np.array([float(v.double().sum()) for v in sd.values()])
    heads["gnet_y_eval"] = y
    np.savez_compressed(os.path.join(HERE, "models.npz"), **heads)
    print("wrote fixtures:", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
