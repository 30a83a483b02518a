"""The CPU oracle (oracle/sq_oracle.py) against the reference's own outputs (tests/golden)."""
import numpy as np
import pytest

import sq_oracle as O
from _golden import cases, load


@pytest.mark.parametrize("case", cases("implicit_loss.npz"), ids=lambda c: str(c["name"]))
def test_implicit_matches_reference(case):
    L, G, per, imgs = O.implicit_loss(case["true"], case["pred"], int(case["R"]), float(case["tau"]),
                                      float(case["s"]))
    assert abs(L - float(case["loss"])) <= 1e-12 * abs(float(case["loss"]))
    # the reference grad is float32 (pred is f32): compare at f32 resolution
    g = case["grad"].astype(np.float64)
    assert np.abs(G - g).max() <= 2e-7 * max(np.abs(g).max(), 1e-30)
    assert np.abs(imgs - case["depth"]).max() <= 1e-12


@pytest.mark.parametrize("case", cases("explicit_loss.npz"), ids=lambda c: str(c["name"]))
def test_explicit_matches_reference(case):
    L, G, _ = O.explicit_loss(case["true"], case["pred"], int(case["R"]))
    assert abs(L - float(case["loss"])) <= 1e-12 * abs(float(case["loss"]))
    g = case["grad"].astype(np.float64)
    assert np.abs(G - g).max() <= 2e-7 * np.abs(g).max()


@pytest.mark.parametrize("case", cases("iou.npz"), ids=lambda c: str(c["name"]))
def test_iou_matches_reference(case):
    R = int(case["R"])
    assert O.iou_accuracy(case["true"], case["pred"], R) == pytest.approx(float(case["iou"]), rel=1e-7)
    np.testing.assert_allclose(O.iou_accuracy(case["true"], case["pred"], R, reduce=False), case["iou_per"],
                               rtol=1e-15)


def test_quaternion_matches_reference():
    d = load("quaternion.npz")
    np.testing.assert_allclose(O.mat_from_quaternion(d["q"]), d["mat"], atol=1e-15)
    np.testing.assert_allclose(O.conjugate(d["q"]), d["conj"], atol=0)
    np.testing.assert_allclose(O.multiply(d["q"], d["q2"]), d["mul"], atol=1e-15)


def test_quaternion_vjp_finite_difference():
    rng = np.random.default_rng(0)
    q = rng.normal(size=4)
    gM = rng.normal(size=(3, 3))
    an = O.mat_from_quaternion_vjp(q, gM)
    fd = np.zeros(4)
    for i in range(4):
        e = np.zeros(4)
        e[i] = 1e-6
        fd[i] = (np.sum(gM * O.mat_from_quaternion(q + e)) - np.sum(gM * O.mat_from_quaternion(q - e))) / 2e-6
    np.testing.assert_allclose(an, fd, rtol=1e-6, atol=1e-8)


def test_nearest_index_rule():
    # 256 -> 64 picks every 4th pixel, 512 -> 64 every 8th, 256 -> 48 floor(i*16/3)
    assert (O.nearest_src_index(64, 256) == np.arange(64) * 4).all()
    assert (O.nearest_src_index(64, 512) == np.arange(64) * 8).all()
    assert (O.nearest_src_index(48, 256) == np.floor(np.arange(48) * np.float32(256 / 48))).all()


def test_kat_example_images_small_loss():
    # scanner renders vs their own labels: every KAT loss is small
    c = [c for c in cases("implicit_loss.npz") if str(c["name"]) == "kat10_R64"][0]
    _, _, per, _ = O.implicit_loss(c["true"], c["pred"], 64, 1.5, 260, need_grad=False)
    assert per.max() < 0.012


@pytest.mark.parametrize("name", ["rand_R16_t1_s100", "clamp_edges_R32", "rand_R48"])
def test_torch_restatement_matches_reference(name):
    # oracle/ref_torch.py (the CPU baseline's loss) against the same golden vectors
    import torch
    import ref_torch
    c = [c for c in cases("implicit_loss.npz") if str(c["name"]) == name][0]
    crit = ref_torch.ImplicitLossRef(int(c["R"]), float(c["tau"]), float(c["s"]))
    p = torch.tensor(c["pred"], requires_grad=True)
    loss = crit(torch.tensor(c["true"]), p)
    loss.backward()
    assert loss.dtype == torch.float64
    assert abs(loss.item() - float(c["loss"])) <= 1e-12 * abs(float(c["loss"]))
    g = c["grad"]
    assert np.abs(p.grad.numpy() - g).max() <= 2e-7 * np.abs(g).max()


def test_torch_restatement_explicit_matches_reference():
    import torch
    import ref_torch
    c = cases("explicit_loss.npz")[0]
    p = torch.tensor(c["pred"], requires_grad=True)
    loss = ref_torch.ExplicitLossRef(int(c["R"]))(torch.tensor(c["true"]), p)
    loss.backward()
    assert abs(loss.item() - float(c["loss"])) <= 1e-12 * abs(float(c["loss"]))
    assert np.abs(p.grad.numpy() - c["grad"]).max() <= 2e-7 * np.abs(c["grad"]).max()
