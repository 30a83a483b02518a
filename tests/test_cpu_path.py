"""The product's host-CPU path (BASELINE config 1: the reference's CPU training run — fp32 ResNetSQ,
float64 losses) against the reference's own fixtures (tests/golden/*.npz) and the CPU
restatement of the network.  CPU only; libsqr is not needed for any of it."""
import numpy as np
import pytest
import torch

from _golden import cases


def _classes():
    import classes
    return classes


@pytest.mark.parametrize("case", cases("implicit_loss.npz"), ids=lambda c: str(c["name"]))
def test_cpu_implicit_vs_golden(case):
    C = _classes()
    crit = C.ImplicitLoss(int(case["R"]), "cpu", float(case["tau"]), float(case["s"]))
    p = torch.tensor(case["pred"], requires_grad=True)
    loss = crit(torch.tensor(case["true"]), p)
    loss.backward()
    assert loss.dtype == torch.float64 and loss.dim() == 0
    assert abs(loss.item() - float(case["loss"])) <= 1e-12 * abs(float(case["loss"]))
    np.testing.assert_allclose(p.grad.numpy(), case["grad"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("case", cases("explicit_loss.npz"), ids=lambda c: str(c["name"]))
def test_cpu_explicit_vs_golden(case):
    C = _classes()
    p = torch.tensor(case["pred"], requires_grad=True)
    loss = C.ExplicitLoss(int(case["R"]), "cpu")(torch.tensor(case["true"]), p)
    loss.backward()
    assert loss.dtype == torch.float64
    assert abs(loss.item() - float(case["loss"])) <= 1e-12 * abs(float(case["loss"]))
    np.testing.assert_allclose(p.grad.numpy(), case["grad"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("case", cases("iou.npz"), ids=lambda c: str(c["name"]))
def test_cpu_iou_vs_golden(case):
    C = _classes()
    R = int(case["R"])
    t, p = torch.tensor(case["true"]), torch.tensor(case["pred"])
    assert C.IoUAccuracy(R, "cpu")(t, p).item() == pytest.approx(float(case["iou"]), rel=1e-6)
    np.testing.assert_allclose(C.IoUAccuracy(R, "cpu", reduce=False)(t, p).numpy(), case["iou_per"], rtol=1e-12)


def test_cpu_render_matches_example_kat():
    """The CPU render of the example images' labels reproduces the reference's KAT losses
    (example_images.npz: scanner images, labels; SURVEY §4 lists the reference values)."""
    from _golden import load
    C = _classes()
    d = load("example_images.npz")
    x = torch.tensor(d["images"][:3], dtype=torch.float32).unsqueeze(1) / 255.0
    y = torch.tensor(d["labels"][:3])
    loss = C.ImplicitLoss(64, "cpu", 1.5, 260)(x, y)
    assert 0.004 < loss.item() < 0.011


def test_resnetsq_cpu_matches_restatement():
    """The product ResNetSQ on CPU tensors (torch's own CPU convs / BatchNorm) == the CPU
    restatement on the same state dict (train and eval mode)."""
    import models
    import ref_torch
    torch.manual_seed(0)
    net = models.ResNetSQ(outputs=4, pretrained=False)
    ref = ref_torch.ResNetSQRef()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(2, 1, 64, 64, generator=torch.Generator().manual_seed(1))
    for train in (True, False):
        net.train(train)
        ref.train(train)
        with torch.no_grad():
            a = torch.cat(net(x), 1)
            b = torch.cat(ref(x), 1)
        assert (a - b).abs().max().item() <= 1e-6


def test_train_py_config1_cpu_explicit(tmp_path):
    """BASELINE config 1: train.py with the explicit loss, batch 4, on the CPU — one epoch of a
    tiny synthetic set, the loss is finite and a checkpoint in the reference format is written."""
    import train
    ckpt = tmp_path / "model.pt"
    losses, val = train.main(["--device", "cpu", "--loss", "explicit", "--synthetic", "10", "--batch-size", "4",
                              "--epochs", "1", "--render-size", "16", "--pretrained", "0",
                              "--model-location", str(ckpt), "--log-interval", "100"])
    assert len(losses) == 1 and np.isfinite(losses[0]) and np.isfinite(val[0])
    sd = torch.load(str(ckpt), map_location="cpu", weights_only=True)
    assert set(sd) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss"}
    assert "encoder.layer1.0.conv1.weight" in sd["model_state_dict"]
