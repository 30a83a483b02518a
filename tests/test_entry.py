"""Drop-in entry points: helpers.read_image_gray (CPU), train.py and test.py (GPU)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def _write_bmp24(path, img):
    """minimal bottom-up 24-bit BMP writer (gray replicated in B, G, R), the scanner's format"""
    h, w = img.shape
    stride = (w * 3 + 3) & ~3
    rows = np.zeros((h, stride), np.uint8)
    rows[:, :w * 3] = np.repeat(img[::-1], 3, axis=1)
    hdr = (b"BM" + (54 + rows.size).to_bytes(4, "little") + b"\0\0\0\0" + (54).to_bytes(4, "little")
           + (40).to_bytes(4, "little") + w.to_bytes(4, "little") + h.to_bytes(4, "little")
           + (1).to_bytes(2, "little") + (24).to_bytes(2, "little") + b"\0" * 24)
    with open(path, "wb") as f:
        f.write(hdr + rows.tobytes())


def test_read_image_gray_roundtrip(tmp_path):
    from helpers import read_image_gray
    img = np.load(os.path.join(GOLDEN, "example_images.npz"))["images"][3]
    p = str(tmp_path / "x.bmp")
    _write_bmp24(p, img)
    assert np.array_equal(read_image_gray(p), img)


def test_train_parse_defaults():
    import train
    a = train.parse_args([])
    assert a.batch_size == 32 and a.lr == 1e-4 and a.render_size == 64  # train.py:26,40,64


@pytest.mark.gpu
def test_train_synthetic_epoch(tmp_path):
    import train
    from helpers import load_model
    from models import ResNetSQ
    ck = str(tmp_path / "m.pt")
    losses, val = train.main(["--synthetic", "80", "--epochs", "2", "--batch-size", "8", "--render-size", "32",
                              "--pretrained", "0", "--model-location", ck])
    assert len(losses) == 2 and all(np.isfinite(losses)) and all(np.isfinite(val))
    assert os.path.exists(ck)
    net = ResNetSQ(outputs=4, pretrained=False).cuda()
    epoch, net, _, hist = load_model(ck, net, None)
    assert epoch in (0, 1) and len(hist["loss"]) >= 1


@pytest.mark.gpu
def test_test_py_predicts(tmp_path):
    import importlib.util
    from conftest import PKG
    spec = importlib.util.spec_from_file_location("sq_test_entry", os.path.join(PKG, "test.py"))
    sq_test = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sq_test)  # not `import test`: that name is also a stdlib package
    img = np.load(os.path.join(GOLDEN, "example_images.npz"))["images"][0]
    p = str(tmp_path / "000000.bmp")
    _write_bmp24(p, img)
    torch.manual_seed(0)
    a, e, t, q = sq_test.main(["--image", p, "--model", str(tmp_path / "missing.pt")])
    assert a.shape == (1, 3) and e.shape == (1, 2) and t.shape == (1, 3) and q.shape == (1, 4)
    assert np.allclose(np.linalg.norm(q, axis=1), 1, atol=1e-5)  # RotationHead normalises
