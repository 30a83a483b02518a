"""Drop-in for torch/helpers.py (timoblak/sq-recovery): checkpoints, label parsing and scanner
command lines — the parts train.py / test.py use.  The reference's plotting and autograd-debug
utilities (plot_render, plot_points, gray_to_jet, plot_grad_flow, getBack, slerp, randquat;
helpers.py:108-320) are out of scope and not restated.

Checkpoint format is the reference's (helpers.py:42-68):
    {'epoch', 'model_state_dict', 'optimizer_state_dict', 'loss'}
with un-prefixed state-dict keys; a DistributedDataParallel model is unwrapped before saving, so
single-GPU and 8-GPU runs write interchangeable files.  The scanner helpers import cv2 lazily (it
is not needed on the training path).
"""
import os

import numpy as np
import torch


def norm_img(img):
    img = img - img.min()
    return img / img.max()


def quat2mat(q):
    """helpers.py:17-24: rotation matrix of the NORMALISED quaternion (xyzw)."""
    q = np.asarray(q, dtype=np.float64)
    x, y, z, w = q / np.sqrt(np.square(q).sum())
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def get_command(scanner_loc, fn, params):
    """helpers.py:27-39: `scanner out.bmp a1 a2 a3 e1 e2 px py pz r11..r33` command line."""
    params = np.asarray(params)
    vals = list(params[:3]) + list(params[3:5]) + list(np.ravel(params[5:8])) + list(np.ravel(params[8:]))
    return scanner_loc + "scanner " + fn + " " + "".join("%f " % v for v in vals) + "\n"


def _unwrap(model):
    return model.module if hasattr(model, "module") and isinstance(model.module, torch.nn.Module) else model


def save_model(path, epoch, model, optimizer, loss, scaler=None):
    """helpers.py:42-48.  scaler (optional, fp16 runs): its state_dict goes under the extra key
    'scaler_state_dict' — the reference's four keys are unchanged, so either side loads the file."""
    ck = {"epoch": epoch, "model_state_dict": _unwrap(model).state_dict(),
          "optimizer_state_dict": optimizer.state_dict(), "loss": loss}
    if scaler is not None:
        ck["scaler_state_dict"] = scaler.state_dict()
    torch.save(ck, path)


def _safe_load(path, map_location):
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except Exception:
        # reference checkpoints keep numpy float64 running means in 'loss' (train.py:170)
        import numpy.core.multiarray as ma
        with torch.serialization.safe_globals([ma.scalar, np.dtype, np.dtypes.Float64DType]):
            return torch.load(path, map_location=map_location, weights_only=True)


def load_model(path, model, optimizer, plot=False, scaler=None):
    """helpers.py:51-68 (map_location cuda:0 when a GPU is present, as the reference).  scaler
    (optional): restored from 'scaler_state_dict' when the checkpoint has it (a resumed fp16 run
    keeps its loss scale and growth tracker)."""
    print("Loading model: " + path)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    checkpoint = _safe_load(path, dev)
    _unwrap(model).load_state_dict(checkpoint["model_state_dict"])
    if optimizer is not None:
        optimizer.load_state_dict(checkpoint["optimizer_state_dict"])
    if scaler is not None and "scaler_state_dict" in checkpoint:
        scaler.load_state_dict(checkpoint["scaler_state_dict"])
    epoch = checkpoint["epoch"]
    loss = checkpoint["loss"]
    if plot:
        from matplotlib import pyplot as plt
        plt.plot(loss["loss"], label="Loss")
        plt.plot(loss["val_loss"], label="Validation Loss")
        plt.title("Progression of loss during training")
        plt.xlabel("# Epochs")
        plt.ylabel("Loss")
        plt.legend()
        plt.show()
    return epoch, model, optimizer, loss


def _scanner_params(p, clip):
    M = quat2mat(p[-4:])
    if clip:
        return np.concatenate((np.clip(p[:3], 0.05, 1) * 255., np.clip(p[3:5], 0.1, 1), np.clip(p[5:8], 0, 1) * 255,
                               M.ravel()))
    return np.concatenate((p[:3] * 255., p[3:5], p[5:8] * 255, M.ravel()))


def save_compare_images(params_true, params_pred):
    """helpers.py:71-81: renders true/predicted SQs with the external `scanner` binary."""
    for i, (true, pred) in enumerate(zip(params_true, params_pred)):
        os.system(get_command("../", "examples/" + str(i) + "_true.bmp", _scanner_params(true, False)))
        os.system(get_command("../", "examples/" + str(i) + "_pred.bmp", _scanner_params(pred, True)))


def compare_images(params_true, params_pred, wait=16):
    """helpers.py:84-100."""
    import cv2
    for true, pred in zip(params_true, params_pred):
        os.system(get_command("../", "true.bmp", _scanner_params(true, False)))
        os.system(get_command("../", "pred.bmp", _scanner_params(pred, True)))
        combined = np.hstack([cv2.imread("true.bmp", 0), cv2.imread("pred.bmp", 0)])
        cv2.imshow("comparison", combined)
        cv2.waitKey(wait)


def read_image_gray(path):
    """cv2.imread(path, 0) for the scanner's 24-bit BMPs without OpenCV (uses cv2 when present for
    other formats).  Gray = the common channel value; genuinely colour BMPs use cv2's weights."""
    with open(path, "rb") as f:
        b = f.read()
    if b[:2] != b"BM" or int.from_bytes(b[28:30], "little") != 24:
        import cv2
        return cv2.imread(path, 0)
    off = int.from_bytes(b[10:14], "little")
    w = int.from_bytes(b[18:22], "little", signed=True)
    h = int.from_bytes(b[22:26], "little", signed=True)
    stride = (w * 3 + 3) & ~3
    rows = np.frombuffer(b[off:off + stride * abs(h)], np.uint8).reshape(abs(h), stride)[:, :w * 3]
    bgr = rows.reshape(abs(h), w, 3)
    if (bgr[..., 0] == bgr[..., 1]).all() and (bgr[..., 1] == bgr[..., 2]).all():
        img = bgr[..., 0]
    else:
        img = np.clip(np.rint(0.114 * bgr[..., 0] + 0.587 * bgr[..., 1] + 0.299 * bgr[..., 2]), 0, 255).astype(np.uint8)
    return np.ascontiguousarray(img[::-1] if h > 0 else img)


def change_lr(opt, lr):
    for g in opt.param_groups:
        g["lr"] = lr


def parse_csv(csvfile):
    """helpers.py:188-218: rows 'fn,a1,a2,a3,e1,e2,t1,t2,t3,m11..m33,q1..q4' ->
    float32 [a/255 (3), e (2), t/255 (3), q (4)] per image."""
    with open(csvfile, "r") as f:
        lines = f.read().split("\n")
    print("Parsing csv " + csvfile)
    labels = []
    for line in lines:
        if line == "":
            continue
        v = line.split(",")
        row = [float(v[i]) / 255.0 if i in (1, 2, 3, 6, 7, 8) else float(v[i]) for i in range(1, 9)]
        row += [float(v[i]) for i in range(-4, 0)]
        labels.append(np.array(row, dtype=np.float32))
    print("Size of data: " + str(len(labels)))
    print("----------------------------------------------------------------")
    return labels
