"""Drop-in for torch/test.py (timoblak/sq-recovery): predict the superquadric parameters of one
depth image with a trained ResNetSQ checkpoint (helpers.load_model format) on MI355X.

    python test.py [--image ../data/example_imgs/000000.bmp] [--model trained_models/model_explicit.pt]

Prints size a and position t in pixel units (x255) like the reference (test.py:40-44).  The
image window of the reference (cv2.imshow) is shown only with --show and OpenCV installed.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from helpers import load_model, read_image_gray  # noqa: E402
from models import ResNetSQ  # noqa: E402


def predict(net, img_u8, device):
    """uint8 [H,W] depth image -> (a, e, t, q) numpy arrays of the single prediction."""
    x = torch.from_numpy(img_u8.astype(np.float32)[None, None] / 255).to(device)
    with torch.no_grad():
        out = net(x)
    return tuple(o.detach().cpu().numpy() for o in out)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", default="../data/example_imgs/000000.bmp")
    ap.add_argument("--model", default="trained_models/model_explicit.pt")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--show", action="store_true")
    args = ap.parse_args(argv)

    net = ResNetSQ(outputs=4, pretrained=False).to(args.device)
    if os.path.exists(args.model):
        _, net, _, _ = load_model(args.model, net, None)
    else:
        print("checkpoint %s not found: using random weights" % args.model)
    net.eval()
    img = read_image_gray(args.image)
    a, e, t, q = predict(net, img, args.device)
    print("Predicted parameters: ")
    print("Size a:", a * 255)
    print("Shape e:", e)
    print("Position t:", t * 255)
    print("Rotation q:", q)
    if args.show:
        import cv2
        cv2.imshow("image", img)
        cv2.waitKey(0)
    return a, e, t, q


if __name__ == "__main__":
    main()
