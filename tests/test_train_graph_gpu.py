"""train.py's captured step (sqr.step.CapturedStep): the whole training step replayed as one HIP graph
on static batch buffers, the loss and the reference's NaN check read back one step behind.  The
run must be bitwise identical to the reference's eager loop (--graph 0): same per-epoch losses, same
checkpoint (parameters and BatchNorm buffers), with the epoch's partial last batch run eagerly in
between replays."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, graph, extra=()):
    import train
    ck = os.path.join(str(tmp_path), "ck_graph%d.pt" % graph)
    torch.manual_seed(0)
    dt = list(extra) or ["--bf16"]
    tl, vl = train.main(["--synthetic", "44", "--batch-size", "8", "--epochs", "2", "--render-size", "32",
                         "--pretrained", "0", "--graph", str(graph), "--model-location", ck,
                         "--log-interval", "1"] + dt)
    return tl, vl, torch.load(ck, map_location="cpu", weights_only=True), ck


@pytest.mark.timeout(300)
def test_train_graph_equals_eager(tmp_path, capsys):
    tl_g, vl_g, ck_g, _ = _run(tmp_path, 1)
    out = capsys.readouterr().out
    assert "HIP graph" in out and "images/s" in out
    tl_e, vl_e, ck_e, _ = _run(tmp_path, 0)
    out_e = capsys.readouterr().out
    assert "eager" in out_e
    # 44 images, 90 % train = 39: 4 full batches of 8 (1 eager warm-up, 1 capture, replays) + 7
    assert tl_g == tl_e and vl_g == vl_e, (tl_g, tl_e, vl_g, vl_e)
    for k, v in ck_e["model_state_dict"].items():
        assert torch.equal(ck_g["model_state_dict"][k], v), k
    assert ck_g["epoch"] == ck_e["epoch"]


@pytest.mark.timeout(300)
def test_train_graph_fp16_scaler_checkpoint(tmp_path):
    """--fp16: the captured step includes the loss scaler; its state rides in the checkpoint under an
    extra key and a resumed run restores it."""
    import helpers
    import models
    from sqr import amp
    from sqr.optim import Adam
    _, _, ck, path = _run(tmp_path, 1, ["--fp16"])
    sd = ck["scaler_state_dict"]
    assert sd["scale"] > 0 and sd["growth_interval"] == 2000
    assert {"epoch", "model_state_dict", "optimizer_state_dict", "loss"} <= set(ck)
    net = models.ResNetSQ(outputs=4, pretrained=False).cuda()
    scaler = amp.GradScaler("cuda")
    scaler.update(new_scale=7.0)
    helpers.load_model(path, net, Adam(net.parameters(), lr=1e-4), scaler=scaler)
    assert scaler.get_scale() == sd["scale"] and scaler.state_dict()["_growth_tracker"] == sd["_growth_tracker"]
