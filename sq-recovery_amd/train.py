"""Drop-in for torch/train.py (timoblak/sq-recovery) on MI355X.

Same loop as the reference (train.py:72-175): per batch zero_grad -> ResNetSQ forward ->
cat(a, e, t, q) -> loss -> backward -> Adam(1e-4) step -> loss.item(); NaN check on
encoder.fc[0].weight.grad; per epoch a validation pass with the loss and IoUAccuracy(64, full=True),
ReduceLROnPlateau(patience 25) on the validation loss, checkpoint (helpers.save_model format)
whenever the validation loss improves.  The loss is the reference's choice (train.py:62-64):
--loss implicit (default: ImplicitLoss(R, tau 1.5, s 260)(images, pred)), explicit
(ExplicitLoss(R)(labels, pred)) or combined (their sum, the visu.py pairing).

MI355X-specific:
  * on CUDA the convs / BatchNorm / losses run on the libsqr HIP kernels (nothing falls back);
    --device cpu runs the reference's CPU configuration (BASELINE config 1) on torch's CPU ops and
    the float64 host losses (sqr/cpu.py);
  * --bf16 / --fp16 run the network under autocast (fp16 with sqr.amp.GradScaler loss scaling); the
    loss kernels always consume fp32 params;
  * data parallel: launch with `torchrun --nproc-per-node 8 train.py ...` — one process per GPU,
    sqr.dist.GraphDataParallel (the bucketed all-reduce on libsqr's RCCL communicator, overlapped
    with backward, captured in the step graph below as in bench.py), each rank trains on its own
    contiguous shard (sqr.dist.shard), rank 0 logs and writes checkpoints (un-prefixed state-dict
    keys); --dp-rehearsal runs that path on one GPU with a world-1 communicator;
  * --synthetic N trains on N rendered SQ images (no dataset files needed); otherwise the
    reference's H5Dataset(dataset_location, parse_csv(labels), 0.9) is used (needs h5py);
  * on CUDA the whole training step (forward, loss, backward, all-reduce, Adam / loss scaler) is
    captured in one HIP graph and replayed per batch (sqr.step.CapturedStep: static batch buffers,
    loss and the NaN check of encoder.fc[0].weight.grad read back one step behind, so the host
    never stalls the device); --graph 0 runs the reference's eager loop;
  * each epoch prints its training throughput (images/s over all ranks, train loop only).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.optim as optim
import torch.utils.data as data

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from classes import ExplicitLoss, H5Dataset, ImplicitLoss, IoUAccuracy, SyntheticDataset  # noqa: E402
from helpers import load_model, parse_csv, save_compare_images, save_model  # noqa: E402
from models import ResNetSQ  # noqa: E402
from sqr import amp, dist  # noqa: E402
from sqr.data import DevicePrefetcher  # noqa: E402
from sqr.optim import Adam  # noqa: E402
from sqr.step import CapturedStep  # noqa: E402
from sqr.tail import cat_heads  # noqa: E402


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dataset-location", default="../data/data/")
    ap.add_argument("--labels", default="../data/annotations/data_labels.csv")
    ap.add_argument("--synthetic", type=int, default=0, help="train on N synthetic images instead of the h5 set")
    ap.add_argument("--model-location", default="trained_models/model_full.pt")
    ap.add_argument("--epochs", type=int, default=20000)
    ap.add_argument("--batch-size", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--render-size", type=int, default=64, help="ImplicitLoss render size (train.py:64)")
    ap.add_argument("--explicit-render-size", type=int, default=32, help="ExplicitLoss render size (train.py:62)")
    ap.add_argument("--log-interval", type=int, default=1)
    ap.add_argument("--running-mean", type=int, default=100)
    ap.add_argument("--pretrained", type=int, default=1)
    ap.add_argument("--continue-training", action="store_true")
    ap.add_argument("--bf16", action="store_true", help="bf16 autocast for the network")
    ap.add_argument("--fp16", action="store_true", help="fp16 autocast + dynamic loss scaling")
    ap.add_argument("--loss", default="implicit", choices=("implicit", "explicit", "combined"),
                    help="training loss (reference train.py:62-64)")
    ap.add_argument("--device", default="auto", choices=("auto", "cuda", "cpu"))
    ap.add_argument("--compare-images", action="store_true",
                    help="render val batch 0 with the external scanner (helpers.save_compare_images)")
    ap.add_argument("--max-steps", type=int, default=0, help="stop an epoch after this many steps (0 = all)")
    ap.add_argument("--graph", type=int, default=1, help="capture the training step in a HIP graph (CUDA; 0 = eager)")
    ap.add_argument("--dist-backend", default="", choices=("", "nccl", "gloo"),
                    help="data-path backend (default: nccl on CUDA = libsqr's RCCL communicator, one GPU per rank, "
                         "host group gloo; gloo on CPU; gloo on CUDA runs several ranks on one GPU, eagerly)")
    ap.add_argument("--dp-rehearsal", action="store_true",
                    help="one CUDA rank: run the N>1 data path (flat gradient buffer, bucketed all-reduce on "
                         "libsqr's RCCL communicator, captured in the step graph) on a world-1 communicator")
    return ap.parse_args(argv)


def _batches(dataset, rank, world, batch_size, device=torch.device("cpu")):
    """This rank's batches of the current split (contiguous shard, no shuffle, like the reference;
    the last batch may be partial, as with the reference's DataLoader)."""
    idx = dist.shard(len(dataset), rank, world)
    if isinstance(dataset, SyntheticDataset):
        off = 0 if dataset.mode == 0 else dataset.n_train
        for i in range(idx.start, idx.stop, batch_size):
            j = min(i + batch_size, idx.stop)
            yield (dataset.images[off + i:off + j], dataset.labels[off + i:off + j])
        return
    # pinned-memory workers + side-stream prefetch of the next batch (sqr.data.DevicePrefetcher)
    loader = data.DataLoader(data.Subset(dataset, list(idx)), batch_size=batch_size, shuffle=False, num_workers=4,
                             pin_memory=device.type == "cuda")
    yield from DevicePrefetcher(loader, device)


def main(argv=None):
    args = parse_args(argv)
    use_cuda = args.device == "cuda" or (args.device == "auto" and torch.cuda.is_available())
    rank, world, device = dist.init(args.dist_backend or ("nccl" if use_cuda else "gloo"),
                                    "cuda" if use_cuda else "cpu")
    main_rank = rank == 0
    if main_rank:
        print("Using device: %s (world size %d)" % (device, world))

    if args.synthetic:
        # every rank renders the same set and trains on its own shard
        dataset = SyntheticDataset(args.synthetic, device, train_split=0.9, seed=0)
    else:
        dataset = H5Dataset(args.dataset_location, parse_csv(args.labels), train_split=0.9, dataset_file="dataset.h5")

    net = ResNetSQ(outputs=4, pretrained=bool(args.pretrained)).to(device)
    # torch.optim.Adam semantics / state_dict on libsqr's fused step (+ 16-bit conv weight packing)
    optimizer = Adam(net.parameters(), lr=args.lr, weight_decay=0)
    amp_dtype = torch.bfloat16 if args.bf16 else (torch.float16 if args.fp16 else None)
    if amp_dtype is not None and use_cuda:
        optimizer.attach(net, amp_dtype)
    scaler = amp.GradScaler(device) if (args.fp16 and use_cuda) else None
    scheduler = optim.lr_scheduler.ReduceLROnPlateau(optimizer, patience=25)
    starting_epoch = 0
    if args.continue_training:
        if main_rank:
            print("Continuing with training...")
        starting_epoch, net, optimizer, _ = load_model(args.model_location, net, optimizer, scaler=scaler)
    # N > 1: bucketed gradient all-reduce overlapped with backward (the same machinery bench.py
    # captures in its step graph); the model itself stays unwrapped (checkpoints keep plain keys)
    if args.dp_rehearsal and world == 1 and use_cuda:
        dist.open_comm(device)
    gdp = dist.GraphDataParallel(net, optimizer, device) if (world > 1 or dist.comm() is not None) else None
    model = net

    implicit = ImplicitLoss(args.render_size, device, 1.5, 260)
    explicit = ExplicitLoss(args.explicit_render_size, device)

    def loss_criterion(images, labels, pred):
        if args.loss == "implicit":
            return implicit(images, pred)
        if args.loss == "explicit":
            return explicit(labels, pred)
        return explicit(labels, pred) + implicit(images, pred)

    accuracy_estimator = IoUAccuracy(render_size=64, device=device, full=True)

    def forward(x):
        with torch.autocast("cuda", dtype=amp_dtype or torch.bfloat16, enabled=amp_dtype is not None and use_cuda):
            out = model(x)
        return cat_heads(out)  # torch.cat of the heads (train.py:88-89; no copy after the fused tail)

    def train_body(x, labels):
        pred_labels = forward(x)
        loss = loss_criterion(x, labels, pred_labels)
        (scaler.scale(loss) if scaler is not None else loss).backward()
        if gdp is not None:
            gdp.allreduce()
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        return loss

    # the reference's per-step NaN check (train.py:115) on encoder.fc[0].weight.grad
    # (a gloo process group on CUDA — several ranks on one GPU — all-reduces through the host: eager)
    stepper = CapturedStep(train_body, optimizer, device, check=lambda: net.encoder.fc[0].weight.grad,
                           graph=bool(args.graph) and dist.capturable())

    best_val_loss = None
    mean_losses, mean_val_losses, mean_val_accs = [], [], []
    for epoch in range(starting_epoch, args.epochs):
        losses, val_losses, val_accuracies = [], [], []
        net.train()
        dataset.set_mode(0)
        n_items = len(dataset)
        sizes = []

        def report(results):
            # (loss, nan) of finished steps in order: the reference's bookkeeping and log lines
            for loss_v, nan in results:
                step_idx = len(losses)
                losses.append(loss_v)
                if nan:
                    print("--------------- NAN GRADS!!!! ---------------")
                if main_rank and step_idx % args.log_interval == 0:
                    sys.stdout.write("\033[K")
                    print("Train Epoch: {} Step: {} [{}/{}]\tLoss: {:,.6f}".format(
                        epoch, step_idx, (step_idx + 1) * sizes[step_idx] * world, n_items,
                        np.mean(losses[-args.running_mean:])), end="\r")

        dist.barrier()
        t0 = time.perf_counter()
        for batch_idx, (x, true_labels) in enumerate(_batches(dataset, rank, world, args.batch_size, device)):
            if args.max_steps and batch_idx >= args.max_steps:
                break
            x, true_labels = x.to(device, non_blocking=True), true_labels.to(device, non_blocking=True)
            sizes.append(len(x))
            stepper.step(x, true_labels)
            # log one step behind: the previous step has finished by the time this one is queued
            report(stepper.drain(stepper.launched - 1 if stepper.graph is not None else None))
        report(stepper.drain())
        dist.barrier()
        secs = dist.max_over_ranks(time.perf_counter() - t0)
        if main_rank and losses:
            sys.stdout.write("\033[K")
            print("Train Epoch: {} throughput: {:.1f} images/s ({} steps, {} ranks, {})".format(
                epoch, sum(sizes) * world / secs, len(sizes), world,
                "HIP graph" if stepper.captures else "eager"))
        train_mean = dist.mean_over_ranks(np.mean(losses)) if losses else float("nan")
        mean_losses.append(train_mean)
        if main_rank:
            sys.stdout.write("\033[K")
            print("-" * 72)
            print("Train Epoch: {} [(100%)]\tLoss: {:.6f}".format(epoch, train_mean))

        net.eval()
        dataset.set_mode(1)
        with torch.no_grad():
            for batch_idx, (x, true_labels) in enumerate(_batches(dataset, rank, world, args.batch_size, device)):
                if args.max_steps and batch_idx >= args.max_steps:
                    break
                x, true_labels = x.to(device), true_labels.to(device)
                pred_labels = forward(x)
                loss = loss_criterion(x, true_labels, pred_labels)
                acc = accuracy_estimator(true_labels, pred_labels)
                if batch_idx == 0 and main_rank and args.compare_images:
                    save_compare_images(true_labels.cpu().numpy(), pred_labels.cpu().numpy())
                val_losses.append(loss.item())
                val_accuracies.append(acc.item())
        val_loss_mean = dist.mean_over_ranks(np.mean(val_losses)) if val_losses else float("nan")
        val_accuracy_mean = dist.mean_over_ranks(np.mean(val_accuracies)) if val_accuracies else float("nan")
        mean_val_accs.append(val_accuracies)
        mean_val_losses.append(val_loss_mean)
        scheduler.step(val_loss_mean)

        if main_rank:
            if best_val_loss is None or val_loss_mean < best_val_loss:
                print("Saving first model.." if best_val_loss is None else "New best loss achieved. Saving model..")
                best_val_loss = val_loss_mean
                os.makedirs(os.path.dirname(args.model_location) or ".", exist_ok=True)
                save_model(args.model_location, epoch, model, optimizer,
                           {"loss": mean_losses, "val_loss": mean_val_losses, "val_acc": mean_val_accs},
                           scaler=scaler)
            print("-" * 72)
            print("Validation Epoch: {}\tLoss: {:,.6f}\tAccuracy: {:,.6f}".format(epoch, val_loss_mean,
                                                                                 val_accuracy_mean))
            print("=" * 72)
        else:
            best_val_loss = val_loss_mean if best_val_loss is None else min(best_val_loss, val_loss_mean)
    if gdp is not None:
        gdp.close(optimizer)
    # ordered teardown: the step graph (with any captured all-reduces) before the process group
    dist.finish(stepper.close())
    return mean_losses, mean_val_losses


if __name__ == "__main__":
    # a CommFailure (aborted RCCL communicator) ends the process at once with status 3
    dist.exit_on_comm_failure(main)
