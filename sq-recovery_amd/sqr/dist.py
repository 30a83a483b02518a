"""Data-parallel plumbing shared by train.py and bench.py.

One process per GPU (torchrun / torch.distributed.run sets RANK, LOCAL_RANK, WORLD_SIZE), backend
"nccl" = RCCL over xGMI on ROCm.  Images are independent, so the only data-path collective is the
gradient all-reduce that DistributedDataParallel buckets and overlaps with backward; BatchNorm keeps
per-rank batch statistics (the reference trains on one GPU; DDP without SyncBN is the documented
multi-GPU semantics: an N-rank step equals the average of N independent per-rank gradients).
"""
import os

import torch
import torch.distributed as dist

# DDP bucket size: 45.5 MB of fp32 ResNetSQ gradients -> 3 buckets; large enough that each ring
# all-reduce runs near xGMI link bandwidth, small enough that the first bucket (layer4 + heads)
# starts while layer3..layer1 backward still runs.
BUCKET_MB = 16


def env():
    """(rank, world_size, local_rank) from the torchrun environment (1 process => 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl"):
    """Set this rank's device and join the process group when WORLD_SIZE > 1.
    Returns (rank, world, device)."""
    rank, world, local = env()
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    return rank, world, device


def is_main():
    return not dist.is_initialized() or dist.get_rank() == 0


def shard(n, rank, world):
    """Indices of rank's shard of n samples: contiguous blocks of size n // world (the remainder
    is dropped so every rank runs the same number of equal batches — the all-reduce average then
    equals the global-batch mean of the per-sample losses, classes.py:293)."""
    per = n // world
    return range(rank * per, (rank + 1) * per)


def wrap(model, device):
    """DistributedDataParallel with the bucket layout above (identity when not distributed)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=BUCKET_MB, gradient_as_bucket_view=True,
               broadcast_buffers=False)


def max_over_ranks(x):
    """max of a host float over all ranks (bench timing: the job is as slow as its slowest rank)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def mean_over_ranks(x):
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.item() / dist.get_world_size()


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def finish():
    if dist.is_initialized():
        dist.destroy_process_group()
