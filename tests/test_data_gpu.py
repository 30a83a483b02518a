"""sqr.data.DevicePrefetcher on the GPU: pinned DataLoader batches arrive on the device, in order and
bit-identical, while the next batch's copy is in flight on a side stream."""
import pytest
import torch
import torch.utils.data as data

pytestmark = pytest.mark.gpu


def test_prefetcher_gpu_batches_identical():
    from sqr.data import DevicePrefetcher
    g = torch.Generator().manual_seed(0)
    x = torch.rand(37, 1, 64, 64, generator=g)
    y = torch.rand(37, 12, generator=g).double()
    loader = data.DataLoader(data.TensorDataset(x, y), batch_size=8, shuffle=False, num_workers=2, pin_memory=True)
    seen = 0
    for bx, by in DevicePrefetcher(loader, "cuda:0"):
        assert bx.is_cuda and by.is_cuda and by.dtype == torch.float64
        # consume on the compute stream (the prefetcher made it wait for the copy)
        s = (bx * 2).sum()
        assert torch.equal(bx.cpu(), x[seen:seen + bx.shape[0]]) and torch.equal(by.cpu(), y[seen:seen + by.shape[0]])
        assert torch.isfinite(s)
        seen += bx.shape[0]
    assert seen == 37
