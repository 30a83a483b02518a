"""sqr.data.DevicePrefetcher on a CPU device: a pass-through of the DataLoader (same batches, same
order, same structure) — the reference's train.py loop (torch/train.py:74-90) sees no difference."""
import torch
import torch.utils.data as data


def test_prefetcher_cpu_passthrough():
    from sqr.data import DevicePrefetcher
    x = torch.arange(40, dtype=torch.float32).view(10, 4)
    y = torch.arange(10)
    loader = data.DataLoader(data.TensorDataset(x, y), batch_size=4, shuffle=False)
    got = list(DevicePrefetcher(loader, "cpu"))
    assert len(got) == 3 and len(DevicePrefetcher(loader, "cpu")) == 3
    assert torch.equal(torch.cat([b[0] for b in got]), x) and torch.equal(torch.cat([b[1] for b in got]), y)
    assert [b[0].shape[0] for b in got] == [4, 4, 2]  # the partial last batch is kept (drop_last=False)
