"""Host -> device batch prefetch for the h5 data path.

The reference feeds train.py from a torch DataLoader over H5Dataset (torch/train.py:24-40,
torch/classes.py:32-101) and copies each batch to the GPU synchronously at the top of the step.
Here the DataLoader's worker processes decode into pinned host memory (pin_memory=True) and
DevicePrefetcher copies batch i+1 to the device on a side HIP stream while batch i trains: the
copy engine and the compute stream overlap, and the compute stream waits only on an event.  On a
CPU device it is a plain pass-through.
"""
import torch


def _to(obj, device):
    if torch.is_tensor(obj):
        return obj.to(device, non_blocking=True)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(o, device) for o in obj)
    return obj


def _record(obj, stream):
    if torch.is_tensor(obj):
        obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record(o, stream)


class DevicePrefetcher:
    """Iterate `loader` (batches of tensors / tuples of tensors) with every batch already on
    `device`: batch i+1's host->device copy runs on a side stream during batch i."""

    def __init__(self, loader, device):
        self.loader = loader
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        if not self.cuda:
            yield from self.loader
            return
        side = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)

        def stage():
            try:
                host = next(it)
            except StopIteration:
                return None
            with torch.cuda.stream(side):
                dev = _to(host, self.device)
                ev = torch.cuda.Event()
                ev.record(side)
            return dev, ev

        nxt = stage()
        while nxt is not None:
            dev, ev = nxt
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            _record(dev, cur)  # the caching allocator must not recycle it before the compute stream is done
            nxt = stage()      # next copy overlaps this batch's compute
            yield dev
