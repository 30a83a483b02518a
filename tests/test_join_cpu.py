"""sqr.conv.ResidualJoin: the residual block input's two gradient contributions (conv1's
backward-data and the identity / downsample branch) reach autograd exactly once, in either
order of the two backward calls (torchvision BasicBlock `out += identity`,
/root/reference/torch/models.py:181 via resnet18).  Pure host logic, no GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sq-recovery_amd"))


def _join():
    from sqr.conv import ResidualJoin
    return ResidualJoin()


def test_branch_first_conv1_accumulates():
    j = _join()
    g_branch = torch.ones(2)
    assert j.deposit(g_branch) is None          # branch hands its gradient to the join
    assert j.take() is g_branch                 # conv1 adds it in its epilogue
    assert j.pending is None and not j.acc_done


def test_conv1_first_branch_returns_to_autograd():
    j = _join()
    assert j.take() is None                     # conv1 found nothing: returns its own dx
    g_branch = torch.ones(2)
    assert j.deposit(g_branch) is g_branch      # branch returns to autograd, which adds
    assert j.pending is None and not j.acc_done


def test_repeated_backward_resets():
    j = _join()
    for branch_first in (True, False, True, False):
        g = torch.full((2,), 3.0)
        if branch_first:
            assert j.deposit(g) is None and j.take() is g
        else:
            assert j.take() is None and j.deposit(g) is g
        assert j.pending is None and not j.acc_done


def test_no_join_off_gpu():
    from sqr.conv import ResidualJoin
    x = torch.zeros(1, 8, 4, 4, dtype=torch.bfloat16, requires_grad=True)
    assert ResidualJoin.make(x) is None  # CPU tensors: torch's own autograd add


def test_untaken_deposit_raises_at_end_of_backward():
    """A deposit that conv1's backward never takes in the same backward pass would silently drop the
    residual branch's gradient: the join's end-of-backward callback raises instead."""
    import pytest
    j = _join()

    class Branch(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 2

        @staticmethod
        def backward(ctx, g):
            return j.deposit(g * 2)

    x = torch.ones(3, requires_grad=True)
    with pytest.raises(RuntimeError, match="ResidualJoin"):
        Branch.apply(x).sum().backward()
    assert j.pending is None

    # taken inside the same pass: no error, and the consumer got it
    got = []

    class Conv1(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 3

        @staticmethod
        def backward(ctx, g):
            add = j.take()
            got.append(add)
            return g * 3 + (add if add is not None else 0)

    x = torch.ones(3, requires_grad=True)
    (Branch.apply(x) + Conv1.apply(x)).sum().backward()
    assert torch.equal(x.grad, torch.full((3,), 5.0))
