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
