"""Graph-captured data parallelism (sqr.dist.GraphDataParallel) on one GPU: an RCCL process group
of world size 1 (the all-reduce runs, as an identity) — gradients land in the flat buffer, the
eager step equals plain training bitwise, and the whole step including the RCCL all-reduce is
captured and replayed as one HIP graph with the same parameter trajectory.

The checks run in a child process (tests/_dp_graph_child.py) that exits without destroying the
communicator: that teardown, after collectives were captured in a graph, aborts intermittently
inside RCCL on this image and would take the whole test session down with it."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_graph_dp_world1(tmp_path):
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dp_graph_child.py")
    r = subprocess.run([sys.executable, "-u", child, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "DP_GRAPH_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
