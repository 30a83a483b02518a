"""Graph-captured data parallelism (sqr.dist.GraphDataParallel) on one GPU, on a world-1 RCCL
communicator owned by libsqr (sqr.dist.Comm / sqr_comm_*): the all-reduce runs, as an identity.
Gradients land in the flat buffer, the eager step equals plain training bitwise, the whole step
including the RCCL all-reduce is captured and replayed as one HIP graph with the same parameter
trajectory, train.py's CapturedStep survives partial batches (eager all-reduces between replays) and a
learning-rate recapture, and train.py --dp-rehearsal matches the plain run.

The checks run in a child process (tests/_dp_graph_child.py) that ends with the product teardown
(sqr.dist.finish) and a normal exit: the test requires every marker and exit status 0, so an abort
anywhere — including from a host thread polling captured work, the round-3 failure of the
ProcessGroupNCCL-based design — fails it."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_graph_dp_world1(tmp_path):
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dp_graph_child.py")
    env = dict(os.environ, NCCL_DEBUG="WARN")  # any RCCL complaint lands in the failure message
    r = subprocess.run([sys.executable, "-u", child, str(tmp_path)], capture_output=True, text=True, timeout=300,
                       env=env)
    marks = ("DP_GRAPH_OK", "DP_STEPPER_OK", "DP_TRAIN_OK", "DP_TEARDOWN_OK")
    ok = r.returncode == 0 and all(m in r.stdout for m in marks)
    key = []
    if not ok:
        # the error text first (a watchdog exception's what() line), then the raw streams in full
        key = [ln for ln in (r.stdout + r.stderr).splitlines()
               if any(w in ln for w in ("what()", "Exception", "Error", "error", "DP_"))
               and "NCCL WARN" not in ln]
        print("\n".join(key))
        print(r.stdout)
        print(r.stderr)
    assert ok, (r.returncode, key[:20])
