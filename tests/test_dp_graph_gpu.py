"""Graph-captured data parallelism (sqr.dist.GraphDataParallel) on one GPU: an RCCL process group
of world size 1 (the all-reduce runs, as an identity) — gradients land in the flat buffer, the
eager step equals plain training bitwise, and the whole step including the RCCL all-reduce is
captured and replayed as one HIP graph with the same parameter trajectory.

The checks run in a child process (tests/_dp_graph_child.py) that ends with the product teardown
(sqr.dist.finish: the step graph destroyed before the RCCL communicator, host barrier, then
destroy_process_group) and a normal exit: the test requires both markers and exit status 0, so an
abort anywhere in the teardown or at interpreter exit fails it (in round 2 an eager RCCL barrier
after CUDAGraph.reset() aborted; host-side synchronisation now runs on a gloo group)."""
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
    ok = r.returncode == 0 and "DP_GRAPH_OK" in r.stdout and "DP_TEARDOWN_OK" in r.stdout
    if not ok:
        # the error text first (a watchdog exception's what() line), then the raw streams in full
        key = [ln for ln in (r.stdout + r.stderr).splitlines()
               if any(w in ln for w in ("what()", "Exception", "Error", "error", "DP_"))
               and "NCCL WARN" not in ln]
        print("\n".join(key))
        print(r.stdout)
        print(r.stderr)
    assert ok, (r.returncode, key[:20])
