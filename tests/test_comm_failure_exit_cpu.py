"""How a rank ends when the RCCL data path gives up, on CPU with stand-ins:

* ``train.py`` run as a script wraps ``main`` in ``sqr.dist.exit_on_comm_failure``: a CommFailure
  raised by the real ``wait_event`` deadline (communicator aborted) prints its traceback and ends
  the process with status 3 at once, instead of unwinding through interpreter shutdown with the
  captured graph and the process group destroyed in garbage-collection order;
* the blocking RCCL host calls (``ncclCommInitRank``, ``ncclCommFinalize/Destroy``) run under the
  host deadline: a call that does not return ends the process with status 3 and says which call."""
import os
import subprocess
import sys

from test_dist_comm_mock_cpu import _Ev, _StallComm  # noqa: F401  (stand-ins reused by the child)
from test_dist_cpu import _paths

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(code):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "sq-recovery_amd"), os.path.join(ROOT, "tests"),
                                         env.get("PYTHONPATH", "")])
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=120)


def test_exit_on_comm_failure_in_process():
    _paths()
    from sqr import dist as sd
    codes = []

    def failing():
        sd.wait_event(_Ev(), timeout=0.02, what="step", comm_=_StallComm())

    sd.exit_on_comm_failure(failing, exit_fn=codes.append)
    assert codes == [3]
    assert sd.exit_on_comm_failure(lambda a: a + 1, 1, exit_fn=codes.append) == 2 and codes == [3]


def test_train_script_exits_3_on_comm_failure():
    # train.py's __main__ guard around a main() whose step wait hits the deadline on a stalled peer
    code = (
        "import textwrap\n"
        "from sqr import dist\n"
        "from test_dist_comm_mock_cpu import _Ev, _StallComm\n"
        "c = _StallComm()\n"
        "def fake_main(argv=None):\n"
        "    dist.wait_event(_Ev(), timeout=0.02, what='train step', comm_=c)\n"
        "import train\n"
        "train.main = fake_main\n"
        "src = open(train.__file__).read().split('if __name__ == \"__main__\":')[1]\n"
        "exec(textwrap.dedent(src), vars(train))\n"
        "print('NOT REACHED')\n")
    r = _child(code)
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    assert "CommFailure" in r.stderr and "did not finish" in r.stderr
    assert "NOT REACHED" not in r.stdout


def test_blocking_rccl_call_deadline():
    r = _child("import time\nfrom sqr import dist\n"
               "dist._blocking_with_deadline(lambda: time.sleep(60), 0.5, 'ncclCommFinalize/Destroy')\n"
               "print('NOT REACHED')\n")
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    assert "ncclCommFinalize/Destroy did not return" in r.stderr
    assert "NOT REACHED" not in r.stdout
    # a call that returns (or raises) in time is transparent
    _paths()
    from sqr import dist as sd
    assert sd._blocking_with_deadline(lambda: 7, 5.0, "x") == 7
    assert sd._blocking_with_deadline(lambda: 8, None, "x") == 8
    try:
        sd._blocking_with_deadline(lambda: 1 / 0, 5.0, "x")
    except ZeroDivisionError:
        pass
    else:
        raise AssertionError("the call's exception must reach the caller")
