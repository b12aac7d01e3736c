"""Failure detection of multi-rank runs (parallel/watchdog.py, used by bench.py for N > 1): a
rank that stalls before its all-reduce ends the job with a non-zero status within the stall
limit, and the diagnostic names the stalled rank."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(env_extra, timeout):
    env = dict(os.environ)
    env.update(env_extra)
    # 12 s: above the start-up skew of two ranks on a loaded CI host (pytest -n 4 saw >6 s)
    env.update(RAG_TEST_STALL_LIMIT="12", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "stall_job.py")]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=timeout)
    return r.returncode, r.stdout, time.time() - t0


def test_healthy_two_rank_job_finishes():
    rc, out, _ = _launch({}, 120)
    assert rc == 0, out[-2000:]
    assert "rank 0 done" in out and "rank 1 done" in out


def test_stalled_rank_is_named_and_job_exits_nonzero():
    rc, out, dt = _launch({"RAG_STALL": "1:5"}, 120)
    assert rc != 0, out[-2000:]
    assert dt < 60, "the stall must end the job within the watchdog limit (took %.0fs)" % dt
    # whichever rank's watchdog fires first (the stalled rank's own thread, or a rank blocked in
    # the collective) prints the diagnostic and ends the job; either must name rank 1
    lines = [ln for ln in out.splitlines() if "[watchdog] rank " in ln and "stalled" in ln]
    assert lines, out[-3000:]
    assert "stalled rank(s): [1]" in lines[0], lines[0]
