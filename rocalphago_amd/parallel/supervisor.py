"""Supervised restart of a training job from its last checkpoint.

The reference has no failure handling at all: a crashed Keras ``fit_generator`` run is simply
lost (/root/reference/AlphaGo/training/supervised_policy_trainer.py:134-135 only *loads*
``--weights`` when a human restarts it). Here a supervisor process owns the job:

    python -m rocalphago_amd.parallel.supervisor --out OUT_DIR [--max-restarts 3]
        [--hang-timeout 600] -- <training command ... OUT_DIR ... --epochs E ...>

* the command (a trainer CLI, or a ``python -m torch.distributed.run ...`` launch of one, i.e.
  one process per GPU over RCCL) runs as a CHILD process in its own process group — the
  supervisor never re-execs itself or the job;
* when the child exits non-zero, or writes no progress for ``--hang-timeout`` seconds (a
  watchdog on the modification time of everything in OUT_DIR, e.g. the per-rank
  ``metrics.rank*.jsonl`` streams, the trainers' ``heartbeat`` file touched every few seconds,
  checkpoints and metadata), the whole process group is killed
  and the job is relaunched from the newest ``weights.NNNNN.hdf5`` in OUT_DIR: ``--weights`` is
  set to that file and ``--epochs`` reduced by the epochs already completed. The trainers
  restore the optimizer step count and data cursor from the ``.opt.json`` sidecar, so the
  resumed run continues the same schedule (tests/test_supervisor.py);
* fault injection (``RAG_FAULT_AT_STEP``) is removed from the environment of restarted
  attempts.
"""
import argparse
import glob
import os
import re
import signal
import subprocess
import sys
import time

_CKPT = re.compile(r"weights\.(\d+)\.hdf5$")


def latest_checkpoint(out_dir):
    """(epoch, basename) of the newest complete ``weights.NNNNN.hdf5`` in ``out_dir``, or None.

    Complete = the weights file has its ``.opt.json`` sidecar (the trainers write the sidecar
    first and each file through an atomic rename, training/supervised.save_checkpoint), so a
    job killed while saving resumes from the previous epoch instead of a truncated file or a
    reset optimizer schedule. Directories whose checkpoints carry no sidecars at all (RL runs)
    fall back to the newest weights file."""
    found = []
    for p in glob.glob(os.path.join(out_dir, "weights.*.hdf5")):
        m = _CKPT.search(os.path.basename(p))
        if m:
            side = os.path.splitext(p)[0] + ".opt.json"
            found.append((int(m.group(1)), os.path.basename(p), os.path.exists(side)))
    if not found:
        return None
    complete = [f for f in found if f[2]]
    pool = complete if complete else found
    best = max(pool)
    return best[0], best[1]


def _get_opt(cmd, names):
    for i, a in enumerate(cmd):
        for n in names:
            if a == n and i + 1 < len(cmd):
                return i, cmd[i + 1]
            if a.startswith(n + "="):
                return i, a.split("=", 1)[1]
    return None, None


def _set_opt(cmd, names, value):
    cmd = list(cmd)
    i, _ = _get_opt(cmd, names)
    if i is None:
        return cmd + [names[0], str(value)]
    if "=" in cmd[i] and cmd[i].split("=", 1)[0] in names:
        cmd[i] = "%s=%s" % (cmd[i].split("=", 1)[0], value)
    else:
        cmd[i + 1] = str(value)
    return cmd


def resume_command(cmd, out_dir, total_epochs):
    """The command that continues ``cmd`` from the newest checkpoint (None: nothing left)."""
    ck = latest_checkpoint(out_dir)
    if ck is None:
        return list(cmd)
    done = ck[0] + 1
    left = total_epochs - done if total_epochs is not None else None
    if left is not None and left <= 0:
        return None
    out = _set_opt(cmd, ["--weights"], ck[1])
    if left is not None:
        out = _set_opt(out, ["--epochs", "-E"], left)
    return out


def _newest_mtime(out_dir):
    t = 0.0
    for p in glob.glob(os.path.join(out_dir, "*")):
        try:
            t = max(t, os.path.getmtime(p))
        except OSError:
            pass
    return t


def _kill_group(proc):
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(timeout=20)
    except (ProcessLookupError, subprocess.TimeoutExpired):
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        proc.wait()


def run(cmd, out_dir, max_restarts=3, hang_timeout=None, poll_s=1.0, log=print):
    """Run ``cmd`` under supervision; returns the final exit code (0 on success)."""
    _, e = _get_opt(cmd, ["--epochs", "-E"])
    total_epochs = int(e) if e is not None else None
    env = dict(os.environ)
    attempt = 0
    cur = list(cmd)
    while True:
        log("[supervisor] attempt %d: %s" % (attempt, " ".join(cur)))
        proc = subprocess.Popen(cur, env=env, start_new_session=True)
        start = time.time()
        hung = False
        while True:
            try:
                rc = proc.wait(timeout=poll_s)
                break
            except subprocess.TimeoutExpired:
                pass
            if hang_timeout:
                last = max(_newest_mtime(out_dir), start)
                if time.time() - last > hang_timeout:
                    log("[supervisor] no progress in %s for %.0fs: killing the job" %
                        (out_dir, hang_timeout))
                    _kill_group(proc)
                    rc, hung = -9, True
                    break
        if rc == 0 and not hung:
            return 0
        attempt += 1
        if attempt > max_restarts:
            log("[supervisor] giving up after %d restarts (rc=%s)" % (max_restarts, rc))
            return rc if rc else 1
        nxt = resume_command(cmd, out_dir, total_epochs)
        if nxt is None:
            log("[supervisor] all epochs checkpointed; done")
            return 0
        env.pop("RAG_FAULT_AT_STEP", None)
        log("[supervisor] job failed (rc=%s); resuming from %s" %
            (rc, latest_checkpoint(out_dir)))
        cur = nxt


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        raise SystemExit("usage: supervisor --out DIR [--max-restarts N] [--hang-timeout S] "
                         "-- <training command>")
    k = argv.index("--")
    ap = argparse.ArgumentParser(prog="rocalphago_amd.parallel.supervisor")
    ap.add_argument("--out", required=True, help="the job's output directory (checkpoints)")
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--hang-timeout", type=float, default=None,
                    help="seconds without any file update in --out before the job is killed")
    args = ap.parse_args(argv[:k])
    return run(argv[k + 1:], args.out, args.max_restarts, args.hang_timeout)


if __name__ == "__main__":
    sys.exit(main())
