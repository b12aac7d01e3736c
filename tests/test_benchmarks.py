"""The CPU plumbing benchmark (BASELINE config #1) runs end to end and reports one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_plumbing_benchmark():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "cpu_plumbing.py"),
                          "--steps", "2", "--warmup", "1", "--positions", "256", "--batch", "16"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    r = json.loads(out.stdout.decode().strip().splitlines()[-1])
    assert r["status"] == "pass" and r["value"] > 0 and r["n_gpus"] == 0
