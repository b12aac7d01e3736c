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


def test_search_efficiency_effective_from_rows(tmp_path):
    """benchmarks/search_efficiency.py --effective --from-rows: the modelled / effective rates of
    earlier efficiency rows from one GPU's serving rate at (wave, depth), capped by rank 0's
    per-wave host ceiling, and the argmax per N (profiles/search_efficiency_r6.json)."""
    import json
    import subprocess
    import sys
    rows = [{"ranks": 8, "gpu_wave": 128, "depth": 2, "efficiency": 0.5},
            {"ranks": 8, "gpu_wave": 512, "depth": 2, "efficiency": 0.3},
            {"ranks": 2, "gpu_wave": 512, "depth": 2, "efficiency": 0.9}]
    prev = tmp_path / "prev.json"
    prev.write_text("noise line\n" + json.dumps({"rows": rows}, indent=1))
    rates = tmp_path / "rates.json"
    rates.write_text(json.dumps({"sims_per_s_by_wave": {"128": 70000.0, "512": 120000.0},
                                 "serving_sims_per_s": {"128": {"2": 80000.0}}}))
    out = subprocess.run([sys.executable, "benchmarks/search_efficiency.py", "--effective",
                          "--from-rows", str(prev), "--gpu-rates", str(rates),
                          "--master-ceiling", "900000", "--master-ceilings", "128:600000"],
                         capture_output=True, text=True, check=True,
                         cwd=str(__import__("pathlib").Path(__file__).parent.parent)).stdout
    res = json.loads(out[out.index("{\n"):])
    by = {(r["ranks"], r["gpu_wave"]): r for r in res["rows"]}
    # serving rate at (128, depth 2) wins over the single-GPU table; capped at 600k
    assert by[8, 128]["modelled_sims_per_s"] == 600000.0
    assert by[8, 128]["effective_sims_per_s"] == 300000.0
    assert by[8, 512]["modelled_sims_per_s"] == 900000.0  # 8 x 120k capped at 900k
    assert by[2, 512]["effective_sims_per_s"] == 216000.0
    assert res["best_by_ranks"]["8"]["gpu_wave"] == 128
