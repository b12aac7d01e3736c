"""One parameterised runner for the GPU-box jobs (replaces the per-experiment shell scripts).

    gpurun --timeout 900 -- 'python tools/gpujob.py OUT STEP [STEP ...]'

Every STEP runs as a child process (never exec) under its own ``timeout -k 10 <s>``, writes
``gpurun_out/OUT/<name>.log``, and the job stops at the first step that fails, times out or
crashes (no GPU step starts after a failed one). A STEP is either a named step from ``STEPS``
below, optionally with ``NAME@KEY=VAL,KEY=VAL`` environment overrides, or an ad-hoc
``name:seconds:command`` string. After each step the last lines of its log (or the JSON lines
it printed) are echoed so gpurun's tail shows the result.

Examples:
    python tools/gpujob.py r4a tests smoke bench
    python tools/gpujob.py ab sl sl@RAG_WINO=0 sl
    python tools/gpujob.py tr trace-sl pmc-sl
    python tools/gpujob.py x 'conv:300:VARIANTS=7 python scripts/dbg/conv_ab.py'
"""
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = "python3 -u"
PMC_SQ = ("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES "
          "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")

PMC_LDS = ("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS "
           "SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT")

# name -> (seconds, command, echo mode); {dir} = gpurun_out/OUT/<step tag> (profiler output)
STEPS = {
    "tests": (900, PY + " -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread",
              "tail2"),
    "smoke": (200, PY + " -c 'import __graft_entry__ as g; g.smoke()'", "tail1"),
    "bench": (400, PY + " bench.py", "json"),
    "sl": (200, PY + " bench.py --no-mcts --steps 60 --warmup 10", "json"),
    "sl-long": (300, PY + " bench.py --no-mcts --steps 5000 --warmup 20", "json"),
    "value": (200, PY + " bench.py --model value --no-mcts", "json"),
    "resnet": (200, PY + " bench.py --model resnet --no-mcts", "json"),
    "cnn128": (200, PY + " bench.py --filters 128 --no-mcts", "json"),
    "mcts": (300, PY + " benchmarks/mcts_bench.py --moves 6", "json"),
    "trace-sl": (300, "rocprofv3 --kernel-trace --stats -d {dir} -o sl -- " + PY +
                 " bench.py --no-mcts --steps 10 --warmup 3", "tail1"),
    "trace-resnet": (300, "rocprofv3 --kernel-trace --stats -d {dir} -o res -- " + PY +
                     " bench.py --model resnet --no-mcts --steps 10 --warmup 3", "tail1"),
    "trace-mcts": (300, "rocprofv3 --kernel-trace -d {dir} -o mcts -- " + PY +
                   " benchmarks/mcts_bench.py --moves 4", "tail1"),
    "pmc-sl": (150, "rocprofv3 --pmc " + PMC_SQ + " --output-format csv -d {dir} -- " +
               PY + " bench.py --no-mcts --steps 6 --warmup 2", "tail1"),
    "pmc-resnet": (150, "rocprofv3 --pmc " + PMC_SQ + " --output-format csv -d {dir} -- "
                   + PY + " bench.py --model resnet --no-mcts --steps 6 --warmup 2", "tail1"),
    "pmc2-sl": (150, "rocprofv3 --pmc " + PMC_LDS + " --output-format csv -d {dir} -- " +
                PY + " bench.py --no-mcts --steps 6 --warmup 2", "tail1"),
    "rl": (300, PY + " benchmarks/rl_bench.py --config 19 --game-batch 256", "json"),
    "trace-rl": (300, "rocprofv3 --kernel-trace -d {dir} -o rl -- " + PY +
                 " benchmarks/rl_bench.py --config 19 --game-batch 256", "tail1"),
    "trace-cnn128": (300, "rocprofv3 --kernel-trace --stats -d {dir} -o cnn -- " + PY +
                     " bench.py --filters 128 --no-mcts --steps 10 --warmup 3", "tail1"),
    "trace-value": (300, "rocprofv3 --kernel-trace --stats -d {dir} -o val -- " + PY +
                    " bench.py --model value --no-mcts --steps 10 --warmup 3", "tail1"),
    "rl512": (300, PY + " benchmarks/rl_bench.py --config 19 --game-batch 512", "json"),
    "valuegen": (300, PY + " benchmarks/value_gen_bench.py", "json"),
    "kernels": (600, PY + " -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py "
                "tests/test_gpu_bench_path.py -m gpu -x -q --timeout 200 "
                "--timeout-method thread", "tail2"),
}


def _echo(log, mode):
    try:
        lines = open(log, errors="replace").read().splitlines()
    except OSError:
        return
    if mode == "json":
        js = [ln for ln in lines if ln.startswith("{")]
        for ln in (js or lines[-3:]):
            print("   ", ln[:1500])
    else:
        for ln in lines[-(2 if mode == "tail2" else 1):]:
            print("   ", ln[:400])


def parse(spec):
    env = {}
    if ":" in spec and spec.split(":", 1)[0] not in STEPS and spec.count(":") >= 2:
        name, secs, cmd = spec.split(":", 2)
        return name, int(secs), cmd.replace("{PMC}", PMC_SQ), "json", env
    if "@" in spec:
        spec, kv = spec.split("@", 1)
        for item in kv.split(","):
            k, v = item.split("=", 1)
            env[k] = v
    secs, cmd, mode = STEPS[spec]
    tag = spec + "".join("_%s%s" % (k.replace("RAG_", "").lower(), os.path.basename(v))
                         for k, v in env.items())
    tag = "".join(c if c.isalnum() or c in "._-" else "_" for c in tag)
    return tag, secs, cmd, mode, env


def main(argv):
    if len(argv) < 2:
        print(__doc__)
        return 2
    out = os.path.join(ROOT, "gpurun_out", argv[0])
    os.makedirs(out, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    seen = {}
    for spec in argv[1:]:
        name, secs, cmd, mode, env = parse(spec)
        seen[name] = seen.get(name, 0) + 1
        if seen[name] > 1:
            name = "%s.%d" % (name, seen[name])
        log = os.path.join(out, name + ".log")
        full = "timeout -k 10 %d %s" % (secs, cmd.replace("{dir}", os.path.join(out, name)))
        e = dict(os.environ)
        e.update(env)
        argv_ = shlex.split(full)
        while len(argv_) > 5 and "=" in argv_[4] and argv_[4].split("=", 1)[0].isupper():
            k, v = argv_.pop(4).split("=", 1)  # leading VAR=value words of an ad-hoc command
            e[k] = v
        t0 = time.time()
        with open(log, "w") as f:
            f.write("# %s\n# env %s\n" % (full, env))
            f.flush()
            rc = subprocess.call(argv_, cwd=ROOT, stdout=f, stderr=subprocess.STDOUT,
                                 env=e)
        print("[%s] rc=%d %.0fs" % (name, rc, time.time() - t0), flush=True)
        _echo(log, mode if rc == 0 else "tail2")
        if rc != 0:
            try:
                print("\n".join(open(log, errors="replace").read().splitlines()[-25:]))
            except OSError:
                pass
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
