"""Build the HIP kernel library with some sources taken from another git revision, for a same-box
A/B against the current tree (the driver's boxes differ by a few percent, so before/after numbers
from two gpurun calls do not compare).

    python tools/ab_build.py REV csrc/hip/conv_tap.hip [...]   -> rocalphago_amd/_hipkernels_ab.so
    RAG_HIP_SO=rocalphago_amd/_hipkernels_ab.so python bench.py ...

Every other source is the working tree's; symbols missing from the old sources are optional in
ops/_abi.py."""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv):
    if len(argv) < 2:
        print(__doc__)
        return 2
    from rocalphago_amd import _build
    rev, files = argv[0], set(argv[1:])
    out = os.path.join(ROOT, "build", "ab")
    os.makedirs(out, exist_ok=True)
    hip = os.path.join(_build.ROCM, "bin", "hipcc")
    inc = os.path.join(ROOT, "csrc", "hip")
    srcs = sorted(glob.glob(os.path.join(inc, "*.hip")))
    jobs = []
    for s in srcs:
        rel = os.path.relpath(s, ROOT)
        src = s
        if rel in files:
            src = os.path.join(out, os.path.basename(s))
            with open(src, "wb") as f:
                f.write(subprocess.check_output(["git", "show", "%s:%s" % (rev, rel)], cwd=ROOT))
        jobs.append((src, os.path.join(out, os.path.basename(s)[:-4] + ".o")))
    flags = ["--offload-arch=" + _build.GPU_ARCH, "-O3", "-std=c++17", "-fPIC",
             "-munsafe-fp-atomics", "-Wno-unused-result", "-I" + inc]

    def cc(j):
        subprocess.check_call([hip] + flags + ["-c", j[0], "-o", j[1]])
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(cc, jobs))
    so = os.path.join(ROOT, "rocalphago_amd", "_hipkernels_ab.so")
    subprocess.check_call([hip, "--offload-arch=" + _build.GPU_ARCH, "-shared", "-fPIC"] +
                          [o for _, o in jobs] + ["-o", so])
    print(so)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
