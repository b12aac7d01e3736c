"""Find compiler-inserted `s_waitcnt vmcnt` waits directly in front of LDS reads in hipcc's .s
output: with global_load_lds prefetch in flight such a wait drains the whole staging pipeline
(MI355X guide §5 'Projection GEMM' item 4; the ds_read_tr16 builtin triggered it in wgrad).

  python tools/check_drains.py csrc/hip/conv_tap.hip [...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def drains(src):
    with tempfile.TemporaryDirectory() as d:
        inc = "-I" + os.path.join(ROOT, "csrc", "hip")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
                        "-fPIC", inc, os.path.abspath(src), "-o", os.path.join(d, "x.o"),
                        "--save-temps"], cwd=d, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        base = os.path.splitext(os.path.basename(src))[0]
        lines = open(os.path.join(d, base + "-hip-amdgcn-amd-amdhsa-gfx950.s")).read().split("\n")
    out = {}
    name, asm = None, False
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            name = m.group(1)
            out.setdefault(name, 0)
        if "ASMSTART" in l:
            asm = True
            continue
        if "ASMEND" in l:
            asm = False
            continue
        if name and not asm and "s_waitcnt vmcnt" in l:
            nxt = [x for x in lines[i + 1:i + 4] if x.strip() and not x.strip().startswith(";")]
            if nxt and "ds_read" in nxt[0]:
                out[name] += 1
    return out


if __name__ == "__main__":
    bad = 0
    for src in sys.argv[1:]:
        for fn, n in drains(src).items():
            if n:
                bad += 1
                print("%s: %s: %d vmcnt wait(s) in front of ds_read" % (src, fn[:70], n))
    sys.exit(1 if bad else 0)
