"""In-tree native build: the C++ engine (pybind11, g++) and the gfx950 HIP kernels (hipcc).

Both artefacts are written next to this file so they travel with the repository snapshot to the
GPU box (see __graft_entry__.build). Rebuilds are incremental on source mtimes.

  rocalphago_amd/_rocgo<EXT_SUFFIX>   C++17: rules engine, features, LZF, APV-MCTS, rollouts
  rocalphago_amd/_hipkernels.so       HIP (gfx950 only): conv implicit-GEMM fwd/dgrad/wgrad,
                                      policy/value heads, SGD, augmentation, features, rollouts
"""
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "csrc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")
ENGINE_SO = os.path.join(HERE, "_rocgo" + EXT_SUFFIX)
HIP_SO = os.path.join(HERE, "_hipkernels.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
GPU_ARCH = "gfx950"


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("native build failed: " + " ".join(cmd[:3]) + " ...")
    return r.stdout


def build_engine(force=False, verbose=False, debug=False, sanitize=None):
    """Compile the C++ engine module with g++ (-O3, threads)."""
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cpp")) +
                  glob.glob(os.path.join(CSRC, "mcts", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "*", "*.hpp"))
    target = ENGINE_SO if sanitize is None else ENGINE_SO.replace("_rocgo", "_rocgo_" + sanitize)
    if not force and not _stale(target, srcs + hdrs):
        return target
    opt = ["-O1", "-g"] if (debug or sanitize) else ["-O3", "-DNDEBUG"]
    cmd = (["g++", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-msse4.2", "-mpopcnt",
            "-pthread", "-Wall", "-Wno-sign-compare"] + opt +
           ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
            "-I" + os.path.join(CSRC, "engine"), "-I" + os.path.join(CSRC, "mcts")] +
           srcs + ["-o", target + ".tmp"])
    if sanitize:
        cmd[1:1] = ["-fsanitize=" + sanitize, "-fno-omit-frame-pointer"]
    _run(cmd, verbose)
    os.replace(target + ".tmp", target)
    return target


def build_hip(force=False, verbose=False, jobs=None):
    """Compile every csrc/hip/*.hip into one gfx950 shared object (C ABI, loaded via ctypes).

    Each source compiles to its own object under build/hip/ (in parallel, incremental on the
    source and header mtimes), then one hipcc link produces the shared object."""
    from concurrent.futures import ThreadPoolExecutor

    srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "hip", "*.h"))
    if not srcs:
        return None
    if not force and not _stale(HIP_SO, srcs + hdrs):
        return HIP_SO
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    flags = ["--offload-arch=" + GPU_ARCH, "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I" + os.path.join(CSRC, "hip")]
    objs = [os.path.join(objdir, os.path.basename(s)[:-4] + ".o") for s in srcs]

    def compile_one(so):
        src, obj = so
        if force or _stale(obj, [src] + hdrs):
            _run([hipcc] + flags + ["-c", src, "-o", obj + ".tmp"], verbose)
            os.replace(obj + ".tmp", obj)

    jobs = jobs or min(len(srcs), max(1, min(os.cpu_count() or 1, 8)))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, zip(srcs, objs)))
    _run([hipcc, "--offload-arch=" + GPU_ARCH, "-shared", "-fPIC"] + objs +
         ["-o", HIP_SO + ".tmp"], verbose)
    os.replace(HIP_SO + ".tmp", HIP_SO)
    return HIP_SO


def build_all(force=False, verbose=False):
    return build_engine(force, verbose), build_hip(force, verbose)


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_all(force=force, verbose=True))
