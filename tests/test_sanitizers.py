"""Native runtime under ThreadSanitizer and Address/UndefinedBehaviorSanitizer.

csrc/tests/native_selftest.cpp drives the engine, features, ladders, multi-threaded rollouts and
the APV search with overlapping asynchronous rollout waves, without Python, so the sanitizer
runtimes need no preloading. Host code only (GPU sanitizers are not available)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "csrc", p) for p in
        ("tests/native_selftest.cpp", "engine/go_engine.cpp", "engine/features.cpp",
         "engine/ladder.cpp", "mcts/rollout.cpp")]


@pytest.mark.slow
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_native_selftest_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
           "-fsanitize=" + san, "-I" + os.path.join(ROOT, "csrc", "engine")] + SRCS + ["-o", exe]
    b = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert b.returncode == 0, b.stderr.decode()[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"native selftest ok" in r.stdout
    assert b"WARNING: ThreadSanitizer" not in r.stderr and b"runtime error" not in r.stderr
