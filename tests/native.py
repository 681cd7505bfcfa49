"""Paths of the native test programs built by tests/c/build.py (0xfec_amd/_bin). They are built
ahead of time on the CPU (__graft_entry__.build()) and travel with the tree; a missing one is
built here, which needs the toolchain of the build container."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "0xfec_amd", "_bin")
# host ASan + UBSan runtime options: stop at the first report; the HIP runtime's own allocations
# outlive main, so leak checking is off on the GPU (it stays on for the CPU-only runs)
SAN_ENV = {"ASAN_OPTIONS": "abort_on_error=0:halt_on_error=1:protect_shadow_gap=0",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def binary(name):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tests", "c", "build.py")])
    return path


def san_env(gpu):
    env = dict(os.environ)
    if "libclang_rt.asan" in env.get("LD_PRELOAD", ""):
        # our own sanitized CPU-suite run (tools/cpu_tests_sanitized.sh) preloads the shared ASan
        # runtime for python; the test programs carry the static one
        del env["LD_PRELOAD"]
    env.update(SAN_ENV)
    if gpu:
        env["ASAN_OPTIONS"] += ":detect_leaks=0"
    return env
