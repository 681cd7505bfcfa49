"""Build lib0xfec_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib0xfec_hip.so")

SOURCES = ["fec_kernels.hip", "fec_capi.cpp", "fec_scheme.cpp", "fec_batch.cpp", "fec_wire.cpp"]
HEADERS = ["fec_kernels.hpp", "gf256.h", "rs_matrix.hpp"]
PUBLIC = ["fec_hip.h", "fec_scheme.h", "fec_batch.h", "fec_batch.hpp", "fec_scheme.hpp", "fec_wire.h"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def _inputs():
    inc = os.path.join(os.path.dirname(HERE), "include")
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(inc, h) for h in PUBLIC]
    return [f for f in files if os.path.exists(f)]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force=False, verbose=False):
    """Compile every HIP/C++ source of the codec into lib0xfec_hip.so (gfx950 only)."""
    if not force and up_to_date():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    # The atomic optimizer turns a single-lane atomicAdd (queue kernels' ticket draw) into a
    # wave-aggregated one whose result is consumed on the spot, which makes the draw a full HBM
    # round trip on the critical path; the tickets are consumed a stage later instead.
    cmd = [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "-I", os.path.join(os.path.dirname(HERE), "include"), "-o", LIB + ".tmp"] + srcs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
