"""Build the native test programs in-tree (0xfec_amd/_bin/), ahead of any GPU run:

  fec_go_harness        the Go binding's C call sequence (tests/test_go_harness.py)
  fec_go_stress         many-block round trips through include/fec_go.h
  fec_go_threads        encoders / decoders created on one thread, driven concurrently from
                        others (Go's goroutine-to-thread migration), checked against the oracle
  fec_batch_lifetime    a connection's queue freed while the batch codec still owes it blocks
  *_san                 the same programs linked against lib0xfec_hip_san.so: the library's host
                        C++ (C-ABI, scheme/batch layers, wire codecs, Go ABI) compiled with
                        AddressSanitizer + UBSan on the host side only (-Xarch_host), kernels
                        unchanged (device code is never instrumented)
  go_batch_bench        host-resident throughput of the batched Go ABI (tools/go_batch_bench.c)
  fuzz_wire             libFuzzer target for the frame parsers (tests/fuzz/fuzz_wire.cpp)

Called by __graft_entry__.build(); rebuilds only what is stale."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "0xfec_amd")
BIN = os.path.join(PKG, "_bin")
SAN = os.path.join(PKG, "_san")
INCLUDE = os.path.join(ROOT, "include")
CLANG = "/opt/rocm/lib/llvm/bin/clang"
HOST_SOURCES = ["fec_capi.cpp", "fec_scheme.cpp", "fec_batch.cpp", "fec_wire.cpp", "fec_go.cpp"]
SAN_HOST = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
            "-Xarch_host", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]
SAN_C = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    subprocess.check_call(cmd)


def _headers():
    return [os.path.join(INCLUDE, h) for h in os.listdir(INCLUDE) if h.endswith((".h", ".hpp"))]


def build_san_lib():
    sys.path.insert(0, PKG)
    import _build  # noqa: the library's own build (objects of the kernels are reused)
    os.makedirs(SAN, exist_ok=True)
    csrc = os.path.join(PKG, "csrc")
    hdrs = _headers() + [os.path.join(csrc, h) for h in os.listdir(csrc) if h.endswith((".hpp", ".h"))]
    cmds, objs = [], []
    for s in _build._sources():
        src = os.path.join(csrc, s)
        if s in HOST_SOURCES:
            obj = os.path.join(SAN, s.rsplit(".", 1)[0] + ".o")
            if _stale(obj, [src] + hdrs):
                cmds.append([_build._hipcc()] + _build.CFLAGS + SAN_HOST + ["-c", "-o", obj, src])
        else:
            obj = _build._obj(s)
        objs.append(obj)
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(_run, cmds))
    lib = os.path.join(SAN, "lib0xfec_hip_san.so")
    if _stale(lib, objs):
        _run([_build._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + SAN_HOST + objs +
             ["-o", lib, "-lpthread"])
    return lib


def build():
    os.makedirs(BIN, exist_ok=True)
    sys.path.insert(0, PKG)
    import _build
    if not _build.up_to_date():
        _build.build()
    san_lib = build_san_lib()
    hdrs = _headers()
    here = os.path.dirname(os.path.abspath(__file__))
    lib = os.path.join(PKG, "lib0xfec_hip.so")
    jobs = []
    # the thread test checks frames against the CPU oracle (test infrastructure, oracle/_build)
    oracle_dir = os.path.join(ROOT, "oracle", "_build")
    if not os.path.exists(os.path.join(oracle_dir, "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    extra = {"fec_go_threads": (["-pthread"], ["-L", oracle_dir, "-loracle", "-Wl,-rpath," + oracle_dir],
                                [os.path.join(oracle_dir, "liboracle.so")])}
    for prog in ("fec_go_harness", "fec_go_stress", "fec_go_threads", "fec_batch_lifetime"):
        src = os.path.join(here, prog + ".c")
        cflags, libs, deps = extra.get(prog, ([], [], []))
        exe = os.path.join(BIN, prog)
        if _stale(exe, [src, lib] + hdrs + deps):
            jobs.append(["gcc", "-std=c11", "-O1", "-Wall", "-Werror"] + cflags + ["-I", INCLUDE, src, "-L", PKG,
                         "-l0xfec_hip", "-Wl,-rpath," + PKG] + libs + ["-o", exe])
        exe = os.path.join(BIN, prog + "_san")
        if _stale(exe, [src, san_lib] + hdrs + deps):
            jobs.append([CLANG, "-std=c11", "-O1", "-Wall", "-Werror"] + SAN_C + cflags +
                        ["-I", INCLUDE, src, "-L", SAN, "-l0xfec_hip_san", "-Wl,-rpath," + SAN] + libs + ["-o", exe])
    gb_src = os.path.join(ROOT, "tools", "go_batch_bench.c")
    gb = os.path.join(BIN, "go_batch_bench")
    if _stale(gb, [gb_src, lib] + hdrs):
        jobs.append(["gcc", "-std=c11", "-O2", "-Wall", "-Werror", "-pthread", "-I", INCLUDE, gb_src, "-L", PKG,
                     "-l0xfec_hip", "-Wl,-rpath," + PKG, "-o", gb])
    fz_src = [os.path.join(ROOT, "tests", "fuzz", "fuzz_wire.cpp"), os.path.join(PKG, "csrc", "fec_wire.cpp")]
    fz = os.path.join(BIN, "fuzz_wire")
    if _stale(fz, fz_src + hdrs):
        jobs.append([CLANG + "++", "-std=c++17", "-O1", "-fsanitize=fuzzer"] + SAN_C + ["-I", INCLUDE] + fz_src +
                    ["-o", fz])
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(_run, jobs))


if __name__ == "__main__":
    build()
