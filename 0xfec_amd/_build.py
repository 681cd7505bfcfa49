"""Build lib0xfec_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

Every source is compiled to its own object in parallel (the kernel translation units carry
many template instances and dominate the build), then linked into one shared library. An
object is rebuilt when its source or any shared header is newer than it.
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "lib0xfec_hip.so")

SOURCES = ["fec_encode.hip", "fec_encode23.hip", "fec_decode.hip", "fec_rebuild.hip", "fec_recover.hip", "fec_plan.hip", "fec_xor.hip", "fec_synth.hip", "fec_pack.hip", "fec_probe.hip", "fec_kernels.hip", "fec_capi.cpp",
           "fec_scheme.cpp", "fec_batch.cpp", "fec_wire.cpp", "fec_go.cpp"]
HEADERS = ["fec_kernels.hpp", "fec_device.hpp", "fec_recon.hpp", "gf256.h", "rs_matrix.hpp", "fec_bitslice.inc"]
PUBLIC = ["fec_hip.h", "fec_scheme.h", "fec_batch.h", "fec_batch.hpp", "fec_scheme.hpp", "fec_wire.h", "fec_go.h", "fec_synth.h", "fec_probe.h"]

# The atomic optimizer would wrap every single-lane atomic (the sticky error words: one lane per
# wave sets them, fec_device.hpp wave_flag) in wave-aggregation code it never needs.
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
          "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-I", INCLUDE]


def source_hash(tu):
    """sha256 (first 16 hex digits) over what the kernels of translation unit `tu` are compiled
    from: its source, the device headers and the compile flags. A PMC traffic profile records it
    (tools/pmc_traffic.py) and bench.py reports the profile's traffic only while it still matches."""
    import hashlib
    h = hashlib.sha256(" ".join(CFLAGS[:-2]).encode())
    for f in [os.path.join(CSRC, tu)] + [os.path.join(CSRC, x) for x in HEADERS]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_code_hashes(lib=LIB):
    """sha256 (first 16 hex digits) of each gfx950 kernel's machine code in the built library:
    {demangled kernel name: hash}. The code objects are read from the clang offload bundles in
    the library's .hip_fatbin data, each kernel's bytes from its symbol in the code object's
    .text. A PMC traffic profile records these (tools/pmc_traffic.py) and bench.py reports the
    profile's traffic only while the kernel it runs has the same code: edits elsewhere (another
    kernel, a host launch knob in a shared header) do not retire a profile, a changed kernel does."""
    import hashlib
    import shutil
    import struct
    with open(lib, "rb") as fh:
        blob = fh.read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    syms = {}
    at = blob.find(magic)
    while at >= 0:
        nent = struct.unpack_from("<Q", blob, at + 24)[0]
        off = at + 32
        for _ in range(nent):
            eo, esz, tl = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if triple.endswith("gfx950") and esz:
                elf = blob[at + eo:at + eo + esz]
                shoff, = struct.unpack_from("<Q", elf, 0x28)
                shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
                secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
                for name_i, typ, _, addr, soff, size, link, _, _, entsize in secs:
                    if typ != 2:   # SHT_SYMTAB
                        continue
                    stroff = secs[link][4]
                    for s in range(size // entsize):
                        st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from(
                            "<IBBHQQ", elf, soff + s * entsize)
                        if st_info & 0xF != 2 or not st_size or st_shndx >= len(secs):   # STT_FUNC
                            continue
                        end = elf.index(b"\0", stroff + st_name)
                        sym = elf[stroff + st_name:end].decode()
                        tsec = secs[st_shndx]
                        start = tsec[4] + (st_value - tsec[3])
                        syms[sym] = hashlib.sha256(elf[start:start + st_size]).hexdigest()[:16]
        at = blob.find(magic, at + 1)
    filt = next((c for c in ("/opt/rocm/lib/llvm/bin/llvm-cxxfilt", shutil.which("llvm-cxxfilt"),
                             shutil.which("c++filt")) if c and os.path.exists(c)), None)
    names = list(syms)
    if filt and names:
        out = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return dict(zip(out.splitlines(), (syms[n] for n in names)))
    return syms


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def _sources():
    return [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _headers():
    files = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, h) for h in PUBLIC]
    return [f for f in files if os.path.exists(f)]


def _obj(src):
    return os.path.join(OBJ, src.rsplit(".", 1)[0] + ".o")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def up_to_date():
    hdrs = _headers()
    srcs = _sources()
    if any(_stale(_obj(s), [os.path.join(CSRC, s)] + hdrs) for s in srcs):
        return False
    return not _stale(LIB, [_obj(s) for s in srcs])


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force=False, verbose=False, jobs=None):
    """Compile every HIP/C++ source of the codec and link lib0xfec_hip.so (gfx950 only)."""
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    srcs = _sources()
    todo = [s for s in srcs if force or _stale(_obj(s), [os.path.join(CSRC, s)] + hdrs)]
    # heaviest translation units first, so they start before the quick host sources
    todo.sort(key=lambda s: not s.endswith(".hip"))
    hipcc = _hipcc()
    cmds = [[hipcc] + CFLAGS + ["-c", "-o", _obj(s), os.path.join(CSRC, s)] for s in todo]
    if cmds:
        jobs = jobs or min(len(cmds), max(1, (os.cpu_count() or 2)))
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for f in [ex.submit(_run, c, verbose) for c in cmds]:
                f.result()
    if force or todo or _stale(LIB, [_obj(s) for s in srcs]):
        _run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB + ".tmp"] + [_obj(s) for s in srcs],
             verbose)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
