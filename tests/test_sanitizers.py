"""Host sanitizers and fuzzing (the GPU kernels are never instrumented).

* fuzz_wire: libFuzzer + ASan + UBSan over the repair / source-symbol frame parsers and the
  varint codec, differential against a byte-at-a-time model of the reference's parsers
  (tests/fuzz/fuzz_wire.cpp: io.EOF exactly where fec_repair_frame.go:16-42 /
  fec_source_symbol_frame.go:19-41 return it, the reader position after it, round trips).
* *_san: the library's host C++ (C-ABI, scheme and batch layers, wire codecs, Go ABI) built
  with ASan + UBSan and driven by the Go-call-sequence harness and the many-block stress
  program: validation paths on the CPU, full GPU round trips on the box.
"""
import os
import subprocess

import pytest

from native import binary, san_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _varint(v):
    for n, pre in ((1, 0x00), (2, 0x40), (4, 0x80), (8, 0xC0)):
        if v < 1 << (8 * n - 2):
            b = bytearray(v.to_bytes(n, "big"))
            b[0] |= pre
            return bytes(b)
    raise ValueError(v)


def _seeds(d):
    """Valid frames (minimal and non-minimal varints), truncations and over-long lengths."""
    seeds = []
    for bid, pid, plen in ((0, 0, 0), (1, 2, 5), (1 << 20, 9, 1200), ((1 << 62) - 1, 63, 64)):
        body = _varint(bid) + _varint(pid) + _varint(plen) + bytes(range(256))[:plen % 256] * (plen // 256 + 1)
        body = body[:len(_varint(bid) + _varint(pid) + _varint(plen)) + plen]
        seeds += [body, body[:-1], body[:3], _varint(bid) + _varint(pid) + _varint(plen + 1)]
    seeds.append(b"\xc0" + b"\x00" * 7 + b"\x40\x01\x00")   # non-minimal 8-byte id
    for i, s in enumerate(seeds):
        (d / ("seed%02d" % i)).write_bytes(s)


def test_fuzz_wire_parsers(tmp_path):
    fz = binary("fuzz_wire")
    corpus = tmp_path / "corpus"
    corpus.mkdir()
    _seeds(corpus)
    p = subprocess.run([fz, "-runs=400000", "-max_len=2048", "-seed=4077", str(corpus)],
                       capture_output=True, text=True, timeout=300, env=san_env(gpu=False), cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-4000:]
    assert "Done 400000 runs" in p.stderr


def test_fuzz_target_detects_a_mutant(tmp_path, fec):
    """The differential check is live: the target built against a model that is off by one at the
    payload-length check (FUZZ_MUTANT) must abort within the seed corpus."""
    if fec.device_count() > 0:
        pytest.skip("built on the CPU container only")
    exe = str(tmp_path / "fuzz_mutant")
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang++", "-std=c++17", "-O1", "-DFUZZ_MUTANT",
                           "-fsanitize=fuzzer,address,undefined", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "fuzz", "fuzz_wire.cpp"),
                           os.path.join(ROOT, "0xfec_amd", "csrc", "fec_wire.cpp"), "-o", exe])
    corpus = tmp_path / "corpus"
    corpus.mkdir()
    _seeds(corpus)
    p = subprocess.run([exe, "-runs=100000", str(corpus)], capture_output=True, text=True, timeout=120,
                       env=san_env(gpu=False), cwd=str(tmp_path))
    assert p.returncode != 0 and "deadly signal" in p.stderr, p.stderr[-2000:]


def test_sanitized_harness_validation_without_device(golden, oracle, fec, tmp_path):
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    import test_go_harness as h
    cases = h._with_oracle_texts(h._golden_cases(golden), oracle)
    results = h._run(binary("fec_go_harness_san"), cases, "batch", tmp_path, env=san_env(gpu=False))
    n = 0
    for r, (kind, blk, k, m, exp, ref) in zip(results, cases):
        if r["err"] == "no HIP device":
            continue
        n += 1
        if exp[0] == "err":
            assert r["err"] == exp[1], ref
    assert n >= 8


def test_sanitized_stress_fails_loudly_without_device(fec):
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    p = subprocess.run([binary("fec_go_stress_san"), "rs", "8", "4", "4", "2", "1"], capture_output=True,
                       text=True, timeout=60, env=san_env(gpu=False))
    assert p.returncode == 1 and "no HIP device" in p.stderr, p.stderr[-2000:]


STRESS = [("rs", 8, 4, 600, 64), ("rs", 20, 10, 300, 32), ("rs", 16, 8, 200, 7), ("rs", 2, 1, 300, 5),
          ("xor", 2, 1, 500, 64), ("xor", 5, 1, 300, 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("san", [False, True], ids=["plain", "asan_ubsan"])
@pytest.mark.parametrize("scheme,k,m,blocks,maxb", STRESS)
def test_stress_roundtrip(scheme, k, m, blocks, maxb, san):
    exe = binary("fec_go_stress_san" if san else "fec_go_stress")
    p = subprocess.run([exe, scheme, str(k), str(m), str(blocks), str(maxb), str(0x5EED + k)],
                       capture_output=True, text=True, timeout=110, env=san_env(gpu=True) if san else None)
    assert p.returncode == 0, p.stderr[-4000:]
    assert p.stdout.startswith("ok blocks=%d" % blocks)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["direct", "batch", "batchref"])
def test_sanitized_harness_golden(golden, oracle, mode, tmp_path):
    import test_go_harness as h
    cases = (h._with_oracle_texts(h._golden_cases(golden), oracle) + h._synthetic_cases(oracle) +
             h._empty_repair_cases(oracle)[0])
    h._check(h._run(binary("fec_go_harness_san"), cases, mode, tmp_path, env=san_env(gpu=True)), cases,
             texts=(mode == "direct"))


def test_loaded_library_is_the_requested_build(fec):
    """Under tools/cpu_tests_sanitized.sh (FEC_LIB_PATH) the process really runs the sanitized
    library: it is the one mapped, and the ASan runtime is live in the process."""
    want = os.environ.get("FEC_LIB_PATH")
    maps = open("/proc/self/maps").read()
    if not want:
        assert os.path.basename(fec._LIB_PATH) == "lib0xfec_hip.so" and fec._LIB_PATH in maps
        return
    assert fec._LIB_PATH == want and want in maps
    import ctypes
    assert hasattr(ctypes.CDLL(None), "__asan_init")


def test_host_suite_under_asan_ubsan(fec):
    """The host-logic CPU tests (C-ABI checks, scheme/batch layers, wire codecs, Go-call harness)
    pass against the ASan+UBSan build of the library (no GPU here: every HIP call fails cleanly)."""
    if fec.device_count() > 0 or os.environ.get("FEC_LIB_PATH"):
        pytest.skip("CPU container only, and not from inside the sanitized run itself")
    tests = ["test_capi_exports.py", "test_batch_host.py", "test_scheme_host.py", "test_wire.py",
             "test_go_harness.py", "test_sanitizers.py::test_loaded_library_is_the_requested_build"]
    p = subprocess.run([os.path.join(ROOT, "tools", "cpu_tests_sanitized.sh"), "-x"] +
                       [os.path.join(ROOT, "tests", t) for t in tests],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert " passed" in p.stdout and "failed" not in p.stdout


def test_threads_program_fails_loudly_without_device(fec):
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    p = subprocess.run([binary("fec_go_threads"), "4", "1"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "no HIP device" in p.stderr, p.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("san", [False, True], ids=["plain", "asan_ubsan"])
def test_go_abi_concurrent_connections(san):
    """Four encoders + four decoders (RS(8,12) twice, RS(20,30), XOR(2,1)) created on one thread
    and driven concurrently from four others, then from swapped threads (connection.go:525 run
    loops; goroutines migrate between OS threads). Each owns its fec_ctx, so no stream, workspace
    or sticky error is shared; frames are checked against the oracle, payloads against the
    originals (tests/c/fec_go_threads.c)."""
    exe = binary("fec_go_threads_san" if san else "fec_go_threads")
    p = subprocess.run([exe, "120", str(0xC0FFEE)], capture_output=True, text=True, timeout=110,
                       env=san_env(gpu=True) if san else None)
    assert p.returncode == 0, p.stderr[-4000:]
    assert p.stdout.startswith("ok connections=4 blocks=960")


def test_batch_lifetime_fails_loudly_without_device(fec):
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    p = subprocess.run([binary("fec_batch_lifetime_san")], capture_output=True, text=True, timeout=60,
                       env=san_env(gpu=False))
    assert p.returncode == 1 and "no HIP device" in p.stderr, p.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("san", [False, True], ids=["plain", "asan_ubsan"])
def test_queue_freed_while_blocks_owed(san):
    """A RepairQueue freed while its frames sit in the encoder's backlog or its batch is in flight,
    and a RecoveredQueue freed while its blocks are in flight: poll and drain drop those blocks
    and touch nothing freed (the backlog entry held the last token reference)."""
    exe = binary("fec_batch_lifetime_san" if san else "fec_batch_lifetime")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=110, env=san_env(gpu=True) if san else None)
    assert p.returncode == 0, p.stderr[-4000:]
    assert p.stdout.startswith("ok backlog inflight mixed decoder")
