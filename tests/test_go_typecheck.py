"""The Go drop-in type-checked on the CPU by a subset Go checker (tests/go_lite.py): there is no
Go toolchain in this image, so these tests stand in for `go vet` / `go build -tags fechip`.

The package checked is the reference's internal/fec (block.go, manager.go patched by
go/patches/manager.go.diff, ...) with go/internal/fec/*.go dropped in, in both build
configurations (-tags fechip: the engine; default: the stubs), against the declarations of the
reference's internal/wire (patched as fec_source_symbol_frame.go.diff / fec_repair_frame.go.diff
patch it) and internal/protocol, and the cgo prototypes of include/*.h.

What a compiler would reject and the checker catches (each seeded below, on a copy of the files,
to prove it does): an unknown field or method, an undefined identifier, a cgo argument of the
wrong C type (int for C.int, *C.uint32_t for *C.size_t, ...), a wrong argument or return count,
an assignment count mismatch, a struct literal field that does not exist, mismatched operand
types, a type that no longer satisfies an interface it is asserted to implement, a local declared
and never read, an unused import, a missing return, a non-boolean condition, and a name declared
twice in one build configuration. Reads /root/reference (skipped where it is absent)."""
import os
import re
import shutil
import subprocess

import pytest

import go_lite

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GO = os.path.join(ROOT, "go", "internal", "fec")
PATCHES = os.path.join(ROOT, "go", "patches")
HEADERS = [os.path.join(ROOT, "include", h) for h in ("fec_hip.h", "fec_scheme.h", "fec_go.h")]

needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not present")


def _read(p):
    with open(p) as fh:
        return fh.read()


def _tags(src):
    m = re.match(r"//go:build (\S+)", src)
    return m.group(1) if m else None


@pytest.fixture(scope="module")
def patched(tmp_path_factory):
    """The reference's internal/{fec,wire,protocol} with the drop-in's patches applied."""
    root = tmp_path_factory.mktemp("goref")
    for sub in ("internal/fec", "internal/wire", "internal/protocol"):
        shutil.copytree(os.path.join(REF, sub), str(root / sub))
    for diff, target in (("manager.go.diff", "internal/fec/manager.go"),
                         ("fec_source_symbol_frame.go.diff", "internal/wire/fec_source_symbol_frame.go"),
                         ("fec_repair_frame.go.diff", "internal/wire/fec_repair_frame.go")):
        r = subprocess.run(["patch", "-p1", "--batch", "--forward", "-i", os.path.join(PATCHES, diff)],
                           cwd=str(root), capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert os.path.exists(str(root / target))
    return str(root)


def _pkg_files(d):
    """A package's files in the linux/amd64 build (go_lite.build_ok), tests excluded."""
    out = []
    for f in sorted(os.listdir(d)):
        if f.endswith(".go") and not f.endswith("_test.go"):
            src = _read(os.path.join(d, f))
            if go_lite.build_ok(f, src):
                out.append((os.path.join(d, f), src))
    return out


def _ours(fechip, overrides=None):
    out = []
    for f in sorted(os.listdir(GO)):
        if not f.endswith(".go"):
            continue
        src = (overrides or {}).get(f) or _read(os.path.join(GO, f))
        tag = _tags(src)
        if tag == "fechip" and not fechip or tag == "!fechip" and fechip:
            continue
        out.append((os.path.join(GO, f), src))
    return out


def _other_pkgs():
    """Declarations of the reference's other packages package quic imports (internal/ackhandler,
    handshake, qerr, utils, ..., logging, quicvarint): more of its selectors and calls typed."""
    out = []
    for sub in sorted(os.listdir(os.path.join(REF, "internal"))):
        d = os.path.join(REF, "internal", sub)
        if os.path.isdir(d) and sub not in ("fec", "wire", "protocol"):
            out += _pkg_files(d)
    for sub in ("logging", "quicvarint"):
        if os.path.isdir(os.path.join(REF, sub)):
            out += _pkg_files(os.path.join(REF, sub))
    return out


# the patched reference files whose bodies are checked too (the rest give declarations only)
CHECKED_REF = ("internal/fec/manager.go", "internal/wire/fec_source_symbol_frame.go",
               "internal/wire/fec_repair_frame.go")


def check(patched, fechip=True, overrides=None):
    files = _pkg_files(os.path.join(patched, "internal", "wire")) + \
        _pkg_files(os.path.join(patched, "internal", "protocol")) + \
        _pkg_files(os.path.join(patched, "internal", "fec"))
    checked = {os.path.join(patched, f) for f in CHECKED_REF}
    decls = [(p, s) for p, s in files if p not in checked]
    ours = _ours(fechip, overrides) + [(p, s) for p, s in files if p in checked]
    uni = go_lite.load_universe([_read(h) for h in HEADERS], decls, ours)
    ck = go_lite.Checker(uni)
    errors = ck.check_all()
    dups = go_lite.duplicate_decls(uni, "fec", [p for p, _ in ours])
    return errors, dups, ck.stats


QUIC_PATCHES = ("connection.go", "packet_packer.go", "repair_queue.go")


def _added_lines(diff_text):
    """New-file line numbers of a unified diff's added lines."""
    out, new = set(), 0
    for ln in diff_text.split("\n"):
        m = re.match(r"@@ -\d+(?:,\d+)? \+(\d+)", ln)
        if m:
            new = int(m.group(1))
            continue
        if ln.startswith("+++") or ln.startswith("---"):
            continue
        if ln.startswith("+"):
            out.add(new)
            new += 1
        elif ln.startswith(" "):
            new += 1
    return out


@pytest.fixture(scope="module")
def patched_quic(patched, tmp_path_factory):
    """The reference's root package (package quic) with the connection / packer / repair-queue
    hooks applied; returns (dir, {file: added line numbers})."""
    root = tmp_path_factory.mktemp("goquic")
    for f in os.listdir(REF):
        if f.endswith(".go") and not f.endswith("_test.go"):
            shutil.copy(os.path.join(REF, f), str(root / f))
    added = {}
    for f in QUIC_PATCHES:
        diff = os.path.join(PATCHES, f + ".diff")
        r = subprocess.run(["patch", "-p1", "--batch", "--forward", "-i", diff], cwd=str(root),
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        added[f] = _added_lines(_read(diff))
    return str(root), added


def check_quic(patched, patched_quic, overrides=None, fechip=True):
    """The functions of package quic the hooks add or change, against package quic's own
    declarations and internal/fec with the drop-in (either build configuration)."""
    qdir, added = patched_quic
    files = _pkg_files(os.path.join(patched, "internal", "wire")) + \
        _pkg_files(os.path.join(patched, "internal", "protocol")) + \
        _pkg_files(os.path.join(patched, "internal", "fec")) + _ours(fechip)
    quic = _pkg_files(qdir)
    uni = go_lite.Universe()
    uni.assertions = []
    for h in HEADERS:
        uni.load_c_header(_read(h))
    for p, s in files + _other_pkgs():
        uni.load_go(p, s)
    for p, s in quic:
        name = os.path.basename(p)
        if name not in added:
            uni.load_go(p, s)
    for p, s in quic:
        name = os.path.basename(p)
        if name in added:
            uni.load_go(p, (overrides or {}).get(name) or s, check=added[name])
    ck = go_lite.Checker(uni)
    return ck.check_all(), ck.stats, [fd.name for _, fd in uni.bodies]


@needs_ref
@pytest.mark.parametrize("fechip", [True, False], ids=["tags_fechip", "default_build"])
def test_patched_quic_package_type_checks(patched, patched_quic, fechip):
    """All of package quic with the hooks applied (not only the functions they change) against
    internal/fec with the drop-in: the patches break nothing around them."""
    qdir, _ = patched_quic
    files = _pkg_files(os.path.join(patched, "internal", "wire")) + \
        _pkg_files(os.path.join(patched, "internal", "protocol")) + \
        _pkg_files(os.path.join(patched, "internal", "fec")) + _ours(fechip) + _other_pkgs()
    uni = go_lite.load_universe([_read(h) for h in HEADERS], files, _pkg_files(qdir))
    ck = go_lite.Checker(uni)
    errors = ck.check_all()
    assert not errors, "\n".join(errors)
    assert ck.stats["stmts"] > 4000


@needs_ref
@pytest.mark.parametrize("fechip", [True, False], ids=["tags_fechip", "default_build"])
def test_quic_hooks_type_check(patched, patched_quic, fechip):
    errors, stats, funcs = check_quic(patched, patched_quic, fechip=fechip)
    assert not errors, "\n".join(errors)
    for fn in ("handleRecoveredFEC", "closeFEC", "pollRepairFrames", "fecSourcePayloadBuffer", "Room", "run"):
        assert fn in funcs, funcs
    assert stats["stmts"] > 200, stats


QUIC_SEEDED = [
    ("packet_packer.go", "poller.PollRepairFrames(p.repairQueue.Room())", "poller.PollRepairFrames()",
     "call: 0 arguments, want 1"),
    ("packet_packer.go", "p.repairQueue.Room()", "p.repairQueue.Space()", "has no field or method Space"),
    ("packet_packer.go", "return make([]byte, 0, protocol.MaxPacketBufferSize)",
     "return make([]int, 0, protocol.MaxPacketBufferSize)", "cannot use []int as []uint8"),
    ("connection.go", "!poller.RecoveryPending()", "!poller.RecoveriesPending()",
     "has no field or method RecoveriesPending"),
    ("connection.go", "recovered, err := poller.PollRecovered(wait)", "recovered := poller.PollRecovered(wait)",
     "assignment mismatch: 1 variables but the call returns 2 values"),
]


@needs_ref
@pytest.mark.parametrize("case", range(len(QUIC_SEEDED)))
def test_quic_seeded_error_is_reported(patched, patched_quic, case):
    f, old, new, msg = QUIC_SEEDED[case]
    src = _read(os.path.join(patched_quic[0], f))
    assert old in src, "seed %d no longer matches %s" % (case, f)
    errors, _, _ = check_quic(patched, patched_quic, {f: src.replace(old, new, 1)})
    assert any(msg in e for e in errors), (msg, errors)


@needs_ref
@pytest.mark.parametrize("fechip", [True, False], ids=["tags_fechip", "default_build"])
def test_drop_in_type_checks(patched, fechip):
    errors, dups, stats = check(patched, fechip)
    assert not errors, "\n".join(errors)
    assert not dups, dups


@needs_ref
@pytest.mark.parametrize("target", ["internal/fec", "internal/wire", "internal/protocol", "."])
def test_checker_is_silent_on_the_reference(target):
    """No false positives: the reference's own packages (Go that compiles) check clean, every
    function body of them (~5 800 statements with package quic, "."), against each other's
    declarations (linux/amd64 build constraints)."""
    decls, files = (_other_pkgs() if target == "." else []), []
    for sub in ("internal/fec", "internal/wire", "internal/protocol", "."):
        if sub == "." and target != ".":
            continue
        (files if sub == target else decls).extend(_pkg_files(os.path.join(REF, sub)))
    uni = go_lite.load_universe([_read(h) for h in HEADERS], decls, files)
    ck = go_lite.Checker(uni)
    errors = ck.check_all()
    assert not errors, "\n".join(errors)
    assert ck.stats["stmts"] > 100


@needs_ref
def test_checker_reach(patched):
    """The checker is not vacuous on these files: it typed nearly every selector, call and cgo
    argument it met (unknown types are the standard library's and cgo runtime helpers')."""
    errors, _, st = check(patched, True)
    assert not errors
    assert st["stmts"] > 300 and st["c_args"] >= 100, st
    assert st["c_args_typed"] == st["c_args"], st
    assert st["selectors_typed"] >= 0.95 * st["selectors"], st
    assert st["calls_typed"] >= 0.9 * st["calls"], st


# Seeded errors: (file, old text, new text, message the checker must report)
SEEDED = [
    ("batch_manager_hip.go", "maxBlocks = maxFrames / m.tx.m", "maxBlocks = maxFrames / m.tx.mm",
     "has no field or method mm"),
    ("batch_manager_hip.go", "bS := m.blockStatuses[blockID]\n\tif bS.isProcessed {",
     "bS := m.blockStatuses[blockID]\n\tif bS.processed {", "has no field or method processed"),
    ("batch_hip.go", "C.size_t(maxBlocks), C.int(hipDevice()), &rc)\n\tif e == nil",
     "maxBlocks, C.int(hipDevice()), &rc)\n\tif e == nil", "C.fec_go_encoder_new argument 4: cannot use int as C.size_t"),
    ("batch_hip.go", "s.lens, C.int(n)))\n\t}", "s.lens, n))\n\t}", "cannot use int as C.int"),
    ("reed_solomon_hip.go", "&mask, &status, C.FEC_HOST)", "&status, &mask, C.FEC_HOST)",
     "cannot use *C.int32_t as *C.uint32_t"),
    ("batch_hip.go", "&r.ids[0], &r.plen[0], &r.offs[0],", "&r.ids[0], &r.offs[0], &r.plen[0],",
     "cannot use *C.uint64_t as *C.uint32_t"),
    ("xor_hip.go", "C.fec_xor_encode_batch(s.ctx, C.int(k), C.size_t(L), 1,",
     "C.fec_xor_encode_batch(s.ctx, C.int(k), C.size_t(L),", "C.fec_xor_encode_batch: 9 arguments, want 10"),
    ("batch_manager_hip.go", "\treturn 2, 1, true\n", "\treturn 2, true\n", "wrong number of return values"),
    ("batch_manager_hip.go", "k, m, ok := hipCode(id)\n\tif !ok || !useHIP() {\n\t\treturn nil, false, nil\n\t}\n\tif hipMode() == \"block\" {\n\t\ts, err := newHIPBlockScheme(id, k, m)\n\t\tif err != nil {\n\t\t\treturn nil, true, err\n\t\t}\n\t\tmgr, err := NewManager(s, k, m)\n\t\tif err != nil {\n\t\t\treturn nil, true, err\n\t\t}\n\t\treturn mgr, true, nil\n\t}\n\tbm, err := newBatchManager(id, k, m, true)",
     "k, m := hipCode(id)\n\tif !useHIP() {\n\t\treturn nil, false, nil\n\t}\n\tif hipMode() == \"block\" {\n\t\ts, err := newHIPBlockScheme(id, k, m)\n\t\tif err != nil {\n\t\t\treturn nil, true, err\n\t\t}\n\t\tmgr, err := NewManager(s, k, m)\n\t\tif err != nil {\n\t\t\treturn nil, true, err\n\t\t}\n\t\treturn mgr, true, nil\n\t}\n\tbm, err := newBatchManager(id, k, m, true)",
     "assignment mismatch: 2 variables but the call returns 3 values"),
    ("batch_hip.go", "Metadata: protocol.BlockMetadata{BlockID: protocol.BlockID(s.ids[d]), ParityID: protocol.ParityID(i)},",
     "Metadata: protocol.BlockMetadata{Block: protocol.BlockID(s.ids[d]), ParityID: protocol.ParityID(i)},",
     "unknown field Block in struct literal"),
    ("batch_hip.go", "ParityID: protocol.ParityID(i)},", "ParityID: i},", "cannot use int as protocol.ParityID"),
    ("batch_manager_hip.go", "func (m *batchManager) RecoveriesInFlight() bool { return m.pending > 0 }",
     "func (m *batchManager) RecoveriesInFlight() int { return m.pending }",
     "does not implement fec.RecoveredPoller (method RecoveriesInFlight has type func() (int)"),
    ("batch_manager_hip.go", "func (m *batchManager) SourcePayloadBuffer() []byte {",
     "func (m *batchManager) SourcePayloadBuf() []byte {", "missing method SourcePayloadBuffer"),
    ("packet_pool_hip.go", "i := int32(off / C.FEC_GO_POOL_SLOT)", "i := off / C.FEC_GO_POOL_SLOT",
     "cannot use uintptr as int32"),
    ("reed_solomon_hip.go", "ssid := b.smallestSSID + protocol.SourceSymbolID(i)\n\t\tif _, ok",
     "ssid := b.smallestSSID + i\n\t\tif _, ok", "mismatched types protocol.SourceSymbolID and int"),
    ("hip_cgo.go", "return errors.New(C.GoString(C.fec_strerror(rc)))", "return errors.New(C.GoString(C.fec_strerr(rc)))",
     "C.fec_strerr is not declared"),
    ("batch_manager_hip.go", "m.release = append(m.release, f.Payload)\n\t\t}\n\t\treturn nil, nil",
     "m.relase = append(m.release, f.Payload)\n\t\t}\n\t\treturn nil, nil", "has no field or method relase"),
    ("xor_hip.go", "payloadLen := uint16(rec[big])<<8 | uint16(rec[big+1])",
     "payloadLen := uint16(rec[bigg])<<8 | uint16(rec[big+1])", "undefined: bigg"),
    ("batch_hip.go", "\tn := 0\n\tadd := func(p []byte) {", "\tn := 0\n\tunused := 3\n\tadd := func(p []byte) {",
     "declared and not used: unused"),
    ("reed_solomon_hip.go", "\t\tshard, err := rs.addLengthToSourceSymbolPayload(b, ssid)\n\t\tif err != nil {\n\t\t\treturn nil, err\n\t\t}\n\t\tcopy(buf[i*L:(i+1)*L], shard)\n\t\tmask",
     "\t\tshard, err := rs.addLengthToSourceSymbolPayload(b, ssid)\n\t\tif err != nil {\n\t\t\treturn nil, err\n\t\t}\n\t\tshard = nil\n\t\tmask",
     "declared and not used: shard"),
    ("packet_pool_hip.go", '\t"sync"\n\t"unsafe"\n', '\t"sync"\n\t"strings"\n\t"unsafe"\n',
     "imported and not used: strings"),
    ("hip_cgo.go", 'os.Getenv("FEC_HIP_DEVICE")); err == nil {\n\t\treturn v\n\t}\n\treturn 0\n}',
     'os.Getenv("FEC_HIP_DEVICE")); err == nil {\n\t\treturn v\n\t}\n}', "missing return"),
    ("packet_pool_hip.go", "\tif len(pp.free) == 0 {\n\t\treturn nil", "\tif len(pp.free) {\n\t\treturn nil",
     "non-boolean condition in if statement (int)"),
    # the round-3 verdict's example: BatchSender.m of another integer type than maxFrames
    ("batch_hip.go", "\tscheme  protocol.DecoderFECScheme\n\tk, m    int\n", "\tscheme  protocol.DecoderFECScheme\n\tk, m    C.int\n",
     "mismatched types int and C.int (operator /)"),
]


@needs_ref
@pytest.mark.parametrize("case", range(len(SEEDED)))
def test_seeded_error_is_reported(patched, case):
    f, old, new, msg = SEEDED[case]
    src = _read(os.path.join(GO, f))
    assert old in src, "seed %d no longer matches %s" % (case, f)
    errors, _, _ = check(patched, True, {f: src.replace(old, new, 1)})
    assert any(msg in e for e in errors), (msg, errors)


@needs_ref
def test_seeded_duplicate_declaration_is_reported(patched):
    """useHIP is declared by hip_cgo.go (fechip) and hip_stub.go (!fechip): dropping the stub's
    build tag puts both in the fechip build."""
    src = _read(os.path.join(GO, "hip_stub.go")).replace("//go:build !fechip\n", "", 1)
    _, dups, _ = check(patched, True, {"hip_stub.go": src})
    assert any(name == "useHIP" for name, _ in dups), dups


def test_checker_on_a_small_package():
    """The checker's own cases, without the reference: scoping, comma-ok, closures, promotion."""
    src = '''package p

type inner struct{ n int }

func (i *inner) Get() int { return i.n }

type outer struct {
	*inner
	m map[string][]byte
}

type Getter interface{ Get() int }

var _ Getter = &outer{}

func use(o *outer, k string) (int, bool) {
	v, ok := o.m[k]
	if !ok {
		return 0, false
	}
	add := func(b []byte) int { return len(b) + o.Get() }
	total := 0
	for i, x := range v {
		total += int(x) + i
	}
	if n := add(v); n > 0 {
		total += n
	}
	return total + o.n, true
}
'''
    uni = go_lite.load_universe([], [], [("p.go", src)])
    ck = go_lite.Checker(uni)
    assert ck.check_all() == []
    bad = src.replace("return total + o.n, true", "return total + o.nn, 1")
    uni = go_lite.load_universe([], [], [("p.go", bad)])
    errs = go_lite.Checker(uni).check_all()
    assert any("no field or method nn" in e for e in errs) and any("cannot use untyped int as bool" in e for e in errs), errs
    bad = src.replace("func (i *inner) Get() int", "func (i *inner) Get() uint")
    uni = go_lite.load_universe([], [], [("p.go", bad)])
    errs = go_lite.Checker(uni).check_all()
    assert any("does not implement" in e for e in errs), errs
