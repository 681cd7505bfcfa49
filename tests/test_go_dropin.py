"""The Go drop-in, checked mechanically on the CPU (there is no Go toolchain in this image).

What is committed (go/):
  go/internal/fec/*.go   files added to the reference's internal/fec: the cgo binding
                         (fechip build tag), the batched managers, the !fechip stubs, and the
                         RepairPoller / RecoveredPoller interfaces (no tag)
  go/patches/*.diff      the hooks in the reference's own files: manager.go (scheme selection,
                         manager.go:50-94), packet_packer.go (:650-664, :1005-1011),
                         connection.go (:218, :594-630, :1341, :1660-1666), repair_queue.go,
                         and the wire parsers' payload allocation (fec_source_symbol_frame.go:34,
                         fec_repair_frame.go:36: the receive side of the registered pool)

These tests tie the three descriptions of the boundary together, so none can drift unnoticed:
  * every diff applies to the reference's files (patch --dry-run, then for real);
  * every C.fec_* call in the Go files names a prototype of include/*.h with the same number of
    arguments, every C constant / type it names is declared there, and the call set equals the
    one tests/c/fec_go_harness.c issues (the harness stands in for the Go files on the GPU);
  * every field the Go files read from a reference type (block, manager, wire.RepairFrame,
    protocol.BlockMetadata) and every protocol / wire identifier they name exists in the
    reference's sources (block.go:23-34, manager.go:35-48, ...);
  * identifiers the patches introduce are declared by the committed Go files, with the same
    signatures on both sides of the fechip build tag;
  * the Go files are lexically well formed (balanced delimiters outside strings and comments).
Reads /root/reference (the build container only; skipped where it is absent).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GO = os.path.join(ROOT, "go", "internal", "fec")
PATCHES = os.path.join(ROOT, "go", "patches")
INCLUDE = os.path.join(ROOT, "include")
HARNESS = os.path.join(ROOT, "tests", "c", "fec_go_harness.c")

PATCH_TARGETS = {"manager.go.diff": "internal/fec/manager.go", "packet_packer.go.diff": "packet_packer.go",
                 "connection.go.diff": "connection.go", "repair_queue.go.diff": "repair_queue.go",
                 "fec_source_symbol_frame.go.diff": "internal/wire/fec_source_symbol_frame.go",
                 "fec_repair_frame.go.diff": "internal/wire/fec_repair_frame.go"}

needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not present")


def _go_files():
    return sorted(os.path.join(GO, f) for f in os.listdir(GO) if f.endswith(".go"))


def _read(p):
    with open(p) as fh:
        return fh.read()


def _strip_go(src):
    """Go source with comments removed and string / rune literals blanked (delimiters inside
    them must not count). The cgo preamble (a comment) is removed with the other comments."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            assert j >= 0, "unterminated block comment"
            out.append("\n" * src.count("\n", i, j))
            i = j + 2
        elif c in "\"'":
            j = i + 1
            while src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(c + c)
            i = j + 1
        elif c == "`":
            j = src.index("`", i + 1)
            out.append('""')
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _c_preamble(src):
    m = re.search(r"/\*(.*?)\*/\s*import \"C\"", src, re.S)
    lines = [ln[3:] if ln.startswith("// ") else ln for ln in src.split("\n")]
    pre = m.group(1) if m else ""
    if not m:   # line-comment preamble: the // lines right above import "C"
        txt = src.split('import "C"')[0].rstrip().split("\n")
        block = []
        for ln in reversed(txt):
            if not ln.startswith("//"):
                break
            block.append(ln[2:].strip())
        pre = "\n".join(reversed(block))
    del lines
    return pre


def _split_args(s):
    """Top-level comma split of a call's argument text."""
    args, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        args.append(cur.strip())
    return args


def _c_calls(code):
    """(name, argument count) of every C.fec_*( call."""
    calls = []
    for m in re.finditer(r"\bC\.(fec_\w+)\(", code):
        i, depth = m.end(), 1
        j = i
        while depth:
            depth += {"(": 1, ")": -1}.get(code[j], 0)
            j += 1
        calls.append((m.group(1), len(_split_args(code[i:j - 1]))))
    return calls


def _header_protos():
    protos, defines, types = {}, set(), set()
    for f in os.listdir(INCLUDE):
        if not f.endswith(".h"):
            continue
        src = _read(os.path.join(INCLUDE, f))
        defines |= set(re.findall(r"#define\s+(\w+)", src))
        types |= set(re.findall(r"typedef\s+struct\s+\w+\s+(\w+)\s*;", src))
        body = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        body = re.sub(r"//[^\n]*", "", body)
        for m in re.finditer(r"\b(fec_\w+)\s*\(([^;{)]*(?:\([^)]*\)[^;{)]*)*)\)\s*;", body):
            params = m.group(2).strip()
            protos[m.group(1)] = 0 if params in ("", "void") else len(_split_args(params))
    return protos, defines, types


# ---------------------------------------------------------------------------- lexical form

@pytest.mark.parametrize("path", _go_files(), ids=os.path.basename)
def test_go_file_is_well_formed(path):
    src = _read(path)
    code = _strip_go(src)
    stack = []
    pairs = {")": "(", "]": "[", "}": "{"}
    for lineno, line in enumerate(code.split("\n"), 1):
        for ch in line:
            if ch in "([{":
                stack.append((ch, lineno))
            elif ch in ")]}":
                assert stack and stack[-1][0] == pairs[ch], "unbalanced %r at line %d" % (ch, lineno)
                stack.pop()
    assert not stack, "unclosed %r from line %d" % stack[-1]
    assert re.search(r"^package fec$", code, re.M), "package clause"
    # cgo files carry the fechip tag; the stubs carry !fechip; the rest (interfaces) none
    if 'import "C"' in src:
        assert src.startswith("//go:build fechip\n"), "cgo file without the fechip build tag"
    for imp in re.findall(r'"(github\.com/quic-go/quic-go/[^"]+)"', src):
        assert imp in ("github.com/quic-go/quic-go/internal/protocol", "github.com/quic-go/quic-go/internal/wire")
        alias = imp.rsplit("/", 1)[1]
        assert re.search(r"\b%s\." % alias, code), "unused import %s" % imp


# ---------------------------------------------------------------------------- the C boundary

def test_c_calls_match_the_headers():
    protos, defines, types = _header_protos()
    assert len(protos) > 40, "header parse found too few prototypes"
    builtin = {"int", "uint", "size_t", "uint8_t", "uint32_t", "int32_t", "uint64_t", "uintptr_t", "malloc",
               "free", "GoString", "char"}
    seen = set()
    for path in _go_files():
        src = _read(path)
        code = _strip_go(src)
        if 'import "C"' not in src:
            assert "C." not in code, "%s uses C without importing it" % path
            continue
        pre = _c_preamble(src)
        included = set(re.findall(r'#include\s+"([^"]+)"', pre))
        for name, nargs in _c_calls(code):
            assert name in protos, "%s calls C.%s, declared by no include/*.h" % (os.path.basename(path), name)
            assert nargs == protos[name], "C.%s: %d args in %s, %d in the header" % (
                name, nargs, os.path.basename(path), protos[name])
            hdr = [h for h in os.listdir(INCLUDE) if re.search(r"\b%s\s*\(" % name, _read(os.path.join(INCLUDE, h)))]
            assert included & set(hdr) or "hip_cgo.go" in path, "%s: C.%s without including %s" % (path, name, hdr)
            seen.add(name)
        for ident in set(re.findall(r"\bC\.(\w+)", code)):
            if ident.startswith("fec_") and ident in protos:
                continue
            assert ident in builtin or ident in defines or ident in types, \
                "%s names C.%s, not declared in include/*.h" % (os.path.basename(path), ident)
    harness = set(re.findall(r"\b(fec_\w+)\s*\(", _strip_go(_read(HARNESS))))
    assert seen <= harness, "C entry points the Go files use but the GPU harness never calls: %s" % (seen - harness)
    assert {"fec_go_encoder_submit", "fec_go_decoder_poll", "fec_rs_reconstruct_batch"} <= seen


# ---------------------------------------------------------------------------- reference types

def _ref_struct_fields(path, name):
    src = _strip_go(_read(path))
    m = re.search(r"type %s struct \{(.*?)\n\}" % name, src, re.S)
    assert m, "%s not found in %s" % (name, path)
    fields = set()
    for line in m.group(1).split("\n"):
        toks = line.strip().split()
        if not toks:
            continue
        if len(toks) == 1:   # embedded
            fields.add(toks[0].lstrip("*").split(".")[-1])
        else:
            fields |= {t.rstrip(",") for t in toks[:-1] if re.match(r"^[A-Za-z_]\w*,?$", t)}
            fields.add(toks[0])
    return fields


def _ref_methods(pkgdir, recv):
    out = set()
    for f in os.listdir(pkgdir):
        if f.endswith(".go") and not f.endswith("_test.go"):
            out |= set(re.findall(r"func \(\w+ \*?%s\) (\w+)\(" % recv, _read(os.path.join(pkgdir, f))))
    return out


@needs_ref
def test_block_and_manager_fields_exist_in_the_reference():
    fecdir = os.path.join(REF, "internal", "fec")
    block = _ref_struct_fields(os.path.join(fecdir, "block.go"), "block") | _ref_methods(fecdir, "block")
    mgr = _ref_struct_fields(os.path.join(fecdir, "manager.go"), "manager") | _ref_methods(fecdir, "manager")
    bstat = _ref_struct_fields(os.path.join(fecdir, "manager.go"), "blockStatus")
    assert {"ssidToSourcePayload", "biggestSourceSymbolLenSoFar", "isComplete"} <= block
    ours = {}
    for path in _go_files():
        code = _strip_go(_read(path))
        ours[path] = code
        for fld in re.findall(r"\bb\.(\w+)", code):
            assert fld in block, "%s reads b.%s, not a field / method of block (block.go:23-95)" % (path, fld)
        for fld in re.findall(r"\bbS\.(\w+)", code):
            assert fld in bstat, "%s: bS.%s not in blockStatus (manager.go:35-39)" % (path, fld)
    bm = ours[os.path.join(GO, "batch_manager_hip.go")]
    own = set(re.findall(r"func \(m \*batchManager\) (\w+)\(", bm)) | _ref_struct_fields(
        os.path.join(GO, "batch_manager_hip.go"), "batchManager")
    assert {"manager", "tx", "rx", "pending", "pool", "held"} <= own
    for fld in re.findall(r"\bm\.(\w+)", bm):
        assert fld in own or fld in mgr, "batch_manager_hip.go: m.%s is neither its own nor manager.go's" % fld


@needs_ref
def test_protocol_and_wire_identifiers_exist_in_the_reference():
    decl = {}
    for pkg in ("protocol", "wire"):
        names = set()
        d = os.path.join(REF, "internal", pkg)
        for f in os.listdir(d):
            if f.endswith(".go") and not f.endswith("_test.go"):
                src = _strip_go(_read(os.path.join(d, f)))
                names |= set(re.findall(r"^\s*(?:type|func|const|var)\s+([A-Z]\w*)", src, re.M))
                names |= set(re.findall(r"^\t([A-Z]\w*)\b", src, re.M))   # const / var block entries
        decl[pkg] = names
    # and what the wire patches declare (the receive-side allocator hook)
    for d in ("fec_source_symbol_frame.go.diff", "fec_repair_frame.go.diff"):
        add = "\n".join(ln[1:] for ln in _read(os.path.join(PATCHES, d)).split("\n")
                        if ln.startswith("+") and not ln.startswith("+++"))
        decl["wire"] |= set(re.findall(r"^\s*(?:type|func|const|var)\s+([A-Z]\w*)", _strip_go(add), re.M))
    texts = [_strip_go(_read(p)) for p in _go_files()]
    texts += ["\n".join(ln[1:] for ln in _read(os.path.join(PATCHES, d)).split("\n") if ln.startswith("+"))
              for d in PATCH_TARGETS]
    used = 0
    for t in texts:
        for pkg in ("protocol", "wire"):
            for ident in re.findall(r"\b%s\.([A-Z]\w*)" % pkg, t):
                assert ident in decl[pkg], "%s.%s is not declared in the reference's internal/%s" % (pkg, ident, pkg)
                used += 1
    assert used > 20
    # composite-literal keys of the reference's frame types
    rf = _ref_struct_fields(os.path.join(REF, "internal", "wire", "fec_repair_frame.go"), "RepairFrame")
    meta_src = [os.path.join(REF, "internal", "protocol", f) for f in os.listdir(os.path.join(REF, "internal", "protocol"))]
    meta = next(_ref_struct_fields(p, "BlockMetadata") for p in meta_src
                if p.endswith(".go") and "type BlockMetadata struct" in _read(p))
    for t in texts:
        for body in re.findall(r"wire\.RepairFrame\{(.*?)\}\s*$", t, re.M | re.S):
            for key in re.findall(r"\b([A-Z]\w*):", body.split("{")[0]):
                assert key in rf, "wire.RepairFrame has no field %s" % key
        for body in re.findall(r"protocol\.BlockMetadata\{([^}]*)\}", t):
            for key in re.findall(r"\b([A-Z]\w*):", body):
                assert key in meta, "protocol.BlockMetadata has no field %s" % key


# ---------------------------------------------------------------------------- the patches

@needs_ref
@pytest.mark.parametrize("diff", sorted(PATCH_TARGETS), ids=lambda d: d.split(".")[0])
def test_patch_applies_to_the_reference(diff, tmp_path):
    target = PATCH_TARGETS[diff]
    dst = tmp_path / target
    dst.parent.mkdir(parents=True, exist_ok=True)
    shutil.copy(os.path.join(REF, target), dst)
    p = os.path.join(PATCHES, diff)
    for dry in (True, False):
        r = subprocess.run(["patch", "-p1", "--batch", "--forward"] + (["--dry-run"] if dry else []) + ["-i", p],
                           cwd=str(tmp_path), capture_output=True, text=True)
        assert r.returncode == 0 and "FAILED" not in r.stdout and "offset" not in r.stdout.lower(), r.stdout + r.stderr
    patched = _read(str(dst))
    assert patched != _read(os.path.join(REF, target))
    code = _strip_go(patched)
    assert code.count("{") == code.count("}") and code.count("(") == code.count(")")


def _decls(code):
    return set(re.findall(r"^func (?:\(\w+ \*?\w+\) )?(\w+)\(", code, re.M)) | \
        set(re.findall(r"^type (\w+) ", code, re.M)) | set(re.findall(r"^\t(\w+)\(", code, re.M))


@needs_ref
def test_patch_identifiers_are_declared():
    """Everything the hooks call into exists: the fec identifiers in internal/fec (our Go files),
    the package-quic ones in the patched files themselves."""
    fec_decl = set()
    for p in _go_files():
        fec_decl |= _decls(_strip_go(_read(p)))
    added = {d: "\n".join(ln[1:] for ln in _read(os.path.join(PATCHES, d)).split("\n")
                          if ln.startswith("+") and not ln.startswith("+++")) for d in PATCH_TARGETS}
    mgr = _strip_go(added["manager.go.diff"])
    for ident in ("newHIPSender", "newHIPReceiver"):
        assert ident in mgr and ident in fec_decl
    quic = _strip_go(added["packet_packer.go.diff"] + "\n" + added["connection.go.diff"])
    ref_fec = os.path.join(REF, "internal", "fec")
    for f in os.listdir(ref_fec):   # the reference package's own declarations (fec.Sender, ...)
        if f.endswith(".go") and not f.endswith("_test.go"):
            fec_decl |= _decls(_strip_go(_read(os.path.join(ref_fec, f))))
    for ident in set(re.findall(r"\bfec\.([A-Z]\w*)", quic)):
        assert ident in fec_decl, "fec.%s used by a hook but not declared in internal/fec" % ident
    for meth in set(re.findall(r"poller\.(\w+)\(", quic)):
        assert meth in fec_decl, "poller.%s is not a method of the poller interfaces (fec_poll.go)" % meth
    assert "Room" in _decls(_strip_go(added["repair_queue.go.diff"]))
    assert re.search(r"repairQueue\.Room\(\)", quic)
    for ident in ("pollRepairFrames", "handleRecoveredFEC", "closeFEC"):
        assert re.search(r"func \(\w \*\w+\) %s\(" % ident, quic)


def _sig(code, name):
    m = re.search(r"^func %s(\(.*?)\{" % name, code, re.M)
    assert m, name
    return re.sub(r"\s+", " ", re.sub(r"\b(\w+) (protocol\.|Sender|Receiver|bool|error)", r"\2", m.group(1))).strip()


def test_stub_and_engine_signatures_agree():
    stub = _strip_go(_read(os.path.join(GO, "hip_stub.go")))
    assert _read(os.path.join(GO, "hip_stub.go")).startswith("//go:build !fechip\n")
    eng = _strip_go(_read(os.path.join(GO, "batch_manager_hip.go")) + _read(os.path.join(GO, "hip_cgo.go")))
    for name in ("newHIPSender", "newHIPReceiver", "useHIP"):
        assert _sig(stub, name) == _sig(eng, name), name
    # the interfaces the hooks assert are untagged, so both builds see them
    poll = _read(os.path.join(GO, "fec_poll.go"))
    assert "go:build" not in poll and "type RepairPoller interface" in poll and "type RecoveredPoller interface" in poll
    bm = _strip_go(_read(os.path.join(GO, "batch_manager_hip.go")))
    for meth in re.findall(r"^\t(\w+)\(", _strip_go(poll), re.M):
        assert re.search(r"func \(m \*batchManager\) %s\(" % meth, bm), meth
