"""The Go binding's call sequence, checked against the reference's golden tables.

go/internal/fec/{reed_solomon_hip,xor_hip,batch_hip}.go cannot be compiled here (no Go
toolchain in the image), so tests/c/fec_go_harness.c restates each Go function's C calls line for
line (same checks, buffer layout, strides, present masks and FEC_HOST flags) and is run over

  * every case of reed_solomon_test.go / xor_test.go (tests/golden/reference_cases.json), and
  * seeded synthetic blocks (RS(20,10) / RS(8,4) / RS(6,2) / RS(2,1) (config #1's code) / XOR(k,1), ragged payload lengths,
    random losses) whose expected frames / payloads / errors come from the oracle's scheme
    layer (oracle/oracle.py, restating reed_solomon.go / xor.go).

`direct` mode = the per-block schemes (hipReedSolomonScheme / hipXorScheme); `batch` mode =
BatchSender / BatchReceiver over include/fec_go.h; `batchref` = the same with the sender's source
payloads in a registered packet-buffer pool, submitted by reference (BatchSender.SubmitRef:
gathered by the device). CPU: the harness compiles, links the library
and the batch mode reports every validation error the reference reports with no device touched;
GPU: every case, bit-exact, plus the reference's error texts in direct mode.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "0xfec_amd")


def _sym_lines(tag, d):
    out = []
    for key in sorted(d, key=int):
        v = d[key]
        out.append("%s %d %d %s" % (tag, int(key), v["cap"], v["hex"] or "-"))
    return out


def _case_text(kind, blk, k, m):
    lines = ["case %s %d %d %d %d %d %d %d %d" % (
        kind, k, m, blk["id"], blk["smallestSSID"], blk["largestSSID"],
        blk["biggestSourceSymbolLenSoFar"], blk["totNumSourceSymbols"], blk["totNumRepairSymbols"])]
    lines += _sym_lines("src", blk["ssidToSourcePayload"])
    lines += _sym_lines("rep", blk["pidToRepairPayload"])
    lines.append("end")
    return "\n".join(lines)


def _golden_cases(golden):
    """(kind, block dict, k, m, expected) with expected = ('err', None) | ('frames', [hex]) |
    ('bytes', hex or None)."""
    cases = []
    for kind in ("rs_repair", "rs_recover", "xor_repair", "xor_recover"):
        for c in golden[kind]:
            blk = c["block"]
            k, m = c["rs_new"] or (blk["totNumSourceSymbols"], blk["totNumRepairSymbols"])
            if c["wantErr"]:
                exp = ("err", None)
            elif "repair" in kind:
                exp = ("frames", [f["Payload"]["hex"] for f in c["want"]["frames"]])
            else:
                exp = ("bytes", None if c["want"] is None else c["want"]["bytes"])
            cases.append((kind, blk, k, m, exp, c["ref"]))
    return cases


def _synthetic_cases(oracle):
    """Seeded blocks as a connection builds them (manager.go:123-227), expected from the oracle."""
    rng = np.random.default_rng(0x60FEC)
    cases = []
    for kind_base, k, m in (("rs", 20, 10), ("rs", 8, 4), ("rs", 6, 2), ("rs", 2, 1), ("xor", 2, 1), ("xor", 5, 1)):
        for t in range(4):
            bid = int(rng.integers(0, 1 << 20))
            lens = rng.integers(0, 1435, k)
            if t == 0:
                lens[:] = 1434
            pay = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in lens]
            smallest = bid * k
            big = int(lens.max())
            src = {str(smallest + i): {"cap": 1452, "hex": pay[i].hex()} for i in range(k)}
            blk = {"id": bid, "smallestSSID": smallest, "largestSSID": smallest + k - 1,
                   "biggestSourceSymbolLenSoFar": big, "totNumSourceSymbols": k,
                   "totNumRepairSymbols": m, "ssidToSourcePayload": src, "pidToRepairPayload": {}}
            ob = oracle.block_from_fixture(blk)
            if kind_base == "rs":
                frames, err = oracle.rs_repair_symbols(ob, k, m)
            else:
                frames, err = oracle.xor_repair_symbols(ob)
            assert err is None
            cases.append((kind_base + "_repair", blk, k, m, ("frames", [f[2].hex() for f in frames]),
                          "synthetic %s(%d,%d) #%d repair" % (kind_base, k, m, t)))
            # the receiver: lose up to m sources (t = 3: too many losses for RS -> error)
            nloss = m + 1 if (t == 3 and kind_base == "rs") else int(rng.integers(1, m + 1))
            lost = set(rng.choice(k, size=min(nloss, k), replace=False).tolist())
            keep_rep = list(range(m))
            rblk = dict(blk)
            rblk["ssidToSourcePayload"] = {s: v for s, v in src.items() if int(s) - smallest not in lost}
            rblk["pidToRepairPayload"] = {str(p): {"cap": len(frames[p][2]), "hex": frames[p][2].hex()}
                                          for p in keep_rep}
            # the receiver's biggest: max of the present sources, overwritten by a repair's len - 2
            rblk["biggestSourceSymbolLenSoFar"] = len(frames[0][2]) - 2
            ob = oracle.block_from_fixture(rblk)
            if kind_base == "rs":
                got, err = oracle.rs_recover_symbol_payloads(ob, k, m)
            else:
                got, err = oracle.xor_recover_symbol_payloads(ob)
            exp = ("err", err) if err is not None else ("bytes", None if got is None else got.hex())
            cases.append((kind_base + "_recover", rblk, k, m, exp,
                          "synthetic %s(%d,%d) #%d recover, %d lost" % (kind_base, k, m, t, len(lost))))
    return cases


def _empty_repair_cases(oracle):
    """RS blocks where a REPAIR arrived with a zero-length payload: klauspost's ReconstructData
    counts a zero-length shard as missing (no ErrShardSize), so the block recovers from the other
    shards, or fails with ErrTooFewShards when too few are left."""
    rng = np.random.default_rng(0xE0FEC)
    cases = []
    for k, m, nlost, empty, keep in ((8, 4, 2, (0,), (0, 1, 2, 3)), (8, 4, 2, (0,), (0, 1)),
                                     (20, 10, 3, (2, 5), tuple(range(10)))):
        bid = int(rng.integers(0, 1 << 20))
        lens = rng.integers(1, 1435, k)
        pay = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in lens]
        smallest = bid * k
        src = {str(smallest + i): {"cap": 1452, "hex": pay[i].hex()} for i in range(k)}
        blk = {"id": bid, "smallestSSID": smallest, "largestSSID": smallest + k - 1,
               "biggestSourceSymbolLenSoFar": int(lens.max()), "totNumSourceSymbols": k,
               "totNumRepairSymbols": m, "ssidToSourcePayload": src, "pidToRepairPayload": {}}
        frames, err = oracle.rs_repair_symbols(oracle.block_from_fixture(blk), k, m)
        assert err is None
        lost = sorted(rng.choice(k, size=nlost, replace=False).tolist())
        rblk = dict(blk)
        rblk["ssidToSourcePayload"] = {s: v for s, v in src.items() if int(s) - smallest not in lost}
        rblk["pidToRepairPayload"] = {str(p): ({"cap": 0, "hex": ""} if p in empty else
                                               {"cap": len(frames[p][2]), "hex": frames[p][2].hex()})
                                      for p in keep}
        rblk["biggestSourceSymbolLenSoFar"] = len(frames[0][2]) - 2
        got, err = oracle.rs_recover_symbol_payloads(oracle.block_from_fixture(rblk), k, m)
        exp = ("err", err) if err is not None else ("bytes", got.hex())
        cases.append(("rs_recover", rblk, k, m, exp, "RS(%d,%d) empty repairs %s, kept %s, lost %s"
                      % (k, m, empty, keep, lost)))
    return cases, pay


def test_empty_repair_is_a_missing_shard(oracle):
    """The oracle restates klauspost's zero-length rule: recovery ignores the empty repair."""
    cases, _ = _empty_repair_cases(oracle)
    kinds = [c[4][0] for c in cases]
    assert kinds == ["bytes", "err", "bytes"]
    assert cases[1][4][1] == "too few shards given"
    for c in (cases[0], cases[2]):   # the recovered bytes are the lost sources, concatenated
        blk, k = c[1], c[2]
        ob = oracle.block_from_fixture(dict(blk, pidToRepairPayload={
            p: v for p, v in blk["pidToRepairPayload"].items() if v["hex"]}))
        got, err = oracle.rs_recover_symbol_payloads(ob, k, c[3])
        assert err is None and got.hex() == c[4][1]


@pytest.fixture(scope="module")
def harness(fec):
    from native import binary
    return binary("fec_go_harness")


def _run(harness, cases, mode, tmp_path, env=None):
    fx = tmp_path / ("cases_%s.txt" % mode)
    fx.write_text("\n".join(_case_text(kind, blk, k, m) for kind, blk, k, m, _, _ in cases) + "\n")
    p = subprocess.run([harness, str(fx), mode], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    out = p.stdout
    results, cur = [], None
    for line in out.splitlines():
        tag, _, rest = line.partition(" ")
        if tag == "result":
            idx, _, tail = rest.partition(" ")
            status, _, text = tail.partition(" ")
            cur = {"status": status, "err": text if status == "err" else None, "frames": [], "bytes": None}
            results.append(cur)
        elif tag == "frame":
            cur["frames"].append(rest.split(" ")[1])
        elif tag == "bytes":
            cur["bytes"] = None if rest == "-" else rest
    assert len(results) == len(cases)
    return results


def _check(results, cases, texts):
    for r, (kind, blk, k, m, exp, ref) in zip(results, cases):
        what, val = exp
        if what == "err":
            assert r["status"] == "err", (ref, r)
            if texts and val is not None:
                assert r["err"] == val, (ref, r["err"], val)
        else:
            assert r["status"] == "ok", (ref, r["err"])
            if what == "frames":
                assert r["frames"] == val, ref
            else:
                # the block-complete case returns nil; an empty recovered payload prints "-" too
                assert (r["bytes"] or None) == (val or None), ref


def _with_oracle_texts(cases, oracle):
    """Error cases of the golden tables carry only wantErr: take the text from the oracle."""
    out = []
    for kind, blk, k, m, exp, ref in cases:
        if exp[0] == "err" and exp[1] is None:
            ob = oracle.block_from_fixture(blk)
            fn = {"rs_repair": lambda: oracle.rs_repair_symbols(ob, k, m),
                  "rs_recover": lambda: oracle.rs_recover_symbol_payloads(ob, k, m),
                  "xor_repair": lambda: oracle.xor_repair_symbols(ob),
                  "xor_recover": lambda: oracle.xor_recover_symbol_payloads(ob)}[kind]
            exp = ("err", fn()[1])
        out.append((kind, blk, k, m, exp, ref))
    return out


def test_harness_builds_and_validates_without_device(harness, golden, oracle, fec, tmp_path):
    """Batch mode with no GPU: the reference's validation errors come back before any device work
    (a block that needs the device fails loudly with the no-device error instead)."""
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    cases = _with_oracle_texts(_golden_cases(golden), oracle)
    results = _run(harness, cases, "batch", tmp_path)
    validated = 0
    for r, (kind, blk, k, m, exp, ref) in zip(results, cases):
        if r["status"] == "err" and r["err"] == "no HIP device":
            continue   # needs the device: fails loudly, no CPU fallback
        validated += 1
        if exp[0] == "err":
            assert r["status"] == "err" and r["err"] == exp[1], (ref, r, exp)
        else:
            assert r["status"] == "ok" and r["bytes"] is None and exp == ("bytes", None), (ref, r)
    assert validated >= 8
    # direct mode: the scheme constructor needs a device (fec_ctx_create) and says so
    for r in _run(harness, cases, "direct", tmp_path):
        assert r == {"status": "err", "err": "no HIP device", "frames": [], "bytes": None}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["direct", "batch", "batchref"])
def test_go_call_sequence_golden(harness, golden, oracle, mode, tmp_path):
    cases = _with_oracle_texts(_golden_cases(golden), oracle)
    _check(_run(harness, cases, mode, tmp_path), cases, texts=(mode == "direct"))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["direct", "batch", "batchref"])
def test_go_call_sequence_synthetic(harness, oracle, mode, tmp_path):
    cases = _synthetic_cases(oracle) + _empty_repair_cases(oracle)[0]
    _check(_run(harness, cases, mode, tmp_path), cases, texts=(mode == "direct"))


def test_synthetic_cases_are_well_formed(oracle):
    """The seeded blocks cover repairs, every loss count up to m, and the too-many-losses error."""
    cases = _synthetic_cases(oracle)
    assert len(cases) == 48
    errs = [c for c in cases if c[4][0] == "err"]
    assert len(errs) == 4 and all(e[4][1] == "not enough present symbols to repair the missing ones" for e in errs)
    assert sum(1 for c in cases if c[4][0] == "bytes" and c[4][1]) == 20
