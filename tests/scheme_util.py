"""Shared helpers: build host-mirror Blocks from the reference's golden table cases."""
import importlib


def scheme_mod():
    importlib.import_module("0xfec_amd")
    return importlib.import_module("0xfec_amd.scheme")


def block_from_case(blk):
    S = scheme_mod()
    return S.Block.literal(
        id=blk["id"], tot_src=blk["totNumSourceSymbols"], tot_rep=blk["totNumRepairSymbols"],
        biggest=blk["biggestSourceSymbolLenSoFar"], smallest=blk["smallestSSID"], largest=blk["largestSSID"],
        sources={int(k): (bytes.fromhex(v["hex"]), v["cap"]) for k, v in blk["ssidToSourcePayload"].items()},
        repairs={int(k): bytes.fromhex(v["hex"]) for k, v in blk["pidToRepairPayload"].items()})


def want_frames(want):
    return [(f["BlockID"], f["ParityID"], bytes.fromhex(f["Payload"]["hex"])) for f in want["frames"]]


def needs_device(case):
    """Cases the reference expects to succeed with output reach the codec (GPU)."""
    return (not case["wantErr"]) and case["want"] is not None
