import importlib, json, os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import torch
import config_bench as cb
fec = importlib.import_module("0xfec_amd")
codec = fec.Codec(0).use_torch_stream()
orig = cb.timed
def med(torch_, fn, iters):
    r = [orig(torch_, fn, iters) for _ in range(5)]
    return sorted(r)[2]
print("orig", json.dumps(cb.run_rs(torch, fec, codec, 2, 1, 65536, 0, 100, 0x0FEC)))
cb.timed = med
print("median-of-5", json.dumps(cb.run_rs(torch, fec, codec, 2, 1, 65536, 0, 100, 0x0FEC)))
print("median-of-5 x50", json.dumps(cb.run_rs(torch, fec, codec, 2, 1, 65536, 0, 50, 0x0FEC)))
