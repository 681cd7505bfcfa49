import importlib, json, os, sys
sys.path.insert(0, os.getcwd())
mode = sys.argv[1]
if mode != "notorch":
    import torch
    torch.cuda.init()
    x = torch.zeros(1, device="cuda")
fec = importlib.import_module("0xfec_amd")
c = fec.Codec(0)
for mib in (512, 1024):
    print(mode, json.dumps(c.probe_link(mib << 20)), flush=True)
if mode == "torchwork":
    c.prepare(8, 4)
    import bench
    r = bench.host_resident(torch, fec, c, 8, 4, 1 << 15, 1)
    print(mode, "after host_resident", json.dumps(c.probe_link(512 << 20)), flush=True)
