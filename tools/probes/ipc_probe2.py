import sys, torch
sys.path.insert(0, ".")
from distributedtensorflowexample_amd.ops import hip
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
for n in (79510, 1 << 20):
    try:
        x = hip().XgmiAllReduce(0, 1, 0, n)
        h = x.handle()
        print("ok", n, len(h))
    except Exception as e:
        print("fail", n, e)
