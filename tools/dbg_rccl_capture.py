"""World-1 RCCL all-reduce captured in a hipGraph on a side stream (the graphed training step's
bucket reduction, grad_buckets.py), step by step with prints, to locate an abort.
mode 'del': graph deleted before destroy_process_group; 'keep': destroyed while the graph lives;
'nodestroy': never destroy (process exit tears down)."""
import os
import socket
import sys

import torch
import torch.distributed as dist

mode = sys.argv[1] if len(sys.argv) > 1 else "del"
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
print("init ok", flush=True)
x = torch.arange(8, device=dev, dtype=torch.float32)
dist.all_reduce(x)
torch.cuda.synchronize()
print("eager all_reduce ok", x.tolist(), flush=True)
side = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
y = torch.ones(1024, device=dev)
torch.cuda.synchronize()
with torch.cuda.graph(g, capture_error_mode=os.environ.get('CAPMODE', 'thread_local')):
    z = y * 2
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    side.wait_event(ev)
    with torch.cuda.stream(side):
        dist.all_reduce(z)
        z.div_(1)
    torch.cuda.current_stream().wait_stream(side)
    w = z + 1
print("capture ok", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", float(w[0]), flush=True)
y.fill_(3.0)
g.replay()
torch.cuda.synchronize()
print("replay 2 ok", float(w[0]), flush=True)
if mode == "del":
    del g
    torch.cuda.synchronize()
    print("graph deleted", flush=True)
if mode != "nodestroy":
    dist.destroy_process_group()
    print("destroy ok", flush=True)
print("done", flush=True)
