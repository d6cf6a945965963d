"""Usage example (reference: ``example.py:1-33``): 2-head attention, d=768, T=4096, offset=64,
MSE loss, one forward + backward on this rank's T/N rows.

    python example.py                                               # 1 GPU (or CPU)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 example.py
"""
import torch
import torch.nn as nn

import xdot
from xdot.parallel import GradSync

comm = xdot.init()  # torchrun env -> RCCL (GPU) / gloo (CPU); single rank otherwise
torch.manual_seed(111)
device = torch.device("cpu")
dtype = torch.float32
if torch.cuda.is_available():
    device = torch.device("cuda", torch.cuda.current_device())
    dtype = torch.bfloat16

module = xdot.DistributedDotProductAttn(768, num_heads=2, offset=64).to(device, dtype)
sync = GradSync(module)  # Sum-allreduce of the replicated parameters' partial gradients
criterion = nn.MSELoss()

length = 4096
world_size = xdot.get_world_size()
x = torch.rand(1, length // world_size, 768, device=device, dtype=dtype)
y = torch.rand(1, length // world_size, 768, device=device, dtype=dtype)
mask = torch.zeros(1, length // world_size, length, device=device).bool()

out = module(x, x, x, mask)
loss = criterion(out, y)
loss.backward()
sync.wait()
if xdot.is_main_process():
    print(f"rank 0/{world_size}: out {tuple(out.shape)} loss {loss.item():.5f} impl={module._pick_impl(x)}")
