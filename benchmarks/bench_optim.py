"""FusedAdamW step time over the headline module's parameters (bf16, 2.4M) vs torch fused AdamW.

    python benchmarks/bench_optim.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import xdot

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = xdot.DistributedDotProductAttn(768, num_heads=8).to(dev, torch.bfloat16)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    for name, opt in (("xdot", xdot.FusedAdamW(m.parameters(), lr=1e-4)),
                      ("torch_fused", torch.optim.AdamW(m.parameters(), lr=1e-4, fused=True))):
        for _ in range(10):
            opt.step()
        ts = []
        for _ in range(100):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            opt.step()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"optimizer": name, "ext": os.environ.get("XDOT_EXT_PATH", "xdot/_C.so"),
                          "us_median": round(statistics.median(ts), 1), "us_min": round(min(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
