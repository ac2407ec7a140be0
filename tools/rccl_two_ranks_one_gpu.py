"""Can two ranks form an RCCL (torch "nccl") group on ONE GPU?  Each rank
all-reduces, all-gathers and all-to-alls a small tensor on cuda:0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tools/rccl_two_ranks_one_gpu.py
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    g = [torch.empty(4, device="cuda") for _ in range(world)]
    dist.all_gather(g, torch.full((4,), float(rank), device="cuda"))
    a = torch.arange(world * 2, device="cuda", dtype=torch.float32) + 100 * rank
    b = torch.empty_like(a)
    dist.all_to_all_single(b, a)
    torch.cuda.synchronize()
    ok = bool(x[0].item() == world * (world + 1) / 2) and \
        [t[0].item() for t in g] == [float(r) for r in range(world)]
    print(json.dumps({"rank": rank, "all_reduce_ok": ok, "a2a": b.tolist()}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
