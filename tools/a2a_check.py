import os, torch, torch.distributed as dist
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
for mb in (900, 1100, 1500):
    n = mb * (1 << 20) // 8
    a = torch.arange(n, dtype=torch.int64, device="cuda")
    b = torch.zeros_like(a)
    dist.all_to_all_single(b, a, output_split_sizes=[n], input_split_sizes=[n])
    torch.cuda.synchronize()
    bad = (a != b).nonzero()
    print(mb, "MiB: mismatches", bad.numel(), "first bad index", int(bad[0]) if bad.numel() else None, flush=True)
dist.destroy_process_group()
