import os, torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
t = torch.full((4,), rank, dtype=torch.uint8, device=dev)
bufs = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
dist.gather(t, bufs, dst=0)
torch.cuda.synchronize()
if rank == 0:
    print("gather ok", [b.tolist() for b in bufs], flush=True)
dist.destroy_process_group()
