import os, torch, torch.distributed as dist
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29677", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.ones(4, device="cuda"); dist.all_reduce(t); torch.cuda.synchronize(); print("ok", t.sum().item())
dist.destroy_process_group()
