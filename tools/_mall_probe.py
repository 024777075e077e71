"""Re-read bandwidth vs footprint: does the Infinity Cache (MALL) serve
repeated reads of a buffer that fits it?  float32 sum over the buffer."""
import json, torch
dev = torch.device("cuda", 0)
res = {}
for mb in (32, 64, 96, 128, 160, 192, 224, 256, 320, 512, 2048):
    n = mb * (1 << 20) // 4
    x = torch.ones(n, dtype=torch.float32, device=dev)
    reps = max(5, int(20000 / mb))
    for _ in range(3):
        x.sum()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        x.sum()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res[mb] = round(n * 4 / ms / 1e9, 1)   # GB/s (ms -> TB/s*1000)
    del x
print(json.dumps({"read_GBps_by_MB": res}))
