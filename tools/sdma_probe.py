import os, time, json, torch
dev = torch.device("cuda", 0)
n = 256 << 20
a = torch.empty(n, dtype=torch.uint8, device=dev); b = torch.empty_like(a)
for _ in range(3): b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): b.copy_(a)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(json.dumps({"blit_env": os.environ.get("GPU_BLIT_ENGINE_TYPE"), "ms": round(ms, 4), "GBps": round(n / ms / 1e6, 1)}))
