import os, sys, time
os.environ["GPU_MAX_HW_QUEUES"] = "1"
sys.path.insert(0, os.getcwd())
import torch, torch.distributed as dist
from akka_allreduce_1_amd._native import C
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
lag = int(sys.argv[1])
slot_mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
f = open(f"gpurun_out/probe_{os.environ.get('PROBE_TAG', 'x')}_r{rank}.log", "w")
def log(m):
    f.write(f"{time.time():.2f} {m}\n"); f.flush()
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=rank, world_size=world)
log("init")
c = C.hip.XgmiComm(rank, world, 0, slot_mib << 20, 64, 20.0, lag + 1 if lag >= 0 else 0)
log(f"alloc slab {c.slab_bytes >> 20} MiB")
h = c.ipc_handle()
log("handle")
hs = [None] * world
dist.all_gather_object(hs, h)
log("gathered")
c.connect(hs)
log("connected")
dist.barrier()
log("done")
