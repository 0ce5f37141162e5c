"""GPU box: cost of the data-parallel step's structure on ONE GPU (nccl group of size 1): the
multi-rank code path (fwd/bwd → RCCL all-reduce → Adam) forced at world 1, eager and hipGraph
replay, against the fused single-GPU step.  Timing only (the forced path scales the gradient as
for 2 ranks)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from cvae_amd import ConditionalTrajectoryVAE  # noqa: E402
from cvae_amd.dist import DataParallelStep  # noqa: E402

torch.manual_seed(0)
m = ConditionalTrajectoryVAE(100, 6, 8)
eng = m.attach(dtype="bf16", max_batch=1024)
x = eng.as_input(torch.randn(1024, 100, 6))
dp = DataParallelStep(eng)
dp.world_size = 2  # force the collective path (timing only)


def timed(fn, k=400):
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6, th / k * 1e6


w, h = timed(lambda: eng.train_step(x))
print(f"fused single-GPU step: wall {w:.1f} us/step, host enqueue {h:.1f} us/step")
w, h = timed(lambda: dp.step(x, batch=1024, global_batch=2048))
print(f"DP path (fwd/bwd, all_reduce, adam) eager: wall {w:.1f} us/step, host enqueue {h:.1f} us/step")
w, h = timed(lambda: (eng.forward_backward(x, batch=1024), eng.adam_step(grad_scale=0.5)))
print(f"DP path without the collective: wall {w:.1f} us/step, host enqueue {h:.1f} us/step")
w, h = timed(lambda: dist.all_reduce(eng.grads))
print(f"all_reduce alone (1 rank): wall {w:.1f} us, host {h:.1f} us")
# the DP step captured once into a hipGraph (kernels + the RCCL all-reduce), replayed per step
try:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            dp.step(x, batch=1024, global_batch=2048)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dp.step(x, batch=1024, global_batch=2048)
    w, h = timed(g.replay)
    print(f"DP path as one hipGraph replay: wall {w:.1f} us/step, host enqueue {h:.1f} us/step")
except Exception as e:  # noqa: BLE001
    print(f"graph capture of the DP step failed: {type(e).__name__}: {e}")
dist.destroy_process_group()
