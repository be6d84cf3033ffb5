"""Micro-benchmark: per-kernel boundary cost on this GPU, eager vs HIP graph, for a
trivial kernel (step_begin, 1 thread) -- tells how much of a step is launch floor."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from cori_intml_examples_amd.ops.hip import kernels

K = kernels()
dev = torch.device("cuda", 0)
st = torch.zeros(K.STEP_STATE_BYTES, dtype=torch.uint8, device=dev)
a = K.StepBeginArgs()
a.st = st.data_ptr()
a.training = 0
a.bs = 1
N = 200


def launch_n():
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(N):
        K.step_begin(a, s)


launch_n()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    launch_n()
torch.cuda.synchronize()
eager = (time.perf_counter() - t) / (10 * N) * 1e6

g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=s):
    launch_n()
torch.cuda.current_stream().wait_stream(s)
g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t) / (10 * N) * 1e6

x = torch.zeros(1, device=dev)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(2000):
    x.add_(1)
torch.cuda.synchronize()
torch_eager = (time.perf_counter() - t) / 2000 * 1e6
print("per-kernel: eager %.2f us, graph %.2f us, torch tiny op eager %.2f us" % (eager, graph, torch_eager))
