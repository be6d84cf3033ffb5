"""Hardware sanity: HBM copy bandwidth, bf16 GEMM rate (torch/hipBLASLt), kernel floor."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

dev = torch.device("cuda", 0)
x = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
y = torch.empty_like(x)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    y.copy_(x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 20
print("copy 256MiB: %.1f us  -> %.2f TB/s (r+w)" % (dt * 1e6, 2 * x.numel() / dt / 1e12))
a = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
b = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
for _ in range(3):
    c = a @ b
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    c = a @ b
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 10
print("bf16 8192^3 GEMM: %.2f ms -> %.0f TFLOP/s" % (dt * 1e3, 2 * 8192 ** 3 / dt / 1e12))
s = torch.zeros(1, device=dev)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5000):
    s.add_(1)
torch.cuda.synchronize()
print("torch tiny op eager: %.2f us/op" % ((time.perf_counter() - t) / 5000 * 1e6))
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=st):
    for _ in range(200):
        s.add_(1)
torch.cuda.current_stream().wait_stream(st)
g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print("torch tiny op in graph: %.2f us/op" % ((time.perf_counter() - t) / 4000 * 1e6))
