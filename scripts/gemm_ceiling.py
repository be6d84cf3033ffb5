"""Library-GEMM reference points for the legacy RPV conv layers (hipBLASLt through
torch.matmul, bf16 in / fp32 accumulate): the plain GEMM of each implicit-GEMM conv's
(M = pixels over the batch, N = Cout, K = 9 * Cin) shape, no im2col cost included -- an upper
bound for what the LDS-gathered implicit GEMM (conv_tile.hip) could reach on the same MFMA
pipes.  Prints us and TFLOP/s per shape; compare with the legacy kernel stats."""
import torch

dev = torch.device("cuda", 0)
B = 128
shapes = {  # name: (M, N, K)
    "conv_fwd1 64->128 s2 (32x32)": (B * 32 * 32, 128, 9 * 64),
    "conv_fwd2 128->256 (32x32)": (B * 32 * 32, 256, 9 * 128),
    "conv_fwd3 256->256 s2 (16x16)": (B * 16 * 16, 256, 9 * 256),
    "dgrad_conv2 256->128 (32x32)": (B * 32 * 32, 128, 9 * 256),
    "wgrad_conv2 (K=pixels)": (9 * 128, 256, B * 32 * 32),
}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print("%-32s M=%7d N=%4d K=%7d  %8.1f us  %7.1f TFLOP/s" % (name, M, N, K, us, 2.0 * M * N * K / us / 1e6))
