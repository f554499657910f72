"""hipBLASLt kernel choice on the encoder GEMM shapes (run under rocprofv3 --kernel-trace to read the names)."""
import torch
for M, N, K in [(36000, 3840, 1280), (36000, 1280, 1280), (36000, 5120, 1280), (36000, 1280, 5120)]:
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    for _ in range(3):
        torch.nn.functional.linear(A, W)
torch.cuda.synchronize()
