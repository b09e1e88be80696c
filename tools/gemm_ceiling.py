"""Library ceiling for the prefill GEMM shapes (diagnostic, not product code): torch.matmul (hipBLASLt / rocBLAS)
on W [N][K] fp16 x H^T [K][2M] fp16 (the hi and lo columns of a chunk of M positions side by side, the same MFMA
work pgemm_kernel issues), fp16 out, fp32 accumulate. Prints us per GEMM and issued TFLOP/s (4 N K M), next to
tools/pgemm_lab's numbers for the hand-written kernel.   python tools/gemm_ceiling.py [M]
"""
import sys

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [("qkv", 12288, 4096), ("gu", 22016, 4096), ("wo", 4096, 4096), ("down", 4096, 11008)]
dev = torch.device("cuda:0")
for name, N, K in shapes:
    ws = [torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02 for _ in range(4)]  # 4 copies: no MALL re-reads
    h = torch.randn(K, 2 * M, device=dev, dtype=torch.float16)
    for w in ws:
        torch.matmul(w, h)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        for w in ws:
            torch.matmul(w, h)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / (it * len(ws))
    tf = 4.0 * N * K * M / (us * 1e-6) / 1e12
    print(f"{name:5s} N {N:6d} K {K:6d} M {M}: {us:8.1f} us  {tf:7.1f} TF issued  W {N * K * 2 / us / 1e3:7.0f} GB/s",
          flush=True)
