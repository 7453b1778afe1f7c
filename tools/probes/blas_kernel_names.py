"""Which library kernels torch.matmul (hipBLASLt) runs for the MLP's GEMM shapes: run under
``rocprofv3 --kernel-trace`` and read the kernel names (Tensile names encode macro tile, MFMA shape, waves, depth-U,
direct-to-LDS, prefetch settings) — design input for the hand-written kernels, nothing of it is linked."""
import torch

shapes = [("fwd1", 8192, 4096, 4096, False, False), ("bwdd1", 8192, 4096, 4096, False, True),
          ("bwdw1", 4096, 4096, 8192, True, False), ("sq8k_nt", 8192, 8192, 8192, False, True)]
for name, M, N, K, a_t, b_t in shapes:
    A = torch.randn(K, M, device="cuda", dtype=torch.bfloat16).t() if a_t else torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t() if b_t else torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(A, B)
    torch.cuda.synchronize()
    print(name, flush=True)
