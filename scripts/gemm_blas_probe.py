"""bf16 projection GEMMs (F.linear) of the AWQ / GPTQ calibration forwards: hipBLASLt vs rocBLAS."""
import torch
import torch.nn.functional as F

dev = 'cuda'
shapes = [(65536, 4096, 4096), (65536, 1024, 4096), (65536, 14336, 4096), (65536, 4096, 14336),
          (262144, 4096, 4096), (262144, 14336, 4096)]
for (M, N, K) in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    res = []
    for lib in ('cublaslt', 'cublas'):
        torch.backends.cuda.preferred_blas_library(lib)
        for _ in range(3):
            F.linear(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            F.linear(x, w)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res.append(f'{lib} {ms:.3f} ms {2 * M * N * K / ms / 1e9:.0f} TF/s')
    print((M, N, K), ' | '.join(res), flush=True)
    del x, w
