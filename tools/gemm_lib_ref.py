"""hipBLASLt (torch.matmul, bf16) on the encoder's GEMM shapes: the library's rate as a yardstick for gemm256_kernel.
Run on the GPU box: python tools/gemm_lib_ref.py"""
import torch

SHAPES = {"qkv": (12000, 3840, 1280), "out": (12000, 1280, 1280), "fc1": (12000, 5120, 1280),
          "fc2": (12000, 1280, 5120), "sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192)}


def main():
    torch.manual_seed(0)
    for name, (m, n, k) in SHAPES.items():
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, w.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            torch.matmul(a, w.t())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(f"{name:7s} M={m} N={n} K={k}: {ms * 1e3:8.1f} us  {2 * m * n * k / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
