"""Run torch.matmul (hipBLASLt) on the BERT-base GEMM shapes a few times each, so a
rocprofv3 --kernel-trace of this script names the Tensile/hipBLASLt kernel (macro tile,
MFMA shape, prefetch / LDS settings) that the library picks per shape.

    rocprofv3 --kernel-trace --output-format csv -d out -o run -- python tools/probes/blaslt_names.py
"""
import torch

T = 128 * 128
SHAPES = [("qkv_fwd", T, 2304, 768, False), ("out_fwd", T, 768, 768, False),
          ("ffn1_fwd", T, 3072, 768, False), ("ffn2_fwd", T, 768, 3072, False),
          ("ffn1_dgrad", T, 768, 3072, False), ("ffn1_wgrad", 3072, 768, T, True),
          ("sq8192", 8192, 8192, 8192, False)]


def main():
    dev = torch.device("cuda:0")
    for name, M, N, K, ta in SHAPES:
        a = torch.randn(*((K, M) if ta else (M, K)), device=dev).to(torch.bfloat16)
        b = torch.randn(N, K, device=dev).to(torch.bfloat16) if not ta else \
            torch.randn(K, N, device=dev).to(torch.bfloat16)
        for _ in range(3):
            c = (a.t() @ b) if ta else (a @ b.t())
        torch.cuda.synchronize()
        print(name, tuple(c.shape), flush=True)


if __name__ == "__main__":
    main()
