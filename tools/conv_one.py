"""Run one residual-conv backward shape repeatedly (GPU dev tool, for rocprofv3 --pmc passes).

    python tools/conv_one.py {fused|dgrad|wgrad|fwd} [T] [dilation] [reps]
B = 32, C = 32, K = 3, bf16, conv input x with ReLU, residual on the data gradient (conv_a of a block).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402


def main():
    op = sys.argv[1]
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    B, C, K = 32, 32, 3
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    res = torch.randn(B, T, C, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(K, C, C, device=dev, generator=g) * 0.1
    b = torch.zeros(C, device=dev)
    dx = torch.empty_like(x)
    dw = torch.empty(K, C, C, device=dev)
    db = torch.empty(C, device=dev)
    pad = d
    for _ in range(reps):
        if op == "fused":
            V.conv1d_bwd_data_weight(dy, w, x, res, dx, dw, db, B, T, T, C, C, K, 1, d, pad,
                                     V.PRE_RELU | V.ADD_RESIDUAL, V.BF16, V.Deferred())
        elif op == "dgrad":
            V.conv1d_bwd_data(dy, w, x, res, dx, B, T, T, C, C, K, 1, d, pad, V.POST_MASK | V.ADD_RESIDUAL, V.BF16)
        elif op == "wgrad":
            V.conv1d_bwd_weight_deferred(x, dy, dw, db, B, T, T, C, C, K, 1, d, pad, V.PRE_RELU, V.BF16,
                                         V.Deferred())
        else:
            V.conv1d_fwd(x, w, b, res, dx, B, T, T, C, C, K, 1, d, pad, V.PRE_RELU | V.ADD_RESIDUAL, V.BF16)
    torch.cuda.synchronize()
    print("ok", op, T, d)


if __name__ == "__main__":
    main()
