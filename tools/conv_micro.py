"""Micro-benchmark of the implicit-GEMM conv kernels on one layer shape (rocprofv3 target).

usage: python tools/conv_micro.py {fwd|dgrad|wgrad} B C H M K pad [bf16] [iters]
  fwd   : y = conv(x, w) + b            (LDS-patch kernel + its weight pack)
  dgrad : dx = conv(dy, flip(w))        (same kernel, flip = 1)
  wgrad : dW, db                        (split-K kernel + fixed-order slice sum)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.ops import native  # noqa: E402

mode = sys.argv[1]
B, C, H, M, K, pad = (int(v) for v in sys.argv[2:8])
bf = int(sys.argv[8]) if len(sys.argv) > 8 else 1
iters = int(sys.argv[9]) if len(sys.argv) > 9 else 50
ext = native.hip()
dev = torch.device("cuda", 0)
OH = H + 2 * pad - K + 1
x = torch.randn(B, C, H, H, device=dev)
w = torch.randn(M, C, K, K, device=dev)
b = torch.randn(M, device=dev)
dy = torch.randn(B, M, OH, OH, device=dev)
s = torch.cuda.current_stream().cuda_stream
if mode == "wgrad":
    dw, db = torch.empty_like(w), torch.empty_like(b)
    part = torch.empty(ext.conv_wgrad_slices(B, C, H, H, M, K, pad) * M * (C * K * K + 1), device=dev)

    def run():
        ext.conv_wgrad(x.data_ptr(), dy.data_ptr(), part.data_ptr(), dw.data_ptr(), db.data_ptr(), B, C, H, H, M, K,
                       pad, bf, s)
elif mode == "fwd":
    y = torch.empty(B, M, OH, OH, device=dev)
    ws = torch.empty(max(16, ext.conv_fwd_workspace(B, C, H, H, M, K, pad, bf, 0)), device=dev, dtype=torch.uint8)

    def run():
        ext.conv_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), ws.data_ptr(), B, C, H, H, M, K, pad, bf,
                     0, s)
else:  # dgrad
    dx = torch.empty_like(x)
    ws = torch.empty(max(16, ext.conv_fwd_workspace(B, M, OH, OH, C, K, K - 1 - pad, bf, 1)), device=dev,
                     dtype=torch.uint8)

    def run():
        ext.conv_fwd(dy.data_ptr(), w.data_ptr(), 0, dx.data_ptr(), ws.data_ptr(), B, M, OH, OH, C, K, K - 1 - pad,
                     bf, 1, s)
for _ in range(iters):
    run()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(iters):
    run()
ev1.record()
torch.cuda.synchronize()
print(f"{mode} B{B} C{C} H{H} M{M} K{K} pad{pad} bf{bf}: {ev0.elapsed_time(ev1) * 1000 / iters:.2f} us/iter")
