"""Micro-benchmark of the implicit-GEMM conv kernels on one layer shape (rocprofv3 target).

usage: python tools/conv_micro.py B C H M K pad [bf16] [iters]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributed_neural_network_amd.ops import native  # noqa: E402

B, C, H, M, K, pad = (int(v) for v in sys.argv[1:7])
bf = int(sys.argv[7]) if len(sys.argv) > 7 else 1
iters = int(sys.argv[8]) if len(sys.argv) > 8 else 50
ext = native.hip()
dev = torch.device("cuda", 0)
OH = H + 2 * pad - K + 1
x = torch.randn(B, C, H, H, device=dev)
dy = torch.randn(B, M, OH, OH, device=dev)
dw = torch.empty(M, C, K, K, device=dev)
db = torch.empty(M, device=dev)
part = torch.empty(ext.conv_wgrad_slices(B, C, H, H, M, K, pad) * M * (C * K * K + 1), device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(iters):
    ext.conv_wgrad(x.data_ptr(), dy.data_ptr(), part.data_ptr(), dw.data_ptr(), db.data_ptr(), B, C, H, H, M, K, pad,
                   bf, s)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(iters):
    ext.conv_wgrad(x.data_ptr(), dy.data_ptr(), part.data_ptr(), dw.data_ptr(), db.data_ptr(), B, C, H, H, M, K, pad,
                   bf, s)
ev1.record()
torch.cuda.synchronize()
print(f"wgrad B{B} C{C} H{H} M{M} K{K} pad{pad} bf{bf}: {ev0.elapsed_time(ev1) * 1000 / iters:.2f} us/iter "
      f"(incl. slice sum)")
