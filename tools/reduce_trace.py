#!/usr/bin/env python3
"""Per-block timeline of the grad_reduce kernel (diagnostic).

Runs fused step + grad_reduce eagerly with the reduce kernel's stamp buffer enabled and
prints, per block role, when blocks start and finish (us from the earliest block start,
medians over repeats).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import LAYOUT  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def main(reps: int = 40, batch: int = 64):
    tr = synthetic(4096, 0)
    e = HipEngine(batch=batch, seed=0, use_graphs=False)
    e.attach(tr)
    st = torch.zeros(2 * 256, dtype=torch.int64, device=e.device)
    rows = []
    for r in range(reps):
        e.begin_epoch(np.roll(np.arange(4096, dtype=np.int32), -64 * (r % 60)))
        s = e._stream()
        e.ext.fused_train(e._p(e.train.images), e._p(e.train.labels), e._p(e.batch_ids), e.order_len, e.batch,
                          e._p(e.state), e._p(e.master), e._p(e.shadow), e._p(e.a0), e._p(e.h1), e._p(e.h2),
                          e._p(e.z1), e._p(e.z2), e._p(e.z3), e._p(e.slab), e._p(e.loss), e._p(e.correct), s)
        e.ext.grad_reduce(e._p(e.a0), e._p(e.h1), e._p(e.h2), e._p(e.z1), e._p(e.z2), e._p(e.z3), e._p(e.slab),
                          e._p(e.loss), e._p(e.correct), e.batch, e._p(e.master), e._p(e.grad), e._p(e.mom),
                          e._p(e.shadow), e._p(e.state), e._p(e.stats), e.lr, e.momentum, 1.0, 1, 0, LAYOUT.total,
                          1, e._p(e.order), e.order_len, e._p(e.batch_ids), s, stamps=st.data_ptr())
        torch.cuda.synchronize()
        rows.append(st.cpu().numpy().reshape(-1, 2).copy())
    a = np.array(rows[5:])  # [reps, blocks, 2]
    nb = int((a[-1, :, 0] > 0).sum())
    a = a[:, :nb]
    t0 = a[:, :, 0].min(axis=1, keepdims=True)
    rel = np.median((a - t0[:, :, None]) * 0.01, axis=0)
    roles = [("fc1 tiles", 0, 50), ("fc2 tiles", 50, 62), ("fc3 tiles", 62, 64), ("fc bias", 64, 68),
             ("conv cols", 68, 113), ("bookkeeping", 113, 114)]  # RT = 256: 960 / 11,488 split slots
    for name, lo, hi in roles:
        if hi <= nb:
            r = rel[lo:hi]
            print(f"{name:12s} start {r[:, 0].min():5.2f}-{r[:, 0].max():5.2f}  end min/med/max "
                  f"{r[:, 1].min():5.2f}/{np.median(r[:, 1]):5.2f}/{r[:, 1].max():5.2f} us")
    print(f"blocks {nb}, last end {rel[:, 1].max():.2f} us")


if __name__ == "__main__":
    main()
