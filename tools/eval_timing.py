import time, torch, numpy as np, sys
sys.path.insert(0, '/root/repo')
from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.runtime import HipEngine, eval_metrics
test = synthetic(10000, 0, False).to('cuda')
e = HipEngine(batch=64, seed=0)
for i in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    loss, corr = e.evaluate_samples(test, 0, 10000)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    m = eval_metrics(loss, corr, 64)
    t2 = time.perf_counter()
    print(f"eval kernel+launch {1e3*(t1-t0):.3f} ms, metrics {1e3*(t2-t1):.3f} ms", m)
