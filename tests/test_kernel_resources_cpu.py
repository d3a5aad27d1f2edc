"""Build-time guard on the gfx950 kernels' register allocation (runs on the CPU: hipcc
cross-compiles).  Every kernel must keep its working set in registers: no private
(scratch) memory.  Round 1 shipped the layer engine's LDS-patch convolution with 112 B of
scratch per lane - arrays of HIP's ``uint4`` / ``float4`` structs were spilled to memory -
and removing it cut the cifar-vgg bf16 step from 354 to ~317 us (profiles/r2/conv_scratch/)."""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["kernels/lenet_fused.hip", "kernels/lenet_f32.hip", "kernels/reduce_sgd.hip", "kernels/layers.hip", "kernels/conv_igemm.hip",
           "kernels/linear.hip", "comm/xgmi_allreduce.hip"]


def _resources(src, tmp):
    out = os.path.join(tmp, os.path.basename(src) + ".o")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "csrc"),
                        "--cuda-device-only", "-c", os.path.join(ROOT, "csrc", src), "-o", out,
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    kernels, name = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            kernels[name] = int(m.group(1))
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC), reason="hipcc not available")
def test_no_kernel_uses_scratch(tmp_path):
    with ThreadPoolExecutor(2) as ex:
        res = list(ex.map(lambda s: _resources(s, str(tmp_path)), SOURCES))
    found = {k: v for r in res for k, v in r.items()}
    assert len(found) > 40, f"resource remarks not parsed: {len(found)} kernels"
    spills = {k: v for k, v in found.items() if v}
    assert not spills, f"kernels using scratch memory: {spills}"
