#!/usr/bin/env python3
"""Build a kernel A/B variant of the HIP extension: the listed sources recompiled with extra
-D flags, linked with the main build's other objects into
distributed_neural_network_amd/ops/variants/NAME.so (``tools/gpu_run.sh useso:NAME`` swaps it in
for the next steps of one GPU call and restores the main build afterwards).

    python tools/build_variant.py NAME -DDNN_SOME_SWITCH=0 [--src lenet_fused.hip ...]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from distributed_neural_network_amd.ops import build as B  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("defines", nargs=argparse.REMAINDER, help="-DNAME=VALUE flags")
    ap.add_argument("--src", nargs="*", default=["lenet_fused.hip"])
    a = ap.parse_args()
    B.build_hip()  # the main build's objects are the base
    objdir = REPO / "build" / "hip"
    vdir = REPO / "build" / "variant" / a.name
    vdir.mkdir(parents=True, exist_ok=True)
    common = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{B.CSRC}"]
    objs = []
    names = set(a.src)
    for src in B.HIP_SOURCES:
        if src.name in names:
            obj = vdir / (src.stem + ".o")
            subprocess.run(common + list(a.defines) + ["-c", str(src), "-o", str(obj)], check=True)
            objs.append(str(obj))
        else:
            objs.append(str(objdir / (src.stem + ".o")))
    for src in B.HOST_SOURCES:
        objs.append(str(objdir / (src.stem + ".o")))
    objs.append(str(objdir / "bindings.o"))
    out = REPO / "distributed_neural_network_amd" / "ops" / "variants" / f"{a.name}.so"
    out.parent.mkdir(exist_ok=True)
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out)] + objs + B.LINK_LIBS,
                   check=True)
    print(out)


if __name__ == "__main__":
    main()
