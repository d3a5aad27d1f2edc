"""In-tree build of the native extensions.

* ``_dnn_hip``: the gfx950 HIP kernels + pybind11 launchers (hipcc, --offload-arch=gfx950).
* ``_dnn_io``: the C++ data runtime (CIFAR-10 binary reader, synthetic generator,
  seeded epoch permutations / shard partitioning) built with g++.

Both land next to this file so a ``gpurun`` snapshot of the repo carries them to the
GPU box.  No hipify, no torch.utils.cpp_extension: device pointers cross the python
boundary as integers, so nothing here depends on libtorch's C++ ABI.

Run ``python -m distributed_neural_network_amd.ops.build [--force]``.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
CSRC = REPO / "csrc"
ARCH = os.environ.get("DNN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

HIP_SOURCES = [
    CSRC / "kernels" / "lenet_fused.hip",
    CSRC / "kernels" / "lenet_f32.hip",
    CSRC / "kernels" / "reduce_sgd.hip",
    CSRC / "kernels" / "layers.hip",
    CSRC / "kernels" / "conv_igemm.hip",
    CSRC / "kernels" / "linear.hip",
    CSRC / "comm" / "xgmi_allreduce.hip",
    CSRC / "kernels" / "diag.hip",
]
HIP_BINDING = CSRC / "bindings.cpp"
HOST_SOURCES = [CSRC / "comm" / "rccl_comm.cpp", CSRC / "runtime" / "aql_dispatch.cpp"]
HIP_HEADERS = sorted((CSRC / "kernels").glob("*.h")) + sorted((CSRC / "runtime").glob("*.h"))
IO_SOURCES = [CSRC / "io" / "dataio.cpp"]
LINK_LIBS = ["-ldl", "-L/opt/rocm/lib", "-lhsa-runtime64"]  # (RCCL is dlopen'ed; HSA: runtime/aql_dispatch)


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def hip_target() -> Path:
    return HERE / f"_dnn_hip{EXT_SUFFIX}"


def io_target() -> Path:
    return HERE / f"_dnn_io{EXT_SUFFIX}"


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_hip(force: bool = False, verbose_resources: bool = False) -> Path:
    target = hip_target()
    deps = HIP_SOURCES + [HIP_BINDING] + HIP_HEADERS + HOST_SOURCES
    if not force and not _stale(target, deps):
        return target
    objdir = REPO / "build" / "hip"
    objdir.mkdir(parents=True, exist_ok=True)
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{CSRC}"]
    jobs, objs = [], []
    for src in HIP_SOURCES:
        obj = objdir / (src.stem + ".o")
        extra = ["-Rpass-analysis=kernel-resource-usage"] if verbose_resources else []
        jobs.append(common + extra + ["-c", str(src), "-o", str(obj)])
        objs.append(str(obj))
    for src in HOST_SOURCES:  # host-only C++ (RCCL via dlopen), compiled as HIP for the headers
        obj = objdir / (src.stem + ".o")
        jobs.append(common + ["-x", "hip", "-c", str(src), "-o", str(obj)])
        objs.append(str(obj))
    bobj = objdir / "bindings.o"
    jobs.append(common + _pybind_includes() + ["-x", "hip", "-c", str(HIP_BINDING), "-o", str(bobj)])
    objs.append(str(bobj))
    # translation units compile in parallel (bounded by MAX_JOBS / the CPU count)
    from concurrent.futures import ThreadPoolExecutor

    width = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 16))
    with ThreadPoolExecutor(width) as ex:
        for f in [ex.submit(_run, j) for j in jobs]:
            f.result()
    tmp = target.with_suffix(".tmp.so")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + objs + LINK_LIBS)
    os.replace(tmp, target)
    return target


def build_io(force: bool = False) -> Path:
    target = io_target()
    if not force and not _stale(target, IO_SOURCES):
        return target
    tmp = target.with_suffix(".tmp.so")
    _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden"] + _pybind_includes()
         + [str(s) for s in IO_SOURCES] + ["-o", str(tmp)])
    os.replace(tmp, target)
    return target


def build_all(force: bool = False) -> None:
    build_io(force)
    build_hip(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
