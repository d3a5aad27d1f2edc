"""Host-code sanitizer run: the native data runtime (csrc/io/dataio.cpp - the
CIFAR-10 binary reader, the synthetic generator, the seeded Fisher-Yates permutations) built with
AddressSanitizer + UndefinedBehaviorSanitizer and driven from a Python subprocess (libasan
preloaded, leak checking off: the interpreter itself is not instrumented).  Any out-of-bounds
access, use-after-free or undefined operation aborts the child with a sanitizer report.

GPU code is not sanitized here: GPU AddressSanitizer / XNACK runs are not available on the
target pool (the kernels' own checks are the CPU resource test and the GPU numerics tests)."""
import os
import subprocess
import sys
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_lib(name):
    r = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


DRIVER = r'''
import os, sys, struct, numpy as np
sys.path.insert(0, sys.argv[1])
import _dnn_io as io
tmp = sys.argv[2]
# CIFAR binary batches: 2 files, then the error paths (missing, bad size, bad label)
rng = np.random.default_rng(0)
paths = []
for f in range(2):
    n = 7 + f
    lab = rng.integers(0, 10, n, dtype=np.uint8)
    img = rng.integers(0, 256, (n, 3072), dtype=np.uint8)
    rec = np.concatenate([lab[:, None], img], 1)
    p = os.path.join(tmp, f"b{f}.bin"); rec.tofile(p); paths.append(p)
im, lb = io.read_cifar_bin(paths)
assert im.shape == (15, 3, 32, 32) and lb.shape == (15,) and lb.max() <= 9
bad = os.path.join(tmp, "bad.bin"); open(bad, "wb").write(b"\x01" * 3074)
badlab = os.path.join(tmp, "badlab.bin"); open(badlab, "wb").write(b"\x0b" + b"\x00" * 3072)
for ps in ([os.path.join(tmp, "missing.bin")], [bad], [badlab], paths + [bad]):
    try:
        io.read_cifar_bin(ps)
        raise SystemExit("expected an error for %s" % ps)
    except RuntimeError:
        pass
# synthetic data: every size class incl. 0, every noise level extreme
for n, noise in ((0, 96), (1, 0), (33, 255), (257, 96)):
    a, b = io.synthetic(n, 5, noise, 1)
    assert a.shape == (n, 3, 32, 32) and b.shape == (n,)
# permutations: 0, 1 and odd sizes, large seeds / epochs / streams
for n in (0, 1, 2, 1001):
    idx = np.arange(n, dtype=np.int32)
    s = io.shuffled(idx, 2**63 + 5, 2**40, 2**31 - 1)
    assert sorted(s.tolist()) == list(range(n))
print("SANITIZED_OK")
'''


@pytest.mark.timeout(600)
def test_data_runtime_under_asan_ubsan(tmp_path):
    asan = _gcc_lib("libasan.so")
    if asan is None:
        pytest.skip("no libasan for g++")
    import pybind11

    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    so = tmp_path / f"_dnn_io{ext}"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"] + inc + [
        os.path.join(ROOT, "csrc", "io", "dataio.cpp"), "-o", str(so)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    # libstdc++ preloaded right after libasan: the interpreter does not link it, and ASan's
    # __cxa_throw interceptor must find the real one when the reader throws on a bad file
    stdcxx = _gcc_lib("libstdc++.so") or "libstdc++.so.6"
    env = dict(os.environ, LD_PRELOAD=f"{asan} {stdcxx}", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", DRIVER, str(tmp_path), str(tmp_path)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "SANITIZED_OK" in r.stdout, (r.stdout + r.stderr)[-4000:]
