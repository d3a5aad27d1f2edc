// Native data runtime: CIFAR-10 binary reader, synthetic CIFAR-shaped generator, and
// seeded epoch permutations.
//
// Capability parity: replaces torchvision.datasets.CIFAR10 (download + PIL decode in
// DataLoader worker processes, data_parallelism_train.py:69-79,88-91) and the
// DataLoader's shuffle=True sampler.  Here the whole split is read ONCE into a
// contiguous uint8 [N][3][32][32] array (the CIFAR binary record order is already
// CHW) that the engine uploads to HBM; normalisation happens inside the fused
// kernel.  Permutations are Fisher-Yates over a splitmix64 stream keyed by
// (seed, epoch, stream id), so every rank / device / CPU oracle draws identical
// orders for identical keys.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kImg = 3 * 32 * 32;
constexpr int kRec = kImg + 1;

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  // unbiased integer in [0, n)
  uint64_t below(uint64_t n) {
    const uint64_t lim = UINT64_MAX - UINT64_MAX % n;
    uint64_t r;
    do { r = next(); } while (r >= lim);
    return r % n;
  }
};

uint64_t mix_key(uint64_t seed, uint64_t epoch, uint64_t stream) {
  SplitMix64 m(seed * 0x100000001B3ull ^ (epoch + 0x51ED270Bull) * 0x9E3779B97F4A7C15ull ^ (stream << 32));
  return m.next();
}

py::tuple read_cifar_bin(const std::vector<std::string>& paths) {
  std::vector<uint8_t> img;
  std::vector<int32_t> lab;
  for (const auto& p : paths) {
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open CIFAR-10 batch file: " + p);
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (sz <= 0 || sz % kRec != 0) {
      std::fclose(f);
      throw std::runtime_error("not a CIFAR-10 binary batch (size % 3073 != 0): " + p);
    }
    const size_t n = (size_t)sz / kRec;
    std::vector<uint8_t> buf((size_t)sz);
    const size_t got = std::fread(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    if (got != buf.size()) throw std::runtime_error("short read: " + p);
    const size_t base = lab.size();
    img.resize((base + n) * kImg);
    lab.resize(base + n);
    for (size_t i = 0; i < n; ++i) {
      const uint8_t* r = buf.data() + i * kRec;
      if (r[0] > 9) throw std::runtime_error("label out of range in " + p);
      lab[base + i] = r[0];
      std::memcpy(img.data() + (base + i) * kImg, r + 1, kImg);
    }
  }
  const py::ssize_t n = (py::ssize_t)lab.size();
  py::array_t<uint8_t> images({n, (py::ssize_t)3, (py::ssize_t)32, (py::ssize_t)32});
  py::array_t<int32_t> labels(n);
  std::memcpy(images.mutable_data(), img.data(), img.size());
  std::memcpy(labels.mutable_data(), lab.data(), lab.size() * sizeof(int32_t));
  return py::make_tuple(images, labels);
}

// Learnable CIFAR-shaped data: each class has a fixed colour/gradient template and
// every image is template + uniform noise, so the CNN's loss actually falls.
py::tuple synthetic(int64_t n, uint64_t seed, int noise, uint64_t split) {
  if (n < 0) throw std::runtime_error("n must be >= 0");
  py::array_t<uint8_t> images({(py::ssize_t)n, (py::ssize_t)3, (py::ssize_t)32, (py::ssize_t)32});
  py::array_t<int32_t> labels((py::ssize_t)n);
  uint8_t* im = images.mutable_data();
  int32_t* lb = labels.mutable_data();
  // class templates
  std::vector<float> tmpl(10 * kImg);
  SplitMix64 tr(mix_key(seed, 0xC1A55, 7));
  for (int k = 0; k < 10; ++k) {
    const float base[3] = {(float)(tr.below(96) + 80), (float)(tr.below(96) + 80), (float)(tr.below(96) + 80)};
    const float gy = ((float)tr.below(81) - 40.f) / 31.f, gx = ((float)tr.below(81) - 40.f) / 31.f;
    for (int c = 0; c < 3; ++c)
      for (int y = 0; y < 32; ++y)
        for (int x = 0; x < 32; ++x)
          tmpl[(size_t)k * kImg + (c * 32 + y) * 32 + x] = base[c] + gy * (y - 15.5f) * (c + 1) - gx * (x - 15.5f);
  }
  {
  py::gil_scoped_release nogil;
  SplitMix64 r(mix_key(seed, 0xDA7A + split, 11));  // per-split sample stream, shared templates
  const int span = 2 * noise + 1;
  for (int64_t i = 0; i < n; ++i) {
    const int k = (int)r.below(10);
    lb[i] = k;
    const float* t = tmpl.data() + (size_t)k * kImg;
    uint8_t* o = im + (size_t)i * kImg;
    for (int j = 0; j < kImg; j += 8) {
      uint64_t bits = r.next();
      for (int u = 0; u < 8; ++u) {
        const int d = (int)((bits >> (8 * u)) & 0xff) % span - noise;
        float v = t[j + u] + (float)d;
        v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
        o[j + u] = (uint8_t)(v + 0.5f);
      }
    }
  }
  }
  return py::make_tuple(images, labels);
}

// Fisher-Yates permutation of `indices` keyed by (seed, epoch, stream).
py::array_t<int32_t> shuffled(py::array_t<int32_t, py::array::c_style | py::array::forcecast> indices, uint64_t seed,
                              uint64_t epoch, uint64_t stream) {
  const py::ssize_t n = indices.size();
  py::array_t<int32_t> out(n);
  int32_t* o = out.mutable_data();
  std::memcpy(o, indices.data(), (size_t)n * sizeof(int32_t));
  SplitMix64 r(mix_key(seed, epoch, stream));
  for (py::ssize_t i = n - 1; i > 0; --i) {
    const py::ssize_t j = (py::ssize_t)r.below((uint64_t)i + 1);
    std::swap(o[i], o[j]);
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_dnn_io, m) {
  m.doc() = "native data runtime: CIFAR-10 binary reader, synthetic data, seeded permutations";
  m.def("read_cifar_bin", &read_cifar_bin, py::arg("paths"));
  m.def("synthetic", &synthetic, py::arg("n"), py::arg("seed"), py::arg("noise") = 96, py::arg("split") = 0);
  m.def("shuffled", &shuffled, py::arg("indices"), py::arg("seed"), py::arg("epoch"), py::arg("stream") = 0);
}
