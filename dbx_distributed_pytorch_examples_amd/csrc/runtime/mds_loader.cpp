// Native MDS batch assembler (host side of the input pipeline).
//
// The reference feeds the GPU from a Python DataLoader with num_workers=0 and per-sample PIL
// transforms in the training process (SURVEY.md §3 "where time goes", item 2). Here a C++
// reader memory-maps the MDS shards once and, for a batch of global sample ids, copies the raw
// `pil`-encoded pixels (or `ndarray:uint8` payloads) and int64 labels straight into a pinned
// uint8 NHWC staging buffer with a thread pool — no decode, no Python per sample, GIL released.
// The Python side (data/loader.py) then issues one async H2D copy on a side stream and the GPU
// kernel `augment_u8` does crop/resize/flip/normalise.
//
// Shard format (data/mds.py): uint32 n, uint32 offsets[n+1] (absolute), samples = uint32 sizes of
// the variable-size columns, then every column's bytes in column order.
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct Shard {
  std::string path;
  const uint8_t* base = nullptr;
  size_t bytes = 0;
  uint32_t n = 0;
  const uint32_t* offs = nullptr;
};

class MDSReader {
 public:
  MDSReader(const std::vector<std::string>& paths, const std::vector<int64_t>& counts,
            const std::vector<std::string>& names, const std::vector<std::string>& encs,
            const std::vector<int64_t>& sizes)
      : names_(names), encs_(encs), sizes_(sizes) {
    if (paths.size() != counts.size()) throw std::invalid_argument("paths/counts length mismatch");
    if (names.size() != encs.size() || names.size() != sizes.size())
      throw std::invalid_argument("column metadata length mismatch");
    cum_.push_back(0);
    for (size_t i = 0; i < paths.size(); ++i) {
      Shard s;
      s.path = paths[i];
      int fd = ::open(paths[i].c_str(), O_RDONLY);
      if (fd < 0) throw std::runtime_error("cannot open shard " + paths[i]);
      struct stat st;
      fstat(fd, &st);
      s.bytes = (size_t)st.st_size;
      void* p = mmap(nullptr, s.bytes, PROT_READ, MAP_SHARED, fd, 0);
      ::close(fd);
      if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + paths[i]);
      s.base = static_cast<const uint8_t*>(p);
      std::memcpy(&s.n, s.base, 4);
      if ((int64_t)s.n != counts[i]) throw std::runtime_error("sample count mismatch in " + paths[i]);
      if (s.bytes < 4 + 4 * ((size_t)s.n + 1)) throw std::runtime_error("truncated shard " + paths[i]);
      s.offs = reinterpret_cast<const uint32_t*>(s.base + 4);
      if (s.offs[s.n] > s.bytes) throw std::runtime_error("offsets past end of " + paths[i]);
      shards_.push_back(s);
      cum_.push_back(cum_.back() + s.n);
    }
    nvar_ = 0;
    for (auto z : sizes_) nvar_ += (z < 0);
  }
  ~MDSReader() {
    for (auto& s : shards_)
      if (s.base) munmap(const_cast<uint8_t*>(s.base), s.bytes);
  }

  int64_t num_samples() const { return cum_.back(); }

  int col(const std::string& name) const {
    for (size_t i = 0; i < names_.size(); ++i)
      if (names_[i] == name) return (int)i;
    throw std::invalid_argument("no MDS column " + name);
  }

  // pointer + size of column c of global sample g
  std::pair<const uint8_t*, size_t> field(int64_t g, int c) const {
    if (g < 0 || g >= cum_.back()) throw std::out_of_range("sample index out of range");
    const size_t si = std::upper_bound(cum_.begin(), cum_.end(), g) - cum_.begin() - 1;
    const Shard& s = shards_[si];
    const uint32_t i = (uint32_t)(g - cum_[si]);
    const uint8_t* rec = s.base + s.offs[i];
    const size_t rec_len = s.offs[i + 1] - s.offs[i];
    const uint32_t* vs = reinterpret_cast<const uint32_t*>(rec);
    size_t pos = 4 * (size_t)nvar_;
    int vi = 0;
    for (int k = 0; k < (int)sizes_.size(); ++k) {
      size_t sz = sizes_[k] < 0 ? vs[vi++] : (size_t)sizes_[k];
      if (k == c) {
        if (pos + sz > rec_len) throw std::runtime_error("corrupt MDS record in " + s.path);
        return {rec + pos, sz};
      }
      pos += sz;
    }
    throw std::invalid_argument("bad column");
  }

  // Gather images (raw `pil` RGB/L or ndarray uint8 of exactly H*W*C bytes) + int labels.
  void gather(py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx, uintptr_t out_ptr,
              uintptr_t label_ptr, int H, int W, int C, const std::string& image_col,
              const std::string& label_col, int nthreads) {
    const int ic = col(image_col), lc = col(label_col);
    const std::string& ienc = encs_[ic];
    const bool pil = ienc == "pil";
    if (!pil && ienc.rfind("ndarray:uint8", 0) != 0)
      throw std::invalid_argument("native gather needs `pil` or `ndarray:uint8` images, got " + ienc);
    const int64_t B = idx.shape(0);
    const int64_t* ids = idx.data();
    uint8_t* out = reinterpret_cast<uint8_t*>(out_ptr);
    int64_t* labels = reinterpret_cast<int64_t*>(label_ptr);
    const size_t img_bytes = (size_t)H * W * C;
    std::string err;
    std::mutex mu;
    {
      py::gil_scoped_release release;
      auto work = [&](int t, int nt) {
        for (int64_t b = t; b < B; b += nt) {
          try {
            auto f = field(ids[b], ic);
            const uint8_t* src = f.first;
            size_t n = f.second;
            if (pil) {
              uint32_t hdr[3];
              std::memcpy(hdr, src, 12);
              const std::string mode(reinterpret_cast<const char*>(src + 12), hdr[2]);
              const int mc = mode == "RGB" ? 3 : (mode == "L" ? 1 : -1);
              if ((int)hdr[0] != W || (int)hdr[1] != H || mc != C)
                throw std::runtime_error("image " + std::to_string(ids[b]) + " is " + mode + " " +
                                         std::to_string(hdr[0]) + "x" + std::to_string(hdr[1]) +
                                         ", loader expects fixed-size raw images");
              src += 12 + hdr[2];
              n -= 12 + hdr[2];
            }
            if (n != img_bytes) throw std::runtime_error("image payload size mismatch");
            std::memcpy(out + (size_t)b * img_bytes, src, img_bytes);
            if (labels) {
              auto l = field(ids[b], lc);
              int64_t v = 0;
              if (l.second == 8) std::memcpy(&v, l.first, 8);
              else if (l.second == 4) { int32_t v32; std::memcpy(&v32, l.first, 4); v = v32; }
              else throw std::runtime_error("unsupported label width");
              labels[b] = v;
            }
          } catch (const std::exception& e) {
            std::lock_guard<std::mutex> g(mu);
            if (err.empty()) err = e.what();
            return;
          }
        }
      };
      const int nt = std::max(1, std::min<int>(nthreads, (int)B));
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back(work, t, nt);
      work(0, nt);
      for (auto& x : th) x.join();
    }
    if (!err.empty()) throw std::runtime_error(err);
  }

  py::bytes raw_field(int64_t g, const std::string& column) const {
    auto f = field(g, col(column));
    return py::bytes(reinterpret_cast<const char*>(f.first), f.second);
  }

 private:
  std::vector<Shard> shards_;
  std::vector<int64_t> cum_;
  std::vector<std::string> names_, encs_;
  std::vector<int64_t> sizes_;
  int nvar_ = 0;
};

}  // namespace

void register_runtime(py::module& m) {
  py::class_<MDSReader>(m, "MDSReader")
      .def(py::init<const std::vector<std::string>&, const std::vector<int64_t>&, const std::vector<std::string>&,
                    const std::vector<std::string>&, const std::vector<int64_t>&>())
      .def("num_samples", &MDSReader::num_samples)
      .def("gather", &MDSReader::gather, py::arg("indices"), py::arg("out_ptr"), py::arg("label_ptr"), py::arg("H"),
           py::arg("W"), py::arg("C"), py::arg("image_col") = "image", py::arg("label_col") = "label",
           py::arg("nthreads") = 8)
      .def("raw_field", &MDSReader::raw_field);
}
