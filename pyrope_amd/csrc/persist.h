// persist.h -- the binary index image behind pyr_index_snapshot / pyr_index_load
// (IVectorIndex.Snapshot / Load, reference Vector/IVectorIndex.cs:26-27).
//
// The reference writes JSON DTOs (BruteForceVectorIndex.cs:58-107, IvfFlatVectorIndex.cs:233-298)
// and composes a Delta snapshot from .head/.tail files plus a manifest written through a temp
// file and a move (DeltaVectorIndex.cs:160-191).  The image keeps the same content -- live rows
// with their ids, the buffer, the inverted lists in order, the quantizer (and for IVF_PQ the
// codebooks and codes) -- as raw little-endian arrays that go to HBM with one copy each:
//
//   header   : char magic[8] = "PYRIDX01", int32 version, kind, dim, metric, uint32 nsections
//   section  : uint32 tag, uint32 reserved, uint64 nbytes, payload (padded to 8 bytes)
//
// The last section is T_NONCE: 16 random bytes per snapshot (pyr_image_nonce reads them back).
//
// Sections are looked up by tag; a section that is absent loads as empty (the reference's
// Load_MissingFields_ShouldHandleGracefully, IvfFlatVectorIndexTests.cs:144-165).  Writes go to
// path + ".tmp", are flushed and fsync'ed, and then renamed over path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace pyr {

// section tags
enum : uint32_t {
  T_BUILT = 1,      // uint8: the IVF lists are in use (_isBuilt)
  T_CENTS = 2,      // float [nlist][dim] coarse quantizer
  T_LCOUNT = 3,     // int32 [nlist] rows per inverted list (list-major order of T_LLABELS / T_LROWS)
  T_LLABELS = 4,    // int64 labels of the list entries, list-major
  T_LROWS = 5,      // float [n][dim] list rows, list-major (IVF_FLAT)
  T_BLABELS = 6,    // int64 labels of the pre-build buffer in enumeration order
  T_BROWS = 7,      // float [n][dim] buffer rows
  T_FLABELS = 8,    // int64 labels of the live FLAT slots in slot order
  T_FROWS = 9,      // float [n][dim] FLAT rows
  T_CODEBOOKS = 10, // float [M][ksub][dim / M] (IVF_PQ)
  T_KSUB = 11,      // int32 codebook size per subspace
  T_LCODES = 12,    // uint8 [n][M] PQ codes, list-major
  T_NONCE = 13,     // uint8 [16] random bytes drawn by every commit(): the image's identity, which
                    // the shim's ".ids" map records so that it never pairs with another image
};

constexpr uint64_t NONCE_BYTES = 16;

struct ImageWriter {
  std::string path, tmp;
  std::FILE *f = nullptr;
  uint32_t nsec = 0;
  bool done = false;
  ImageWriter(const std::string &path, int32_t kind, int32_t dim, int32_t metric);
  ~ImageWriter();
  void host(uint32_t tag, const void *p, uint64_t nbytes);
  // device bytes, copied through a bounded host buffer
  void device(uint32_t tag, const void *dp, uint64_t nbytes, hipStream_t st);
  void commit();  // append T_NONCE, flush + fsync + rename(tmp, path)

 private:
  void put(const void *p, size_t n);
  void begin(uint32_t tag, uint64_t nbytes);
  void pad(uint64_t nbytes);
};

struct ImageReader {
  std::FILE *f = nullptr;
  int32_t kind = -1, dim = 0, metric = 0;
  std::map<uint32_t, std::pair<uint64_t, uint64_t>> sec;  // tag -> (offset, nbytes)
  explicit ImageReader(const std::string &path);  // throws PYR_E_NOT_FOUND / PYR_E_FORMAT
  ~ImageReader();
  bool has(uint32_t tag) const { return sec.count(tag) != 0; }
  uint64_t size(uint32_t tag) const;  // 0 if absent
  void host(uint32_t tag, void *p, uint64_t nbytes);  // the section must hold exactly nbytes
  template <class T>
  std::vector<T> vec(uint32_t tag) {
    const uint64_t n = size(tag);
    if (n % sizeof(T)) throw_format("section size is not a whole number of elements");
    std::vector<T> v(n / sizeof(T));
    if (n) host(tag, v.data(), n);
    return v;
  }
  void device(uint32_t tag, void *dp, uint64_t nbytes, hipStream_t st);
  [[noreturn]] static void throw_format(const std::string &m);
};

}  // namespace pyr
