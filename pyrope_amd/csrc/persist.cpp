// persist.cpp -- binary index image I/O (persist.h).
#include "persist.h"

#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <random>

#include "engine.h"

namespace pyr {

namespace {
constexpr char MAGIC[8] = {'P', 'Y', 'R', 'I', 'D', 'X', '0', '1'};
constexpr int32_t VERSION = 1;
constexpr size_t CHUNK = size_t(64) << 20;  // host bounce buffer for device sections
}  // namespace

ImageWriter::ImageWriter(const std::string &p, int32_t kind, int32_t dim, int32_t metric) : path(p), tmp(p + ".tmp") {
  if (path.empty()) throw Error(PYR_E_ARG, "Path cannot be empty.");
  f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw Error(PYR_E_IO, "cannot create " + tmp + ": " + std::strerror(errno));
  put(MAGIC, 8);
  const int32_t h[4] = {VERSION, kind, dim, metric};
  put(h, sizeof(h));
  put(&nsec, 4);  // patched by commit()
}

ImageWriter::~ImageWriter() {
  if (f) std::fclose(f);
  if (!done) std::remove(tmp.c_str());
}

void ImageWriter::put(const void *p, size_t n) {
  if (n && std::fwrite(p, 1, n, f) != n) throw Error(PYR_E_IO, "write to " + tmp + " failed");
}

void ImageWriter::begin(uint32_t tag, uint64_t nbytes) {
  const uint32_t t[2] = {tag, 0};
  put(t, 8);
  put(&nbytes, 8);
  nsec++;
}

void ImageWriter::pad(uint64_t nbytes) {
  static const char z[8] = {0};
  put(z, (8 - nbytes % 8) % 8);
}

void ImageWriter::host(uint32_t tag, const void *p, uint64_t nbytes) {
  begin(tag, nbytes);
  put(p, nbytes);
  pad(nbytes);
}

void ImageWriter::device(uint32_t tag, const void *dp, uint64_t nbytes, hipStream_t st) {
  begin(tag, nbytes);
  std::vector<char> buf(std::min<uint64_t>(nbytes, CHUNK));
  for (uint64_t o = 0; o < nbytes; o += buf.size()) {
    const uint64_t n = std::min<uint64_t>(buf.size(), nbytes - o);
    HIPCHK(hipMemcpyAsync(buf.data(), static_cast<const char *>(dp) + o, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    put(buf.data(), n);
  }
  pad(nbytes);
}

void ImageWriter::commit() {
  std::random_device rd;  // the image's identity (T_NONCE), fresh for every snapshot
  uint32_t nonce[NONCE_BYTES / 4];
  for (auto &w : nonce) w = rd();
  host(T_NONCE, nonce, NONCE_BYTES);
  if (std::fseek(f, 8 + 16, SEEK_SET) != 0) throw Error(PYR_E_IO, "seek in " + tmp + " failed");
  put(&nsec, 4);
  if (std::fflush(f) != 0 || fsync(fileno(f)) != 0) throw Error(PYR_E_IO, "flush of " + tmp + " failed");
  std::fclose(f);
  f = nullptr;
  // the temp file replaces the old image in one step (DeltaVectorIndex.cs:172-185 temp + move)
  if (std::rename(tmp.c_str(), path.c_str()) != 0)
    throw Error(PYR_E_IO, "rename " + tmp + " -> " + path + " failed: " + std::strerror(errno));
  done = true;
}

void ImageReader::throw_format(const std::string &m) { throw Error(PYR_E_FORMAT, "not a valid index image: " + m); }

ImageReader::ImageReader(const std::string &path) {
  if (path.empty()) throw Error(PYR_E_ARG, "Path cannot be empty.");
  f = std::fopen(path.c_str(), "rb");
  if (!f) throw Error(PYR_E_NOT_FOUND, "Snapshot file not found: " + path);
  char m[8];
  int32_t h[4];
  uint32_t n = 0;
  if (std::fread(m, 1, 8, f) != 8 || std::memcmp(m, MAGIC, 8) != 0) throw_format("bad magic");
  if (std::fread(h, 1, sizeof(h), f) != sizeof(h) || std::fread(&n, 1, 4, f) != 4) throw_format("short header");
  if (h[0] != VERSION) throw_format("unsupported version " + std::to_string(h[0]));
  kind = h[1];
  dim = h[2];
  metric = h[3];
  if (std::fseek(f, 0, SEEK_END) != 0) throw_format("unreadable");
  const long fend = std::ftell(f);
  if (fend < 0) throw_format("unreadable");
  const uint64_t fsize = (uint64_t)fend;
  uint64_t off = 8 + 16 + 4;
  if (std::fseek(f, (long)off, SEEK_SET) != 0) throw_format("short header");
  for (uint32_t i = 0; i < n; i++) {
    uint32_t t[2];
    uint64_t nb;
    if (std::fread(t, 1, 8, f) != 8 || std::fread(&nb, 1, 8, f) != 8) throw_format("short section header");
    off += 16;
    // every section lies inside the file (untrusted sizes: no wrap-around of off)
    if (off > fsize || nb > fsize - off) throw_format("section " + std::to_string(t[0]) + " runs past the end");
    sec[t[0]] = {off, nb};
    off += nb + (8 - nb % 8) % 8;
    if (std::fseek(f, (long)std::min(off, fsize), SEEK_SET) != 0) throw_format("short section");
  }
}

ImageReader::~ImageReader() {
  if (f) std::fclose(f);
}

uint64_t ImageReader::size(uint32_t tag) const {
  auto it = sec.find(tag);
  return it == sec.end() ? 0 : it->second.second;
}

void ImageReader::host(uint32_t tag, void *p, uint64_t nbytes) {
  auto it = sec.find(tag);
  if (it == sec.end() || it->second.second != nbytes) throw_format("section " + std::to_string(tag) + " size");
  if (std::fseek(f, (long)it->second.first, SEEK_SET) != 0 || std::fread(p, 1, nbytes, f) != nbytes)
    throw_format("short read");
}

void ImageReader::device(uint32_t tag, void *dp, uint64_t nbytes, hipStream_t st) {
  auto it = sec.find(tag);
  if (it == sec.end() || it->second.second != nbytes) throw_format("section " + std::to_string(tag) + " size");
  if (std::fseek(f, (long)it->second.first, SEEK_SET) != 0) throw_format("short read");
  std::vector<char> buf(std::min<uint64_t>(nbytes, CHUNK));
  for (uint64_t o = 0; o < nbytes; o += buf.size()) {
    const uint64_t n = std::min<uint64_t>(buf.size(), nbytes - o);
    if (std::fread(buf.data(), 1, n, f) != n) throw_format("short read");
    HIPCHK(hipMemcpyAsync(static_cast<char *>(dp) + o, buf.data(), n, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  }
}

}  // namespace pyr
