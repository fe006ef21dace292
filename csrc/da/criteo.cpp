// Criteo click-log featurisation, native.
//
// Reference (cerebro_gpdb/preprocessing/criteo/preprocessing_criteo.py:48-110):
// a TSV row = label, 13 integer features, 26 categorical hex strings.  After
// pandas fillna(0) a feature participates iff it is truthy:
//   * continuous f (0..12): bucket = first j with value < 1.5**j - 0.51
//     (j < 50, else 49) -> column f*50 + bucket
//   * categorical f (13..38): mmh3.hash(str) % 256 (Python modulo of the
//     signed 32-bit MurmurHash3_x86_32, seed 0) -> column 650 + (f-13)*256 + h
// giving <= 39 active columns of 7306.  Rows with a field count other than
// 40 yield no features and label 0 (the reference's `len(features) != 39`
// branch).  Output here is the compact form: ids [rows][39] int32 padded
// with -1, plus labels; ``tools.preprocess_criteo`` can expand it to the
// reference's dense f32 [N, 7307] .npy.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kCont = 13, kFields = 39, kBuckets = 50, kHash = 256;

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

}  // namespace

extern "C" {

// MurmurHash3_x86_32 (Austin Appleby, public domain algorithm), seed given
uint32_t cer_murmur3_32(const uint8_t* data, int64_t len, uint32_t seed) {
  const int64_t nblocks = len / 4;
  uint32_t h1 = seed;
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  for (int64_t i = 0; i < nblocks; ++i) {
    uint32_t k1;
    std::memcpy(&k1, data + 4 * i, 4);  // little-endian load
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= (uint32_t)tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= (uint32_t)tail[1] << 8; [[fallthrough]];
    case 1:
      k1 ^= tail[0];
      k1 *= c1;
      k1 = rotl32(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

int cer_criteo_bucket(double v) {
  for (int j = 0; j < kBuckets; ++j)
    if (v < std::pow(1.5, j) - 0.51) return j;
  return kBuckets - 1;
}

}  // extern "C"

namespace {

// featurise one line [b, e) -> ids (kFields, -1 padded); returns label
int featurize(const char* b, const char* e, int32_t* ids) {
  const char* f[kFields + 1];
  const char* fe[kFields + 1];
  int n = 0;
  const char* s = b;
  for (const char* p = b;; ++p) {
    if (p == e || *p == '\t') {
      if (n <= kFields) {
        f[n] = s;
        fe[n] = p;
      }
      ++n;
      s = p + 1;
      if (p == e) break;
    }
  }
  for (int i = 0; i < kFields; ++i) ids[i] = -1;
  if (n != kFields + 1) return 0;
  int label = (fe[0] > f[0]) ? std::atoi(std::string(f[0], fe[0]).c_str()) : 0;
  int k = 0;
  for (int i = 0; i < kCont; ++i) {
    const char* a = f[1 + i];
    const char* z = fe[1 + i];
    if (a == z) continue;                       // NaN -> 0 -> falsy
    const long v = std::strtol(std::string(a, z).c_str(), nullptr, 10);
    if (v == 0) continue;                       // literal 0 is falsy too
    ids[k++] = i * kBuckets + cer_criteo_bucket((double)v);
  }
  for (int i = kCont; i < kFields; ++i) {
    const char* a = f[1 + i];
    const char* z = fe[1 + i];
    if (a == z) continue;
    const int32_t h = (int32_t)cer_murmur3_32((const uint8_t*)a, z - a, 0);
    const int m = ((h % kHash) + kHash) % kHash;  // Python modulo
    ids[k++] = kCont * kBuckets + (i - kCont) * kHash + m;
  }
  return label;
}

}  // namespace

extern "C" {

// Parse up to max_rows '\n'-terminated lines of buf; returns rows written.
int64_t cer_criteo_featurize(const char* buf, int64_t len, int32_t* ids, int32_t* labels,
                             int64_t max_rows, int nthreads) {
  std::vector<const char*> starts;
  const char* p = buf;
  const char* end = buf + len;
  while (p < end && (int64_t)starts.size() < max_rows) {
    starts.push_back(p);
    const char* nl = (const char*)std::memchr(p, '\n', end - p);
    p = nl ? nl + 1 : end;
  }
  const int64_t rows = (int64_t)starts.size();
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < nthreads; ++t) {
    pool.emplace_back([&, t]() {
      for (int64_t r = t; r < rows; r += nthreads) {
        const char* b = starts[r];
        const char* nl = (const char*)std::memchr(b, '\n', end - b);
        const char* e = nl ? nl : end;
        while (e > b && e[-1] == '\r') --e;
        labels[r] = featurize(b, e, ids + r * kFields);
      }
    });
  }
  for (auto& th : pool) th.join();
  return rows;
}

}  // extern "C"
