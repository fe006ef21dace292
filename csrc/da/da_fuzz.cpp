// Sanitizer harness for the DA reader and pglz (ASan/UBSan
// builds of the C++ reader fuzzed with corrupted pages, TSan over the
// reader's thread pool).  Built and run by tests/test_sanitizers.py:
//   g++ -O1 -g -fsanitize=address,undefined  -> every mutation must end in a
//                                               clean error, never a fault
//   g++ -O1 -g -fsanitize=thread             -> the multi-threaded read of a
//                                               valid partition is race-free
// usage: da_fuzz DIR ITERATIONS SEED
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "da.h"

extern "C" {
const char* cer_da_last_error();
void* cer_da_open(const char* heap_base, const char* toast_base);
int cer_da_count(void* h);
int cer_da_info(void* h, int i, int32_t* dist_key, int32_t* buffer_id, int64_t* indep_raw,
                int64_t* dep_raw);
int cer_da_read(void* h, int n, const int* idx, uint8_t** indep_out, uint8_t** dep_out,
                int nthreads);
void cer_da_close(void* h);
void* cer_da_writer_open(const char* heap_base, const char* toast_base, uint32_t toastrelid,
                         uint32_t first_valueid, int64_t seg_bytes);
int cer_da_writer_add(void* hw, int32_t dist_key, int32_t buffer_id, const uint8_t* indep,
                      int64_t indep_n, const uint8_t* dep, int64_t dep_n, int dep_inline);
int cer_da_writer_close(void* hw);
int64_t cer_criteo_featurize(const char* buf, int64_t len, int32_t* ids, int32_t* labels,
                             int64_t max_rows, int nthreads);
}

static std::vector<uint8_t> slurp(const std::string& p) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f) return b;
  std::fseek(f, 0, SEEK_END);
  b.resize((size_t)std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (!b.empty() && std::fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
  std::fclose(f);
  return b;
}

static void spit(const std::string& p, const std::vector<uint8_t>& b) {
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) { std::perror(p.c_str()); std::exit(2); }
  std::fwrite(b.data(), 1, b.size(), f);
  std::fclose(f);
}

// open + read everything; returns tuples read or -1 on a (clean) error
static int read_all(const std::string& heap, const std::string& toast, int nthreads) {
  void* h = cer_da_open(heap.c_str(), toast.c_str());
  if (!h) return -1;
  const int n = cer_da_count(h);
  std::vector<std::vector<uint8_t>> ind((size_t)n), dep((size_t)n);
  std::vector<uint8_t*> pi((size_t)n), pd((size_t)n);
  std::vector<int> idx((size_t)n);
  for (int i = 0; i < n; ++i) {
    int32_t dk, bid;
    int64_t ir, dr;
    if (cer_da_info(h, i, &dk, &bid, &ir, &dr) || ir < 0 || dr < 0 || ir > (1 << 28) ||
        dr > (1 << 28)) {
      cer_da_close(h);
      return -1;
    }
    ind[(size_t)i].resize((size_t)ir + 1);
    dep[(size_t)i].resize((size_t)dr + 1);
    pi[(size_t)i] = ind[(size_t)i].data();
    pd[(size_t)i] = dep[(size_t)i].data();
    idx[(size_t)i] = i;
  }
  const int rc = n ? cer_da_read(h, n, idx.data(), pi.data(), pd.data(), nthreads) : 0;
  cer_da_close(h);
  return rc ? -1 : n;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s DIR ITERATIONS SEED\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int iters = std::atoi(argv[2]);
  std::mt19937 rng((uint32_t)std::atoi(argv[3]));
  const std::string heap = dir + "/heap", toast = dir + "/toast";

  // 1) a valid partition: compressible images (external, TOAST-chunked) and labels
  void* w = cer_da_writer_open(heap.c_str(), toast.c_str(), 4242u, 100u, (int64_t)1 << 30);
  if (!w) { std::fprintf(stderr, "writer: %s\n", cer_da_last_error()); return 2; }
  const int ntup = 6;
  std::vector<std::vector<uint8_t>> want_ind;
  for (int t = 0; t < ntup; ++t) {
    std::vector<uint8_t> img(20000 + 4000 * t), lab(64);
    for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)((i / 7 + t) & 0x3f);
    for (size_t i = 0; i < lab.size(); ++i) lab[i] = (uint8_t)(rng() & 1);
    if (cer_da_writer_add(w, t % 3, t, img.data(), (int64_t)img.size(), lab.data(),
                          (int64_t)lab.size(), t & 1)) {
      std::fprintf(stderr, "writer add: %s\n", cer_da_last_error());
      return 2;
    }
    want_ind.push_back(img);
  }
  if (cer_da_writer_close(w)) { std::fprintf(stderr, "writer close\n"); return 2; }

  // 2) threaded read of the valid partition (the TSan target)
  for (int rep = 0; rep < 4; ++rep) {
    if (read_all(heap, toast, 4) != ntup) {
      std::fprintf(stderr, "valid partition unreadable: %s\n", cer_da_last_error());
      return 1;
    }
  }

  // 2b) Criteo featurisation on its thread pool (TSan), then garbage lines (ASan)
  {
    std::string tsv;
    for (int r = 0; r < 257; ++r) {
      tsv += std::to_string(r & 1);
      for (int f = 0; f < 13; ++f) tsv += "\t" + ((r + f) % 5 ? std::to_string((r * 31 + f) % 1000 - 3) : "");
      for (int f = 0; f < 26; ++f) tsv += "\t" + ((r + f) % 7 ? std::to_string(r * 131 + f * 7) : "");
      tsv += (r % 3) ? "\n" : "\r\n";
    }
    std::vector<int32_t> ids(257 * 39), labels(257);
    if (cer_criteo_featurize(tsv.data(), (int64_t)tsv.size(), ids.data(), labels.data(), 257, 4) !=
        257) {
      std::fprintf(stderr, "criteo featurize row count\n");
      return 1;
    }
    for (int it = 0; it < iters / 10 + 1; ++it) {
      std::string g = tsv;
      for (int k = 0; k < 20; ++k) g[rng() % g.size()] = (char)(rng() & 0xff);
      (void)cer_criteo_featurize(g.data(), (int64_t)g.size(), ids.data(), labels.data(), 257,
                                 1 + (int)(rng() % 4));
    }
  }

  // 3) pglz: random round trips and corrupted streams
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> raw(1 + rng() % 5000);
    const int alpha = 1 + (int)(rng() % 16);
    for (auto& b : raw) b = (uint8_t)(rng() % alpha);
    std::vector<uint8_t> comp(raw.size() * 2 + 64), back(raw.size());
    const int64_t cl = cer_pglz_compress(raw.data(), (int64_t)raw.size(), comp.data(),
                                         (int64_t)comp.size());
    if (cl > 0) {
      if (cer_pglz_decompress(comp.data(), cl, back.data(), (int64_t)back.size()) !=
              (int64_t)raw.size() ||
          back != raw) {
        std::fprintf(stderr, "pglz round trip failed\n");
        return 1;
      }
      comp.resize((size_t)cl);
      for (int k = 0; k < 1 + (int)(rng() % 8); ++k) comp[rng() % comp.size()] ^= (uint8_t)(1 + rng() % 255);
      if (rng() & 1) comp.resize(comp.size() - rng() % comp.size());
      (void)cer_pglz_decompress(comp.data(), (int64_t)comp.size(), back.data(),
                                (int64_t)back.size());
    }
  }

  // 4) corrupted pages: every mutation must be read or rejected cleanly
  const std::vector<uint8_t> h0 = slurp(heap), t0 = slurp(toast);
  const std::string mh = dir + "/mheap", mt = dir + "/mtoast";
  int rejected = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> h = h0, t = t0;
    std::vector<uint8_t>& v = (rng() & 1) ? h : t;
    const int nmut = 1 + (int)(rng() % 6);
    for (int k = 0; k < nmut; ++k) {
      // page headers + line pointers (head of a page), tuple headers / TOAST
      // pointers / varlena headers (tail of the first page), or anywhere
      const size_t page0 = (size_t)(rng() % (v.size() / da::kBlck)) * da::kBlck;
      const int where = (int)(rng() % 3);
      const size_t pos = where == 0   ? page0 + rng() % 512
                         : where == 1 ? page0 + da::kBlck - 1 - rng() % 512
                                      : rng() % v.size();
      v[pos] = (rng() & 1) ? (uint8_t)rng() : (uint8_t)(v[pos] ^ (1u << (rng() % 8)));
    }
    spit(mh, h);
    spit(mt, t);
    if (read_all(mh, mt, 1 + (int)(rng() % 4)) < 0) ++rejected;
  }
  std::printf("ok: %d tuples, %d mutations, %d rejected cleanly\n", ntup, iters, rejected);
  return 0;
}
