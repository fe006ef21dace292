// Direct-Access page reader / writer.  See da.h for
// the on-disk format.
//
// Reader: every segment file of the heap and TOAST relations is mmap-ed (no
// read into a private copy: round 3 fread the whole relation -- 13 GB for a
// full ImageNet-112 partition -- on one thread into a zero-filled vector,
// which is where the decode wall time went, profiles/r4_da_etl.md); heap
// pages are parsed into tuples; the TOAST pages are scanned into a chunk
// index keyed by value id on a thread pool (page ranges per thread, only ids
// referenced by the heap, merged once); buffers are then detoasted +
// pglz-decompressed in parallel, straight into caller-provided (pinned) host
// memory.  Each phase is timed (cer_da_stats).  Integrity checks follow the
// reference: line-pointer area multiple of 4, no special space on TOAST
// pages, chunk counts / sizes, final size, pglz end-of-stream.
//
// Writer: builds the same format from raw buffers (compressing with pglz),
// for tests and for generating synthetic DA partitions.
#include <arpa/inet.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "da.h"

using namespace da;

namespace {

thread_local std::string g_err;

bool set_err(const std::string& e) {
  g_err = e;
  return false;
}

std::vector<std::string> segment_files(const std::string& base) {
  std::vector<std::string> out;
  FILE* f = std::fopen(base.c_str(), "rb");
  if (!f) return out;
  std::fclose(f);
  out.push_back(base);
  for (int i = 1;; ++i) {
    std::string p = base + "." + std::to_string(i);
    FILE* g = std::fopen(p.c_str(), "rb");
    if (!g) break;
    std::fclose(g);
    out.push_back(p);
  }
  return out;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// One relation (heap or TOAST): its segment files mapped read-only, and the
// address of every page in relation order.
struct Relation {
  struct Seg {
    void* base = nullptr;
    size_t len = 0;
  };
  std::vector<Seg> segs;
  std::vector<const uint8_t*> pages;
  ~Relation() {
    for (auto& g : segs)
      if (g.base && g.len) munmap(g.base, g.len);
  }
};

bool map_relation(const std::string& base, Relation* rel, bool required) {
  auto files = segment_files(base);
  if (files.empty()) return required ? set_err("no segment files at " + base) : true;
  for (auto& path : files) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return set_err("cannot open " + path);
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
      close(fd);
      return set_err("cannot stat " + path);
    }
    const size_t n = (size_t)sb.st_size;
    if (n % kBlck) {
      close(fd);
      return set_err("segment size not a multiple of BLCKSZ: " + path);
    }
    Relation::Seg g;
    if (n) {
      g.base = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      if (g.base == MAP_FAILED) {
        close(fd);
        return set_err("cannot mmap " + path);
      }
      g.len = n;
      madvise(g.base, n, MADV_WILLNEED);     // start the page-cache reads now
    }
    close(fd);
    rel->segs.push_back(g);
    for (size_t o = 0; o < n; o += kBlck)
      rel->pages.push_back(static_cast<const uint8_t*>(g.base) + o);
  }
  return true;
}

inline uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline int32_t rdi32(const uint8_t* p) { int32_t v; std::memcpy(&v, p, 4); return v; }
inline void wr16(uint8_t* p, uint16_t v) { std::memcpy(p, &v, 2); }
inline void wr32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
inline uint32_t varsize_4b(const uint8_t* p) { return ntohl(rd32(p)) & 0x3FFFFFFFu; }

struct PageHdr {
  uint16_t lower, upper, special;
};

inline PageHdr page_header(const uint8_t* page) {
  return PageHdr{rd16(page + 12), rd16(page + 14), rd16(page + 16)};
}

struct ExtPtr {
  int32_t rawsize, extsize;
  uint32_t valueid, toastrelid;
};

struct Datum {
  bool external = false;
  ExtPtr ptr{};
  const uint8_t* inl = nullptr;  // inline compressed varlena (4B_C)
};

struct Tuple {
  int32_t dist_key = 0, buffer_id = 0;
  Datum indep, dep;
};

struct Chunk {
  int32_t seq;
  const uint8_t* data;
  uint32_t size;
};

bool parse_datum(const uint8_t* p, const uint8_t* end, Datum* d, int64_t* consumed) {
  if (p >= end) return set_err("datum beyond tuple end");
  if (p[0] == 0x80) {  // 1B_E external TOAST pointer
    if (p + kExtPtr > end) return set_err("truncated TOAST pointer");
    d->external = true;
    d->ptr.rawsize = rdi32(p + 4);
    d->ptr.extsize = rdi32(p + 8);
    d->ptr.valueid = rd32(p + 12);
    d->ptr.toastrelid = rd32(p + 16);
    // sizes straight from the file: reject what no writer produces (a 1 GB
    // datum limit, as in PostgreSQL) before anything is allocated from them
    if (d->ptr.rawsize < 4 || d->ptr.extsize <= 0 || d->ptr.extsize > (1 << 30) ||
        d->ptr.rawsize > (1 << 30) + 4)
      return set_err("bad TOAST pointer sizes");
    *consumed = kExtPtr;
    return true;
  }
  if ((p[0] & 0xC0) == 0x40) {  // inline 4B compressed
    if (p + 8 > end) return set_err("truncated inline datum header");
    uint32_t vs = varsize_4b(p);
    if (vs < 8 || p + vs > end) return set_err("truncated inline datum");
    if (rd32(p + 4) > (1u << 30)) return set_err("bad inline raw size");
    d->external = false;
    d->inl = p;
    *consumed = vs;
    return true;
  }
  return set_err("unsupported varlena header");
}

}  // namespace

// ---------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------
struct DAReader {
  Relation heap, toast;
  std::vector<Tuple> tuples;
  std::unordered_map<uint32_t, std::vector<Chunk>> chunks;
  int nthreads = 8;
  // phase timings (seconds): open = map + heap parse + TOAST index; read =
  // the last cer_da_read (wall) and its workers' busy / copy / pglz sums
  double map_s = 0, heap_s = 0, index_s = 0;
  double read_wall_s = 0, read_busy_s = 0, read_copy_s = 0, read_pglz_s = 0;
  int read_threads = 0;
};

static bool parse_heap(DAReader* r) {
  for (const uint8_t* page : r->heap.pages) {
    PageHdr h = page_header(page);
    if (h.lower < kPageHeader || h.lower > kBlck) return set_err("bad pd_lower");
    if ((h.lower - kPageHeader) % kItemId) return set_err("line pointer area not a multiple of 4");
    const int n = (h.lower - kPageHeader) / kItemId;
    for (int i = 0; i < n; ++i) {
      const uint32_t lp = rd32(page + kPageHeader + kItemId * i);
      const uint32_t lp_off = lp & 0x7FFF, lp_flags = (lp >> 15) & 3, lp_len = lp >> 17;
      if (lp_flags != 1) continue;  // LP_NORMAL only
      if (lp_off + lp_len > (uint32_t)kBlck || lp_len < (uint32_t)kTupleHeader)
        return set_err("line pointer out of page");
      const uint8_t* tup = page + lp_off;
      const uint8_t t_hoff = tup[22];
      const uint8_t* data = tup + t_hoff;
      const uint8_t* end = tup + lp_len;
      if (data + 8 > end) return set_err("tuple too short");
      Tuple t;
      t.dist_key = rdi32(data);
      int64_t used = 0;
      if (!parse_datum(data + 4, end, &t.indep, &used)) return false;
      const uint8_t* q = data + 4 + used;
      if (!parse_datum(q, end, &t.dep, &used)) return false;
      t.buffer_id = rdi32(end - 4);
      r->tuples.push_back(t);
    }
  }
  return true;
}

// scan TOAST pages [p0, p1): chunks of wanted value ids, in page order
static bool index_toast_range(const DAReader* r, const std::unordered_set<uint32_t>& want,
                              size_t p0, size_t p1,
                              std::vector<std::pair<uint32_t, Chunk>>* out) {
  for (size_t pg = p0; pg < p1; ++pg) {
    const uint8_t* page = r->toast.pages[pg];
    PageHdr h = page_header(page);
    if (h.special != kBlck) return set_err("THERE SHALL NOT BE INDICES (special space on TOAST page)");
    if (h.lower < kPageHeader || h.lower > kBlck || (h.lower - kPageHeader) % kItemId)
      return set_err("bad TOAST line pointer area");
    const int n = (h.lower - kPageHeader) / kItemId;
    int64_t off = h.upper;
    for (int i = 0; i < n; ++i) {
      off = maxalign(off);
      if (off + kTupleHeader > kBlck) return set_err("TOAST item beyond page");
      const uint8_t* item = page + off;
      const uint8_t t_hoff = item[22];
      if (off + t_hoff + 12 > kBlck) return set_err("TOAST chunk header beyond page");
      const uint8_t* tup = item + t_hoff;
      const uint32_t chunk_id = rd32(tup), chunk_seq = rd32(tup + 4);
      const uint8_t* cv = tup + 8;
      const uint32_t csize = varsize_4b(cv);
      if (cv[0] & 0xC0) return set_err("TOAST chunk must be a plain 4B varlena");
      if (csize < 4) return set_err("TOAST chunk shorter than its header");
      if (off + t_hoff + 8 + csize > (uint32_t)kBlck) return set_err("TOAST chunk beyond page");
      if (want.count(chunk_id))
        out->emplace_back(chunk_id, Chunk{(int32_t)chunk_seq, cv + 4, csize - 4});
      off += t_hoff + 8 + csize;
    }
  }
  return true;
}

static bool index_toast(DAReader* r) {
  std::unordered_set<uint32_t> want;
  for (auto& t : r->tuples) {
    if (t.indep.external) want.insert(t.indep.ptr.valueid);
    if (t.dep.external) want.insert(t.dep.ptr.valueid);
  }
  const size_t np = r->toast.pages.size();
  const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)r->nthreads, np / 64 + 1));
  std::vector<std::vector<std::pair<uint32_t, Chunk>>> part((size_t)nt);
  std::vector<std::string> errs((size_t)nt);
  std::vector<char> ok((size_t)nt, 1);
  auto work = [&](int t) {
    const size_t p0 = np * (size_t)t / (size_t)nt, p1 = np * (size_t)(t + 1) / (size_t)nt;
    part[(size_t)t].reserve((p1 - p0) * 4);
    if (!index_toast_range(r, want, p0, p1, &part[(size_t)t])) {
      ok[(size_t)t] = 0;
      errs[(size_t)t] = g_err;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (int t = 0; t < nt; ++t)
    if (!ok[(size_t)t]) return set_err(errs[(size_t)t]);
  r->chunks.reserve(want.size());
  for (auto& v : part)
    for (auto& kv : v) r->chunks[kv.first].push_back(kv.second);
  return true;
}

static bool detoast(const DAReader* r, const Datum& d, uint8_t* out, int64_t out_size,
                    std::vector<uint8_t>* scratch, double* copy_s, double* pglz_s) {
  if (!d.external) {
    const uint8_t* p = d.inl;
    const uint32_t vs = varsize_4b(p);
    const uint32_t raw = rd32(p + 4);
    if ((int64_t)raw != out_size) return set_err("inline raw size does not match");
    const double t0 = now_s();
    if (cer_pglz_decompress(p + 8, vs - 8, out, raw) < 0) return set_err("compressed data is corrupt");
    *pglz_s += now_s() - t0;
    return true;
  }
  const double tc = now_s();
  auto it = r->chunks.find(d.ptr.valueid);
  if (it == r->chunks.end()) return set_err("missing TOAST value " + std::to_string(d.ptr.valueid));
  std::vector<Chunk> cs = it->second;
  std::sort(cs.begin(), cs.end(), [](const Chunk& a, const Chunk& b) { return a.seq < b.seq; });
  const int64_t ext = d.ptr.extsize;
  const int64_t nchunks = (ext - 1) / kToastMaxChunk + 1;
  if ((int64_t)cs.size() != nchunks) return set_err("TOAST chunk count mismatch");
  for (int64_t i = 0; i < nchunks; ++i) {
    const Chunk& c = cs[(size_t)i];
    if (c.seq != i) return set_err("TOAST chunk sequence gap");
    if (i < nchunks - 1 && c.size != (uint32_t)kToastMaxChunk) return set_err("unexpected chunk size");
    if (i == nchunks - 1 && i * kToastMaxChunk + (int64_t)c.size != ext)
      return set_err("unexpected last chunk size");
  }
  const bool compressed = ext < (int64_t)d.ptr.rawsize - 4;
  if (!compressed) {
    if (ext != out_size) return set_err("external raw size mismatch");
    int64_t pos = 0;
    for (const Chunk& c : cs) {
      std::memcpy(out + pos, c.data, c.size);
      pos += c.size;
    }
    *copy_s += now_s() - tc;
    return true;
  }
  if (ext < 4) return set_err("external compressed datum shorter than its header");
  // the stream is read in place from the chunks (pglz_decompress_pieces): no
  // copy of the compressed value into a scratch buffer first
  std::vector<const uint8_t*> ptrs(cs.size());
  std::vector<int64_t> lens(cs.size());
  for (size_t i = 0; i < cs.size(); ++i) {
    ptrs[i] = cs[i].data;
    lens[i] = cs[i].size;
  }
  uint8_t hdr[4];
  for (int64_t k = 0, i = 0, o = 0; k < 4; ++k) {     // rawsize u32 (may straddle chunks)
    while (o >= lens[(size_t)i]) {
      ++i;
      o = 0;
    }
    hdr[k] = ptrs[(size_t)i][o++];
  }
  const uint32_t raw = rd32(hdr);
  if ((int64_t)raw != out_size) return set_err("external raw size does not match");
  const double tp = now_s();
  *copy_s += tp - tc;
  if (cer_pglz_decompress_pieces(ptrs.data(), lens.data(), (int)cs.size(), 4, out, raw) < 0)
    return set_err("compressed data is corrupt");
  *pglz_s += now_s() - tp;
  (void)scratch;
  return true;
}

static int64_t raw_size(const Datum& d) {
  if (!d.external) return rd32(d.inl + 4);
  return (int64_t)d.ptr.rawsize - 4;
}

extern "C" {

const char* cer_da_last_error() { return g_err.c_str(); }

// nthreads: TOAST-index threads (0: 16)
void* cer_da_open2(const char* heap_base, const char* toast_base, int nthreads) {
  auto* r = new DAReader();
  r->nthreads = nthreads > 0 ? nthreads : 16;
  double t0 = now_s();
  if (!map_relation(heap_base, &r->heap, true) || !map_relation(toast_base, &r->toast, false)) {
    delete r;
    return nullptr;
  }
  double t1 = now_s();
  r->map_s = t1 - t0;
  if (!parse_heap(r)) {
    delete r;
    return nullptr;
  }
  double t2 = now_s();
  r->heap_s = t2 - t1;
  if (!index_toast(r)) {
    delete r;
    return nullptr;
  }
  r->index_s = now_s() - t2;
  return r;
}

void* cer_da_open(const char* heap_base, const char* toast_base) {
  return cer_da_open2(heap_base, toast_base, 0);
}

// phase timings: out[0..8] = map, heap parse, TOAST index (open), read wall,
// read busy (sum over workers), read TOAST copy (sum), read pglz (sum),
// read threads, TOAST-index threads
int cer_da_stats(void* h, double* out) {
  auto* r = static_cast<DAReader*>(h);
  const double v[9] = {r->map_s, r->heap_s, r->index_s, r->read_wall_s, r->read_busy_s,
                       r->read_copy_s, r->read_pglz_s, (double)r->read_threads,
                       (double)r->nthreads};
  for (int i = 0; i < 9; ++i) out[i] = v[i];
  return 9;
}

int cer_da_count(void* h) { return (int)static_cast<DAReader*>(h)->tuples.size(); }

int cer_da_info(void* h, int i, int32_t* dist_key, int32_t* buffer_id, int64_t* indep_raw,
                int64_t* dep_raw) {
  auto* r = static_cast<DAReader*>(h);
  if (i < 0 || i >= (int)r->tuples.size()) return -1;
  const Tuple& t = r->tuples[(size_t)i];
  *dist_key = t.dist_key;
  *buffer_id = t.buffer_id;
  *indep_raw = raw_size(t.indep);
  *dep_raw = raw_size(t.dep);
  return 0;
}

// Detoast + decompress tuples idx[0..n) into indep_out[j] / dep_out[j]
// (buffers of the raw sizes reported by cer_da_info) on `nthreads` threads.
int cer_da_read(void* h, int n, const int* idx, uint8_t** indep_out, uint8_t** dep_out,
                int nthreads) {
  auto* r = static_cast<DAReader*>(h);
  std::atomic<int> next(0), failed(0);
  std::string first_err;
  std::atomic<bool> have_err(false);
  nthreads = std::max(1, std::min(nthreads, n));
  std::vector<double> busy((size_t)nthreads, 0.0), copy((size_t)nthreads, 0.0),
      pglz((size_t)nthreads, 0.0);
  // largest values first: a partition's buffers are few and large (a
  // pglz stream is serial), so the last round of a size-blind order leaves
  // most threads idle
  std::vector<int> order(idx, idx + n);
  std::vector<int> slot((size_t)n);
  for (int j = 0; j < n; ++j) slot[(size_t)j] = j;
  std::stable_sort(slot.begin(), slot.end(), [&](int a, int b) {
    return raw_size(r->tuples[(size_t)order[(size_t)a]].indep) >
           raw_size(r->tuples[(size_t)order[(size_t)b]].indep);
  });
  auto work = [&](int w) {
    std::vector<uint8_t> scratch;
    for (;;) {
      int q = next.fetch_add(1);
      if (q >= n || failed.load()) break;
      const int j = slot[(size_t)q];
      const double t0 = now_s();
      const Tuple& t = r->tuples[(size_t)idx[j]];
      bool ok = detoast(r, t.indep, indep_out[j], raw_size(t.indep), &scratch, &copy[(size_t)w],
                        &pglz[(size_t)w]) &&
                detoast(r, t.dep, dep_out[j], raw_size(t.dep), &scratch, &copy[(size_t)w],
                        &pglz[(size_t)w]);
      busy[(size_t)w] += now_s() - t0;
      if (!ok) {
        failed.store(1);
        bool expected = false;
        if (have_err.compare_exchange_strong(expected, true)) first_err = g_err;
      }
    }
  };
  const double t0 = now_s();
  std::vector<std::thread> pool;
  for (int i = 1; i < nthreads; ++i) pool.emplace_back(work, i);
  work(0);
  for (auto& t : pool) t.join();
  r->read_wall_s = now_s() - t0;
  r->read_busy_s = r->read_copy_s = r->read_pglz_s = 0;
  for (int i = 0; i < nthreads; ++i) {
    r->read_busy_s += busy[(size_t)i];
    r->read_copy_s += copy[(size_t)i];
    r->read_pglz_s += pglz[(size_t)i];
  }
  r->read_threads = nthreads;
  if (failed.load()) {
    g_err = first_err;
    return -1;
  }
  return 0;
}

void cer_da_close(void* h) { delete static_cast<DAReader*>(h); }

}  // extern "C"

// ---------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------
namespace {

struct SegWriter {
  std::string base;
  int64_t seg_bytes;
  int seg = 0;
  int64_t in_seg = 0;
  FILE* f = nullptr;
  bool open_next() {
    if (f) std::fclose(f);
    std::string p = seg == 0 ? base : base + "." + std::to_string(seg);
    f = std::fopen(p.c_str(), "wb");
    in_seg = 0;
    ++seg;
    return f != nullptr || set_err("cannot create " + p);
  }
  bool write_page(const uint8_t* page) {
    if (!f || in_seg + kBlck > seg_bytes)
      if (!open_next()) return false;
    if (std::fwrite(page, 1, kBlck, f) != (size_t)kBlck) return set_err("write failed");
    in_seg += kBlck;
    return true;
  }
  void close() {
    if (f) std::fclose(f);
    f = nullptr;
  }
};

struct PageBuilder {
  uint8_t page[kBlck];
  uint16_t lower, upper;
  uint32_t blkno = 0;
  void reset() {
    std::memset(page, 0, kBlck);
    lower = kPageHeader;
    upper = kBlck;
  }
  bool fits(int64_t len) const { return (int64_t)upper - maxalign(len) >= (int64_t)lower + kItemId; }
  uint16_t nitems() const { return (uint16_t)((lower - kPageHeader) / kItemId); }
  void add(const uint8_t* item, int64_t len) {
    upper = (uint16_t)(upper - maxalign(len));
    std::memcpy(page + upper, item, (size_t)len);
    const uint32_t lp = (uint32_t)upper | (1u << 15) | ((uint32_t)len << 17);
    wr32(page + lower, lp);
    lower = (uint16_t)(lower + kItemId);
  }
  void finish() {
    wr16(page + 12, lower);
    wr16(page + 14, upper);
    wr16(page + 16, (uint16_t)kBlck);                 // pd_special: no special space
    wr16(page + 18, (uint16_t)(kBlck | 4));           // pd_pagesize_version
  }
};

void tuple_header(uint8_t* h, uint32_t blk, uint16_t pos, uint16_t natts) {
  std::memset(h, 0, 24);
  wr32(h + 0, 2);  // xmin = FrozenTransactionId
  wr16(h + 12, (uint16_t)(blk >> 16));
  wr16(h + 14, (uint16_t)(blk & 0xffff));
  wr16(h + 16, pos);
  wr16(h + 18, natts);
  wr16(h + 20, 0x0802);  // HEAP_HASVARWIDTH | HEAP_XMAX_INVALID
  h[22] = 24;            // t_hoff = MAXALIGN(23)
}

}  // namespace

struct DAWriter {
  SegWriter heap, toast;
  PageBuilder hp, tp;
  uint32_t toastrelid, next_valueid;
  std::vector<uint8_t> comp;
};

static bool flush_page(SegWriter* w, PageBuilder* p) {
  if (p->nitems() == 0) return true;
  p->finish();
  if (!w->write_page(p->page)) return false;
  p->reset();
  ++p->blkno;
  return true;
}

// compress `n` bytes into a datum body = rawsize u32 | pglz (or raw if it does not shrink)
static void make_body(const uint8_t* src, int64_t n, std::vector<uint8_t>* body, bool* compressed) {
  body->resize((size_t)n + 4);
  int64_t c = cer_pglz_compress(src, n, body->data() + 4, n - 1);
  if (c > 0 && c + 4 < n) {
    wr32(body->data(), (uint32_t)n);
    body->resize((size_t)c + 4);
    *compressed = true;
  } else {
    std::memcpy(body->data(), src, (size_t)n);
    body->resize((size_t)n);
    *compressed = false;
  }
}

static bool toast_value(DAWriter* w, const std::vector<uint8_t>& body, uint32_t valueid) {
  const int64_t ext = (int64_t)body.size();
  const int64_t nchunks = (ext - 1) / kToastMaxChunk + 1;
  std::vector<uint8_t> item(24 + 8 + 4 + kToastMaxChunk);
  for (int64_t s = 0; s < nchunks; ++s) {
    const int64_t off = s * kToastMaxChunk;
    const int64_t sz = std::min<int64_t>(kToastMaxChunk, ext - off);
    const int64_t len = 24 + 8 + 4 + sz;
    if (!w->tp.fits(len))
      if (!flush_page(&w->toast, &w->tp)) return false;
    tuple_header(item.data(), w->tp.blkno, (uint16_t)(w->tp.nitems() + 1), 3);
    wr32(item.data() + 24, valueid);
    wr32(item.data() + 28, (uint32_t)s);
    wr32(item.data() + 32, htonl((uint32_t)(sz + 4)));  // 4B uncompressed varlena
    std::memcpy(item.data() + 36, body.data() + off, (size_t)sz);
    w->tp.add(item.data(), len);
  }
  return true;
}

extern "C" {

void* cer_da_writer_open(const char* heap_base, const char* toast_base, uint32_t toastrelid,
                         uint32_t first_valueid, int64_t seg_bytes) {
  auto* w = new DAWriter();
  w->heap.base = heap_base;
  w->toast.base = toast_base;
  w->heap.seg_bytes = w->toast.seg_bytes = std::max<int64_t>(seg_bytes / kBlck, 1) * kBlck;
  w->toastrelid = toastrelid;
  w->next_valueid = first_valueid;
  w->hp.reset();
  w->tp.reset();
  if (!w->heap.open_next() || !w->toast.open_next()) {
    delete w;
    return nullptr;
  }
  return w;
}

// Append one packed buffer.  `dep_inline`: store dependent_var inline
// (compressed) when it fits in a heap page, like small one-hot label arrays.
}  // extern "C"

// one tuple from an already built independent_var body (compressed or raw)
static int add_tuple(DAWriter* w, int32_t dist_key, int32_t buffer_id,
                     const std::vector<uint8_t>& ibody, int64_t indep_n, const uint8_t* dep,
                     int64_t dep_n, int dep_inline) {
  std::vector<uint8_t> tup(24 + 4 + kExtPtr + 8 + 4);
  std::vector<uint8_t> dep_datum;
  std::vector<uint8_t> body;
  bool comp = false;
  // independent_var: always external
  const uint32_t v_indep = w->next_valueid++;
  if (!toast_value(w, ibody, v_indep)) return -1;
  uint8_t ptr_indep[kExtPtr] = {0};
  ptr_indep[0] = 0x80;
  ptr_indep[1] = 18;
  wr32(ptr_indep + 4, (uint32_t)(indep_n + 4));
  wr32(ptr_indep + 8, (uint32_t)ibody.size());
  wr32(ptr_indep + 12, v_indep);
  wr32(ptr_indep + 16, w->toastrelid);
  // dependent_var
  make_body(dep, dep_n, &body, &comp);
  const bool inl = dep_inline && comp && (int64_t)body.size() + 4 + 96 < kBlck / 4;
  if (inl) {
    dep_datum.resize(body.size() + 4);
    wr32(dep_datum.data(), htonl((uint32_t)(dep_datum.size()) | 0x40000000u));
    std::memcpy(dep_datum.data() + 4, body.data(), body.size());
  } else {
    const uint32_t v_dep = w->next_valueid++;
    if (!toast_value(w, body, v_dep)) return -1;
    dep_datum.assign(kExtPtr, 0);
    dep_datum[0] = 0x80;
    dep_datum[1] = 18;
    wr32(dep_datum.data() + 4, (uint32_t)(dep_n + 4));
    wr32(dep_datum.data() + 8, (uint32_t)body.size());
    wr32(dep_datum.data() + 12, v_dep);
    wr32(dep_datum.data() + 16, w->toastrelid);
  }
  // heap tuple: header | dist_key | indep ptr | dep | pad to 4 | buffer_id
  int64_t dlen = 4 + kExtPtr + (int64_t)dep_datum.size();
  dlen = (dlen + 3) & ~(int64_t)3;
  const int64_t len = 24 + dlen + 4;
  tup.assign((size_t)len, 0);
  if (!w->hp.fits(len))
    if (!flush_page(&w->heap, &w->hp)) return -1;
  tuple_header(tup.data(), w->hp.blkno, (uint16_t)(w->hp.nitems() + 1), 4);
  wr32(tup.data() + 24, (uint32_t)dist_key);
  std::memcpy(tup.data() + 28, ptr_indep, kExtPtr);
  std::memcpy(tup.data() + 28 + kExtPtr, dep_datum.data(), dep_datum.size());
  wr32(tup.data() + len - 4, (uint32_t)buffer_id);
  w->hp.add(tup.data(), len);
  return 0;
}

extern "C" {

int cer_da_writer_add(void* hw, int32_t dist_key, int32_t buffer_id, const uint8_t* indep,
                      int64_t indep_n, const uint8_t* dep, int64_t dep_n, int dep_inline) {
  std::vector<uint8_t> body;
  bool comp = false;
  make_body(indep, indep_n, &body, &comp);
  return add_tuple(static_cast<DAWriter*>(hw), dist_key, buffer_id, body, indep_n, dep, dep_n,
                   dep_inline);
}

// Append n buffers: their independent_var bodies are pglz-compressed on
// `nthreads` threads (one whole datum per thread, as Greenplum compresses a
// datum in one stream), then the tuples are laid out in order.  A full
// ImageNet-112 partition is ~24 GB of float32 payload: one compressor
// thread writes ~40 MB/s.
int cer_da_writer_add_batch(void* hw, int n, const int32_t* dist_keys, const int32_t* buffer_ids,
                            const uint8_t* const* indep, const int64_t* indep_n,
                            const uint8_t* const* dep, const int64_t* dep_n, int dep_inline,
                            int nthreads) {
  auto* w = static_cast<DAWriter*>(hw);
  std::vector<std::vector<uint8_t>> bodies((size_t)n);
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int i = next++; i < n; i = next++) {
      bool comp = false;
      make_body(indep[i], indep_n[i], &bodies[(size_t)i], &comp);
    }
  };
  const int nt = std::max(1, std::min(nthreads, n));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  for (int i = 0; i < n; ++i) {
    const int rc = add_tuple(w, dist_keys[i], buffer_ids[i], bodies[(size_t)i], indep_n[i],
                             dep[i], dep_n[i], dep_inline);
    std::vector<uint8_t>().swap(bodies[(size_t)i]);
    if (rc != 0) return rc;
  }
  return 0;
}

int cer_da_writer_close(void* hw) {
  auto* w = static_cast<DAWriter*>(hw);
  bool ok = flush_page(&w->heap, &w->hp) && flush_page(&w->toast, &w->tp);
  w->heap.close();
  w->toast.close();
  delete w;
  return ok ? 0 : -1;
}

}  // extern "C"
