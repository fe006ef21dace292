// PostgreSQL LZ (pglz) codec — compressor and decompressor.
//
// Format (what the reference decodes in Python, cerebro_gpdb/pg_page_reader.py
// :191-231, and in its unused C, pg_lzcompress.c:49-143): a control byte
// announces 8 items, LSB first; bit 1 = back-reference of 2 or 3 bytes
//   b0 = ((off >> 4) & 0xf0) | (len - 3)   (len - 3 in 0..14)
//   b0 = ((off >> 4) & 0xf0) | 0x0f, b2 = len - 18   (len 18 .. 273)
//   b1 = off & 0xff,  off in 1..4095
// bit 0 = one literal byte.  References may overlap their output (RLE).
//
// The decompressor is the hot path of Direct-Access ETL (83 525 s at 1 worker
// in the reference, pure Python); it runs here as a tight native loop, one
// value per thread (values are independent; a value is inherently serial).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "da.h"

namespace {

constexpr int kMaxOff = 4095;
constexpr int kMinMatch = 3;
constexpr int kMaxMatch = 273;
constexpr int kHashBits = 13;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kChainDepth = 16;

inline uint32_t hash3(const uint8_t* p) {
  uint32_t v = (uint32_t)p[0] << 16 | (uint32_t)p[1] << 8 | p[2];
  return (v * 2654435761u) >> (32 - kHashBits);
}

}  // namespace

// Returns the number of compressed bytes written to dst, or -1 if the output
// would not fit in `cap` (the caller then stores the value uncompressed).
extern "C" int64_t cer_pglz_compress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  if (n <= 0) return 0;
  std::vector<int32_t> head(kHashSize, -1);
  std::vector<int32_t> prev((size_t)n, -1);
  int64_t sp = 0, dp = 0;
  int64_t ctrl_pos = -1;
  int ctrl_bit = 8;
  auto emit_ctrl_slot = [&](bool match) -> bool {
    if (ctrl_bit == 8) {
      if (dp >= cap) return false;
      ctrl_pos = dp++;
      dst[ctrl_pos] = 0;
      ctrl_bit = 0;
    }
    if (match) dst[ctrl_pos] |= (uint8_t)(1u << ctrl_bit);
    ++ctrl_bit;
    return true;
  };
  auto insert = [&](int64_t pos) {
    if (pos + 2 < n) {
      uint32_t h = hash3(src + pos);
      prev[pos] = head[h];
      head[h] = (int32_t)pos;
    }
  };
  while (sp < n) {
    int best_len = 0, best_off = 0;
    if (sp + kMinMatch <= n) {
      uint32_t h = hash3(src + sp);
      int32_t cand = head[h];
      int depth = 0;
      const int64_t max_len = std::min<int64_t>(kMaxMatch, n - sp);
      while (cand >= 0 && depth < kChainDepth && sp - cand <= kMaxOff) {
        int len = 0;
        while (len < max_len && src[cand + len] == src[sp + len]) ++len;
        if (len > best_len) {
          best_len = len;
          best_off = (int)(sp - cand);
          if (len == max_len) break;
        }
        cand = prev[cand];
        ++depth;
      }
    }
    if (best_len >= kMinMatch) {
      if (!emit_ctrl_slot(true)) return -1;
      if (best_len >= 18) {
        if (dp + 3 > cap) return -1;
        dst[dp++] = (uint8_t)(((best_off >> 4) & 0xf0) | 0x0f);
        dst[dp++] = (uint8_t)(best_off & 0xff);
        dst[dp++] = (uint8_t)(best_len - 18);
      } else {
        if (dp + 2 > cap) return -1;
        dst[dp++] = (uint8_t)(((best_off >> 4) & 0xf0) | (best_len - 3));
        dst[dp++] = (uint8_t)(best_off & 0xff);
      }
      for (int i = 0; i < best_len; ++i) insert(sp + i);
      sp += best_len;
    } else {
      if (!emit_ctrl_slot(false)) return -1;
      if (dp >= cap) return -1;
      dst[dp++] = src[sp];
      insert(sp);
      ++sp;
    }
  }
  return dp;
}

// Decompress `srclen` bytes of pglz data (WITHOUT the 8-byte varlena+rawsize
// header) into exactly `rawsize` bytes.  Returns rawsize, or -1 if corrupt
// (output overrun / underrun or input not fully consumed — the reference's
// end-of-stream corruption check).
namespace {

constexpr int64_t kGroupIn = 1 + 8 * 3;              // input bytes of one control group, at most
constexpr int64_t kGroupOut = 8 * kMaxMatch + 16;    // output bytes (+ copy overshoot), at most

// One control group with no bounds checks: the caller guarantees kGroupIn
// input bytes at sp and kGroupOut output bytes at dp.  An all-literal group
// is one 8-byte copy; a back-reference copies in 16- / 8-byte steps (the
// overshoot stays inside the slack) unless it overlaps closer than 8 bytes
// (byte loop: run-length).  False: a reference before the start of dst.
inline bool group_fast(const uint8_t*& sp, uint8_t*& dp, const uint8_t* dst) {
  uint8_t ctrl = *sp++;
  if (ctrl == 0) {
    std::memcpy(dp, sp, 8);
    dp += 8;
    sp += 8;
    return true;
  }
  for (int k = 0; k < 8; ++k, ctrl >>= 1) {
    if (ctrl & 1) {
      int32_t len = (sp[0] & 0x0f) + 3;
      const int32_t off = ((sp[0] & 0xf0) << 4) | sp[1];
      sp += 2;
      if (len == 18) len += *sp++;
      if (off == 0 || off > dp - dst) return false;
      const uint8_t* from = dp - off;
      if (off >= 16) {
        for (int32_t i = 0; i < len; i += 16) std::memcpy(dp + i, from + i, 16);
      } else if (off >= 8) {
        for (int32_t i = 0; i < len; i += 8) std::memcpy(dp + i, from + i, 8);
      } else {
        for (int32_t i = 0; i < len; ++i) dp[i] = from[i];
      }
      dp += len;
    } else {
      *dp++ = *sp++;
    }
  }
  return true;
}

// every item checked; continues a stream whose output so far is [dst, dp)
int64_t decode_checked(const uint8_t* sp, const uint8_t* srcend, const uint8_t* dst, uint8_t* dp,
                       uint8_t* destend) {
  while (sp < srcend && dp < destend) {
    uint8_t ctrl = *sp++;
    for (int ctrlc = 0; ctrlc < 8 && sp < srcend; ++ctrlc) {
      if (ctrl & 1) {
        if (sp + 1 >= srcend) return -1;
        int32_t len = (sp[0] & 0x0f) + 3;
        int32_t off = ((sp[0] & 0xf0) << 4) | sp[1];
        sp += 2;
        if (len == 18) {
          if (sp >= srcend) return -1;
          len += *sp++;
        }
        if (off == 0 || off > dp - dst) return -1;
        if (dp + len > destend) return -1;
        const uint8_t* from = dp - off;
        if (off >= len) {
          std::memcpy(dp, from, (size_t)len);
          dp += len;
        } else {
          while (len--) *dp++ = *from++;  // overlapping copy (run-length)
        }
      } else {
        if (dp >= destend) return -1;
        *dp++ = *sp++;
      }
      ctrl >>= 1;
    }
  }
  if (dp != destend || sp != srcend) return -1;
  return destend - dst;
}

}  // namespace

extern "C" int64_t cer_pglz_decompress(const uint8_t* src, int64_t srclen, uint8_t* dst,
                                       int64_t rawsize) {
  const uint8_t* sp = src;
  const uint8_t* const srcend = src + srclen;
  uint8_t* dp = dst;
  uint8_t* const destend = dst + rawsize;
  // fast path while a whole control group cannot run past either buffer
  while (srcend - sp >= kGroupIn && destend - dp >= kGroupOut)
    if (!group_fast(sp, dp, dst)) return -1;
  return decode_checked(sp, srcend, dst, dp, destend) < 0 ? -1 : rawsize;
}

// Decompress a pglz stream stored in pieces (the TOAST chunks of a value, in
// order) without first copying them into one buffer: ptrs[i] / lens[i] are
// the pieces, the stream starts `skip` bytes into piece 0.  A control group
// that straddles a piece boundary is decoded from a small stitch buffer; the
// last bytes (within a group of the end of the input or output) go through
// the checked decoder.  Same result and corruption checks as
// cer_pglz_decompress on the concatenated pieces.
extern "C" int64_t cer_pglz_decompress_pieces(const uint8_t* const* ptrs, const int64_t* lens,
                                              int n, int64_t skip, uint8_t* dst,
                                              int64_t rawsize) {
  if (n <= 0) return rawsize == 0 ? 0 : -1;
  int si = 0;
  while (si < n && skip >= lens[si]) skip -= lens[si++];
  if (si >= n) return rawsize == 0 ? 0 : -1;
  const uint8_t* sp = ptrs[si] + skip;
  const uint8_t* se = ptrs[si] + lens[si];
  uint8_t* dp = dst;
  uint8_t* const destend = dst + rawsize;
  uint8_t stitch[2 * kGroupIn];
  while (destend - dp >= kGroupOut) {
    if (se - sp >= kGroupIn) {
      if (!group_fast(sp, dp, dst)) return -1;
      continue;
    }
    // the group straddles the end of piece si: stitch its tail with the
    // next pieces' head
    const int64_t r = se - sp;
    std::memcpy(stitch, sp, (size_t)r);
    int64_t m = r;
    int sj = si + 1;
    int64_t oj = 0;
    while (m < kGroupIn && sj < n) {
      const int64_t take = std::min<int64_t>(kGroupIn - m, lens[sj] - oj);
      std::memcpy(stitch + m, ptrs[sj] + oj, (size_t)take);
      m += take;
      oj += take;
      if (oj == lens[sj]) {
        ++sj;
        oj = 0;
      }
    }
    if (m < kGroupIn) break;                     // near the end of the input
    const uint8_t* q = stitch;
    if (!group_fast(q, dp, dst)) return -1;
    int64_t c = q - stitch;
    if (c < r) {
      sp += c;
      continue;
    }
    c -= r;                                      // bytes consumed past piece si
    ++si;
    while (si < n && c >= lens[si]) c -= lens[si++];
    if (si >= n) {
      sp = se = nullptr;
      break;
    }
    sp = ptrs[si] + c;
    se = ptrs[si] + lens[si];
  }
  // the rest (bounded: within one group of the end of the output or input)
  std::vector<uint8_t> rest;
  if (sp) {
    rest.insert(rest.end(), sp, se);
    for (int j = si + 1; j < n; ++j) rest.insert(rest.end(), ptrs[j], ptrs[j] + lens[j]);
  }
  return decode_checked(rest.data(), rest.data() + rest.size(), dst, dp, destend) < 0 ? -1
                                                                                     : rawsize;
}
