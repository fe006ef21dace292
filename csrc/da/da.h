// Direct-Access (DA) reader for Greenplum/PostgreSQL heap + TOAST segment
// files, and a writer producing the same format (synthetic DA partitions).
//
// On-disk format, as the reference reads it (cerebro_gpdb/pg_page_reader.py):
//  * pages of BLCKSZ = 32768 bytes; 1-GB segment files relfilenode, .1, .2 ...
//  * page header 24 B: pd_lsn u64, pd_tli u16, pd_flags u16, pd_lower u16,
//    pd_upper u16, pd_special u16, pd_pagesize_version u16, pd_prune_xid u32
//  * line pointers (4 B) from byte 24 to pd_lower: lp_off:15 | lp_flags:2 | lp_len:15
//    (LSB first)
//  * heap tuple header 23 B (xmin, xmax, field3, ctid(3 x u16), infomask2,
//    infomask, t_hoff u8); user data at t_hoff (MAXALIGNed)
//  * packed-table tuple data: __dist_key__ int4 | independent_var TOAST
//    pointer (20 B: 0x80 1B_E header, tag, 2 pad, va_rawsize, va_extsize,
//    va_valueid, va_toastrelid) | dependent_var pointer or inline compressed
//    varlena | buffer_id int4 (last 4 bytes)
//  * varlena headers are big-endian (ntohl): 4B uncompressed 0x00.., 4B
//    compressed 0x40.., 1B external 0x80
//  * compressed datum = 4B_C header | rawsize u32 | pglz stream
//  * TOAST tuple: chunk_id u32 | chunk_seq u32 | 4B varlena chunk (<= 8140 B),
//    items packed upward from pd_upper with MAXALIGN between them
#pragma once
#include <cstdint>

extern "C" {
int64_t cer_pglz_compress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t cer_pglz_decompress(const uint8_t* src, int64_t srclen, uint8_t* dst, int64_t rawsize);
int64_t cer_pglz_decompress_pieces(const uint8_t* const* ptrs, const int64_t* lens, int n,
                                   int64_t skip, uint8_t* dst, int64_t rawsize);
}

namespace da {
constexpr int kBlck = 32768;
constexpr int kPageHeader = 24;
constexpr int kItemId = 4;
constexpr int kTupleHeader = 23;
constexpr int kMaxAlign = 8;
constexpr int kToastMaxChunk = 8140;
constexpr int kExtPtr = 20;

inline int64_t maxalign(int64_t x) { return (x + kMaxAlign - 1) & ~(int64_t)(kMaxAlign - 1); }
}  // namespace da
