// rp_codec.hip — compression::compressor::uncompress on the device
// (compression/compression.cc:34-55):
//   * LZ4 frames: lz4_frame_compressor::uncompress / do_uncompressed
//     (compression/internal/lz4_frame_compressor.cc:115-213) over lz4 1.9.3's
//     LZ4F state machine and LZ4_decompress_safe_usingDict;
//   * snappy: snappy_java_compressor::uncompress
//     (compression/internal/snappy_java_compressor.cc:76-129), falling back to
//     snappy_standard_compressor (compression/snappy_standard_compressor.cc:
//     43-78) over snappy 1.1.8 RawUncompress.
// The control flow is the oracle's (oracle/rp_oracle.c), which restates those
// libraries; every accept/reject decision is kept.
//
// One wave per payload.  Control state (positions, tokens, lengths) is
// uniform; input bytes are read through a 256-byte window held one dword per
// lane (v_readlane), literal and match copies are spread over the 64 lanes.
// A match reads output this wave stored earlier: a workgroup-scope
// release/acquire fence makes those stores visible first, issued only when
// the match source overlaps output written since the last fence.
#include "rp_device.h"
#ifdef RPGPU_CHECKED
#include <cstdio>
#endif

namespace rp {

// ---------------------------------------------------------------------------
// input window
// ---------------------------------------------------------------------------
struct In {
    const uint8_t* src;  // stream start
    int64_t n;           // stream bytes
    int64_t base;        // stream offset of the window start
    uint32_t w;          // this lane's window dword
};

DEV void in_init(In& in, const uint8_t* src, int64_t n) {
    in.src = src;
    in.n = n;
    in.base = -(1ll << 60);
    in.w = 0;
}

DEV void in_load(In& in, int64_t ip) {
    const uintptr_t a = ((uintptr_t)(in.src + ip)) & ~(uintptr_t)3;
    in.base = (int64_t)(a - (uintptr_t)in.src);
    const uintptr_t mine = a + 4u * lane();
    const uintptr_t end = (uintptr_t)(in.src + in.n);
    in.w = mine < end ? *(const uint32_t*)mine : 0u;
}

// byte ip of the stream (uniform ip >= 0; bytes past the stream read as the
// memory that follows it or zero, never faulting)
DEV uint32_t in_byte(In& in, int64_t ip) {
    int64_t o = ip - in.base;
    if (o < 0 || o >= 256) {
        in_load(in, ip);
        o = ip - in.base;
    }
    return (rl(in.w, (int)(o >> 2)) >> (8 * (uint32_t)(o & 3))) & 0xFFu;
}
DEV uint32_t in_le16(In& in, int64_t ip) { return in_byte(in, ip) | (in_byte(in, ip + 1) << 8); }
DEV uint32_t in_le32(In& in, int64_t ip) { return in_le16(in, ip) | (in_le16(in, ip + 2) << 16); }

// ---------------------------------------------------------------------------
// wave-cooperative copies
// ---------------------------------------------------------------------------
DEV void vis_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Loads of output this wave wrote: agent-scope relaxed loads (sc1) skip the
// vector L1, which may hold a copy of the line taken by another wave of the
// CU before these bytes were stored (arena slots and blocks are adjacent;
// the workgroup-scope acquire does not invalidate L1).  The release in
// vis_fence has put the stores in L2 first.
DEV uint32_t ld_out8(const uint8_t* p) {
    return __hip_atomic_load(const_cast<uint8_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint32_t ld_out32(const uint8_t* p) {  // 4 bytes at any address
    const uintptr_t a = (uintptr_t)p;
    uint32_t* q = (uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t hi = sh ? __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Output of one decode: the arena, plus an optional per-wave LDS ring of the
// last kRing output bytes.  Near matches (offset + length <= kRing) read the
// ring: LDS is in order within a wave, so no fence and no round trip through
// L2.  Far matches read the arena behind a fence with L1-bypassing loads.
typedef __attribute__((address_space(3))) uint8_t lds_u8;
#ifndef RPGPU_RING_BYTES
#define RPGPU_RING_BYTES 4096
#endif
constexpr int64_t kRing = RPGPU_RING_BYTES > 0 ? RPGPU_RING_BYTES : 1;  // 0: no ring
constexpr uint32_t kRingWaves = 4;  // waves per workgroup of the decode kernels

struct Out {
    uint8_t* dst;
    lds_u8* ring;    // nullptr: no ring
    int64_t fenced;  // arena bytes below this are visible to loads
};

DEV void out_init(Out& o, uint8_t* dst, lds_u8* ring) {
    o.dst = dst;
    o.ring = ring;
    o.fenced = 0;
}

DEV void put(Out& o, int64_t at, uint32_t v, bool valid) {
    if (valid) {
        o.dst[at] = (uint8_t)v;
        if (o.ring) o.ring[at & (kRing - 1)] = (uint8_t)v;
    }
}

// Bulk copy of bytes this decode does not write (its input) to the output at
// op: bytes up to the destination's 16-byte alignment, then 16 bytes per lane
// (1 KiB per wave store, four stores' loads issued together) assembled from
// aligned dword loads of the source, then the < 16-byte tail.  The ring
// receives the copy's last kRing bytes.  (Byte-per-lane copies moved 64 bytes
// per load round trip: 0.03 B/cycle per wave on stored LZ4 blocks.)
DEV uint4 ld16_any(const uint8_t* s) {
    const uint32_t* q = (const uint32_t*)((uintptr_t)s & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    const uint32_t w4 = sh ? q[4] : 0u;  // holds byte 15 only when the source is unaligned
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

DEV void copy_bulk(Out& o, int64_t op, const uint8_t* src, int64_t len) {
    if (len <= 0) return;
    const int64_t l = (int64_t)lane();
    int64_t head = (int64_t)((16u - ((uintptr_t)(o.dst + op) & 15u)) & 15u);
    if (head > len) head = len;
    if (l < head) put(o, op + l, src[l], true);
    const int64_t mid_end = head + ((len - head) & ~15ll);
    const int64_t ring_from = len - kRing;  // bytes before this never reach the ring
    for (int64_t c = head; c < mid_end; c += 4096) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t k = c + 1024 * u + 16 * l;
            if (k < mid_end) v[u] = ld16_any(src + k);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t k = c + 1024 * u + 16 * l;
            if (k < mid_end) {
                *(uint4*)(o.dst + op + k) = v[u];
                if (o.ring && k + 16 > ring_from) {
                    const int64_t at = op + k;
                    if (((uintptr_t)o.dst & 15u) == 0) {  // ring slot 16-byte aligned as well
                        typedef __attribute__((address_space(3))) uint32_t lds_u32;
                        lds_u32* r = (lds_u32*)(o.ring + (at & (kRing - 1)));
                        r[0] = v[u].x;
                        r[1] = v[u].y;
                        r[2] = v[u].z;
                        r[3] = v[u].w;
                    } else {
                        const uint32_t wv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                        for (int b = 0; b < 16; b++) o.ring[(at + b) & (kRing - 1)] = (uint8_t)(wv[b >> 2] >> (8 * (b & 3)));
                    }
                }
            }
        }
    }
    if (l < len - mid_end) put(o, op + mid_end + l, src[mid_end + l], true);
}

// literals: src[ip, ip + len) -> out[op, ...).  Bytes inside the 256-byte
// input window come from its registers (ds_bpermute), the rest from memory;
// long runs take the bulk copy.
DEV void copy_lit(Out& o, int64_t op, In& in, const uint8_t* src, int64_t ip, int64_t len) {
    if (len <= 0) return;
    if (len >= 256) {
        copy_bulk(o, op, src + ip, len);
        return;
    }
    if (ip < in.base || ip >= in.base + 192) in_load(in, ip);
    for (int64_t c = 0; c < len; c += 64) {
        const int64_t k = c + (int64_t)lane();
        const bool valid = k < len;
        const int64_t w = ip + k - in.base;
        const bool inwin = w >= 0 && w < 256;
        const uint32_t word = (uint32_t)__shfl((int)in.w, (int)((w >> 2) & 63), 64);
        uint32_t v = (word >> (8 * (uint32_t)(w & 3))) & 0xFFu;
        if (valid && !inwin) v = src[ip + k];
        put(o, op + k, v, valid);
    }
}

// raw bytes straight from memory (stored LZ4 blocks)
DEV void copy_raw(Out& o, int64_t op, const uint8_t* src, int64_t ip, int64_t len) { copy_bulk(o, op, src + ip, len); }

// forward copy out[op + k] = out[op + k - off] (k < len): with off < len the
// source repeats with period off; off == 0 writes zeros (as liblz4's
// write32(op, 0) / LZ4_memcpy_using_offset_base produce)
DEV void copy_match(Out& o, int64_t op, int64_t off, int64_t len) {
    if (len <= 0) return;
    if (off == 0) {
        for (int64_t c = 0; c < len; c += 64) put(o, op + c + lane(), 0u, c + (int64_t)lane() < len);
        return;
    }
    const int64_t s0 = op - off;
    if (o.ring && off + len <= kRing) {
        // every source byte is below op and within the ring
        for (int64_t c = 0; c < len; c += 64) {
            const int64_t k = c + (int64_t)lane();
            const bool valid = k < len;
            const int64_t sk = off >= len ? k : (int64_t)((uint32_t)k % (uint32_t)off);
            const uint32_t v = valid ? (uint32_t)o.ring[(s0 + sk) & (kRing - 1)] : 0u;
            put(o, op + k, v, valid);
        }
        return;
    }
    const int64_t span = off < len ? off : len;
    if (s0 + span > o.fenced) {
        vis_fence();
        o.fenced = op;
    }
    for (int64_t c = 0; c < len; c += 64) {
        const int64_t k = c + (int64_t)lane();
        const bool valid = k < len;
        const int64_t sk = off >= len ? k : (int64_t)((uint32_t)k % (uint32_t)off);
        const uint32_t v = valid ? ld_out8(o.dst + s0 + sk) : 0u;
        put(o, op + k, v, valid);
    }
}

// XXH32 (lz4 1.9.3 xxhash.c), uniform over global memory
DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
template <bool OUT>
DEV uint32_t xxh32_t(const uint8_t* p, int64_t n, uint32_t seed);
DEV uint32_t xxh32_dev(const uint8_t* p, int64_t n, uint32_t seed) { return xxh32_t<false>(p, n, seed); }
DEV uint32_t xxh32_out(const uint8_t* p, int64_t n, uint32_t seed) { return xxh32_t<true>(p, n, seed); }

// OUT: p is output this wave (or this kernel) wrote: L1-bypassing loads
template <bool OUT>
DEV uint32_t xxh32_t(const uint8_t* p, int64_t n, uint32_t seed) {
    const uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
    int64_t i = 0;
    uint32_t h;
    if (n >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; i + 16 <= n; i += 16) {
            v1 = rotl32(v1 + (OUT ? ld_out32(p + i) : ldu32(p + i)) * P2, 13) * P1;
            v2 = rotl32(v2 + (OUT ? ld_out32(p + i + 4) : ldu32(p + i + 4)) * P2, 13) * P1;
            v3 = rotl32(v3 + (OUT ? ld_out32(p + i + 8) : ldu32(p + i + 8)) * P2, 13) * P1;
            v4 = rotl32(v4 + (OUT ? ld_out32(p + i + 12) : ldu32(p + i + 12)) * P2, 13) * P1;
        }
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    for (; i + 4 <= n; i += 4) h = rotl32(h + (OUT ? ld_out32(p + i) : ldu32(p + i)) * P3, 17) * P4;
    for (; i < n; i++) h = rotl32(h + (OUT ? ld_out8(p + i) : (uint32_t)p[i]) * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return uni32(h);
}

// ---------------------------------------------------------------------------
// LZ4 block: rpo_lz4_block_decode (oracle) = lz4 1.9.3 LZ4_decompress_generic
// for LZ4_decompress_safe_usingDict (fast loop + safe loop, every check).
// Returns the decoded length or -1.  H = history bytes before dst.
// ---------------------------------------------------------------------------
constexpr int64_t kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12, kFastSafeDistance = 64;

DEV uint32_t lz_read_var(In& in, int64_t& ip, int64_t lencheck, bool loop_check, bool initial_check, int& err) {
    uint32_t length = 0, b;
    err = 0;
    if (initial_check && ip >= lencheck) {
        err = 1;
        return length;
    }
    do {
        b = in_byte(in, ip);
        ip++;
        length += b;
        if (loop_check && ip >= lencheck) {
            err = 2;
            return length;
        }
    } while (b == 255);
    return length;
}

DEV int64_t lz4_block(In& in, const uint8_t* src, int64_t n, Out& o, int64_t obase, int64_t oend, int64_t H) {
    const int64_t iend = n;
    int64_t ip = 0, op = 0;
    const int64_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    uint32_t token;
    int64_t length, offset, cpy;
    int err;

    if (oend == 0) return (n == 1 && in_byte(in, 0) == 0) ? 0 : -1;
    if (n == 0) return -1;

    if (oend - op < kFastSafeDistance) goto safe_decode;
    for (;;) {
        token = in_byte(in, ip++);
        length = token >> 4;
        if (length == 15) {
            length += lz_read_var(in, ip, iend - 15, true, true, err);
            if (err == 1) return -1;
            cpy = op + length;
            if (cpy > oend - 32 || ip + length > iend - 32) goto safe_literal_copy;
            copy_lit(o, obase + op, in, src, ip, length);
            ip += length;
            op = cpy;
        } else {
            cpy = op + length;
            if (ip > iend - (16 + 1)) goto safe_literal_copy;
            copy_lit(o, obase + op, in, src, ip, length);
            ip += length;
            op = cpy;
        }
        offset = in_le16(in, ip);
        ip += 2;
        length = token & 15;
        if (length == 15) {
            if (offset > op + H) return -1;
            length += lz_read_var(in, ip, iend - kLastLiterals + 1, true, false, err);
            if (err) return -1;
            length += kMinMatch;
            if (op + length >= oend - kFastSafeDistance) goto safe_match_copy;
        } else {
            length += kMinMatch;
            if (op + length >= oend - kFastSafeDistance) goto safe_match_copy;
            if (offset <= op + H && offset >= 8) {
                copy_match(o, obase + op, offset, length);
                op += length;
                continue;
            }
        }
        if (offset > op + H) return -1;
        copy_match(o, obase + op, offset, length);
        op += length;
    }

safe_decode:
    for (;;) {
        token = in_byte(in, ip++);
        length = token >> 4;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            copy_lit(o, obase + op, in, src, ip, length);
            op += length;
            ip += length;
            length = token & 15;
            offset = in_le16(in, ip);
            ip += 2;
            if (length != 15 && offset >= 8 && offset <= op + H) {
                copy_match(o, obase + op, offset, length + kMinMatch);
                op += length + kMinMatch;
                continue;
            }
            goto lbl_copy_match;
        }
        if (length == 15) {
            length += lz_read_var(in, ip, iend - 15, true, true, err);
            if (err == 1) return -1;
        }
        cpy = op + length;
    safe_literal_copy:
        if (cpy > oend - kMfLimit || ip + length > iend - (2 + 1 + kLastLiterals)) {
            if (ip + length != iend || cpy > oend) return -1;
            copy_lit(o, obase + op, in, src, ip, length);
            ip += length;
            op += length;
            break;
        }
        copy_lit(o, obase + op, in, src, ip, length);
        ip += length;
        op = cpy;
        offset = in_le16(in, ip);
        ip += 2;
        length = token & 15;
    lbl_copy_match:
        if (length == 15) {
            length += lz_read_var(in, ip, iend - kLastLiterals + 1, true, false, err);
            if (err) return -1;
        }
        length += kMinMatch;
    safe_match_copy:
        if (offset > op + H) return -1;
        if (offset > op) {
            // match starts in the history (prefix / external dictionary)
            if (op + length > oend - kLastLiterals) return -1;
            copy_match(o, obase + op, offset, length);
            op += length;
            continue;
        }
        cpy = op + length;
        if (cpy > oend - kMfLimit) {
            if (cpy > oend - kLastLiterals) return -1;
        }
        copy_match(o, obase + op, offset, length);
        op = cpy;
    }
    return op;
}

// ---------------------------------------------------------------------------
// LZ4 frame: rpo_lz4f_uncompress (oracle) — LZ4F_getFrameInfo + the
// LZ4F_decompress loop of do_uncompressed, including its output-buffer
// estimate (contentSize, or 4x the input; grown 1.5x + 1 KiB whenever a call
// returns with it full), which decides how much of a truncated frame is
// returned.  dst has room for the planned capacity (decode_capacity_dev).
// Returns 0 (out_len set) or -1 where the reference throws.
// ---------------------------------------------------------------------------
DEV int lz4f_decode(In& in, const uint8_t* s, int64_t n, Out& o, int64_t& out_len) {
    out_len = 0;
    if (n < 7) return -1;                                        // frameHeader_incomplete
    const uint32_t magic = in_le32(in, 0);
    int64_t pos;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {                  // skippable frame
        if (n < 8) return -1;
        pos = 4;
        if (n - pos < 4) return 0;
        const uint32_t sz = in_le32(in, pos);
        pos += 4;
        if (n - pos < (int64_t)sz) return 0;
        pos += sz;
        return pos < n ? -1 : 0;
    }
    if (magic != 0x184D2204u) return -1;                         // frameType_unknown
    const uint32_t flg = in_byte(in, 4);
    const int64_t hsize = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
    if (n < hsize) return -1;
    if ((flg >> 1) & 1) return -1;                               // reservedFlag_set
    if (((flg >> 6) & 3) != 1) return -1;                        // headerVersion_wrong
    const uint32_t bd = in_byte(in, 5);
    if ((bd >> 7) & 1) return -1;
    const uint32_t bsid = (bd >> 4) & 7;
    if (bsid < 4) return -1;                                     // maxBlockSize_invalid
    if (bd & 15) return -1;
    if (((xxh32_dev(s + 4, hsize - 5, 0) >> 8) & 0xFFu) != in_byte(in, hsize - 1)) return -1;  // headerChecksum_invalid
    const bool linked = !((flg >> 5) & 1);
    const bool bcs = (flg >> 4) & 1;
    const bool ccs = (flg >> 2) & 1;
    const bool csf = (flg >> 3) & 1;
    const uint64_t content_size = csf ? ((uint64_t)in_le32(in, 6) | ((uint64_t)in_le32(in, 10) << 32)) : 0;
    const int64_t bmax = bsid == 4 ? (64 << 10) : bsid == 5 ? (256 << 10) : bsid == 6 ? (1 << 20) : (4 << 20);
    pos = hsize;
    // compute_frame_uncompressed_size (lz4_frame_compressor.cc:115-121)
    uint64_t est = (content_size == 0 || content_size > (uint64_t)n * 255) ? (uint64_t)n * 4 : content_size;
    uint64_t remaining = content_size;
    int64_t out = 0;
    for (;;) {
        if (n - pos < 4) { out_len = out; return 0; }            // waiting for a block header
        const uint32_t bh = in_le32(in, pos);
        pos += 4;
        if (bh == 0) break;                                      // end mark
        const int64_t bsz = bh & 0x7FFFFFFFu;
        if (bsz > bmax) return -1;                               // maxBlockSize_invalid
        if (bh & 0x80000000u) {
            // dstage_copyDirect: streamed, partial data is emitted
            int64_t left = bsz;
            const int64_t blk = pos;
            for (;;) {
                const int64_t space = (int64_t)(est - (uint64_t)out), avail = n - pos;
                int64_t k = left < avail ? left : avail;
                if (k > space) k = space;
                copy_raw(o, out, s, pos, k);
                out += k;
                pos += k;
                left -= k;
                if (content_size) remaining -= (uint64_t)k;
                if (left == 0) break;
                if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
                if (pos == n) { out_len = out; return 0; }
            }
            if (bcs) {
                if (n - pos < 4) { out_len = out; return 0; }
                if (in_le32(in, pos) != xxh32_dev(s + blk, bsz, 0)) return -1;
                pos += 4;
            }
            continue;
        }
        if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
        if (pos == n) { out_len = out; return 0; }
        const int64_t need = bsz + (bcs ? 4 : 0);
        if (n - pos < need) { out_len = out; return 0; }         // dstage_storeCBlock: wait
        if (bcs && in_le32(in, pos + bsz) != xxh32_dev(s + pos, bsz, 0)) return -1;
        In bin;
        in_init(bin, s + pos, bsz);
        const int64_t d = lz4_block(bin, s + pos, bsz, o, out, bmax, linked ? out : 0);
        if (d < 0) return -1;                                    // decompressionFailed
        pos += need;
        if (content_size) remaining -= (uint64_t)d;
        const int64_t space = (int64_t)(est - (uint64_t)out);
        if (space >= bmax || d <= space) { out += d; continue; }
        // decoded into tmpOut: `space` bytes flushed now, the rest on later
        // calls — which only happen while input remains
        int64_t pending = d - space;
        out += space;
        while (pending) {
            if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
            if (pos == n) { out_len = out; return 0; }
            const int64_t sp = (int64_t)(est - (uint64_t)out), f = pending < sp ? pending : sp;
            out += f;
            pending -= f;
        }
    }
    if (remaining) return -1;                                    // frameSize_wrong
    if (ccs) {
        if (n - pos < 4) { out_len = out; return 0; }
        vis_fence();
        if (in_le32(in, pos) != xxh32_out(o.dst, out, 0)) return -1;
        pos += 4;
    }
    out_len = out;
    return pos < n ? -1 : 0;                                     // input left over: throw
}

// ---------------------------------------------------------------------------
// snappy 1.1.8 (oracle: snappy_varint32 / snappy_decode_tags /
// snappy_raw_checked / rpo_snappy_*_uncompress)
// ---------------------------------------------------------------------------
DEV int snappy_varint_in(In& in, int64_t pos, int64_t n, uint32_t& v, int64_t& used) {
    uint32_t r = 0;
    for (int64_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        const uint32_t b = in_byte(in, pos + i);
        if (i < 4) {
            r |= (b & 127) << (7 * i);
            if (b < 128) { v = r; used = i + 1; return 0; }
        } else {
            r |= (b & 127) << 28;
            if (b < 16) { v = r; used = 5; return 0; }
            return -1;
        }
    }
    return -1;
}

// DecompressAllTags over [ip, n): succeeds iff the tags end exactly at n and
// exactly ulen bytes come out
DEV int snappy_tags(In& in, const uint8_t* s, int64_t n, int64_t ip, Out& o, int64_t obase, int64_t ulen) {
    int64_t op = 0;
    while (ip < n) {
        const uint32_t c = in_byte(in, ip);
        int64_t extra;
        if ((c & 3) == 0) extra = ((c >> 2) >= 60) ? (int64_t)((c >> 2) - 59) : 0;
        else if ((c & 3) == 1) extra = 1;
        else if ((c & 3) == 2) extra = 2;
        else extra = 4;
        if (n - ip < 1 + extra) return -1;
        ip++;
        if ((c & 3) == 0) {
            int64_t lit = (int64_t)(c >> 2) + 1;
            if (lit >= 61) {
                const int64_t ll = lit - 60;
                uint32_t v = 0;
                for (int64_t k = 0; k < ll; k++) v |= in_byte(in, ip + k) << (8 * k);
                lit = (int64_t)v + 1;
                ip += ll;
            }
            if (n - ip < lit) return -1;       // premature end of input
            if (ulen - op < lit) return -1;    // SnappyArrayWriter::Append overflow
            copy_lit(o, obase + op, in, s, ip, lit);
            op += lit;
            ip += lit;
        } else {
            int64_t len, off;
            if ((c & 3) == 1) {
                len = 4 + ((c >> 2) & 7);
                off = ((int64_t)(c >> 5) << 8) | in_byte(in, ip);
            } else if ((c & 3) == 2) {
                len = (int64_t)(c >> 2) + 1;
                off = in_le16(in, ip);
            } else {
                len = (int64_t)(c >> 2) + 1;
                off = in_le32(in, ip);
            }
            ip += extra;
            // AppendFromSelf: Produced() <= offset - 1u || op_end > op_limit_
            if (off == 0 || op < off || ulen - op < len) return -1;
            copy_match(o, obase + op, off, len);
            op += len;
        }
    }
    return op == ulen ? 0 : -1;
}

DEV int snappy_raw_checked(In& in, const uint8_t* s, int64_t n, Out& o, int64_t obase, int64_t& out_len) {
    uint32_t ulen;
    int64_t used;
    if (snappy_varint_in(in, 0, n, ulen, used)) return -1;
    // no tag sequence expands more than 64/3 per input byte
    if ((uint64_t)ulen > 22ull * (uint64_t)n + 64) return -1;
    if (snappy_tags(in, s, n, used, o, obase, ulen)) return -1;
    out_len = ulen;
    return 0;
}

DEV int snappy_raw(In& in, const uint8_t* s, int64_t n, Out& o, int64_t& out_len) {
    uint32_t ulen;
    int64_t used;
    out_len = 0;
    if (snappy_varint_in(in, 0, n, ulen, used)) return -1;
    if (ulen == 0) return 0;  // "empty frame": RawUncompress is not called
    return snappy_raw_checked(in, s, n, o, 0, out_len);
}

DEV int snappy_java(In& in, const uint8_t* s, int64_t n, Out& o, int64_t& out_len) {
    out_len = 0;
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    bool java = n >= 16;
    for (int i = 0; i < 8 && java; i++) java = in_byte(in, i) == magic[i];
    if (!java) return snappy_raw(in, s, n, o, out_len);
    const int32_t min_version = (int32_t)in_le32(in, 12);  // native little endian
    if (min_version < 1) return -1;
    int64_t pos = 16, out = 0;
    while (pos != n) {
        if (n - pos < 4) return -1;                         // consume_be_type out_of_range
        const int32_t clen = (int32_t)((in_byte(in, pos) << 24) | (in_byte(in, pos + 1) << 16) |
                                       (in_byte(in, pos + 2) << 8) | in_byte(in, pos + 3));
        pos += 4;
        if (clen < 0) return -1;
        if (n - pos < (int64_t)clen) return -1;             // consume_to out_of_range
        In cin;
        in_init(cin, s + pos, clen);
        int64_t got = 0;
        if (snappy_raw_checked(cin, s + pos, clen, o, out, got)) return -1;
        out += got;
        pos += clen;
    }
    out_len = out;
    return 0;
}

// compression::compressor::uncompress dispatch (compression/compression.cc:34-55)
DEV int decode_payload(int codec, const uint8_t* s, int64_t n, uint8_t* dst, lds_u8* ring, int64_t& out_len) {
    out_len = 0;
    if (n == 0) return -1;
    In in;
    in_init(in, s, n);
    Out o;
    out_init(o, dst, ring);
    if (codec == RPGPU_CODEC_SNAPPY) return snappy_java(in, s, n, o, out_len);
    if (codec == RPGPU_CODEC_LZ4) return lz4f_decode(in, s, n, o, out_len);
    return -1;
}

// ---------------------------------------------------------------------------
// Block-parallel decode.  A payload whose pieces are independent and whose
// frame is structurally complete decodes to the concatenation of its pieces
// (or fails when any piece fails): that is the sequential decoder's result
// for such frames, since every flush of do_uncompressed happens while input
// remains.  Those frames are split into BlockItems at the plan rule's
// positions (decode_capacity_dev); everything else (linked LZ4 blocks,
// truncated or malformed frames, raw snappy) takes the sequential path.
// ---------------------------------------------------------------------------

// reserve `nb` items (wave-uniform); UINT32_MAX when the list is full
DEV uint32_t reserve_blocks(const DeviceJob& j, uint32_t nb) {
    uint32_t first = 0;
    if (lane() == 0) first = atomicAdd(&j.counters[4], nb);
    first = rl(first, 0);
    return ((uint64_t)first + nb <= j.block_capacity) ? first : 0xFFFFFFFFu;
}

// LZ4F frame of independent blocks (lz4_frame_compressor.cc:115-200 over
// lz4 1.9.3): returns true and fills the plan when eligible
DEV bool plan_lz4f(const DeviceJob& j, In& in, int64_t n, uint64_t src_abs, uint64_t dst_abs, FramePlan& fp) {
    if (n < 7) return false;
    if (in_le32(in, 0) != 0x184D2204u) return false;
    const uint32_t flg = in_byte(in, 4);
    const int64_t hsize = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
    if (n < hsize || ((flg >> 1) & 1) || ((flg >> 6) & 3) != 1) return false;
    if (!((flg >> 5) & 1)) return false;  // linked blocks: sequential
    const uint32_t bd = in_byte(in, 5);
    const uint32_t bsid = (bd >> 4) & 7;
    if (((bd >> 7) & 1) || bsid < 4 || (bd & 15)) return false;
    if (((xxh32_dev(in.src + 4, hsize - 5, 0) >> 8) & 0xFFu) != in_byte(in, hsize - 1)) return false;
    const bool bcs = (flg >> 4) & 1, ccs = (flg >> 2) & 1, csf = (flg >> 3) & 1;
    const int64_t bmax = bsid == 4 ? (64 << 10) : bsid == 5 ? (256 << 10) : bsid == 6 ? (1 << 20) : (4 << 20);
    // structure: every block present, the end mark, the content checksum,
    // and nothing after it
    int64_t pos = hsize;
    uint32_t nb = 0;
    bool end = false;
    while (n - pos >= 4) {
        const uint32_t bh = in_le32(in, pos);
        pos += 4;
        if (bh == 0) { end = true; break; }
        const int64_t bsz = bh & 0x7FFFFFFFu;
        if (bsz > bmax) return false;
        const int64_t need = bsz + (bcs ? 4 : 0);
        if (n - pos < need) return false;
        pos += need;
        nb++;
    }
    if (!end) return false;
    uint32_t ccs_val = 0;
    if (ccs) {
        if (n - pos < 4) return false;
        ccs_val = in_le32(in, pos);
        pos += 4;
    }
    if (pos != n || nb == 0) return false;
    const uint32_t first = reserve_blocks(j, nb);
    if (first == 0xFFFFFFFFu) return false;
    pos = hsize;
    uint64_t plan = 0;
    for (uint32_t k = 0; k < nb; k++) {
        const uint32_t bh = in_le32(in, pos);
        const int64_t bsz = bh & 0x7FFFFFFFu;
        const bool raw = (bh & 0x80000000u) != 0;
        if (lane() == 0) {
            BlockItem it;
            it.src = src_abs + (uint64_t)pos + 4;
            it.dst = dst_abs + plan;
            it.csize = (uint32_t)bsz;
            it.kind = (raw ? kBlkRaw : 0u) | (bcs ? kBlkChecksum : 0u);
            it.out = -1;
            it.cap = raw ? (uint32_t)bsz : (uint32_t)bmax;
            j.blocks[first + k] = it;
        }
        plan += raw ? (uint64_t)bsz : (uint64_t)bmax;
        pos += 4 + bsz + (bcs ? 4 : 0);
    }
    fp.mode = 1;
    fp.first = first;
    fp.nb = nb;
    fp.ccs = ccs;
    fp.ccs_val = ccs_val;
    fp.csf = csf;
    fp.content_size = csf ? ((uint64_t)in_le32(in, 6) | ((uint64_t)in_le32(in, 10) << 32)) : 0;
    return true;
}

// snappy-java stream (snappy_java_compressor.cc:76-129): chunks are
// independent raw snappy blocks at exact offsets (their length varints)
DEV bool plan_snappy_java(const DeviceJob& j, In& in, int64_t n, uint64_t src_abs, uint64_t dst_abs, FramePlan& fp) {
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    if (n < 16) return false;
    for (int i = 0; i < 8; i++)
        if (in_byte(in, i) != magic[i]) return false;
    if ((int32_t)in_le32(in, 12) < 1) return false;
    int64_t pos = 16;
    uint32_t nb = 0;
    while (pos != n) {
        if (n - pos < 4) return false;
        const int32_t clen = (int32_t)((in_byte(in, pos) << 24) | (in_byte(in, pos + 1) << 16) |
                                       (in_byte(in, pos + 2) << 8) | in_byte(in, pos + 3));
        pos += 4;
        if (clen < 0 || n - pos < (int64_t)clen) return false;
        uint32_t ulen;
        int64_t used;
        if (snappy_varint_in(in, pos, clen, ulen, used)) return false;
        if ((uint64_t)ulen > 22ull * (uint64_t)clen + 64) return false;
        pos += clen;
        nb++;
    }
    if (nb == 0) return false;
    const uint32_t first = reserve_blocks(j, nb);
    if (first == 0xFFFFFFFFu) return false;
    pos = 16;
    uint64_t plan = 0;
    for (uint32_t k = 0; k < nb; k++) {
        const int32_t clen = (int32_t)((in_byte(in, pos) << 24) | (in_byte(in, pos + 1) << 16) |
                                       (in_byte(in, pos + 2) << 8) | in_byte(in, pos + 3));
        pos += 4;
        uint32_t ulen;
        int64_t used;
        snappy_varint_in(in, pos, clen, ulen, used);
        if (lane() == 0) {
            BlockItem it;
            it.src = src_abs + (uint64_t)pos;
            it.dst = dst_abs + plan;
            it.csize = (uint32_t)clen;
            it.kind = kBlkSnappy;
            it.out = -1;
            it.cap = ulen;
            j.blocks[first + k] = it;
        }
        plan += ulen;
        pos += clen;
    }
    fp.mode = 2;
    fp.first = first;
    fp.nb = nb;
    fp.ccs = 0;
    fp.ccs_val = 0;
    fp.csf = 0;
    fp.content_size = 0;
    return true;
}

// ---------------------------------------------------------------------------
// k_decode: one wave per compressed batch of the job (work list built by
// k_emit), claimed dynamically.  Block-parallel frames are only planned here;
// the rest are decoded on the spot.  Each item writes only its own batch
// result, its own plan and its own planned arena slot.
// ---------------------------------------------------------------------------
#if RPGPU_RING_BYTES > 0
#define RP_WAVE_RING(name)                              \
    __shared__ uint8_t name##_lds[kRingWaves * kRing]; \
    lds_u8* name = (lds_u8*)(name##_lds + (threadIdx.x >> 6) * kRing)
#else
#define RP_WAVE_RING(name) lds_u8* name = nullptr
#endif

__global__ __launch_bounds__(256) void k_decode(DeviceJob j) {
    RP_WAVE_RING(ring);
    const uint32_t count = j.counters[2];
    for (;;) {
        uint32_t item = 0;
        if (lane() == 0) item = atomicAdd(&j.counters[3], 1u);
        item = rl(item, 0);
        if (item >= count) break;
        const uint64_t b = j.decode_list[item];
        rpgpu_batch_result* R = &j.batches[b];
        const uint32_t seg = uni32(R->segment);
        const uint64_t S = uni64(j.seg_off[seg]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
        const int64_t n = (int64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
        const int codec = (int)(uni32((uint32_t)(uint16_t)R->attrs) & 7u);
        const uint64_t doff = uni64(j.dcap[b]);
        const uint64_t cap = uni64(j.dcap[b + 1]) - doff;
        uint32_t addf = 0, dl = 0;
        FramePlan fp;
        fp.mode = 0;
        if (doff + cap > j.decoded_capacity) {
            addf = RPGPU_F_DECODE_OVERFLOW;
        } else {
            In in;
            in_init(in, j.data + S, n);
            bool planned = false;
            if (n > 0 && j.block_capacity) {
                if (codec == RPGPU_CODEC_LZ4) planned = plan_lz4f(j, in, n, S, doff, fp);
                else if (codec == RPGPU_CODEC_SNAPPY) planned = plan_snappy_java(j, in, n, S, doff, fp);
            }
            if (!planned) {
                fp.mode = 0;
                int64_t got = 0;
                if (decode_payload(codec, j.data + S, n, j.decoded + doff, ring, got) == 0) {
                    addf = RPGPU_F_CODEC_OK;
                    dl = (uint32_t)got;
                }
            }
        }
        if (lane() == 0) {
            if (j.block_capacity) j.plans[item] = fp;
            if (addf) {
                R->flags = R->flags | addf;
                if (addf & RPGPU_F_CODEC_OK) R->decoded_len = dl;
            }
        }
    }
}

// one wave per BlockItem, wave-strided (a dynamic lane-0 atomic claim here
// compiled to a loop that never terminated on gfx950)
__global__ __launch_bounds__(256) void k_decode_blocks(DeviceJob j) {
    RP_WAVE_RING(ring);
    const uint32_t reserved = j.counters[4];
    const uint32_t count = reserved < j.block_capacity ? reserved : j.block_capacity;
#ifdef RPGPU_CHECKED
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) printf("RPGPU_CHECK blocks reserved=%u cap=%u\n", reserved, j.block_capacity);
#endif
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6); item < count; item += nw) {
#ifdef RPGPU_CHECKED
        if (__builtin_amdgcn_s_memtime() - t_start > 20000000000ull) {
            if (lane() == 0) printf("RPGPU_CHECK blocks timeout at item %u\n", item);
            break;
        }
#endif
        const BlockItem it = j.blocks[item];
        const uint64_t srcp = uni64(it.src), dstp = uni64(it.dst);
        const uint32_t csize = uni32(it.csize), kind = uni32(it.kind), bcap = uni32(it.cap);
#ifdef RPGPU_CHECKED
        if (lane() == 0)
            printf("RPGPU_CHECK block %u src=%llu dst=%llu csize=%u kind=%u cap=%u dlen=%llu dcap=%llu\n", item,
                   (unsigned long long)srcp, (unsigned long long)dstp, csize, kind, bcap,
                   (unsigned long long)j.data_len, (unsigned long long)j.decoded_capacity);
#endif
        const uint8_t* src = j.data + srcp;
        uint8_t* dst = j.decoded + dstp;
        int64_t out = -1;
        In in;
        in_init(in, src, csize);
        Out o;
        out_init(o, dst, ring);
        if (kind & kBlkSnappy) {
            int64_t got = 0;
            if (snappy_raw_checked(in, src, csize, o, 0, got) == 0) out = got;
        } else {
            // dstage_getBlockChecksum before the block is used
            bool ok = true;
            if (kind & kBlkChecksum) {
                In cin;
                in_init(cin, src + csize, 4);
                ok = in_le32(cin, 0) == xxh32_dev(src, csize, 0);
            }
            if (ok) {
                if (kind & kBlkRaw) {
                    copy_raw(o, 0, src, 0, csize);
                    out = csize;
                } else {
                    out = lz4_block(in, src, csize, o, 0, bcap, 0);
                }
            }
        }
        if (lane() == 0) j.blocks[item].out = (int32_t)(out < 0 ? -1 : out);
    }
}

// one wave per block-parallel frame: all pieces decoded, moved together
// when an earlier one came out short, content size / checksum checked
__global__ __launch_bounds__(256) void k_decode_finish(DeviceJob j) {
    const uint32_t count = j.counters[2];
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6); item < count; item += nw) {
        const FramePlan fp = j.plans[item];
        if (uni32(fp.mode) == 0) continue;
        const uint32_t first = uni32(fp.first), nb = uni32(fp.nb);
        const uint64_t b = j.decode_list[item];
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t d0 = uni64(j.dcap[b]);
        bool ok = true;
        uint64_t run = d0;  // where the next piece belongs
        for (uint32_t k = 0; k < nb; k++) {
            const BlockItem it = j.blocks[first + k];
            const int32_t out = (int32_t)uni32((uint32_t)it.out);
            if (out < 0) { ok = false; break; }
            const uint64_t at = uni64(it.dst);
            if (at != run) {
                // forward move to a lower address, 64 bytes per step: each
                // step loads before it stores
                uint8_t* d = j.decoded;
                for (int64_t o = 0; o < out; o += 64) {
                    const int64_t k2 = o + lane();
                    uint8_t v = 0;
                    if (k2 < out) v = (uint8_t)ld_out8(d + at + k2);
                    __builtin_amdgcn_s_waitcnt(0);
                    if (k2 < out) d[run + k2] = v;
                }
            }
            run += (uint64_t)out;
        }
        const uint64_t total = run - d0;
        if (ok && uni32(fp.mode) == 1) {
            if (uni32(fp.csf) && total != uni64(fp.content_size)) ok = false;  // frameSize_wrong
            if (ok && uni32(fp.ccs)) {
                vis_fence();
                if (xxh32_out(j.decoded + d0, (int64_t)total, 0) != uni32(fp.ccs_val)) ok = false;
            }
        }
        if (lane() == 0 && ok) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
        }
    }
}

__global__ __launch_bounds__(64) void k_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst,
                                                       int64_t* res) {
    RP_WAVE_RING(ring);
    int64_t got = 0;
    const int rc = decode_payload(codec, src, (int64_t)n, dst, ring, got);
    if (lane() == 0) {
        res[0] = rc;
        res[1] = got;
    }
}

hipError_t launch_decode(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_decode_blocks(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    if (j.block_capacity) hipLaunchKernelGGL(k_decode_blocks, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_decode_finish(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    if (j.block_capacity) hipLaunchKernelGGL(k_decode_finish, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, int64_t* res,
                                 hipStream_t s) {
    (void)cap;
    hipLaunchKernelGGL(k_uncompress_one, dim3(1), dim3(64), 0, s, codec, src, n, dst, res);
    return hipGetLastError();
}

}  // namespace rp
