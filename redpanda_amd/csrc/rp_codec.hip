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

DEV void copy_lit(uint8_t* dst, int64_t op, const uint8_t* src, int64_t ip, int64_t len) {
    for (int64_t k = lane(); k < len; k += 64) dst[op + k] = src[ip + k];
}

// forward copy dst[op + k] = dst[op + k - off] (k < len): with off < len the
// source repeats with period off; off == 0 writes zeros (as liblz4's
// write32(op, 0) / LZ4_memcpy_using_offset_base produce).  `fenced`: output
// positions below it are visible to loads.
DEV void copy_match(uint8_t* dst, int64_t op, int64_t off, int64_t len, int64_t& fenced) {
    if (len <= 0) return;
    if (off == 0) {
        for (int64_t k = lane(); k < len; k += 64) dst[op + k] = 0;
        return;
    }
    const int64_t s0 = op - off;
    const int64_t span = off < len ? off : len;
    if (s0 + span > fenced) {
        vis_fence();
        fenced = op;
    }
    if (off >= len) {
        for (int64_t k = lane(); k < len; k += 64) dst[op + k] = dst[s0 + k];
    } else {
        const uint32_t uo = (uint32_t)off;
        for (int64_t k = lane(); k < len; k += 64) dst[op + k] = dst[s0 + (int64_t)((uint32_t)k % uo)];
    }
}

// XXH32 (lz4 1.9.3 xxhash.c), uniform over global memory
DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
DEV uint32_t xxh32_dev(const uint8_t* p, int64_t n, uint32_t seed) {
    const uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
    int64_t i = 0;
    uint32_t h;
    if (n >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; i + 16 <= n; i += 16) {
            v1 = rotl32(v1 + ldu32(p + i) * P2, 13) * P1;
            v2 = rotl32(v2 + ldu32(p + i + 4) * P2, 13) * P1;
            v3 = rotl32(v3 + ldu32(p + i + 8) * P2, 13) * P1;
            v4 = rotl32(v4 + ldu32(p + i + 12) * P2, 13) * P1;
        }
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    for (; i + 4 <= n; i += 4) h = rotl32(h + ldu32(p + i) * P3, 17) * P4;
    for (; i < n; i++) h = rotl32(h + p[i] * P5, 11) * P1;
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

DEV int64_t lz4_block(In& in, const uint8_t* src, int64_t n, uint8_t* dst, int64_t oend, int64_t H, int64_t& fenced) {
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
            copy_lit(dst, op, src, ip, length);
            ip += length;
            op = cpy;
        } else {
            cpy = op + length;
            if (ip > iend - (16 + 1)) goto safe_literal_copy;
            copy_lit(dst, op, src, ip, length);
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
                copy_match(dst, op, offset, length, fenced);
                op += length;
                continue;
            }
        }
        if (offset > op + H) return -1;
        copy_match(dst, op, offset, length, fenced);
        op += length;
    }

safe_decode:
    for (;;) {
        token = in_byte(in, ip++);
        length = token >> 4;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            copy_lit(dst, op, src, ip, length);
            op += length;
            ip += length;
            length = token & 15;
            offset = in_le16(in, ip);
            ip += 2;
            if (length != 15 && offset >= 8 && offset <= op + H) {
                copy_match(dst, op, offset, length + kMinMatch, fenced);
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
            copy_lit(dst, op, src, ip, length);
            ip += length;
            op += length;
            break;
        }
        copy_lit(dst, op, src, ip, length);
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
            copy_match(dst, op, offset, length, fenced);
            op += length;
            continue;
        }
        cpy = op + length;
        if (cpy > oend - kMfLimit) {
            if (cpy > oend - kLastLiterals) return -1;
        }
        copy_match(dst, op, offset, length, fenced);
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
DEV int lz4f_decode(In& in, const uint8_t* s, int64_t n, uint8_t* dst, int64_t& out_len) {
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
    int64_t fenced = 0;
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
                copy_lit(dst, out, s, pos, k);
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
        // earlier blocks (the linked history) must be visible to matches
        vis_fence();
        fenced = 0;
        In bin;
        in_init(bin, s + pos, bsz);
        const int64_t d = lz4_block(bin, s + pos, bsz, dst + out, bmax, linked ? out : 0, fenced);
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
        if (in_le32(in, pos) != xxh32_dev(dst, out, 0)) return -1;
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
DEV int snappy_tags(In& in, const uint8_t* s, int64_t n, int64_t ip, uint8_t* dst, int64_t ulen) {
    int64_t op = 0, fenced = 0;
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
            copy_lit(dst, op, s, ip, lit);
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
            copy_match(dst, op, off, len, fenced);
            op += len;
        }
    }
    return op == ulen ? 0 : -1;
}

DEV int snappy_raw_checked(In& in, const uint8_t* s, int64_t n, uint8_t* dst, int64_t& out_len) {
    uint32_t ulen;
    int64_t used;
    if (snappy_varint_in(in, 0, n, ulen, used)) return -1;
    // no tag sequence expands more than 64/3 per input byte
    if ((uint64_t)ulen > 22ull * (uint64_t)n + 64) return -1;
    if (snappy_tags(in, s, n, used, dst, ulen)) return -1;
    out_len = ulen;
    return 0;
}

DEV int snappy_raw(In& in, const uint8_t* s, int64_t n, uint8_t* dst, int64_t& out_len) {
    uint32_t ulen;
    int64_t used;
    out_len = 0;
    if (snappy_varint_in(in, 0, n, ulen, used)) return -1;
    if (ulen == 0) return 0;  // "empty frame": RawUncompress is not called
    return snappy_raw_checked(in, s, n, dst, out_len);
}

DEV int snappy_java(In& in, const uint8_t* s, int64_t n, uint8_t* dst, int64_t& out_len) {
    out_len = 0;
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    bool java = n >= 16;
    for (int i = 0; i < 8 && java; i++) java = in_byte(in, i) == magic[i];
    if (!java) return snappy_raw(in, s, n, dst, out_len);
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
        if (snappy_raw_checked(cin, s + pos, clen, dst + out, got)) return -1;
        out += got;
        pos += clen;
    }
    out_len = out;
    return 0;
}

// compression::compressor::uncompress dispatch (compression/compression.cc:34-55)
DEV int decode_payload(int codec, const uint8_t* s, int64_t n, uint8_t* dst, int64_t& out_len) {
    out_len = 0;
    if (n == 0) return -1;
    In in;
    in_init(in, s, n);
    if (codec == RPGPU_CODEC_SNAPPY) return snappy_java(in, s, n, dst, out_len);
    if (codec == RPGPU_CODEC_LZ4) return lz4f_decode(in, s, n, dst, out_len);
    return -1;
}

// ---------------------------------------------------------------------------
// k_decode: one wave per compressed batch of the job (work list built by
// k_emit), claimed dynamically so 64 KiB and 1 MiB payloads balance.  Each
// item writes only its own batch result and its own planned arena slot.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_decode(DeviceJob j) {
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
        if (doff + cap > j.decoded_capacity) {
            addf = RPGPU_F_DECODE_OVERFLOW;
        } else {
            int64_t got = 0;
            if (decode_payload(codec, j.data + S, n, j.decoded + doff, got) == 0) {
                addf = RPGPU_F_CODEC_OK;
                dl = (uint32_t)got;
            }
        }
        if (lane() == 0 && addf) {
            R->flags = R->flags | addf;
            if (addf & RPGPU_F_CODEC_OK) R->decoded_len = dl;
        }
    }
}

__global__ __launch_bounds__(64) void k_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst,
                                                       int64_t* res) {
    int64_t got = 0;
    const int rc = decode_payload(codec, src, (int64_t)n, dst, got);
    if (lane() == 0) {
        res[0] = rc;
        res[1] = got;
    }
}

hipError_t launch_decode(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, int64_t* res,
                                 hipStream_t s) {
    (void)cap;
    hipLaunchKernelGGL(k_uncompress_one, dim3(1), dim3(64), 0, s, codec, src, n, dst, res);
    return hipGetLastError();
}

}  // namespace rp
