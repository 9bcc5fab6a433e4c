// rp_compress.hip — compression::compressor::compress on the device for lz4
// and snappy (compression/compression.cc:17-33), the write side's
// storage::internal::compress_batch (storage/parser_utils.cc:97-111):
//   * lz4: lz4_frame_compressor::compress (compression/internal/
//     lz4_frame_compressor.cc:72-113) — an LZ4 frame {independent 64 KiB
//     blocks, content size}, each block liblz4 1.9.3's
//     LZ4_compress_generic(byU16, noDict, limitedOutput, acceleration 1)
//     into srcSize - 1 bytes, a raw block when that does not fit;
//   * snappy: snappy_java_compressor::compress (compression/internal/
//     snappy_java_compressor.cc:58-75) — the snappy-java header, then per
//     iobuf fragment a big-endian length and snappy 1.1.8 RawCompress
//     (varint length + CompressFragment per 64 KiB block, fresh table each).
// The algorithm is the oracle's (oracle/rp_oracle.c rpo_lz4_compress_block /
// rpo_snappy_compress_block), itself pinned byte for byte against the
// libraries through oracle/_ref.
//
// Execution model.  Every 64 KiB block of every payload is independent (a
// fresh hash table), so blocks are the unit: one WAVE per block with the
// hash table in LDS (8192 u16 for lz4, up to 16384 u16 for snappy).  The
// match search is a serial chain (each probe updates the table the next one
// reads), run uniformly by the whole wave (every lane holds the same scalar
// state; table reads broadcast, lane 0 writes); the parts with width are
// wave-parallel: match extension compares 64 bytes per step (ballot of
// mismatches), literals are copied 64 bytes per step.  Blocks compress into
// fixed scratch slots; k_compress_pack then lays each payload's frame out
// (one wave per payload: header, per-block size words / fragment lengths,
// coalesced copies of the block outputs).
// Byte work only: no MFMA.
#include "rp_device.h"

namespace rp {
namespace {

typedef __attribute__((address_space(3))) uint16_t lds_u16;

// 4 bytes at s + i (s = a block of a fragment staged 16-byte aligned; reads
// up to 7 bytes past i)
DEV uint32_t g32(const uint8_t* __restrict__ s, uint32_t i) {
    const uint32_t* w = (const uint32_t*)(s + (i & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], i & 3);
}

DEV void put16(lds_u16* T, uint32_t h, uint32_t v) {
    if (lane() == 0) T[h] = (uint16_t)v;
}

// LZ4_count / FindMatchLength: equal bytes of s[a..] and s[m..] before limit
// (a < limit), 64 per step
DEV uint32_t wave_count(const uint8_t* __restrict__ s, uint32_t a, uint32_t m, uint32_t limit) {
    const uint32_t l = lane();
    uint32_t c = 0;
    for (;;) {
        const uint32_t k = a + c + l;
        const bool diff = k >= limit || s[k] != s[m + c + l];
        const uint64_t mask = __ballot(diff);
        if (mask) return c + (uint32_t)__builtin_ctzll(mask);
        c += 64;
    }
}

DEV void wave_copy(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, uint32_t n) {
    for (uint32_t k = lane(); k < n; k += 64) d[k] = s[k];
}

DEV void put8(uint8_t* d, uint32_t at, uint32_t v) {
    if (lane() == 0) d[at] = (uint8_t)v;
}

constexpr uint32_t kLzHashLog = 13;
DEV uint32_t lz_hash(uint32_t v) { return (v * 2654435761u) >> (32 - kLzHashLog); }

// rpo_lz4_compress_block: LZ4_compress_generic_validated (lz4 1.9.3) with
// byU16 / noDict / noDictIssue / limitedOutput / acceleration 1 on a zeroed
// table; the size, or 0 when it does not fit in cap bytes
DEV int32_t lz4c_block(const uint8_t* __restrict__ s, uint32_t n, uint8_t* __restrict__ d, int32_t cap, lds_u16* T) {
    uint32_t ip = 0, anchor = 0, match = 0, fh = 0, fv = 0, tokv = 0;
    const uint32_t mfl1 = n - 12 + 1, mlimit = n - 5;
    int32_t op = 0, token = 0;
    if (n < 13) goto last_literals;
    put16(T, lz_hash(g32(s, 0)), 0);
    ip = 1;
    fv = g32(s, 1);  // the 4 bytes at the next probe position (kept: ip's bytes at the compare)
    fh = lz_hash(fv);
    for (;;) {
        {
            uint32_t fip = ip, step = 1, nb = 64;
            for (;;) {
                const uint32_t h = fh, cur = fip, iv = fv;
                const uint32_t mi = T[h];
                ip = fip;
                fip += step;
                step = nb++ >> 6;
                if (fip > mfl1) goto last_literals;
                match = mi;
                fv = g32(s, fip);
                fh = lz_hash(fv);
                put16(T, h, cur);
                if (g32(s, match) == iv) break;
            }
        }
        while (ip > anchor && match > 0 && s[ip - 1] == s[match - 1]) {
            ip--;
            match--;
        }
        {
            const uint32_t lit = ip - anchor;
            token = op++;
            if (op + (int32_t)lit + 8 + (int32_t)(lit / 255) > cap) return 0;
            if (lit >= 15) {
                uint32_t len = lit - 15;
                tokv = 15u << 4;
                for (; len >= 255; len -= 255) put8(d, op++, 255);
                put8(d, op++, len);
            } else {
                tokv = lit << 4;
            }
            wave_copy(d + op, s + anchor, lit);
            op += (int32_t)lit;
        }
    next_match:
        put8(d, op, ip - match);
        put8(d, op + 1, (ip - match) >> 8);
        op += 2;
        {
            uint32_t mc = wave_count(s, ip + 4, match + 4, mlimit);
            ip += mc + 4;
            if (op + 6 + (int32_t)((mc + 240) / 255) > cap) return 0;
            if (mc >= 15) {
                tokv += 15;
                mc -= 15;
                for (; mc >= 255; mc -= 255) put8(d, op++, 255);
                put8(d, op++, mc);
            } else {
                tokv += mc;
            }
            put8(d, token, tokv);
        }
        anchor = ip;
        if (ip >= mfl1) break;
        put16(T, lz_hash(g32(s, ip - 2)), ip - 2);
        {
            const uint32_t h = lz_hash(g32(s, ip));
            match = T[h];
            put16(T, h, ip);
            if (g32(s, match) == g32(s, ip)) {
                token = op++;
                tokv = 0;
                goto next_match;
            }
        }
        fv = g32(s, ++ip);
        fh = lz_hash(fv);
    }
last_literals : {
    const uint32_t last = n - anchor;
    if (op + (int32_t)last + 1 + (int32_t)((last + 255 - 15) / 255) > cap) return 0;
    if (last >= 15) {
        uint32_t acc = last - 15;
        put8(d, op++, 15u << 4);
        for (; acc >= 255; acc -= 255) put8(d, op++, 255);
        put8(d, op++, acc);
    } else {
        put8(d, op++, last << 4);
    }
    wave_copy(d + op, s + anchor, last);
    op += (int32_t)last;
}
    return op;
}

// snappy 1.1.8
DEV uint32_t sn_hash(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }
DEV int log2f32(uint32_t x) { return 31 - __builtin_clz(x); }

DEV uint32_t sn_literal(uint8_t* __restrict__ d, uint32_t op, const uint8_t* __restrict__ lit, uint32_t len) {
    const uint32_t nn = len - 1;
    if (nn < 60) {
        put8(d, op++, nn << 2);
    } else {
        const int count = (log2f32(nn) >> 3) + 1;
        put8(d, op++, (uint32_t)(59 + count) << 2);
        for (int i = 0; i < count; i++) put8(d, op++, nn >> (8 * i));
    }
    wave_copy(d + op, lit, len);
    return op + len;
}

// EmitCopyAtMost64
DEV uint32_t sn_copy64(uint8_t* d, uint32_t op, uint32_t offset, uint32_t len) {
    if (len < 12 && offset < 2048) {
        put8(d, op, 1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
        put8(d, op + 1, offset);
        return op + 2;
    }
    put8(d, op, 2 + ((len - 1) << 2));
    put8(d, op + 1, offset);
    put8(d, op + 2, offset >> 8);
    return op + 3;
}

DEV uint32_t sn_copy(uint8_t* d, uint32_t op, uint32_t offset, uint32_t len) {
    if (len < 12) return sn_copy64(d, op, offset, len);
    while (len >= 68) {
        op = sn_copy64(d, op, offset, 64);
        len -= 64;
    }
    if (len > 64) {
        op = sn_copy64(d, op, offset, 60);
        len -= 60;
    }
    return sn_copy64(d, op, offset, len);
}

// rpo_snappy_compress_block: CompressFragment of one block (<= 64 KiB)
DEV uint32_t snappyc_block(const uint8_t* __restrict__ s, uint32_t n, uint8_t* __restrict__ d, lds_u16* T, int shift) {
    uint32_t ip = 0, next_emit = 0, op = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        uint32_t next_val = g32(s, ++ip);  // the bytes at next_ip (ip's at the compare)
        uint32_t next_hash = sn_hash(next_val, shift);
        for (;;) {
            uint32_t skip = 32, next_ip = ip, candidate, iv;
            do {
                ip = next_ip;
                iv = next_val;
                const uint32_t hash = next_hash;
                const uint32_t between = skip >> 5;
                skip += between;
                next_ip = ip + between;
                if (next_ip > ip_limit) goto emit_remainder;
                next_val = g32(s, next_ip);
                next_hash = sn_hash(next_val, shift);
                candidate = T[hash];
                put16(T, hash, ip);
            } while (iv != g32(s, candidate));
            op = sn_literal(d, op, s + next_emit, ip - next_emit);
            uint32_t cand_bytes, cur;
            do {
                const uint32_t base = ip;
                const uint32_t matched = 4 + wave_count(s, ip + 4, candidate + 4, n);
                ip += matched;
                op = sn_copy(d, op, base - candidate, matched);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                put16(T, sn_hash(g32(s, ip - 1), shift), ip - 1);
                cur = g32(s, ip);
                const uint32_t cur_hash = sn_hash(cur, shift);
                candidate = T[cur_hash];
                cand_bytes = g32(s, candidate);
                put16(T, cur_hash, ip);
            } while (cur == cand_bytes);
            next_val = g32(s, ip + 1);
            next_hash = sn_hash(next_val, shift);
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < n) op = sn_literal(d, op, s + next_emit, n - next_emit);
    return op;
}

// one kernel per codec: the LDS table is 16 KiB for lz4 (10 waves per CU),
// 32 KiB for snappy (5); a wave given the other codec's block leaves
template <uint32_t kCodec>
__global__ __launch_bounds__(64) void k_compress_blocks(const uint8_t* __restrict__ in, const CompBlock* __restrict__ blocks,
                                                        uint32_t nb, uint8_t* __restrict__ scratch,
                                                        uint32_t* __restrict__ sizes) {
    __shared__ uint16_t table[kCodec == RPGPU_CODEC_SNAPPY ? 16384 : (1u << kLzHashLog)];
    lds_u16* T = (lds_u16*)table;
    const uint32_t b = blockIdx.x;
    if (b >= nb) return;
    const uint32_t codec = uni32(blocks[b].codec);
    if (codec != kCodec) return;
    const uint64_t src = uni64(blocks[b].src);
    const uint32_t n = uni32(blocks[b].n);
    const uint8_t* s = in + src;
    uint8_t* d = scratch + (uint64_t)b * kCompSlot;
    uint32_t tsize = 1u << kLzHashLog;
    int shift = 0;
    if (kCodec == RPGPU_CODEC_SNAPPY) {
        // CalculateTableSize
        tsize = n > 16384u ? 16384u : n < 256u ? 256u : 2u << log2f32(n - 1);
        shift = 32 - log2f32(tsize);
    }
    for (uint32_t k = lane(); k < tsize; k += 64) T[k] = 0;
    __syncthreads();
    uint32_t r;
    if (kCodec == RPGPU_CODEC_SNAPPY) r = snappyc_block(s, n, d, T, shift);
    else r = (uint32_t)lz4c_block(s, n, d, (int32_t)n - 1, T);
    if (lane() == 0) sizes[b] = r;
}

// XXH32 of at most 15 bytes (the LZ4F header checksum)
DEV uint32_t xxh32_small(const uint8_t* p, uint32_t len) {
    constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
    uint32_t h = P5 + len;
    uint32_t i = 0;
    for (; i + 4 <= len; i += 4) {
        const uint32_t v = p[i] | (p[i + 1] << 8) | (p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
        h += v * P3;
        h = ((h << 17) | (h >> 15)) * P4;
    }
    for (; i < len; i++) {
        h += p[i] * P5;
        h = ((h << 11) | (h >> 21)) * P1;
    }
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

DEV void put_le32(uint8_t* d, uint64_t at, uint32_t v) {
    if (lane() == 0)
        for (int i = 0; i < 4; i++) d[at + i] = (uint8_t)(v >> (8 * i));
}

// one wave per payload: the frame from the block outputs
__global__ __launch_bounds__(64) void k_compress_pack(const uint8_t* __restrict__ in, const CompPayload* __restrict__ pay,
                                                      uint32_t np, const CompBlock* __restrict__ blocks,
                                                      const uint8_t* __restrict__ scratch,
                                                      const uint32_t* __restrict__ sizes, uint8_t* __restrict__ out,
                                                      uint64_t* __restrict__ out_len) {
    const uint32_t p = blockIdx.x;
    if (p >= np) return;
    const uint32_t l = lane();
    const uint64_t n = uni64(pay[p].n), base = uni64(pay[p].out);
    const uint32_t first = uni32(pay[p].first), nbk = uni32(pay[p].nblocks), codec = uni32(pay[p].codec);
    uint8_t* d = out + base;
    uint64_t o = 0;
    if (codec == RPGPU_CODEC_LZ4) {
        // LZ4F_compressBegin: magic, FLG (version 01, independent blocks,
        // content size when non-zero), BD (max64KB), content size, HC
        uint8_t h[15];
        h[0] = 0x04; h[1] = 0x22; h[2] = 0x4D; h[3] = 0x18;
        h[4] = (uint8_t)(0x60 | (n ? 0x08 : 0));
        h[5] = 0x40;
        uint32_t hl = 6;
        if (n) {
            for (int i = 0; i < 8; i++) h[6 + i] = (uint8_t)(n >> (8 * i));
            hl = 14;
        }
        h[hl] = (uint8_t)((xxh32_small(h + 4, hl - 4) >> 8) & 0xFF);
        hl++;
        if (l == 0)
            for (uint32_t i = 0; i < hl; i++) d[i] = h[i];
        o = hl;
        for (uint32_t k = 0; k < nbk; k++) {
            const uint32_t b = first + k;
            const uint32_t c = uni32(sizes[b]), bn = uni32(blocks[b].n);
            if (c == 0) {  // LZ4F_makeBlock: does not fit -> raw block
                put_le32(d, o, bn | 0x80000000u);
                wave_copy(d + o + 4, in + uni64(blocks[b].src), bn);
                o += 4 + bn;
            } else {
                put_le32(d, o, c);
                wave_copy(d + o + 4, scratch + (uint64_t)b * kCompSlot, c);
                o += 4 + c;
            }
        }
        put_le32(d, o, 0);  // end mark
        o += 4;
    } else {
        // snappy-java header: magic, version 1, min version 1 (LE, as the
        // reference appends them)
        if (l == 0) {
            const uint8_t hdr[16] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0, 1, 0, 0, 0, 1, 0, 0, 0};
            for (int i = 0; i < 16; i++) d[i] = hdr[i];
        }
        o = 16;
        for (uint32_t k = 0; k < nbk;) {
            // a fragment: its blocks, then BE32 length + RawCompress output
            const uint32_t b0 = first + k;
            const uint32_t fb = uni32(blocks[b0].frag_blocks);
            const uint32_t flen = uni32(blocks[b0].frag_len);
            uint32_t vl = 1;
            for (uint32_t v = flen; v >= 128; v >>= 7) vl++;
            uint32_t tot = vl;
            for (uint32_t j = 0; j < fb; j++) tot += uni32(sizes[b0 + j]);
            if (l == 0) {
                d[o] = (uint8_t)(tot >> 24);
                d[o + 1] = (uint8_t)(tot >> 16);
                d[o + 2] = (uint8_t)(tot >> 8);
                d[o + 3] = (uint8_t)tot;
                uint32_t v = flen;
                uint64_t q = o + 4;
                while (v >= 128) { d[q++] = (uint8_t)(v | 128); v >>= 7; }
                d[q] = (uint8_t)v;
            }
            o += 4 + vl;
            for (uint32_t j = 0; j < fb; j++) {
                const uint32_t c = uni32(sizes[b0 + j]);
                wave_copy(d + o, scratch + (uint64_t)(b0 + j) * kCompSlot, c);
                o += c;
            }
            k += fb;
        }
    }
    if (l == 0) out_len[p] = o;
}

}  // namespace

hipError_t launch_compress(const uint8_t* in, const CompBlock* blocks, uint32_t nb, const CompPayload* pay, uint32_t np,
                           uint8_t* scratch, uint32_t* sizes, uint8_t* out, uint64_t* out_len, hipStream_t s) {
    if (nb) {
        hipLaunchKernelGGL(k_compress_blocks<RPGPU_CODEC_LZ4>, dim3(nb), dim3(64), 0, s, in, blocks, nb, scratch, sizes);
        hipLaunchKernelGGL(k_compress_blocks<RPGPU_CODEC_SNAPPY>, dim3(nb), dim3(64), 0, s, in, blocks, nb, scratch, sizes);
    }
    if (np) hipLaunchKernelGGL(k_compress_pack, dim3(np), dim3(64), 0, s, in, pay, np, blocks, scratch, sizes, out, out_len);
    return hipGetLastError();
}

}  // namespace rp
