/*
 * rp_oracle.c — CPU restatement of the reference's record-batch hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rp_oracle.h).  Never linked into the product.
 * Written for clarity over speed (bytewise CRC, scalar decoders), except the
 * SSE4.2 CRC used as the timed CPU baseline.
 */
#define _GNU_SOURCE
#include "rp_oracle.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

/* ======================================================================== */
/* CRC32C — google crc32c::Extend semantics (hashing/crc32c.h:27 calls       */
/* ::crc32c::Extend(_crc, data, size); crc32c @47b40d22, cmake/oss.cmake.in:195-197). */
/* ======================================================================== */
#define RPO_CRC32C_POLY 0x82F63B78u

static uint32_t g_crc_table[256];
static int g_crc_init = 0;

static void crc_init(void) {
    if (g_crc_init) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ RPO_CRC32C_POLY : c >> 1;
        g_crc_table[i] = c;
    }
    g_crc_init = 1;
}

uint32_t rpo_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
    crc_init();
    uint32_t l = crc ^ 0xFFFFFFFFu; /* kCRC32Xor */
    for (size_t i = 0; i < n; i++) l = g_crc_table[(l ^ p[i]) & 0xFF] ^ (l >> 8);
    return l ^ 0xFFFFFFFFu;
}

/* GF(2) multiply of two reflected polynomials mod P (zlib multmodp shape). */
static uint32_t gf_mulmod(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ RPO_CRC32C_POLY : b >> 1;
    }
    return p;
}

/* x^(8*len) mod P in the reflected domain. */
static uint32_t x8n_mod(uint64_t len) {
    uint32_t r = 1u << 31;       /* x^0 */
    uint32_t sq = 1u << 23;      /* x^8 (reflected: bit 31-8) */
    while (len) {
        if (len & 1) r = gf_mulmod(r, sq);
        sq = gf_mulmod(sq, sq);
        len >>= 1;
    }
    return r;
}

uint32_t rpo_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return gf_mulmod(x8n_mod(len_b), crc_a) ^ crc_b;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2")))
static uint32_t hw_raw(uint32_t l, const uint8_t* p, size_t n) {
    while (n && ((uintptr_t)p & 7)) { l = _mm_crc32_u8(l, *p++); n--; }
    /* three interleaved streams of `blk` bytes, merged by x^(8*blk) shifts */
    const size_t blk = 4096;
    static uint32_t k1 = 0, k2 = 0;
    if (!k1) { k1 = x8n_mod(blk); k2 = x8n_mod(2 * blk); }
    while (n >= 3 * blk) {
        uint64_t a = l, b = 0, c = 0;
        const uint64_t* q = (const uint64_t*)p;
        for (size_t i = 0; i < blk / 8; i++) {
            a = _mm_crc32_u64(a, q[i]);
            b = _mm_crc32_u64(b, q[i + blk / 8]);
            c = _mm_crc32_u64(c, q[i + 2 * blk / 8]);
        }
        l = gf_mulmod(k2, (uint32_t)a) ^ gf_mulmod(k1, (uint32_t)b) ^ (uint32_t)c;
        p += 3 * blk;
        n -= 3 * blk;
    }
    uint64_t v = l;
    while (n >= 8) { v = _mm_crc32_u64(v, *(const uint64_t*)p); p += 8; n -= 8; }
    l = (uint32_t)v;
    while (n) { l = _mm_crc32_u8(l, *p++); n--; }
    return l;
}
uint32_t rpo_crc32c_extend_hw(uint32_t crc, const uint8_t* p, size_t n) {
    crc_init();
    return hw_raw(crc ^ 0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu;
}
#else
uint32_t rpo_crc32c_extend_hw(uint32_t crc, const uint8_t* p, size_t n) { return rpo_crc32c_extend(crc, p, n); }
#endif

/* ======================================================================== */
/* XXH32 (lz4 1.9.3 lib/xxhash.c, XXH32())                                  */
/* ======================================================================== */
#define XP1 0x9E3779B1u
#define XP2 0x85EBCA77u
#define XP3 0xC2B2AE3Du
#define XP4 0x27D4EB2Fu
#define XP5 0x165667B1u
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

uint32_t rpo_xxh32(const uint8_t* p, size_t n, uint32_t seed) {
    const uint8_t* end = p + n;
    uint32_t h;
    if (n >= 16) {
        uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        const uint8_t* lim = end - 16;
        do {
            v1 = rotl32(v1 + rd32(p) * XP2, 13) * XP1; p += 4;
            v2 = rotl32(v2 + rd32(p) * XP2, 13) * XP1; p += 4;
            v3 = rotl32(v3 + rd32(p) * XP2, 13) * XP1; p += 4;
            v4 = rotl32(v4 + rd32(p) * XP2, 13) * XP1; p += 4;
        } while (p <= lim);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + XP5;
    }
    h += (uint32_t)n;
    while (p + 4 <= end) { h += rd32(p) * XP3; h = rotl32(h, 17) * XP4; p += 4; }
    while (p < end) { h += (*p) * XP5; h = rotl32(h, 11) * XP1; p++; }
    h ^= h >> 15; h *= XP2; h ^= h >> 13; h *= XP3; h ^= h >> 16;
    return h;
}

/* ======================================================================== */
/* vint (utils/vint.h)                                                       */
/* ======================================================================== */
int64_t rpo_vint_deserialize(const uint8_t* p, size_t avail, size_t* bytes_read) {
    /* utils/vint.h:82-98: stops after shift 63 (10 bytes) even if the
     * continuation bit is set; at end of input returns what it has. */
    uint64_t result = 0, shift = 0;
    size_t br = 0;
    for (size_t i = 0; shift <= 63 && i < avail; i++) {
        uint64_t byte = p[i];
        br++;
        if (byte & 128) {
            result |= ((byte & 127) << shift);
        } else {
            result |= byte << shift;
            break;
        }
        shift += 7;
    }
    *bytes_read = br;
    /* decode_zigzag (utils/vint.h:37-39) */
    return (int64_t)((result >> 1) ^ (~(result & 1) + 1));
}

size_t rpo_vint_serialize(int64_t x, uint8_t* out) {
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    size_t n = 0;
    while (v >= 0x80) { out[n++] = (uint8_t)(v | 0x80); v >>= 7; }
    out[n++] = (uint8_t)v;
    return n;
}

/* ======================================================================== */
/* Headers and CRCs                                                          */
/* ======================================================================== */
void rpo_header_from_disk(const uint8_t* p, rpo_header* h) {
    /* storage/parser.cc:36-76, reflection::adl little endian */
    h->header_crc = rd32(p + 0);
    h->size_bytes = (int32_t)rd32(p + 4);
    h->base_offset = (int64_t)rd64(p + 8);
    h->type = (int8_t)p[16];
    h->crc = (int32_t)rd32(p + 17);
    h->attrs = (int16_t)rd16(p + 21);
    h->last_offset_delta = (int32_t)rd32(p + 23);
    h->first_timestamp = (int64_t)rd64(p + 27);
    h->max_timestamp = (int64_t)rd64(p + 35);
    h->producer_id = (int64_t)rd64(p + 43);
    h->producer_epoch = (int16_t)rd16(p + 51);
    h->base_sequence = (int32_t)rd32(p + 53);
    h->record_count = (int32_t)rd32(p + 57);
}

static inline uint64_t be_n(const uint8_t* p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

/* kafka_batch_adapter::read_header (kafka/protocol/kafka_batch_adapter.cc:
 * 32-91): big-endian v2 header; size_bytes = batch_length + 12 (int32
 * arithmetic, :57-63), type raft_data, partition_leader_epoch ignored.
 * Returns the magic byte. */
int rpo_header_from_wire(const uint8_t* p, rpo_header* h) {
    h->header_crc = 0;
    h->base_offset = (int64_t)be_n(p, 8);
    h->size_bytes = (int32_t)((uint32_t)be_n(p + 8, 4) + 12u);
    h->type = 1;
    h->crc = (int32_t)(uint32_t)be_n(p + 17, 4);
    h->attrs = (int16_t)(uint16_t)be_n(p + 21, 2);
    h->last_offset_delta = (int32_t)(uint32_t)be_n(p + 23, 4);
    h->first_timestamp = (int64_t)be_n(p + 27, 8);
    h->max_timestamp = (int64_t)be_n(p + 35, 8);
    h->producer_id = (int64_t)be_n(p + 43, 8);
    h->producer_epoch = (int16_t)(uint16_t)be_n(p + 51, 2);
    h->base_sequence = (int32_t)(uint32_t)be_n(p + 53, 4);
    h->record_count = (int32_t)(uint32_t)be_n(p + 57, 4);
    return (int8_t)p[16];
}

static void wr_le(uint8_t* p, uint64_t v, int n) { for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i)); }
static void wr_be(uint8_t* p, uint64_t v, int n) { for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * (n - 1 - i))); }

void rpo_header_to_disk(const rpo_header* h, uint8_t* o) {
    wr_le(o + 0, h->header_crc, 4);
    wr_le(o + 4, (uint32_t)h->size_bytes, 4);
    wr_le(o + 8, (uint64_t)h->base_offset, 8);
    o[16] = (uint8_t)h->type;
    wr_le(o + 17, (uint32_t)h->crc, 4);
    wr_le(o + 21, (uint16_t)h->attrs, 2);
    wr_le(o + 23, (uint32_t)h->last_offset_delta, 4);
    wr_le(o + 27, (uint64_t)h->first_timestamp, 8);
    wr_le(o + 35, (uint64_t)h->max_timestamp, 8);
    wr_le(o + 43, (uint64_t)h->producer_id, 8);
    wr_le(o + 51, (uint16_t)h->producer_epoch, 2);
    wr_le(o + 53, (uint32_t)h->base_sequence, 4);
    wr_le(o + 57, (uint32_t)h->record_count, 4);
}

uint32_t rpo_internal_header_only_crc(const rpo_header* h) {
    /* model/record_utils.cc:34-55: the 57 bytes after header_crc, LE */
    uint8_t b[61];
    rpo_header_to_disk(h, b);
    return rpo_crc32c_extend(0, b + 4, 57);
}

static void be_prefix(const rpo_header* h, uint8_t* o) {
    /* model/record_utils.cc:68-80: attrs..record_count, big endian (40 B) */
    wr_be(o + 0, (uint16_t)h->attrs, 2);
    wr_be(o + 2, (uint32_t)h->last_offset_delta, 4);
    wr_be(o + 6, (uint64_t)h->first_timestamp, 8);
    wr_be(o + 14, (uint64_t)h->max_timestamp, 8);
    wr_be(o + 22, (uint64_t)h->producer_id, 8);
    wr_be(o + 30, (uint16_t)h->producer_epoch, 2);
    wr_be(o + 32, (uint32_t)h->base_sequence, 4);
    wr_be(o + 36, (uint32_t)h->record_count, 4);
}

uint32_t rpo_crc_record_batch(const rpo_header* h, const uint8_t* payload, size_t n) {
    uint8_t pre[40];
    be_prefix(h, pre);
    uint32_t c = rpo_crc32c_extend(0, pre, 40);
    return rpo_crc32c_extend(c, payload, n);
}

static uint32_t crc_record_batch_hw(const rpo_header* h, const uint8_t* payload, size_t n) {
    uint8_t pre[40];
    be_prefix(h, pre);
    uint32_t c = rpo_crc32c_extend_hw(0, pre, 40);
    return rpo_crc32c_extend_hw(c, payload, n);
}

/* ======================================================================== */
/* Record walk                                                               */
/* ======================================================================== */
typedef struct walk_cur {
    const uint8_t* p;
    uint64_t n;
    uint64_t pos;
} walk_cur;

/* iobuf_parser_base::read_varlong (bytes/iobuf_parser.h:48-52): deserialize
 * then skip(bytes_read) — never throws (bytes_read <= available). */
static int64_t rd_varlong(walk_cur* c) {
    size_t br;
    int64_t v = rpo_vint_deserialize(c->p + c->pos, c->n - c->pos, &br);
    c->pos += br;
    return v;
}

/* iobuf_const_parser::copy(len) -> iobuf_copy (bytes/iobuf.cc:133-157):
 * `int bytes_left = len` truncates; a negative int reaches
 * ss_next_allocation_size((size_t)neg) -> 2^63-byte temporary_buffer ->
 * bad_alloc; zero copies nothing; positive copies min(len, available) and
 * never throws. Returns 0 or -1 (throw). */
static int copy_bytes(walk_cur* c, int64_t len) {
    int32_t bl = (int32_t)(uint32_t)(uint64_t)len;
    if (bl < 0) return -1;
    uint64_t left = c->n - c->pos;
    c->pos += ((uint64_t)bl < left) ? (uint64_t)bl : left;
    return 0;
}

uint32_t rpo_walk_records(const uint8_t* payload, size_t n, int32_t record_count,
                          uint32_t batch_ordinal, rpgpu_record_index* index,
                          uint64_t index_cap, uint8_t* parse_err, uint64_t* trailing) {
    walk_cur c = {payload, n, 0};
    uint32_t parsed = 0;
    *parse_err = RPGPU_PARSE_ERR_NONE;
    *trailing = 0;
    /* model/record.h:619: for (auto i = 0; i < record_count; i++) */
    for (int32_t i = 0; i < record_count; i++) {
        rpgpu_record_index e;
        memset(&e, 0, sizeof e);
        e.batch = batch_ordinal;
        e.rec_pos = (uint32_t)c.pos;
        /* parse_record_meta_from_buffer (model/record_utils.cc:147-160) */
        int64_t record_size = rd_varlong(&c);
        if (c.pos >= c.n) { *parse_err = RPGPU_PARSE_ERR_ATTR_EOF; return parsed; }
        int8_t attr = (int8_t)c.p[c.pos++];
        /* do_parse_one_record_from_buffer (model/record_utils.cc:116-145) */
        int64_t ts = rd_varlong(&c);
        int64_t off = rd_varlong(&c);
        int64_t klen = rd_varlong(&c);
        e.key_pos = (uint32_t)c.pos;
        if (klen > 0 && copy_bytes(&c, klen)) { *parse_err = RPGPU_PARSE_ERR_COPY_NEGATIVE; return parsed; }
        int64_t vlen = rd_varlong(&c);
        e.val_pos = (uint32_t)c.pos;
        if (vlen > 0 && copy_bytes(&c, vlen)) { *parse_err = RPGPU_PARSE_ERR_COPY_NEGATIVE; return parsed; }
        /* parse_record_headers (model/record_utils.cc:94-114) */
        int64_t hcount = rd_varlong(&c);
        e.hdr_pos = (uint32_t)c.pos;
        /* headers.reserve(header_count): length_error for negative counts,
         * bad_alloc above the pinned reservation limit */
        if (hcount < 0 || hcount > RPGPU_MAX_HEADER_RESERVE) { *parse_err = RPGPU_PARSE_ERR_HEADER_RESERVE; return parsed; }
        for (int64_t h = 0; h < hcount; h++) {
            if (c.pos >= c.n) break; /* remaining iterations read {0,0}: no-ops */
            int64_t hk = rd_varlong(&c);
            if (hk > 0 && copy_bytes(&c, hk)) { *parse_err = RPGPU_PARSE_ERR_COPY_NEGATIVE; return parsed; }
            int64_t hv = rd_varlong(&c);
            if (hv > 0 && copy_bytes(&c, hv)) { *parse_err = RPGPU_PARSE_ERR_COPY_NEGATIVE; return parsed; }
        }
        e.length = (int32_t)record_size;
        e.attrs = attr;
        e.ts_delta = ts;
        e.offset_delta = (int32_t)off;
        e.key_len = (int32_t)klen;
        e.val_len = (int32_t)vlen;
        e.hdr_count = (int32_t)hcount;
        e.end_pos = (uint32_t)c.pos;
        if (index && (uint64_t)parsed < index_cap) index[parsed] = e;
        parsed++;
    }
    *trailing = c.n - c.pos;
    return parsed;
}

/* ======================================================================== */
/* LZ4 block decode — restates lz4 1.9.3 LZ4_decompress_generic for         */
/* LZ4_decompress_safe_usingDict (endOnInputSize, decode_full_block,         */
/* LZ4_FAST_DEC_LOOP on x86-64).  Control flow and every acceptance check    */
/* are kept; copies use canonical forward-copy semantics (offset 0 -> zeros, */
/* as LZ4_memcpy_using_offset_base / the safe loop's write32(op,0) produce). */
/* ======================================================================== */
#define LZ_MINMATCH 4
#define LZ_LASTLITERALS 5
#define LZ_MFLIMIT 12
#define LZ_FASTLOOP_SAFE_DISTANCE 64

/* read_variable_length: returns added length; *err: 0 ok, 1 initial, 2 loop */
static uint32_t lz_read_var(const uint8_t* s, int64_t* ip, int64_t lencheck, int loop_check,
                            int initial_check, int* err) {
    uint32_t length = 0, b;
    *err = 0;
    if (initial_check && *ip >= lencheck) { *err = 1; return length; }
    do {
        b = s[*ip];
        (*ip)++;
        length += b;
        if (loop_check && *ip >= lencheck) { *err = 2; return length; }
    } while (b == 255);
    return length;
}

static void lz_match_copy(uint8_t* dst, int64_t op, int64_t offset, int64_t length) {
    if (offset == 0) {
        memset(dst + op, 0, (size_t)length);
        return;
    }
    for (int64_t i = 0; i < length; i++) dst[op + i] = dst[op + i - offset];
}

int rpo_lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap,
                         size_t history) {
    const int64_t iend = (int64_t)n, oend = (int64_t)dst_cap;
    int64_t ip = 0, op = 0;
    const int64_t H = (int64_t)history;
    const int64_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    uint32_t token;
    int64_t length, offset, cpy;
    int err;

    if (oend == 0) return (n == 1 && src[0] == 0) ? 0 : -1;
    if (n == 0) return -1;

    if (oend - op < LZ_FASTLOOP_SAFE_DISTANCE) goto safe_decode;
    for (;;) {
        token = src[ip++];
        length = token >> 4;
        if (length == 15) {
            length += lz_read_var(src, &ip, iend - 15, 1, 1, &err);
            if (err == 1) return -1;
            cpy = op + length;
            if (cpy > oend - 32 || ip + length > iend - 32) goto safe_literal_copy;
            memcpy(dst + op, src + ip, (size_t)length);
            ip += length;
            op = cpy;
        } else {
            cpy = op + length;
            if (ip > iend - (16 + 1)) goto safe_literal_copy;
            memcpy(dst + op, src + ip, (size_t)length);
            ip += length;
            op = cpy;
        }
        offset = rd16(src + ip);
        ip += 2;
        length = token & 15;
        if (length == 15) {
            if (offset > op + H) return -1;
            length += lz_read_var(src, &ip, iend - LZ_LASTLITERALS + 1, 1, 0, &err);
            if (err) return -1;
            length += LZ_MINMATCH;
            if (op + length >= oend - LZ_FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
        } else {
            length += LZ_MINMATCH;
            if (op + length >= oend - LZ_FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
            if (offset <= op + H && offset >= 8) {
                lz_match_copy(dst, op, offset, length);
                op += length;
                continue;
            }
        }
        if (offset > op + H) return -1;
        /* external-dictionary end-of-block rule cannot trigger here
         * (op + length < oend - 64) */
        lz_match_copy(dst, op, offset, length);
        op += length;
    }

safe_decode:
    for (;;) {
        token = src[ip++];
        length = token >> 4;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            memcpy(dst + op, src + ip, (size_t)length);
            op += length;
            ip += length;
            length = token & 15;
            offset = rd16(src + ip);
            ip += 2;
            if (length != 15 && offset >= 8 && offset <= op + H) {
                lz_match_copy(dst, op, offset, length + LZ_MINMATCH);
                op += length + LZ_MINMATCH;
                continue;
            }
            goto copy_match;
        }
        if (length == 15) {
            length += lz_read_var(src, &ip, iend - 15, 1, 1, &err);
            if (err == 1) return -1;
        }
        cpy = op + length;
    safe_literal_copy:
        if (cpy > oend - LZ_MFLIMIT || ip + length > iend - (2 + 1 + LZ_LASTLITERALS)) {
            if (ip + length != iend || cpy > oend) return -1;
            memmove(dst + op, src + ip, (size_t)length);
            ip += length;
            op += length;
            break;
        }
        memcpy(dst + op, src + ip, (size_t)length);
        ip += length;
        op = cpy;
        offset = rd16(src + ip);
        ip += 2;
        length = token & 15;
    copy_match:
        if (length == 15) {
            length += lz_read_var(src, &ip, iend - LZ_LASTLITERALS + 1, 1, 0, &err);
            if (err) return -1;
        }
        length += LZ_MINMATCH;
    safe_match_copy:
        if (offset > op + H) return -1;
        if (offset > op) {
            /* match starts in the history (external dictionary or prefix):
             * LZ4_decompress_generic rejects op+length > oend-LASTLITERALS in
             * extDict mode; the in-block rule below rejects the same ends. */
            if (op + length > oend - LZ_LASTLITERALS) return -1;
            lz_match_copy(dst, op, offset, length);
            op += length;
            continue;
        }
        cpy = op + length;
        if (cpy > oend - LZ_MFLIMIT) {
            if (cpy > oend - LZ_LASTLITERALS) return -1;
        }
        lz_match_copy(dst, op, offset, length);
        op = cpy;
    }
    return (int)op;
}

/* ======================================================================== */
/* LZ4 frame — restates compression/internal/lz4_frame_compressor.cc:115-200 */
/* (do_uncompressed: LZ4F_getFrameInfo + LZ4F_decompress loop until code==0,  */
/* throw if input remains) over lz4 1.9.3 lz4frame.c's state machine.        */
/* Running out of input before the end mark is NOT an error there: the loop  */
/* exits with bytes_remaining == src_size and the partial output is returned. */
/* ======================================================================== */
static size_t lz4f_block_max(unsigned id) {
    switch (id) {
    case 4: return 64u << 10;
    case 5: return 256u << 10;
    case 6: return 1u << 20;
    case 7: return 4u << 20;
    }
    return 0;
}

/* Parses the frame header (LZ4F_headerSize + LZ4F_decodeHeader via
 * LZ4F_getFrameInfo).  Returns header bytes consumed, 0 for a skippable frame
 * (4 bytes consumed), -1 on error. */
typedef struct lz4f_info {
    int skippable;
    unsigned block_linked, block_checksum, content_checksum, content_size_flag;
    uint64_t content_size;
    size_t block_max;
} lz4f_info;

static int64_t lz4f_parse_header(const uint8_t* s, size_t n, lz4f_info* fi) {
    memset(fi, 0, sizeof *fi);
    if (n < 7) return -1;                                  /* frameHeader_incomplete */
    uint32_t magic = rd32(s);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {            /* skippable */
        if (n < 8) return -1;
        fi->skippable = 1;
        return 4;
    }
    if (magic != 0x184D2204u) return -1;                   /* frameType_unknown */
    uint8_t flg = s[4];
    size_t hsize = 7 + ((flg >> 3) & 1 ? 8 : 0) + ((flg & 1) ? 4 : 0);
    if (n < hsize) return -1;                              /* frameHeader_incomplete */
    if ((flg >> 1) & 1) return -1;                         /* reservedFlag_set */
    if (((flg >> 6) & 3) != 1) return -1;                  /* headerVersion_wrong */
    uint8_t bd = s[5];
    if ((bd >> 7) & 1) return -1;
    unsigned bsid = (bd >> 4) & 7;
    if (bsid < 4) return -1;                               /* maxBlockSize_invalid */
    if (bd & 15) return -1;
    uint8_t hc = (uint8_t)((rpo_xxh32(s + 4, hsize - 5, 0) >> 8) & 0xFF);
    if (hc != s[hsize - 1]) return -1;                     /* headerChecksum_invalid */
    fi->block_linked = !((flg >> 5) & 1);
    fi->block_checksum = (flg >> 4) & 1;
    fi->content_checksum = (flg >> 2) & 1;
    fi->content_size_flag = (flg >> 3) & 1;
    if (fi->content_size_flag) fi->content_size = rd64(s + 6);
    fi->block_max = lz4f_block_max(bsid);
    return (int64_t)hsize;
}

/* do_uncompressed drives LZ4F_decompress with an output buffer of
 * `est` bytes (contentSize, or 4x the input when unknown / >255x), growing it
 * to 1 KiB + 1.5x whenever a call returns with the buffer exactly full, and
 * stops calling as soon as all input has been handed over.  A compressed
 * block is decoded straight into the buffer only when at least maxBlockSize
 * bytes of room remain; otherwise liblz4 decodes it into its tmpOut and
 * flushes what fits, returning early.  If the input is exhausted at that
 * point (a frame truncated right after such a block), the unflushed tail is
 * never delivered — the reference returns the flushed prefix.  This
 * restatement tracks est/consumed to reproduce that exactly. */
int rpo_lz4f_uncompress(const uint8_t* s, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    lz4f_info fi;
    *out_len = 0;
    int64_t h = lz4f_parse_header(s, n, &fi);
    if (h < 0) return -1;
    size_t pos = (size_t)h, out = 0;
    if (fi.skippable) {
        /* dstage_getSFrameSize / dstage_skipSkippable */
        if (n - pos < 4) return 0;
        uint32_t sz = rd32(s + pos);
        pos += 4;
        if (n - pos < sz) return 0;        /* still skipping: input exhausted, no error */
        pos += sz;
        return pos < n ? -1 : 0;           /* frame done (code 0), input left -> throw */
    }
    /* compute_frame_uncompressed_size (lz4_frame_compressor.cc:115-121) */
    uint64_t est = (fi.content_size == 0 || fi.content_size > (uint64_t)n * 255) ? (uint64_t)n * 4 : fi.content_size;
#define LZ4F_GROW() (est = 1024 + ((est * 3) + 1) / 2)
    uint64_t remaining = fi.content_size; /* frameRemainingSize */
    for (;;) {
        if (n - pos < 4) return (*out_len = out, 0);      /* waiting for block header */
        uint32_t bh = rd32(s + pos);
        pos += 4;
        if (bh == 0) break;                                /* end mark -> dstage_getSuffix */
        size_t bsz = bh & 0x7FFFFFFFu;
        if (bsz > fi.block_max) return -1;                 /* maxBlockSize_invalid */
        if (bh & 0x80000000u) {
            /* dstage_copyDirect: streamed, partial data is emitted */
            size_t left = bsz;
            const uint8_t* blk = s + pos;
            for (;;) {
                size_t space = (size_t)(est - out), avail = n - pos;
                size_t k = left < avail ? left : avail;
                if (k > space) k = space;
                if (out + k > cap) return -2;
                memcpy(dst + out, s + pos, k);
                out += k;
                pos += k;
                left -= k;
                if (fi.content_size) remaining -= k;
                if (left == 0) break;
                if (out == est) LZ4F_GROW();               /* call returned, buffer full */
                if (pos == n) return (*out_len = out, 0);  /* input exhausted */
            }
            if (fi.block_checksum) {
                if (n - pos < 4) return (*out_len = out, 0);
                if (rd32(s + pos) != rpo_xxh32(blk, bsz, 0)) return -1;
                pos += 4;
            }
            continue;
        }
        /* compressed block header read: the call returns if dst is full or
         * the input is exhausted (dstage_getBlockHeader) */
        if (out == est) LZ4F_GROW();
        if (pos == n) return (*out_len = out, 0);
        size_t need = bsz + (fi.block_checksum ? 4 : 0);
        if (n - pos < need) return (*out_len = out, 0);  /* dstage_storeCBlock: wait */
        if (fi.block_checksum && rd32(s + pos + bsz) != rpo_xxh32(s + pos, bsz, 0)) return -1;
        size_t hist = fi.block_linked ? out : 0;
        if (out + fi.block_max > cap) {
            /* decode into a bounded scratch so an overflow is reported, not written */
            size_t hk = hist < 65536 ? hist : 65536;
            uint8_t* tmp = (uint8_t*)malloc(fi.block_max + 65536);
            memcpy(tmp, dst + out - hk, hk);
            int d = rpo_lz4_block_decode(s + pos, bsz, tmp + hk, fi.block_max, hk);
            if (d < 0) { free(tmp); return -1; }
            if (out + (size_t)d > cap) { free(tmp); return -2; }
            memcpy(dst + out, tmp + hk, (size_t)d);
            free(tmp);
            pos += need;
            if (fi.content_size) remaining -= (uint64_t)d;
            size_t space = (size_t)(est - out);
            if (space >= fi.block_max || (size_t)d <= space) { out += (size_t)d; continue; }
            /* tmpOut flush path: same bookkeeping as below */
            size_t pending = (size_t)d - space;
            out += space;
            while (pending) {
                if (out == est) LZ4F_GROW();
                if (pos == n) return (*out_len = out, 0);
                size_t sp = (size_t)(est - out), f = pending < sp ? pending : sp;
                out += f;
                pending -= f;
            }
            continue;
        }
        int d = rpo_lz4_block_decode(s + pos, bsz, dst + out, fi.block_max, hist);
        if (d < 0) return -1;                              /* decompressionFailed */
        pos += need;
        if (fi.content_size) remaining -= (uint64_t)d;
        size_t space = (size_t)(est - out);
        if (space >= fi.block_max || (size_t)d <= space) {
            out += (size_t)d;                              /* direct, or fully flushed */
            continue;
        }
        /* decoded into tmpOut: `space` bytes flushed now, the rest on later
         * calls — which only happen while input remains */
        size_t pending = (size_t)d - space;
        out += space;
        while (pending) {
            if (out == est) LZ4F_GROW();
            if (pos == n) return (*out_len = out, 0);      /* tail never flushed */
            size_t sp = (size_t)(est - out), f = pending < sp ? pending : sp;
            out += f;
            pending -= f;
        }
    }
#undef LZ4F_GROW
    /* dstage_getSuffix */
    if (remaining) return -1;                              /* frameSize_wrong */
    if (fi.content_checksum) {
        if (n - pos < 4) return (*out_len = out, 0);       /* storeSuffix: wait */
        if (rd32(s + pos) != rpo_xxh32(dst, out, 0)) return -1;
        pos += 4;
    }
    *out_len = out;
    return pos < n ? -1 : 0; /* "could not consume all input bytes" */
}

/* ======================================================================== */
/* snappy 1.1.8 raw decode (snappy.cc: GetUncompressedLength ->              */
/* Varint::Parse32WithLimit; RawUncompress -> SnappyDecompressor::            */
/* DecompressAllTags into SnappyArrayWriter).                                 */
/* ======================================================================== */
static int snappy_varint32(const uint8_t* s, size_t n, uint32_t* v, size_t* used) {
    uint32_t r = 0;
    for (size_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        uint32_t b = s[i];
        if (i < 4) {
            r |= (b & 127) << (7 * i);
            if (b < 128) { *v = r; *used = i + 1; return 0; }
        } else {
            r |= (b & 127) << 28;
            if (b < 16) { *v = r; *used = 5; return 0; }
            return -1;
        }
    }
    return -1;
}

/* DecompressAllTags restated over one contiguous input.  Succeeds iff the
 * tags end exactly at the end of input and exactly ulen bytes come out. */
static int snappy_decode_tags(const uint8_t* s, size_t n, size_t ip, uint8_t* dst, size_t ulen) {
    size_t op = 0;
    while (ip < n) {
        uint8_t c = s[ip];
        size_t extra;
        if ((c & 3) == 0) extra = ((c >> 2) >= 60) ? (size_t)((c >> 2) - 59) : 0;
        else if ((c & 3) == 1) extra = 1;
        else if ((c & 3) == 2) extra = 2;
        else extra = 4;
        if (n - ip < 1 + extra) return -1; /* RefillTag cannot stitch the tag */
        ip++;
        if ((c & 3) == 0) {
            size_t lit = (size_t)(c >> 2) + 1;
            if (lit >= 61) {
                size_t ll = lit - 60;
                uint32_t v = 0;
                for (size_t k = 0; k < ll; k++) v |= (uint32_t)s[ip + k] << (8 * k);
                lit = (size_t)v + 1;
                ip += ll;
            }
            if (n - ip < lit) return -1;   /* premature end of input */
            if (ulen - op < lit) return -1; /* SnappyArrayWriter::Append overflow */
            memcpy(dst + op, s + ip, lit);
            op += lit;
            ip += lit;
        } else {
            size_t len, off;
            if ((c & 3) == 1) {
                len = 4 + ((c >> 2) & 7);
                off = ((size_t)(c >> 5) << 8) | s[ip];
            } else if ((c & 3) == 2) {
                len = (size_t)(c >> 2) + 1;
                off = rd16(s + ip);
            } else {
                len = (size_t)(c >> 2) + 1;
                off = rd32(s + ip);
            }
            ip += extra;
            /* AppendFromSelf: Produced() <= offset - 1u || op_end > op_limit_ */
            if (off == 0 || op < off || ulen - op < len) return -1;
            for (size_t k = 0; k < len; k++) dst[op + k] = dst[op + k - off];
            op += len;
        }
    }
    return op == ulen ? 0 : -1; /* decompressor->eof() && writer->CheckLength() */
}

/* snappy::RawUncompress on one buffer (length varint + tags) */
static int snappy_raw_checked(const uint8_t* s, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    uint32_t ulen;
    size_t used;
    if (snappy_varint32(s, n, &ulen, &used)) return -1;
    /* no tag sequence expands more than 64/3 per input byte: a longer
     * declared length can never be produced exactly -> RawUncompress fails */
    if ((uint64_t)ulen > 22ull * (uint64_t)n + 64) return -1;
    if (ulen > cap) return -2;
    if (snappy_decode_tags(s, n, used, dst, ulen)) return -1;
    *out_len = ulen;
    return 0;
}

int rpo_snappy_raw_uncompress(const uint8_t* s, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    /* compression/snappy_standard_compressor.cc:43-65 (do_uncompressed) */
    uint32_t ulen;
    size_t used;
    *out_len = 0;
    if (snappy_varint32(s, n, &ulen, &used)) return -1;
    if (ulen == 0) return 0; /* "empty frame": RawUncompress is not called */
    return snappy_raw_checked(s, n, dst, cap, out_len);
}

static const uint8_t k_snappy_java_magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

int rpo_snappy_java_uncompress(const uint8_t* s, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    /* compression/internal/snappy_java_compressor.cc:76-129 */
    *out_len = 0;
    if (n < 16) return rpo_snappy_raw_uncompress(s, n, dst, cap, out_len);
    if (memcmp(s, k_snappy_java_magic, 8) != 0) return rpo_snappy_raw_uncompress(s, n, dst, cap, out_len);
    int32_t min_version = (int32_t)rd32(s + 12); /* native little endian */
    if (min_version < 1) return -1;
    size_t pos = 16, out = 0;
    while (pos != n) {
        if (n - pos < 4) return -1;                       /* consume_be_type out_of_range */
        int32_t clen = (int32_t)(((uint32_t)s[pos] << 24) | ((uint32_t)s[pos + 1] << 16) |
                                 ((uint32_t)s[pos + 2] << 8) | s[pos + 3]);
        pos += 4;
        if (clen < 0) return -1;                          /* sstring overflow */
        if (n - pos < (size_t)clen) return -1;            /* consume_to out_of_range */
        size_t got = 0;
        int r = snappy_raw_checked(s + pos, (size_t)clen, dst + out, cap - out, &got);
        if (r) return r;
        out += got;
        pos += (size_t)clen;
    }
    *out_len = out;
    return 0;
}

/* ======================================================================== */
/* gzip: zlib 1.2.11 inflate as gzip_compressor::uncompress drives it         */
/* ======================================================================== */
/* The reference (compression/internal/gzip_compressor.cc:161-230) runs
 * inflateInit2(15 + 32) twice over the whole payload: a sizing pass through a
 * 512-byte buffer (buffer_for_input: total_out), then the real pass into a
 * buffer of exactly that size.  Its loop only throws on Z_STREAM_ERROR /
 * Z_NEED_DICT / Z_DATA_ERROR / Z_MEM_ERROR, so:
 *   - an error anywhere before the end of the first member throws;
 *   - a stream that runs out of input is NOT an error: the output is every
 *     symbol zlib could decode from the bytes present (a literal as soon as
 *     its code is complete, a match once its length, distance and extra bits
 *     are), stored blocks byte by byte;
 *   - bytes after the first member are ignored.
 * The state machine below follows zlib's inflate() (inflate.c HEAD ..
 * DONE) and inflate_table()'s acceptance rules (over-subscribed codes are
 * errors, incomplete ones only allowed for a single 1-bit literal/length or
 * distance code; an all-zero code-length code decodes 1 bit per symbol as
 * length 0, zlib's "wait for decoding to report error" table).  Bits are
 * pulled one byte at a time exactly when zlib's NEEDBITS / PULLBYTE would,
 * so truncation is detected at the same symbol.  gz_header fields are not
 * kept (the reference passes an uninitialised gz_header to inflateGetHeader;
 * the name / extra / comment copies it would make are undefined there and
 * have no effect on the output here). */
typedef struct {
    const uint8_t* s;
    size_t n, pos;     /* input and bytes pulled */
    uint64_t hold;
    unsigned bits;
} rpo_zbits;

static int zb_need(rpo_zbits* b, unsigned k) {
    while (b->bits < k) {
        if (b->pos >= b->n) return 0;
        b->hold |= (uint64_t)b->s[b->pos++] << b->bits;
        b->bits += 8;
    }
    return 1;
}
static unsigned zb_peek(const rpo_zbits* b, unsigned k) { return (unsigned)(b->hold & ((1ull << k) - 1)); }
static void zb_drop(rpo_zbits* b, unsigned k) { b->hold >>= k; b->bits -= k; }

static uint32_t g_crc32_table[256];
static void crc32_ieee_init(void) {
    if (g_crc32_table[1]) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        g_crc32_table[i] = c;
    }
}
/* zlib crc32(crc, p, n) */
static uint32_t crc32_ieee(uint32_t crc, const uint8_t* p, size_t n) {
    crc32_ieee_init();
    crc = ~crc;
    for (size_t i = 0; i < n; i++) crc = g_crc32_table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}
/* zlib adler32(adler, p, n) */
static uint32_t adler32_z(uint32_t adler, const uint8_t* p, size_t n) {
    uint32_t a = adler & 0xFFFF, b = adler >> 16;
    for (size_t i = 0; i < n; i++) {
        a = (a + p[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return (b << 16) | a;
}

/* canonical Huffman code (deflate's bit-reversed packing) */
typedef struct {
    uint16_t count[16];   /* codes per length */
    uint16_t sym[320];    /* symbols ordered by (length, value) */
    int empty;            /* no codes at all (zlib's max == 0 table) */
} rpo_huff;

/* inflate_table acceptance (zlib 1.2.11 inftrees.c): 0 ok, -1 error.
 * type: 0 CODES, 1 LENS, 2 DISTS */
static int huff_build(rpo_huff* h, const uint16_t* lens, unsigned n, int type) {
    memset(h->count, 0, sizeof h->count);
    for (unsigned i = 0; i < n; i++) h->count[lens[i]]++;
    unsigned max = 15;
    while (max >= 1 && h->count[max] == 0) max--;
    h->empty = max == 0;
    if (max == 0) return 0;
    int left = 1;
    for (unsigned len = 1; len <= 15; len++) {
        left <<= 1;
        left -= h->count[len];
        if (left < 0) return -1;             /* over-subscribed */
    }
    if (left > 0 && (type == 0 || max != 1)) return -1;  /* incomplete */
    uint16_t offs[16];
    offs[1] = 0;
    for (unsigned len = 1; len < 15; len++) offs[len + 1] = offs[len] + h->count[len];
    for (unsigned i = 0; i < n; i++)
        if (lens[i]) h->sym[offs[lens[i]]++] = (uint16_t)i;
    return 0;
}

/* Decode one symbol: 1 decoded (*sym, bits dropped), 0 needs more input,
 * -1 an invalid code (bits dropped).  zlib looks codes up with the bits it
 * holds (missing ones read as zero) and pulls a byte whenever the entry
 * found needs more bits than it holds; that is: the shortest code matching
 * the zero-extended bits decodes once all its bits are present. */
static int huff_decode(const rpo_huff* h, rpo_zbits* b, unsigned* sym) {
    for (;;) {
        if (h->empty) {  /* zlib's table for no codes: op 64, bits 1 */
            if (!zb_need(b, 1)) return 0;
            zb_drop(b, 1);
            *sym = 0;
            return -1;
        }
        /* canonical decode over the bits held */
        int code = 0, first = 0, index = 0;
        unsigned len;
        for (len = 1; len <= 15; len++) {
            code |= (len <= b->bits) ? (int)((b->hold >> (len - 1)) & 1) : 0;
            int count = h->count[len];
            if (code - count < first) {
                if (len > b->bits) break;  /* the code needs bits not held yet */
                *sym = h->sym[index + (code - first)];
                zb_drop(b, len);
                return 1;
            }
            index += count;
            first += count;
            first <<= 1;
            code <<= 1;
        }
        if (len > 15) {
            /* no code matches: only possible for an incomplete single 1-bit
             * code (zlib fills the hole with op 64, bits 1) */
            if (b->bits < 1 && !zb_need(b, 1)) return 0;
            zb_drop(b, 1);
            return -1;
        }
        if (b->pos >= b->n) return 0;
        b->hold |= (uint64_t)b->s[b->pos++] << b->bits;
        b->bits += 8;
    }
}

static const uint16_t k_len_base[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                        35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t k_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                        3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t k_dist_base[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
                                         6145, 8193, 12289, 16385, 24577};
static const uint8_t k_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                         6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t k_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* emit a byte (counted always, stored while it fits) */
#define ZOUT(byte)                                   \
    do {                                             \
        const uint8_t zb_ = (uint8_t)(byte);         \
        if (total < cap) dst[total] = zb_;           \
        total++;                                     \
    } while (0)


int rpo_gzip_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    rpo_zbits b = {src, n, 0, 0, 0};
    size_t total = 0;
    int err = 0, gz = 0;
    unsigned flags = 0;
    uint32_t hcheck = 0;
    rpo_huff lencode, distcode, codecode;
    rpo_huff* L = &lencode; rpo_huff* D = &distcode; rpo_huff* C = &codecode;
    *out_len = 0;
    /* HEAD */
    if (!zb_need(&b, 16)) goto done;
    if ((b.hold & 0xFFFF) == 0x8b1f) {
        gz = 1;
        hcheck = crc32_ieee(0, src, 2);
        zb_drop(&b, 16);
        /* FLAGS */
        if (!zb_need(&b, 16)) goto done;
        flags = (unsigned)(b.hold & 0xFFFF);
        if ((flags & 0xff) != 8) { err = 1; goto done; }     /* unknown compression method */
        if (flags & 0xe000) { err = 1; goto done; }           /* unknown header flags set */
        if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + b.pos - 2, 2);
        zb_drop(&b, 16);
        /* TIME, OS */
        if (!zb_need(&b, 32)) goto done;
        if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + b.pos - 4, 4);
        zb_drop(&b, 32);
        if (!zb_need(&b, 16)) goto done;
        if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + b.pos - 2, 2);
        zb_drop(&b, 16);
        if (flags & 0x0400) {  /* EXLEN, EXTRA */
            if (!zb_need(&b, 16)) goto done;
            size_t xlen = (size_t)(b.hold & 0xFFFF);
            if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + b.pos - 2, 2);
            zb_drop(&b, 16);
            size_t have = n - b.pos, copy = xlen < have ? xlen : have;
            if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + b.pos, copy);
            b.pos += copy;
            if (copy < xlen) goto done;
        }
        for (unsigned f = 0x0800; f <= 0x1000; f <<= 1) {  /* NAME, COMMENT */
            if (!(flags & f)) continue;
            if (b.pos >= n) goto done;
            size_t start = b.pos;
            uint8_t c;
            do c = src[b.pos++]; while (c && b.pos < n);
            if (flags & 0x0200) hcheck = crc32_ieee(hcheck, src + start, b.pos - start);
            if (c) goto done;
        }
        if (flags & 0x0200) {  /* HCRC */
            if (!zb_need(&b, 16)) goto done;
            if ((b.hold & 0xFFFF) != (hcheck & 0xFFFF)) { err = 1; goto done; }  /* header crc mismatch */
            zb_drop(&b, 16);
        }
    } else {
        /* zlib wrapper */
        const unsigned hold = (unsigned)(b.hold & 0xFFFF);
        if ((((hold & 0xFF) << 8) + (hold >> 8)) % 31) { err = 1; goto done; }  /* incorrect header check */
        if ((hold & 0x0F) != 8) { err = 1; goto done; }                          /* unknown compression method */
        if (((hold >> 4) & 0x0F) + 8 > 15) { err = 1; goto done; }              /* invalid window size */
        zb_drop(&b, 16);
        if (hold & 0x2000) {  /* FDICT: DICTID then Z_NEED_DICT */
            if (!zb_need(&b, 32)) goto done;
            err = 1;
            goto done;
        }
    }
    /* blocks */
    for (;;) {
        if (!zb_need(&b, 3)) goto done;
        const unsigned last = zb_peek(&b, 1);
        const unsigned type = (unsigned)((b.hold >> 1) & 3);
        zb_drop(&b, 3);
        if (type == 0) {  /* STORED */
            zb_drop(&b, b.bits & 7);
            if (!zb_need(&b, 32)) goto done;
            if ((b.hold & 0xFFFF) != (((b.hold >> 16) & 0xFFFF) ^ 0xFFFF)) { err = 1; goto done; }
            size_t length = (size_t)(b.hold & 0xFFFF);
            zb_drop(&b, 32);  /* INITBITS: the hold is empty (whole bytes were pulled exactly) */
            while (length) {
                if (b.pos >= n) goto done;
                ZOUT(src[b.pos++]);
                length--;
            }
        } else if (type == 3) {
            err = 1;  /* invalid block type */
            goto done;
        } else {
            if (type == 1) {  /* fixed codes */
                uint16_t lens[320];
                unsigned i = 0;
                for (; i < 144; i++) lens[i] = 8;
                for (; i < 256; i++) lens[i] = 9;
                for (; i < 280; i++) lens[i] = 7;
                for (; i < 288; i++) lens[i] = 8;
                huff_build(L, lens, 288, 1);
                for (i = 0; i < 32; i++) lens[i] = 5;
                huff_build(D, lens, 32, 2);
            } else {  /* TABLE */
                if (!zb_need(&b, 14)) goto done;
                const unsigned nlen = zb_peek(&b, 5) + 257;
                zb_drop(&b, 5);
                const unsigned ndist = zb_peek(&b, 5) + 1;
                zb_drop(&b, 5);
                const unsigned ncode = zb_peek(&b, 4) + 4;
                zb_drop(&b, 4);
                if (nlen > 286 || ndist > 30) { err = 1; goto done; }  /* too many length or distance symbols */
                uint16_t lens[320];
                unsigned have = 0;
                while (have < ncode) {
                    if (!zb_need(&b, 3)) goto done;
                    lens[k_clen_order[have++]] = (uint16_t)zb_peek(&b, 3);
                    zb_drop(&b, 3);
                }
                while (have < 19) lens[k_clen_order[have++]] = 0;
                if (huff_build(C, lens, 19, 0)) { err = 1; goto done; }  /* invalid code lengths set */
                have = 0;
                while (have < nlen + ndist) {
                    unsigned sym;
                    int r = huff_decode(C, &b, &sym);
                    if (r == 0) goto done;
                    if (r < 0) sym = 0;  /* zlib's CODELENS does not check op: an invalid entry is length 0 */
                    if (sym < 16) {
                        lens[have++] = (uint16_t)sym;
                        continue;
                    }
                    /* the code's bits are already dropped; zlib needs code + extra bits
                     * together (NEEDBITS(here.bits + k)) before dropping the code: the
                     * same truncation point, since the code bits were present */
                    unsigned len = 0, copy;
                    if (sym == 16) {
                        if (!zb_need(&b, 2)) goto done;
                        if (have == 0) { err = 1; goto done; }  /* invalid bit length repeat */
                        len = lens[have - 1];
                        copy = 3 + zb_peek(&b, 2);
                        zb_drop(&b, 2);
                    } else if (sym == 17) {
                        if (!zb_need(&b, 3)) goto done;
                        copy = 3 + zb_peek(&b, 3);
                        zb_drop(&b, 3);
                    } else {
                        if (!zb_need(&b, 7)) goto done;
                        copy = 11 + zb_peek(&b, 7);
                        zb_drop(&b, 7);
                    }
                    if (have + copy > nlen + ndist) { err = 1; goto done; }  /* invalid bit length repeat */
                    while (copy--) lens[have++] = (uint16_t)len;
                }
                if (lens[256] == 0) { err = 1; goto done; }  /* invalid code -- missing end-of-block */
                if (huff_build(L, lens, nlen, 1)) { err = 1; goto done; }       /* invalid literal/lengths set */
                if (huff_build(D, lens + nlen, ndist, 2)) { err = 1; goto done; } /* invalid distances set */
            }
            /* LEN .. MATCH */
            for (;;) {
                unsigned sym;
                int r = huff_decode(L, &b, &sym);
                if (r == 0) goto done;
                if (r < 0 || sym > 285) { err = 1; goto done; }  /* invalid literal/length code */
                if (sym < 256) { ZOUT(sym); continue; }
                if (sym == 256) break;
                sym -= 257;
                unsigned length = k_len_base[sym];
                if (k_len_extra[sym]) {
                    if (!zb_need(&b, k_len_extra[sym])) goto done;
                    length += zb_peek(&b, k_len_extra[sym]);
                    zb_drop(&b, k_len_extra[sym]);
                }
                r = huff_decode(D, &b, &sym);
                if (r == 0) goto done;
                if (r < 0 || sym > 29) { err = 1; goto done; }  /* invalid distance code */
                unsigned dist = k_dist_base[sym];
                if (k_dist_extra[sym]) {
                    if (!zb_need(&b, k_dist_extra[sym])) goto done;
                    dist += zb_peek(&b, k_dist_extra[sym]);
                    zb_drop(&b, k_dist_extra[sym]);
                }
                if (dist > total) { err = 1; goto done; }  /* invalid distance too far back */
                for (unsigned k = 0; k < length; k++) {
                    const size_t from = total - dist;
                    ZOUT(from < cap ? dst[from] : 0);
                }
            }
        }
        if (last) break;
    }
    /* CHECK, LENGTH */
    zb_drop(&b, b.bits & 7);
    if (!zb_need(&b, 32)) goto done;
    {
        const uint32_t w = (uint32_t)(b.hold & 0xFFFFFFFFu);
        if (gz) {
            if (total <= cap && w != crc32_ieee(0, dst, total)) { err = 1; goto done; }   /* incorrect data check */
        } else {
            const uint32_t be = (w >> 24) | ((w >> 8) & 0xFF00u) | ((w << 8) & 0xFF0000u) | (w << 24);
            if (total <= cap && be != adler32_z(1, dst, total)) { err = 1; goto done; }
        }
        if (total > cap) err = 2;  /* the check needs the bytes: the caller resizes and retries */
        zb_drop(&b, 32);
    }
    if (gz && err == 0) {
        if (!zb_need(&b, 32)) goto done;
        if ((uint32_t)(b.hold & 0xFFFFFFFFu) != (uint32_t)total) { err = 1; goto done; }  /* incorrect length check */
    }
done:
    *out_len = total;
    if (err == 1) { *out_len = 0; return -1; }
    if (total > cap) return -2;
    return 0;
}
#undef ZOUT

/* ======================================================================== */
/* zstd: stream_zstd::do_uncompress (compression/stream_zstd.cc:152-178)      */
/* over libzstd (a system dependency; dlopen'd, the library not restated)     */
/* ======================================================================== */
typedef struct { const void* src; size_t size, pos; } rpo_zin;
typedef struct { void* dst; size_t size, pos; } rpo_zout;
static struct {
    int tried;
    size_t (*estimate)(size_t);
    void* (*init_static)(void*, size_t);
    size_t (*decompress_stream)(void*, rpo_zout*, rpo_zin*);
    unsigned (*is_error)(size_t);
} g_zstd;

static int zstd_load(void) {
    if (!g_zstd.tried) {
        g_zstd.tried = 1;
        void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            g_zstd.estimate = (size_t(*)(size_t))dlsym(h, "ZSTD_estimateDStreamSize");
            g_zstd.init_static = (void* (*)(void*, size_t))dlsym(h, "ZSTD_initStaticDCtx");
            g_zstd.decompress_stream = (size_t(*)(void*, rpo_zout*, rpo_zin*))dlsym(h, "ZSTD_decompressStream");
            g_zstd.is_error = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
        }
    }
    return g_zstd.estimate && g_zstd.init_static && g_zstd.decompress_stream && g_zstd.is_error;
}

/* The reference's loop: a static DCtx over ZSTD_estimateDStreamSize(8 MiB)
 * of workspace (zstd_decompress_workspace_bytes, config/configuration.cc:
 * 911-916), a 64 KiB output buffer appended whenever it fills while input
 * remains; an error only counts when the output buffer is not full. */
int rpo_zstd_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (!zstd_load()) return -3;
    const size_t ws = g_zstd.estimate((size_t)8 << 20);
    void* mem = malloc(ws + (64u << 10));
    if (!mem) return -1;
    uint8_t* obuf = (uint8_t*)mem + ws;
    void* dctx = g_zstd.init_static(mem, ws);
    int rc = dctx ? 0 : -1;
    size_t total = 0;
    rpo_zout o = {obuf, 64u << 10, 0};
    rpo_zin i = {src, n, 0};
    while (rc == 0 && i.pos != i.size) {
        const size_t err = g_zstd.decompress_stream(dctx, &o, &i);
        if (i.pos != i.size && o.pos == o.size) {
            if (total + o.size <= cap) memcpy(dst + total, obuf, o.size);
            total += o.size;
            o.size = 64u << 10;
            o.pos = 0;
        } else if (g_zstd.is_error(err)) {
            rc = -1;
        }
    }
    if (rc == 0) {
        if (total + o.pos <= cap) memcpy(dst + total, obuf, o.pos);
        total += o.pos;
        *out_len = total;
        if (total > cap) rc = -2;
    }
    free(mem);
    return rc;
}

int rpo_uncompress(int codec, const uint8_t* s, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    /* compression/compression.cc:34-55 */
    *out_len = 0;
    if (n == 0) return -1;
    switch (codec) {
    case RPGPU_CODEC_GZIP: return rpo_gzip_uncompress(s, n, dst, cap, out_len);
    case RPGPU_CODEC_SNAPPY: return rpo_snappy_java_uncompress(s, n, dst, cap, out_len);
    case RPGPU_CODEC_LZ4: return rpo_lz4f_uncompress(s, n, dst, cap, out_len);
    case RPGPU_CODEC_ZSTD: return rpo_zstd_uncompress(s, n, dst, cap, out_len);
    default: return -1;
    }
}

/* Engine plan rule for a gzip member (not reference semantics; the reference
 * sizes its buffer with the same decode, gzip_compressor.cc:187-195): the
 * bytes the sizing pass yields rounded up to 16, 0 when it rejects.  The
 * sizing pass holds no output, so it stops short of the trailer checks. */
uint64_t rpo_gzip_plan(const uint8_t* s, size_t n) {
    size_t total = 0;
    if (n == 0) return 0;
    if (rpo_gzip_uncompress(s, n, NULL, 0, &total) == -1) return 0;
    return ((uint64_t)total + 15) & ~(uint64_t)15;
}

/* ... and for a host-decoded zstd payload: its decoded size rounded up to
 * 16, 0 when the reference throws */
uint64_t rpo_zstd_plan(const uint8_t* s, size_t n) {
    size_t total = 0;
    if (n == 0) return 0;
    const int rc = rpo_zstd_uncompress(s, n, NULL, 0, &total);
    if (rc != 0 && rc != -2) return 0;
    return ((uint64_t)total + 15) & ~(uint64_t)15;
}

static uint64_t decode_capacity_raw(int codec, const uint8_t* s, size_t n);

/* Engine plan rule (not reference semantics): bytes reserved in the decoded
 * arena for one compressed payload, from its frame structure alone, rounded
 * up to 16 so every slot starts 16-byte aligned. */
uint64_t rpo_decode_capacity(int codec, const uint8_t* s, size_t n) {
    return (decode_capacity_raw(codec, s, n) + 15) & ~(uint64_t)15;
}

static uint64_t decode_capacity_raw(int codec, const uint8_t* s, size_t n) {
    if (n == 0) return 0;
    if (codec == RPGPU_CODEC_LZ4) {
        lz4f_info fi;
        int64_t h = lz4f_parse_header(s, n, &fi);
        if (h < 0 || fi.skippable) return 0;
        uint64_t cap = 0;
        size_t pos = (size_t)h;
        while (n - pos >= 4) {
            uint32_t bh = rd32(s + pos);
            if (bh == 0) break;
            size_t bsz = bh & 0x7FFFFFFFu;
            if (bsz > fi.block_max) break;
            cap += (bh & 0x80000000u) ? bsz : fi.block_max;
            pos += 4;
            size_t adv = bsz + (fi.block_checksum ? 4 : 0);
            if (n - pos < adv) break;
            pos += adv;
        }
        return cap;
    }
    if (codec == RPGPU_CODEC_SNAPPY) {
        uint32_t ulen;
        size_t used;
        if (n < 16 || memcmp(s, k_snappy_java_magic, 8) != 0) {
            if (snappy_varint32(s, n, &ulen, &used)) return 0;
            return ((uint64_t)ulen <= 22ull * n + 64) ? ulen : 0;
        }
        uint64_t cap = 0;
        size_t pos = 16;
        while (n - pos >= 4) {
            int32_t clen = (int32_t)(((uint32_t)s[pos] << 24) | ((uint32_t)s[pos + 1] << 16) |
                                     ((uint32_t)s[pos + 2] << 8) | s[pos + 3]);
            if (clen <= 0 || n - pos - 4 < (size_t)clen) break;
            if (snappy_varint32(s + pos + 4, (size_t)clen, &ulen, &used)) break;
            if ((uint64_t)ulen > 22ull * (uint64_t)clen + 64) break;
            cap += ulen;
            pos += 4 + (size_t)clen;
        }
        return cap;
    }
    return 0;
}

/* ======================================================================== */
/* Segment pipeline                                                          */
/* ======================================================================== */
int rpo_batch_valid_layout(const rpgpu_batch_result* b, uint32_t job_flags, uint32_t layout) {
    if (layout == RPGPU_LAYOUT_WIRE && !(b->flags & RPGPU_F_WIRE_V2)) return 0;
    return rpo_batch_valid(b, job_flags);
}

int rpo_batch_valid(const rpgpu_batch_result* b, uint32_t job_flags) {
    uint32_t f = b->flags;
    if (!(f & RPGPU_F_HEADER_OK) || !(f & RPGPU_F_COMPLETE) || !(f & RPGPU_F_CRC_OK)) return 0;
    if (f & RPGPU_F_CODEC_INVALID) return 0;
    if ((f & RPGPU_F_COMPRESSED) && (job_flags & RPGPU_JOB_DECODE) &&
        !(f & RPGPU_F_CODEC_UNSUPPORTED) && !(f & RPGPU_F_CODEC_OK)) return 0;
    if ((f & RPGPU_F_PARSED) && !(f & RPGPU_F_PARSE_OK)) return 0;
    return 1;
}

static void fill_result_header(rpgpu_batch_result* r, const rpo_header* h) {
    r->base_offset = h->base_offset;
    r->first_timestamp = h->first_timestamp;
    r->max_timestamp = h->max_timestamp;
    r->producer_id = h->producer_id;
    r->size_bytes = h->size_bytes;
    r->record_count = h->record_count;
    r->last_offset_delta = h->last_offset_delta;
    r->base_sequence = h->base_sequence;
    r->header_crc = h->header_crc;
    r->crc = (uint32_t)h->crc;
    r->attrs = h->attrs;
    r->producer_epoch = h->producer_epoch;
    r->type = h->type;
}

/* One segment.  Disk layout: continuous_batch_parser + checksumming_consumer
 * (storage/parser.cc:96-254, storage/log_replayer.cc:27-114).  Wire layout:
 * kafka::batch_reader over one record set (kafka/protocol/batch_reader.cc:
 * 50-156) adapting each batch with kafka_batch_adapter::adapt
 * (kafka_batch_adapter.cc:126-188): the chain is structural (batch_length +
 * 12 per batch); first_bad is the first batch do_load_slice would reject
 * (not v2, crc mismatch, codec bits 5-7 -- compressed() throws --, or a sync
 * record parse failure of an uncompressed batch). */
int64_t rpo_scan_segment_layout(const uint8_t* seg, uint64_t len, uint32_t segment, uint32_t job_flags,
                                uint32_t layout, rpgpu_batch_result* batches, uint64_t batch_cap,
                                rpgpu_record_index* index, uint64_t index_cap,
                                uint8_t* decoded, uint64_t decoded_cap,
                                rpgpu_segment_summary* sm, rpo_job_state* st) {
    const int wire = layout == RPGPU_LAYOUT_WIRE;
    memset(sm, 0, sizeof *sm);
    sm->first_batch = st->batch_base;
    uint64_t pos = 0, phys = 0;
    uint64_t nb = 0;
    int64_t first_bad = -1;
    uint64_t seg_records = 0;
    for (;;) {
        /* read_header_impl (storage/parser.cc:139-176) */
        uint64_t rem = len - pos;
        if (rem == 0) { sm->terminal_errc = RPGPU_ERRC_END_OF_STREAM; sm->terminal_eof = 1; break; }
        if (rem < RPGPU_HEADER_SIZE) { sm->terminal_errc = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES; sm->terminal_eof = 1; break; }
        rpo_header h;
        int v2 = 0;
        uint32_t hc;
        if (wire) {
            /* read_record_batch_info (batch_reader.cc:50-88) needs 61 bytes;
             * adapt() then reads the 61-byte header out of the batch's own
             * batch_length + 12 bytes: a smaller batch throws */
            v2 = rpo_header_from_wire(seg + pos, &h) == 2;
            if ((int64_t)(int32_t)be_n(seg + pos + 8, 4) + 12 < (int64_t)RPGPU_HEADER_SIZE) {
                sm->terminal_errc = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES;
                break;
            }
            hc = rpo_internal_header_only_crc(&h); /* the header_crc the batch gets on disk */
        } else {
            rpo_header_from_disk(seg + pos, &h);
            if (h.header_crc == 0) { sm->terminal_errc = RPGPU_ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER; break; }
            hc = rpo_internal_header_only_crc(&h);
            if (hc != h.header_crc) { sm->terminal_errc = RPGPU_ERRC_HEADER_ONLY_CRC_MISSMATCH; break; }
        }
        if (st->batch_base + nb >= batch_cap) { st->overflow |= 1; sm->terminal_errc = RPGPU_ERRC_NONE; break; }
        rpgpu_batch_result* r = &batches[st->batch_base + nb];
        memset(r, 0, sizeof *r);
        r->file_pos = pos;
        r->segment = segment;
        fill_result_header(r, &h);
        r->header_crc_computed = hc;
        r->flags = RPGPU_F_HEADER_OK;
        if (wire && v2) r->flags |= RPGPU_F_WIRE_V2;
        /* consume_records: size_bytes - 61 computed unsigned (storage/parser.cc:207) */
        uint64_t need = (uint32_t)((uint32_t)h.size_bytes - RPGPU_HEADER_SIZE);
        const uint8_t* payload = seg + pos + RPGPU_HEADER_SIZE;
        uint32_t codec = (uint16_t)h.attrs & 7;
        if (rem - RPGPU_HEADER_SIZE < need) {
            /* short read -> input_stream_not_enough_bytes with eof() set */
            r->index_base = st->index_base;
            r->decoded_off = st->decoded_base;
            if (codec) r->flags |= RPGPU_F_COMPRESSED;
            if (codec >= 5) r->flags |= RPGPU_F_CODEC_INVALID;
            nb++;
            if (first_bad < 0) first_bad = (int64_t)nb - 1;
            sm->terminal_errc = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES;
            sm->terminal_eof = 1;
            sm->terminal_pos = pos;
            phys += (uint64_t)(int64_t)h.size_bytes;
            goto done;
        }
        r->flags |= RPGPU_F_COMPLETE;
        /* the BE40 prefix is wire bytes [21, 61) as they stand: on the wire
         * this is CRC32C(wire[21..end)) (kafka_batch_adapter.cc:94-124); there
         * valid_crc is only computed for v2 batches */
        r->crc_computed = rpo_crc_record_batch(&h, payload, need);
        if (r->crc_computed == (uint32_t)h.crc && (!wire || v2)) r->flags |= RPGPU_F_CRC_OK;
        else if (!wire && first_bad < 0) first_bad = (int64_t)nb;
        /* adapt() parses records only after the v2 and crc checks */
        const int may_walk = !wire || (r->flags & RPGPU_F_CRC_OK);
        if (codec) r->flags |= RPGPU_F_COMPRESSED;
        if (codec >= 5) r->flags |= RPGPU_F_CODEC_INVALID;
        /* zstd: decoded in DECODE jobs (on the device, or on the host with
         * RPGPU_JOB_HOST_CODECS: the same plan and verdicts) */
        if (codec == RPGPU_CODEC_ZSTD && !(job_flags & RPGPU_JOB_DECODE)) r->flags |= RPGPU_F_CODEC_UNSUPPORTED;

        /* Plan (engine rule, see DESIGN.md "index and arena planning"): the
         * record-index slots and decode-arena bytes of a batch are reserved
         * from its header and payload structure alone, before any decode, so
         * the GPU can assign them with prefix sums.  Reservations never depend
         * on whether the decode or the walk later succeed. */
        uint64_t slots = 0, cap = 0;
        int decodable = (codec == RPGPU_CODEC_LZ4 || codec == RPGPU_CODEC_SNAPPY || codec == RPGPU_CODEC_GZIP ||
                         codec == RPGPU_CODEC_ZSTD) &&
                        (job_flags & RPGPU_JOB_DECODE);
        if (codec == 0) {
            if ((job_flags & RPGPU_JOB_PARSE) && h.record_count > 0 && (uint64_t)h.record_count <= need)
                slots = (uint64_t)h.record_count;
        } else if (decodable) {
            cap = codec == RPGPU_CODEC_GZIP ? rpo_gzip_plan(payload, need)
                : codec == RPGPU_CODEC_ZSTD ? rpo_zstd_plan(payload, need)
                : rpo_decode_capacity((int)codec, payload, need);
            if ((job_flags & RPGPU_JOB_PARSE) && h.record_count > 0 && (uint64_t)h.record_count <= cap)
                slots = (uint64_t)h.record_count;
        }
        r->index_base = st->index_base;
        r->decoded_off = st->decoded_base;
        st->index_base += slots;
        st->decoded_base += cap;
        seg_records += slots;
        int idx_ok = r->index_base + slots <= index_cap;
        if (!idx_ok) st->overflow |= 2;

        const uint8_t* walk = NULL;
        uint64_t walk_len = 0;
        int do_walk = 0;
        if (codec == 0) {
            r->decoded_len = (uint32_t)need;
            walk = payload;
            walk_len = need;
            do_walk = (job_flags & RPGPU_JOB_PARSE) && may_walk;
        } else if (decodable) {
            if (r->decoded_off + cap > decoded_cap) {
                st->overflow |= 4;
                r->flags |= RPGPU_F_DECODE_OVERFLOW;
            } else {
                size_t got = 0;
                int rc = rpo_uncompress((int)codec, payload, need, decoded + r->decoded_off, cap, &got);
                if (rc == -2) {
                    r->flags |= RPGPU_F_DECODE_OVERFLOW; /* cannot happen with the planned cap */
                } else if (rc == 0) {
                    r->flags |= RPGPU_F_CODEC_OK;
                    r->decoded_len = (uint32_t)got;
                    /* reset_size_checksum_metadata (storage/parser_utils.cc:114-120) */
                    rpo_header nh = h;
                    nh.attrs = (int16_t)((uint16_t)nh.attrs & ~7u);
                    nh.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + got);
                    nh.crc = (int32_t)rpo_crc_record_batch(&nh, decoded + r->decoded_off, got);
                    nh.header_crc = rpo_internal_header_only_crc(&nh);
                    r->decoded_crc = (uint32_t)nh.crc;
                    r->decoded_header_crc = nh.header_crc;
                    walk = decoded + r->decoded_off;
                    walk_len = got;
                    do_walk = (job_flags & RPGPU_JOB_PARSE) && may_walk;
                }
            }
        }
        if (do_walk) {
            uint8_t perr;
            uint64_t trailing;
            r->records_parsed = rpo_walk_records(walk, walk_len, h.record_count, (uint32_t)(st->batch_base + nb),
                                                 idx_ok ? index + r->index_base : NULL, idx_ok ? slots : 0, &perr, &trailing);
            r->flags |= RPGPU_F_PARSED;
            r->parse_err = perr;
            if (perr == RPGPU_PARSE_ERR_NONE) {
                r->flags |= RPGPU_F_PARSE_ASYNC_OK;
                if (trailing == 0) r->flags |= RPGPU_F_PARSE_OK;
                else r->parse_err = RPGPU_PARSE_ERR_TRAILING;
            }
            if (r->flags & RPGPU_F_PARSE_OK) {
                if (idx_ok) r->flags |= RPGPU_F_INDEX_WRITTEN;
                else r->parse_err = RPGPU_PARSE_ERR_INDEX_CAPACITY;
            }
        }
        if (wire && first_bad < 0) {
            const uint32_t f = r->flags;
            const int accepted = (f & RPGPU_F_CRC_OK) && !(f & RPGPU_F_CODEC_INVALID) &&
                                 !(codec == 0 && (f & RPGPU_F_PARSED) && !(f & RPGPU_F_PARSE_OK));
            if (!accepted) first_bad = (int64_t)nb;
        }
        nb++;
        phys += (uint64_t)(int64_t)h.size_bytes;
        pos += RPGPU_HEADER_SIZE + need;
        if (pos > len) pos = len; /* cannot happen: need <= rem - 61 */
    }
    sm->terminal_pos = pos;
done:
    sm->n_batches = nb;
    sm->n_records = seg_records;
    /* checksumming_consumer checkpoint (storage/log_replayer.cc:62-79) */
    uint64_t good = (first_bad < 0) ? nb : (uint64_t)first_bad;
    sm->first_bad = (uint32_t)good;
    sm->bytes_consumed = 0;
    /* disk: continuous_batch_parser also counts the batch it stopped in;
     * wire: batch_reader consumed the accepted prefix */
    uint64_t upto = (first_bad < 0) ? nb : (uint64_t)first_bad + (wire ? 0 : 1);
    for (uint64_t i = 0; i < upto; i++)
        sm->bytes_consumed += (uint64_t)(int64_t)batches[st->batch_base + i].size_bytes;
    if (good > 0) {
        const rpgpu_batch_result* g = &batches[st->batch_base + good - 1];
        sm->has_checkpoint = 1;
        sm->ckpt_last_offset = (int64_t)((uint64_t)g->base_offset + (uint64_t)(int64_t)g->last_offset_delta);
        /* _file_pos_to_end_of_batch = size_on_disk + physical_base_offset,
         * physical offsets accumulate size_bytes (storage/parser.cc:118-128) */
        uint64_t ph = 0;
        for (uint64_t i = 0; i < good - 1; i++) ph += (uint64_t)(int64_t)batches[st->batch_base + i].size_bytes;
        sm->ckpt_truncate_pos = ph + (uint64_t)(int64_t)g->size_bytes;
    }
    (void)phys;
    st->batch_base += nb;
    return (int64_t)nb;
}

int64_t rpo_scan_segment(const uint8_t* seg, uint64_t len, uint32_t segment, uint32_t job_flags,
                         rpgpu_batch_result* batches, uint64_t batch_cap,
                         rpgpu_record_index* index, uint64_t index_cap,
                         uint8_t* decoded, uint64_t decoded_cap,
                         rpgpu_segment_summary* sm, rpo_job_state* st) {
    return rpo_scan_segment_layout(seg, len, segment, job_flags, RPGPU_LAYOUT_DISK, batches, batch_cap, index,
                                   index_cap, decoded, decoded_cap, sm, st);
}

int rpo_run_job(const uint8_t* data, const uint64_t* seg_offsets, uint32_t n_segments,
                uint32_t job_flags, rpgpu_batch_result* batches, uint64_t batch_cap,
                rpgpu_record_index* index, uint64_t index_cap, uint8_t* decoded,
                uint64_t decoded_cap, rpgpu_segment_summary* summaries,
                rpgpu_job_totals* totals, uint64_t* valid_bitmap) {
    return rpo_run_job_layout(data, seg_offsets, n_segments, job_flags, RPGPU_LAYOUT_DISK, batches, batch_cap, index,
                              index_cap, decoded, decoded_cap, summaries, totals, valid_bitmap);
}

int rpo_run_job_layout(const uint8_t* data, const uint64_t* seg_offsets, uint32_t n_segments,
                       uint32_t job_flags, uint32_t layout, rpgpu_batch_result* batches, uint64_t batch_cap,
                       rpgpu_record_index* index, uint64_t index_cap, uint8_t* decoded,
                       uint64_t decoded_cap, rpgpu_segment_summary* summaries,
                       rpgpu_job_totals* totals, uint64_t* valid_bitmap) {
    rpo_job_state st = {0, 0, 0, 0};
    for (uint32_t s = 0; s < n_segments; s++) {
        rpo_scan_segment_layout(data + seg_offsets[s], seg_offsets[s + 1] - seg_offsets[s], s, job_flags, layout,
                                batches, batch_cap, index, index_cap, decoded, decoded_cap, &summaries[s], &st);
    }
    memset(totals, 0, sizeof *totals);
    totals->n_batches = st.batch_base;
    totals->n_records = st.index_base;
    totals->decoded_bytes = st.decoded_base;
    totals->overflow = st.overflow;
    if (valid_bitmap) {
        for (uint64_t i = 0; i < st.batch_base; i++) {
            if (rpo_batch_valid_layout(&batches[i], job_flags, layout)) valid_bitmap[i >> 6] |= 1ull << (i & 63);
            else valid_bitmap[i >> 6] &= ~(1ull << (i & 63));
        }
    }
    return 0;
}

/* ======================================================================== */
/* CPU baseline (timed on the GPU box's host cores by bench.py)              */
/* ======================================================================== */
typedef struct base_task {
    const uint8_t* data;
    const uint64_t* seg_offsets;
    uint32_t seg_lo, seg_hi;
    int hw;
    int64_t batches;
    uint64_t bytes;
} base_task;

static void* base_worker(void* arg) {
    base_task* t = (base_task*)arg;
    rpgpu_record_index* scratch = (rpgpu_record_index*)malloc(sizeof(rpgpu_record_index) * 65536);
    for (uint32_t s = t->seg_lo; s < t->seg_hi; s++) {
        const uint8_t* seg = t->data + t->seg_offsets[s];
        uint64_t len = t->seg_offsets[s + 1] - t->seg_offsets[s], pos = 0;
        while (len - pos >= RPGPU_HEADER_SIZE) {
            rpo_header h;
            rpo_header_from_disk(seg + pos, &h);
            if (h.header_crc == 0) break;
            uint8_t b[61];
            memcpy(b, seg + pos, 61);
            uint32_t hc = t->hw ? rpo_crc32c_extend_hw(0, b + 4, 57) : rpo_crc32c_extend(0, b + 4, 57);
            if (hc != h.header_crc) break;
            uint64_t need = (uint32_t)((uint32_t)h.size_bytes - RPGPU_HEADER_SIZE);
            if (len - pos - RPGPU_HEADER_SIZE < need) break;
            const uint8_t* payload = seg + pos + RPGPU_HEADER_SIZE;
            uint32_t c = t->hw ? crc_record_batch_hw(&h, payload, need) : rpo_crc_record_batch(&h, payload, need);
            if (c != (uint32_t)h.crc) break;
            if (((uint16_t)h.attrs & 7) == 0) {
                uint8_t perr;
                uint64_t trailing;
                rpo_walk_records(payload, need, h.record_count, 0, scratch, 65536, &perr, &trailing);
            }
            t->batches++;
            t->bytes += RPGPU_HEADER_SIZE + need;
            pos += RPGPU_HEADER_SIZE + need;
        }
    }
    free(scratch);
    return NULL;
}

int64_t rpo_baseline_validate(const uint8_t* data, const uint64_t* seg_offsets,
                              uint32_t n_segments, int threads, int use_hw_crc,
                              double* seconds, uint64_t* bytes) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n_segments) threads = (int)n_segments;
    base_task* tasks = (base_task*)calloc((size_t)threads, sizeof(base_task));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    crc_init();
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        tasks[i].data = data;
        tasks[i].seg_offsets = seg_offsets;
        tasks[i].seg_lo = (uint32_t)((uint64_t)n_segments * (uint64_t)i / (uint64_t)threads);
        tasks[i].seg_hi = (uint32_t)((uint64_t)n_segments * (uint64_t)(i + 1) / (uint64_t)threads);
        tasks[i].hw = use_hw_crc;
        pthread_create(&th[i], NULL, base_worker, &tasks[i]);
    }
    int64_t nb = 0;
    uint64_t by = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        nb += tasks[i].batches;
        by += tasks[i].bytes;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    *bytes = by;
    free(tasks);
    free(th);
    return nb;
}

/* ------------------------------------------------------------------------ */
/* Segment index rebuild (recovery).                                         */
/* ------------------------------------------------------------------------ */

/* index_state::maybe_index (storage/index_state.cc:48-95) for one batch;
 * `acc` is segment_index::_acc after `_acc += hdr.size_bytes`
 * (storage/segment_index.cc:60-61).  Returns 1 when the batch was indexed. */
static int rpo_maybe_index(rpgpu_index_state* st, uint64_t acc, uint64_t step, uint64_t filepos,
                           const rpgpu_batch_result* b, uint32_t* rel_offset, uint32_t* rel_time,
                           uint64_t* position) {
    const int64_t last_offset = (int64_t)((uint64_t)b->base_offset + (uint64_t)(int64_t)b->last_offset_delta);
    int retval = 0;
    if (st->n_entries == 0) { /* empty(): index_state.cc:66-70 */
        st->base_timestamp = b->first_timestamp;
        st->max_timestamp = b->first_timestamp;
        retval = 1;
    }
    st->max_offset = last_offset; /* :73 */
    /* last_timestamp = max(first, last) (:77); max_timestamp = max(...) (:78) */
    const int64_t last_ts = b->max_timestamp > b->first_timestamp ? b->max_timestamp : b->first_timestamp;
    if (last_ts > st->max_timestamp) st->max_timestamp = last_ts;
    if (acc >= step || retval) { /* :80-87, add_entry (index_state.h:70-74) */
        const uint64_t k = st->first_entry + st->n_entries;
        rel_offset[k] = (uint32_t)((uint64_t)b->base_offset - (uint64_t)st->base_offset);
        rel_time[k] = (uint32_t)((uint64_t)last_ts - (uint64_t)st->base_timestamp);
        position[k] = filepos;
        st->n_entries++;
        retval = 1;
    }
    return retval;
}

int rpo_segment_index(const rpgpu_batch_result* batches, uint64_t batch_cap,
                      const rpgpu_segment_summary* summaries, uint32_t n_segments, uint64_t step,
                      rpgpu_index_state* states, uint32_t* rel_offset, uint32_t* rel_time,
                      uint64_t* position) {
    for (uint32_t s = 0; s < n_segments; s++) {
        const rpgpu_segment_summary* sm = &summaries[s];
        rpgpu_index_state* st = &states[s];
        /* checksumming_consumer's constructor: _seg->index().reset() keeps
         * only base_offset (storage/segment_index.cc:44-49) */
        const int64_t base = st->base_offset;
        memset(st, 0, sizeof(*st));
        st->base_offset = base;
        st->first_entry = sm->first_batch;
        st->assert_batch = -1;
        uint64_t n = sm->first_bad; /* consume_batch_end tracks only crc-good batches, stops at the first bad */
        const uint64_t avail = sm->first_batch < batch_cap ? batch_cap - sm->first_batch : 0;
        if (n > avail) { /* the job overflowed its batch capacity */
            n = avail;
            st->assert_batch = -2;
        }
        uint64_t acc = 0; /* segment_index::_acc */
        for (uint64_t i = 0; i < n; i++) {
            const rpgpu_batch_result* b = &batches[sm->first_batch + i];
            if (b->base_offset < st->base_offset) { /* vassert (index_state.cc:57-63) */
                st->assert_batch = (int64_t)i;
                break;
            }
            acc += (uint64_t)(int64_t)b->size_bytes; /* _acc += hdr.size_bytes */
            /* physical_base_offset = end - size_bytes = the header's position (log_replayer.cc:68-70) */
            if (rpo_maybe_index(st, acc, step, b->file_pos, b, rel_offset, rel_time, position)) acc = 0;
            st->tracked++;
        }
    }
    return 0;
}

/* ======================================================================== */
/* Write side, in batch order, in place:            */
/*   RPO_STAMP_OFFSETS: disk_log_appender::operator()                        */
/*     (storage/disk_log_appender.cc:72-74): base_offset = _idx, then         */
/*     _idx = last_offset + 1 (:113-119);                                     */
/*   RPO_STAMP_CRC: storage::internal::reset_size_checksum_metadata          */
/*     (storage/parser_utils.cc:114-120): size_bytes = 61 + payload,          */
/*     crc = crc_record_batch(hdr, payload);                                  */
/*   then header_crc = internal_header_only_crc (model/record_utils.cc:34-55).*/
/* ======================================================================== */
void rpo_stamp_batches(uint8_t* data, const uint64_t* pos, const uint32_t* plen, uint32_t n, int64_t next_offset,
                       uint32_t flags) {
    int64_t idx = next_offset;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t* p = data + pos[i];
        rpo_header h;
        rpo_header_from_disk(p, &h);
        if (flags & 1u) {
            h.base_offset = idx;
            idx = (int64_t)((uint64_t)h.base_offset + (uint64_t)(int64_t)h.last_offset_delta + 1u);
        }
        if (flags & 2u) {
            h.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + plen[i]);
            h.crc = (int32_t)rpo_crc_record_batch(&h, p + RPGPU_HEADER_SIZE, plen[i]);
        }
        h.header_crc = rpo_internal_header_only_crc(&h);
        rpo_header_to_disk(&h, p);
    }
}

/* ========================================================================== */
/* Write side: compression::compressor::compress for lz4 and snappy          */
/* (compression/compression.cc:17-33).                                       */
/*                                                                           */
/* lz4: lz4_frame_compressor::compress (compression/internal/                */
/* lz4_frame_compressor.cc:72-113): LZ4F_compressBegin / Update (one call    */
/* per iobuf fragment) / End with prefs {compressionLevel 1, blockMode       */
/* independent, contentSize = input size}, everything else 0.  liblz4 1.9.3  */
/* (the reference's system dependency, compression/CMakeLists.txt) then      */
/* frames the input as 64 KiB blocks (LZ4F_max64KB, the default block size   */
/* id), whatever the fragmentation: Update buffers partial blocks.  Each     */
/* block is LZ4F_makeBlock -> LZ4F_compressBlock ->                          */
/* LZ4_compress_fast_extState_fastReset(acceleration 1, dstCapacity =        */
/* srcSize - 1) on a table LZ4_prepareTable clears (every block is >= 4 KiB  */
/* or follows a 64 KiB one), i.e. LZ4_compress_generic(byU16, noDict,        */
/* noDictIssue, limitedOutput); 0 ("does not fit") makes a raw block.        */
/*                                                                           */
/* snappy: snappy_java_compressor::compress (compression/internal/           */
/* snappy_java_compressor.cc:58-75): magic, version 1 and min version 1      */
/* (little endian, as the reference appends them), then per iobuf fragment   */
/* a big-endian int32 length and snappy::RawCompress of the fragment:        */
/* libsnappy 1.1.8 Compress = varint length + CompressFragment per 64 KiB    */
/* block with a fresh hash table of CalculateTableSize(block) entries.       */
/*                                                                           */
/* Pinned against the libraries through oracle/_ref (codec_ref.c            */
/* ref_lz4f_compress_stream / ref_snappy_java_compress: the reference's      */
/* driver loops) in tests/test_compress.py.                                  */
/* ========================================================================== */
enum { LZC_MINMATCH = 4, LZC_LASTLITERALS = 5, LZC_MFLIMIT = 12, LZC_MINLENGTH = 13, LZC_SKIPTRIGGER = 6,
       LZC_HASHLOG_U16 = 13 };

static inline uint32_t lz4_hash_u16(uint32_t seq) { return (seq * 2654435761u) >> (32 - LZC_HASHLOG_U16); }

/* LZ4_count(pIn, pMatch, pInLimit) */
static uint32_t lz4_count(const uint8_t* s, uint32_t in, uint32_t match, uint32_t limit) {
    uint32_t start = in;
    while (in < limit && s[in] == s[match]) { in++; match++; }
    return in - start;
}

/* LZ4_compress_generic_validated (lz4 1.9.3 lz4.c), byU16 / noDict /
 * noDictIssue / limitedOutput / acceleration 1, on a zeroed table: the
 * compressed size, or 0 when it does not fit in cap bytes. */
int rpo_lz4_compress_block(const uint8_t* s, int n, uint8_t* dst, int cap) {
    uint16_t table[1 << LZC_HASHLOG_U16];
    memset(table, 0, sizeof table);
    if (n > 65547 - 1) return 0;
    uint32_t ip = 0, anchor = 0;
    const uint32_t iend = (uint32_t)n, mflimit_plus_one = iend - LZC_MFLIMIT + 1, matchlimit = iend - LZC_LASTLITERALS;
    int64_t op = 0;
    const int64_t olimit = cap;
    uint32_t forward_h = 0, match = 0;
    if (n < LZC_MINLENGTH) goto last_literals;
    table[lz4_hash_u16(rd32(s + ip))] = (uint16_t)ip;
    ip++;
    forward_h = lz4_hash_u16(rd32(s + ip));
    for (;;) {
        int64_t token;
        {
            uint32_t forward_ip = ip;
            int step = 1, search_match_nb = 1 << LZC_SKIPTRIGGER;
            for (;;) {
                const uint32_t h = forward_h, current = forward_ip;
                const uint32_t match_index = table[h];
                ip = forward_ip;
                forward_ip += (uint32_t)step;
                step = search_match_nb++ >> LZC_SKIPTRIGGER;
                if (forward_ip > mflimit_plus_one) goto last_literals;
                match = match_index;
                forward_h = lz4_hash_u16(rd32(s + forward_ip));
                table[h] = (uint16_t)current;
                /* byU16 with LZ4_DISTANCE_MAX == 65535: no distance test */
                if (rd32(s + match) == rd32(s + ip)) break;
            }
        }
        /* catch up */
        while (ip > anchor && match > 0 && s[ip - 1] == s[match - 1]) { ip--; match--; }
        {
            const uint32_t lit = ip - anchor;
            token = op++;
            if (op + lit + (2 + 1 + LZC_LASTLITERALS) + lit / 255 > olimit) return 0;
            if (lit >= 15) {
                int64_t len = (int64_t)lit - 15;
                dst[token] = 15 << 4;
                for (; len >= 255; len -= 255) dst[op++] = 255;
                dst[op++] = (uint8_t)len;
            } else {
                dst[token] = (uint8_t)(lit << 4);
            }
            memcpy(dst + op, s + anchor, lit);
            op += lit;
        }
    next_match:
        dst[op] = (uint8_t)(ip - match);
        dst[op + 1] = (uint8_t)((ip - match) >> 8);
        op += 2;
        {
            uint32_t mc = lz4_count(s, ip + LZC_MINMATCH, match + LZC_MINMATCH, matchlimit);
            ip += mc + LZC_MINMATCH;
            if (op + (1 + LZC_LASTLITERALS) + (mc + 240) / 255 > olimit) return 0;
            if (mc >= 15) {
                dst[token] += 15;
                mc -= 15;
                /* LZ4_write32(0xFFFFFFFF) strides: 255 bytes, then mc % 255 */
                while (mc >= 255) { dst[op++] = 255; mc -= 255; }
                dst[op++] = (uint8_t)mc;
            } else {
                dst[token] += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimit_plus_one) break;
        table[lz4_hash_u16(rd32(s + ip - 2))] = (uint16_t)(ip - 2);
        {
            const uint32_t h = lz4_hash_u16(rd32(s + ip));
            const uint32_t match_index = table[h];
            match = match_index;
            table[h] = (uint16_t)ip;
            if (rd32(s + match) == rd32(s + ip)) {
                token = op++;
                dst[token] = 0;
                goto next_match;
            }
        }
        forward_h = lz4_hash_u16(rd32(s + ++ip));
    }
last_literals: {
        const uint64_t last = iend - anchor;
        if (op + (int64_t)last + 1 + (int64_t)((last + 255 - 15) / 255) > olimit) return 0;
        if (last >= 15) {
            uint64_t acc = last - 15;
            dst[op++] = 15 << 4;
            for (; acc >= 255; acc -= 255) dst[op++] = 255;
            dst[op++] = (uint8_t)acc;
        } else {
            dst[op++] = (uint8_t)(last << 4);
        }
        memcpy(dst + op, s + anchor, last);
        op += (int64_t)last;
    }
    return (int)op;
}

/* bytes lz4_frame_compressor::compress produces at most */
size_t rpo_lz4f_compress_bound(size_t n) {
    const size_t nb = (n + 65535) / 65536;
    return 15 + nb * (4 + 65536) + 4;
}

static void wr32le(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }

/* the frame; returns its size (cap >= rpo_lz4f_compress_bound(n)) */
size_t rpo_lz4f_compress(const uint8_t* s, size_t n, uint8_t* dst) {
    size_t o = 0;
    wr32le(dst, 0x184D2204u);
    o = 4;
    dst[o++] = (uint8_t)(0x40 | 0x20 | (n > 0 ? 0x08 : 0));  /* version 01, independent blocks, content size */
    dst[o++] = 0x40;                                        /* max64KB */
    if (n > 0) {
        wr32le(dst + o, (uint32_t)n);
        wr32le(dst + o + 4, (uint32_t)((uint64_t)n >> 32));
        o += 8;
    }
    dst[o] = (uint8_t)((rpo_xxh32(dst + 4, o - 4, 0) >> 8) & 0xFF);
    o++;
    for (size_t b = 0; b < n; b += 65536) {
        const int len = (int)(n - b < 65536 ? n - b : 65536);
        const int c = rpo_lz4_compress_block(s + b, len, dst + o + 4, len - 1);
        if (c == 0) {
            wr32le(dst + o, (uint32_t)len | 0x80000000u);
            memcpy(dst + o + 4, s + b, (size_t)len);
            o += 4 + (size_t)len;
        } else {
            wr32le(dst + o, (uint32_t)c);
            o += 4 + (size_t)c;
        }
    }
    wr32le(dst + o, 0);
    return o + 4;
}

/* snappy 1.1.8 */
static inline uint32_t snappy_hash(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }
static int log2_floor(uint32_t x) { int r = -1; while (x) { x >>= 1; r++; } return r; }

static size_t snappy_emit_literal(uint8_t* op, const uint8_t* lit, uint32_t len) {
    const uint32_t nn = len - 1;
    size_t o = 0;
    if (nn < 60) {
        op[o++] = (uint8_t)(nn << 2);
    } else {
        const int count = (log2_floor(nn) >> 3) + 1;
        op[o++] = (uint8_t)((59 + count) << 2);
        for (int i = 0; i < count; i++) op[o++] = (uint8_t)(nn >> (8 * i));
    }
    memcpy(op + o, lit, len);
    return o + len;
}

/* EmitCopyAtMost64 */
static size_t snappy_copy64(uint8_t* op, uint32_t offset, uint32_t len) {
    if (len < 12 && offset < 2048) {
        op[0] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
        op[1] = (uint8_t)(offset & 0xff);
        return 2;
    }
    op[0] = (uint8_t)(2 + ((len - 1) << 2));
    op[1] = (uint8_t)offset;
    op[2] = (uint8_t)(offset >> 8);
    return 3;
}

static size_t snappy_emit_copy(uint8_t* op, uint32_t offset, uint32_t len) {
    size_t o = 0;
    if (len < 12) return snappy_copy64(op, offset, len);
    while (len >= 68) { o += snappy_copy64(op + o, offset, 64); len -= 64; }
    if (len > 64) { o += snappy_copy64(op + o, offset, 60); len -= 60; }
    o += snappy_copy64(op + o, offset, len);
    return o;
}

/* CompressFragment over one block of at most 64 KiB */
size_t rpo_snappy_compress_block(const uint8_t* s, uint32_t n, uint8_t* op) {
    uint16_t table[1 << 14];
    uint32_t tsize = 256;
    if (n > (1u << 14)) tsize = 1u << 14;
    else if (n >= 256) tsize = 2u << log2_floor(n - 1);
    if (tsize < 256) tsize = 256;
    memset(table, 0, tsize * sizeof(uint16_t));
    const int shift = 32 - log2_floor(tsize);
    uint32_t ip = 0, next_emit = 0;
    size_t o = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        uint32_t next_hash = snappy_hash(rd32(s + ++ip), shift);
        for (;;) {
            uint32_t skip = 32, next_ip = ip, candidate;
            do {
                ip = next_ip;
                const uint32_t hash = next_hash;
                const uint32_t between = skip >> 5;
                skip += between;
                next_ip = ip + between;
                if (next_ip > ip_limit) goto emit_remainder;
                next_hash = snappy_hash(rd32(s + next_ip), shift);
                candidate = table[hash];
                table[hash] = (uint16_t)ip;
            } while (rd32(s + ip) != rd32(s + candidate));
            o += snappy_emit_literal(op + o, s + next_emit, ip - next_emit);
            uint32_t cand_bytes;
            do {
                const uint32_t base = ip;
                uint32_t matched = 4;
                while (ip + matched < n && s[candidate + matched] == s[ip + matched]) matched++;
                ip += matched;
                o += snappy_emit_copy(op + o, base - candidate, matched);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                table[snappy_hash(rd32(s + ip - 1), shift)] = (uint16_t)(ip - 1);
                const uint32_t cur_hash = snappy_hash(rd32(s + ip), shift);
                candidate = table[cur_hash];
                cand_bytes = rd32(s + candidate);
                table[cur_hash] = (uint16_t)ip;
            } while (rd32(s + ip) == cand_bytes);
            next_hash = snappy_hash(rd32(s + ip + 1), shift);
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < n) o += snappy_emit_literal(op + o, s + next_emit, n - next_emit);
    return o;
}

/* snappy::RawCompress: varint length + the blocks */
size_t rpo_snappy_raw_compress(const uint8_t* s, size_t n, uint8_t* dst) {
    size_t o = 0;
    uint32_t v = (uint32_t)n;
    while (v >= 128) { dst[o++] = (uint8_t)(v | 128); v >>= 7; }
    dst[o++] = (uint8_t)v;
    for (size_t b = 0; b < n; b += 65536) {
        const uint32_t len = (uint32_t)(n - b < 65536 ? n - b : 65536);
        o += rpo_snappy_compress_block(s + b, len, dst + o);
    }
    return o;
}

/* snappy::MaxCompressedLength */
static size_t snappy_max_len(size_t n) { return 32 + n + n / 6; }

/* fragments of frag bytes (0: one fragment) */
size_t rpo_snappy_java_compress_bound(size_t n, size_t frag) {
    if (frag == 0 || frag > n) frag = n ? n : 1;
    const size_t nf = n ? (n + frag - 1) / frag : 0;
    return 16 + nf * (4 + snappy_max_len(frag));
}

size_t rpo_snappy_java_compress(const uint8_t* s, size_t n, size_t frag, uint8_t* dst) {
    static const uint8_t hdr[16] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0, 1, 0, 0, 0, 1, 0, 0, 0};
    memcpy(dst, hdr, 16);
    size_t o = 16;
    if (frag == 0) frag = n ? n : 1;
    for (size_t f = 0; f < n; f += frag) {
        const size_t len = n - f < frag ? n - f : frag;
        const size_t c = rpo_snappy_raw_compress(s + f, len, dst + o + 4);
        dst[o] = (uint8_t)(c >> 24);
        dst[o + 1] = (uint8_t)(c >> 16);
        dst[o + 2] = (uint8_t)(c >> 8);
        dst[o + 3] = (uint8_t)c;
        o += 4 + c;
    }
    return o;
}


/* ======================================================================== */
/* kafka::writer_serialize_batch (kafka/protocol/response_writer.h:241-276)  */
/* ======================================================================== */
/* Batches [first, first + n) of a job's results as a Kafka v2 record set:
 * base_offset, batch_length = size_bytes - 61 + 61 - 8 - 4, partition leader
 * epoch 0, magic 2, crc, attrs, last_offset_delta, first / max timestamp,
 * producer id / epoch, base_sequence, record_count (each big endian), then
 * the payload as stored.  Returns the bytes written (out may be NULL to
 * size). */
static size_t put_be(uint8_t* o, uint64_t v, int k) {
    if (o)
        for (int i = 0; i < k; i++) o[i] = (uint8_t)(v >> (8 * (k - 1 - i)));
    return (size_t)k;
}

uint64_t rpo_serialize_wire(const uint8_t* data, const uint64_t* seg_offsets, const rpgpu_batch_result* batches,
                            uint64_t first, uint64_t n, uint8_t* out) {
    uint64_t at = 0;
    for (uint64_t i = first; i < first + n; i++) {
        const rpgpu_batch_result* b = &batches[i];
        uint8_t* o = out ? out + at : NULL;
        size_t k = 0;
        const int32_t size = b->size_bytes - RPGPU_HEADER_SIZE + RPGPU_HEADER_SIZE - 8 - 4;
        k += put_be(o ? o + k : NULL, (uint64_t)b->base_offset, 8);
        k += put_be(o ? o + k : NULL, (uint32_t)size, 4);
        k += put_be(o ? o + k : NULL, 0, 4);
        k += put_be(o ? o + k : NULL, 2, 1);
        k += put_be(o ? o + k : NULL, b->crc, 4);
        k += put_be(o ? o + k : NULL, (uint16_t)b->attrs, 2);
        k += put_be(o ? o + k : NULL, (uint32_t)b->last_offset_delta, 4);
        k += put_be(o ? o + k : NULL, (uint64_t)b->first_timestamp, 8);
        k += put_be(o ? o + k : NULL, (uint64_t)b->max_timestamp, 8);
        k += put_be(o ? o + k : NULL, (uint64_t)b->producer_id, 8);
        k += put_be(o ? o + k : NULL, (uint16_t)b->producer_epoch, 2);
        k += put_be(o ? o + k : NULL, (uint32_t)b->base_sequence, 4);
        k += put_be(o ? o + k : NULL, (uint32_t)b->record_count, 4);
        const uint64_t plen = (uint64_t)(uint32_t)(b->size_bytes - RPGPU_HEADER_SIZE);
        if (o) memcpy(o + k, data + seg_offsets[b->segment] + b->file_pos + RPGPU_HEADER_SIZE, plen);
        at += k + plen;
    }
    return at;
}
