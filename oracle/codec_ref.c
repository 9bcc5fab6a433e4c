/*
 * codec_ref.c — pins the oracle's LZ4F / snappy restatements against the
 * reference's actual codec libraries (liblz4 1.9.3, libsnappy 1.1.8 from
 * /opt/conda, the system dependencies of compression/CMakeLists.txt:2-3).
 *
 * TEST INFRASTRUCTURE ONLY: built into oracle/_ref/, loaded by tests and the
 * golden-fixture script, never by the product.  The driver loops below call
 * the libraries exactly the way the reference's wrappers do:
 *   ref_lz4f_uncompress   <- lz4_frame_compressor.cc:115-200 (do_uncompressed)
 *   ref_snappy_java       <- snappy_java_compressor.cc:76-129
 *   ref_snappy_raw        <- snappy_standard_compressor.cc:43-65
 *   ref_gzip_uncompress   <- gzip_compressor.cc:161-230 (zlib 1.2.11: a sizing
 *                            pass through a 512-byte buffer, then the decode)
 *   ref_zstd_uncompress   <- stream_zstd.cc:152-178 (libzstd 1.4.8: static
 *                            DCtx over estimateDStreamSize(8 MiB), 64 KiB
 *                            output buffer appended when full)
 * (gzip / zstd are used by the C6 CPU baseline only; their verdicts are
 * pinned by the oracle's own tests.)
 * Return 0 ok, -1 where the reference throws, -2 output capacity too small.
 */
#define _POSIX_C_SOURCE 199309L
#include <lz4.h>
#include <lz4frame.h>
#include <snappy-c.h>
#include <zlib.h>
#define ZSTD_STATIC_LINKING_ONLY
#include <zstd.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int ref_lz4f_uncompress(const uint8_t* src, size_t src_size, uint8_t* dst, size_t cap, size_t* out_len) {
    LZ4F_dctx* ctx = NULL;
    *out_len = 0;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&ctx, LZ4F_VERSION))) return -1;
    LZ4F_frameInfo_t fi;
    size_t in_sz = src_size;
    size_t code = LZ4F_getFrameInfo(ctx, &fi, src, &in_sz);
    if (LZ4F_isError(code)) { LZ4F_freeDecompressionContext(ctx); return -1; }
    /* the reference grows a temporary buffer; decode into a private growing
     * buffer, copy out at the end */
    size_t est = (fi.contentSize == 0 || fi.contentSize > src_size * 255) ? src_size * 4 : fi.contentSize;
    if (est == 0) est = 1;
    uint8_t* out = (uint8_t*)malloc(est);
    size_t bytes_remaining = in_sz, consumed = 0;
    while (bytes_remaining < src_size) {
        size_t step_out = est - consumed;
        size_t step_in = src_size - bytes_remaining;
        code = LZ4F_decompress(ctx, out + consumed, &step_out, src + bytes_remaining, &step_in, NULL);
        if (LZ4F_isError(code)) { free(out); LZ4F_freeDecompressionContext(ctx); return -1; }
        consumed += step_out;
        bytes_remaining += step_in;
        if (code == 0) break;
        if (consumed == est) {
            size_t next = 1024 + ((est * 3) + 1) / 2;
            uint8_t* t = (uint8_t*)malloc(next);
            memcpy(t, out, consumed);
            free(out);
            out = t;
            est = next;
        }
    }
    LZ4F_freeDecompressionContext(ctx);
    if (bytes_remaining < src_size) { free(out); return -1; }
    if (consumed > cap) { free(out); *out_len = consumed; return -2; }
    memcpy(dst, out, consumed);
    free(out);
    *out_len = consumed;
    return 0;
}

int ref_snappy_raw(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    size_t ulen = 0;
    *out_len = 0;
    if (snappy_uncompressed_length((const char*)src, n, &ulen) != SNAPPY_OK) return -1;
    if (ulen == 0) return 0;
    if (ulen > cap) {
        if (ulen > (256u << 20)) return -1;
        char* tmp = (char*)malloc(ulen);
        size_t got = ulen;
        int ok = snappy_uncompress((const char*)src, n, tmp, &got) == SNAPPY_OK;
        free(tmp);
        if (!ok) return -1;
        *out_len = ulen;
        return -2;
    }
    size_t got = ulen;
    if (snappy_uncompress((const char*)src, n, (char*)dst, &got) != SNAPPY_OK) return -1;
    *out_len = got;
    return 0;
}

static const uint8_t k_magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

int ref_snappy_java(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (n < 16 || memcmp(src, k_magic, 8) != 0) return ref_snappy_raw(src, n, dst, cap, out_len);
    int32_t min_version;
    memcpy(&min_version, src + 12, 4);
    if (min_version < 1) return -1;
    size_t pos = 16, out = 0;
    while (pos != n) {
        if (n - pos < 4) return -1;
        int32_t clen = (int32_t)(((uint32_t)src[pos] << 24) | ((uint32_t)src[pos + 1] << 16) |
                                 ((uint32_t)src[pos + 2] << 8) | src[pos + 3]);
        pos += 4;
        if (clen < 0) return -1;
        if (n - pos < (size_t)clen) return -1;
        size_t ulen = 0;
        if (snappy_uncompressed_length((const char*)src + pos, (size_t)clen, &ulen) != SNAPPY_OK) return -1;
        size_t got = ulen;
        if (ulen > cap - out) {
            /* the reference reserves output_size and lets RawUncompress
             * decide; do the same in a scratch buffer when it is sane */
            if (ulen > (256u << 20)) return -1;
            char* tmp = (char*)malloc(ulen ? ulen : 1);
            int ok = snappy_uncompress((const char*)src + pos, (size_t)clen, tmp, &got) == SNAPPY_OK;
            free(tmp);
            if (!ok) return -1;
            *out_len = out + ulen;
            return -2;
        }
        if (snappy_uncompress((const char*)src + pos, (size_t)clen, (char*)dst + out, &got) != SNAPPY_OK) return -1;
        out += got;
        pos += (size_t)clen;
    }
    *out_len = out;
    return 0;
}

/* Raw LZ4 block decode through the library (for block-level fuzzing). */
int ref_lz4_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
    return LZ4_decompress_safe((const char*)src, (char*)dst, (int)n, (int)cap);
}

/* Compressors, used only to build golden fixtures and fuzz seeds. */
size_t ref_lz4f_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, int block_linked,
                         int block_checksum, int content_checksum, int content_size, int block_size_id) {
    LZ4F_preferences_t prefs;
    memset(&prefs, 0, sizeof prefs);
    prefs.compressionLevel = 1;
    prefs.frameInfo.blockMode = block_linked ? LZ4F_blockLinked : LZ4F_blockIndependent;
    prefs.frameInfo.blockChecksumFlag = block_checksum ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
    prefs.frameInfo.contentChecksumFlag = content_checksum ? LZ4F_contentChecksumEnabled : LZ4F_noContentChecksum;
    prefs.frameInfo.contentSize = content_size ? n : 0;
    prefs.frameInfo.blockSizeID = (LZ4F_blockSizeID_t)block_size_id;
    size_t r = LZ4F_compressFrame(dst, cap, src, n, &prefs);
    return LZ4F_isError(r) ? 0 : r;
}

size_t ref_lz4f_bound(size_t n) {
    LZ4F_preferences_t prefs;
    memset(&prefs, 0, sizeof prefs);
    prefs.frameInfo.contentChecksumFlag = LZ4F_contentChecksumEnabled;
    prefs.frameInfo.blockChecksumFlag = LZ4F_blockChecksumEnabled;
    return LZ4F_compressFrameBound(n, &prefs) + 64;
}

size_t ref_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
    size_t out = cap;
    if (snappy_compress((const char*)src, n, (char*)dst, &out) != SNAPPY_OK) return 0;
    return out;
}

size_t ref_snappy_bound(size_t n) { return snappy_max_compressed_length(n); }

/* lz4_frame_compressor::compress (lz4_frame_compressor.cc:72-113): Begin,
 * one Update per iobuf fragment (frag bytes each; 0 = one fragment), End.
 * Returns the frame size, 0 on an lz4 error. */
size_t ref_lz4f_compress_stream(const uint8_t* src, size_t n, size_t frag, uint8_t* dst, size_t cap) {
    LZ4F_cctx* ctx = NULL;
    if (LZ4F_isError(LZ4F_createCompressionContext(&ctx, LZ4F_VERSION))) return 0;
    LZ4F_preferences_t prefs;
    memset(&prefs, 0, sizeof prefs);
    prefs.compressionLevel = 1;
    prefs.frameInfo.blockMode = LZ4F_blockIndependent;
    prefs.frameInfo.contentSize = n;
    size_t need = LZ4F_compressBound(n, &prefs) + 4 + 19;
    size_t r = 0;
    if (need > cap) goto out;
    size_t o = LZ4F_compressBegin(ctx, dst, cap, &prefs);
    if (LZ4F_isError(o)) goto out;
    if (frag == 0) frag = n ? n : 1;
    for (size_t f = 0; f < n; f += frag) {
        size_t len = n - f < frag ? n - f : frag;
        size_t c = LZ4F_compressUpdate(ctx, dst + o, cap - o, src + f, len, NULL);
        if (LZ4F_isError(c)) goto out;
        o += c;
    }
    {
        size_t c = LZ4F_compressEnd(ctx, dst + o, cap - o, NULL);
        if (LZ4F_isError(c)) goto out;
        r = o + c;
    }
out:
    LZ4F_freeCompressionContext(ctx);
    return r;
}

/* snappy_java_compressor::compress (snappy_java_compressor.cc:58-75) over
 * frag-byte fragments (0 = one fragment); snappy_compress = RawCompress. */
size_t ref_snappy_java_compress(const uint8_t* src, size_t n, size_t frag, uint8_t* dst, size_t cap) {
    static const uint8_t hdr[16] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0, 1, 0, 0, 0, 1, 0, 0, 0};
    if (cap < 16) return 0;
    memcpy(dst, hdr, 16);
    size_t o = 16;
    if (frag == 0) frag = n ? n : 1;
    for (size_t f = 0; f < n; f += frag) {
        size_t len = n - f < frag ? n - f : frag;
        if (o + 4 + snappy_max_compressed_length(len) > cap) return 0;
        size_t c = snappy_max_compressed_length(len);
        if (snappy_compress((const char*)src + f, len, (char*)dst + o + 4, &c) != SNAPPY_OK) return 0;
        dst[o] = (uint8_t)(c >> 24);
        dst[o + 1] = (uint8_t)(c >> 16);
        dst[o + 2] = (uint8_t)(c >> 8);
        dst[o + 3] = (uint8_t)c;
        o += 4 + c;
    }
    return o;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline of the decode path (bench.py cpu_baseline, C2 / C5): per     */
/* batch of a disk segment, what the reference does on recovery + decode:   */
/*   checksumming_consumer crc over BE40 ++ stored payload                   */
/*     (storage/log_replayer.cc:48-79, model/record_utils.cc:68-91),          */
/*   compressor::uncompress with the reference's codec libraries and driver  */
/*     loops above (compression/compression.cc:34-55),                        */
/*   reset_size_checksum_metadata's crc over BE40 ++ decoded bytes           */
/*     (storage/parser_utils.cc:114-120).                                     */
/* CRC32C with SSE4.2 crc32 instructions, as google crc32c's x86 path.       */
/* One pthread per core, batches dealt round-robin; the clock covers the     */
/* decode loop only (data preloaded).                                        */
/* ------------------------------------------------------------------------ */
#include <nmmintrin.h>
#include <pthread.h>
#include <time.h>

__attribute__((target("sse4.2"))) static uint32_t hw_crc(uint32_t crc, const uint8_t* p, size_t n) {
    uint64_t l = crc ^ 0xFFFFFFFFu;
    while (n && ((uintptr_t)p & 7)) { l = _mm_crc32_u8((uint32_t)l, *p++); n--; }
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        l = _mm_crc32_u64(l, v);
        p += 8;
        n -= 8;
    }
    uint32_t s = (uint32_t)l;
    while (n) { s = _mm_crc32_u8(s, *p++); n--; }
    return s ^ 0xFFFFFFFFu;
}

static void be40(const uint8_t* h, uint8_t* be) {
    static const int f[8][2] = {{21, 2}, {23, 4}, {27, 8}, {35, 8}, {43, 8}, {51, 2}, {53, 4}, {57, 4}};
    int o = 0;
    for (int k = 0; k < 8; k++)
        for (int i = 0; i < f[k][1]; i++) be[o++] = h[f[k][0] + f[k][1] - 1 - i];
}

/* gzip_compressor::uncompress: inflateInit2(15 + 32) twice, the first pass
 * only counting total_out through a 512-byte buffer (buffer_for_input) */
int ref_gzip_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    *out_len = 0;
    uint8_t small[512];
    size_t total = 0;
    for (int pass = 0; pass < 2; pass++) {
        z_stream z;
        memset(&z, 0, sizeof(z));
        if (inflateInit2(&z, 15 + 32) != Z_OK) return -1;
        z.next_in = (Bytef*)src;
        z.avail_in = (uInt)n;
        int rc = Z_OK;
        if (pass == 0) {
            do {
                z.next_out = small;
                z.avail_out = sizeof(small);
                rc = inflate(&z, Z_NO_FLUSH);
            } while (rc == Z_OK && z.avail_in > 0);
            total = z.total_out;
        } else {
            if (total > cap) { inflateEnd(&z); return -2; }
            z.next_out = dst;
            z.avail_out = (uInt)total;
            rc = inflate(&z, Z_NO_FLUSH);
            *out_len = z.total_out;
        }
        inflateEnd(&z);
        if (rc == Z_DATA_ERROR || rc == Z_NEED_DICT || rc == Z_STREAM_ERROR || rc == Z_MEM_ERROR) return -1;
    }
    return 0;
}

/* stream_zstd::do_uncompress; ws: ZSTD_estimateDStreamSize(8 MiB) + 64 KiB
 * bytes of the caller's (the reference keeps one static workspace) */
size_t ref_zstd_workspace(void) { return ZSTD_estimateDStreamSize((size_t)8 << 20) + (64u << 10); }
int ref_zstd_uncompress(void* ws, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    const size_t ws_size = ZSTD_estimateDStreamSize((size_t)8 << 20);
    *out_len = 0;
    uint8_t* obuf = (uint8_t*)ws + ws_size;
    ZSTD_DCtx* d = ZSTD_initStaticDCtx(ws, ws_size);
    if (!d) return -1;
    ZSTD_outBuffer o = {obuf, 64u << 10, 0};
    ZSTD_inBuffer i = {src, n, 0};
    size_t total = 0;
    while (i.pos != i.size) {
        const size_t err = ZSTD_decompressStream(d, &o, &i);
        if (i.pos != i.size && o.pos == o.size) {
            if (total + o.size <= cap) memcpy(dst + total, obuf, o.size);
            total += o.size;
            o.pos = 0;
        } else if (ZSTD_isError(err)) {
            return -1;
        }
    }
    if (total + o.pos <= cap) memcpy(dst + total, obuf, o.pos);
    total += o.pos;
    *out_len = total;
    return total > cap ? -2 : 0;
}

typedef struct {
    const uint8_t* seg;
    const uint64_t* pos;
    uint64_t n;
    uint64_t* next;  /* shared claim cursor over pos (largest batches first) */
    uint64_t stored, decoded, ok;
} dec_task;

static void* dec_worker(void* arg) {
    dec_task* t = (dec_task*)arg;
    size_t cap = 4u << 20;
    uint8_t* buf = (uint8_t*)malloc(cap);
    void* zws = malloc(ref_zstd_workspace());
    for (;;) {
        const uint64_t i = __atomic_fetch_add(t->next, 1, __ATOMIC_RELAXED);
        if (i >= t->n) break;
        const uint8_t* h = t->seg + t->pos[i];
        int32_t size;
        memcpy(&size, h + 4, 4);
        const size_t n = (size_t)size - 61;
        uint8_t be[40];
        be40(h, be);
        uint32_t c = hw_crc(hw_crc(0, be, 40), h + 61, n);
        uint32_t stored_crc;
        memcpy(&stored_crc, h + 17, 4);
        t->stored += (uint64_t)size;
        const int codec = h[21] & 7;
        size_t out = 0;
        int rc = -1;
        if (codec == 3) rc = ref_lz4f_uncompress(h + 61, n, buf, cap, &out);
        else if (codec == 2) rc = ref_snappy_java(h + 61, n, buf, cap, &out);
        else if (codec == 1) rc = ref_gzip_uncompress(h + 61, n, buf, cap, &out);
        else if (codec == 4) rc = ref_zstd_uncompress(zws, h + 61, n, buf, cap, &out);
        else if (codec == 0) { rc = 0; out = 0; }
        if (rc == 0 && codec) {
            be[1] &= (uint8_t)~7u; /* codec bits cleared */
            c ^= hw_crc(hw_crc(0, be, 40), buf, out);
            t->decoded += out;
        }
        t->ok += (c != stored_crc) ? 1u : 0u; /* keeps both CRCs live */
    }
    free(zws);
    free(buf);
    return NULL;
}

static const uint8_t* g_sort_seg;
static int by_size_desc(const void* a, const void* b) {
    int32_t sa, sb;
    memcpy(&sa, g_sort_seg + *(const uint64_t*)a + 4, 4);
    memcpy(&sb, g_sort_seg + *(const uint64_t*)b + 4, 4);
    return sa < sb ? 1 : sa > sb ? -1 : 0;
}

/* pos[n]: file positions of the batches to process (all complete, in one
 * segment buffer).  Returns seconds; stored/decoded byte totals out. */
double ref_baseline_decode(const uint8_t* seg, const uint64_t* pos, uint64_t n, int threads, uint64_t* stored,
                           uint64_t* decoded) {
    if (threads < 1) threads = 1;
    dec_task* t = (dec_task*)calloc((size_t)threads, sizeof(dec_task));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    /* largest batches first, claimed dynamically: a 1 MiB gzip batch takes
     * milliseconds and would otherwise set the tail */
    uint64_t* order = (uint64_t*)malloc((size_t)(n ? n : 1) * sizeof(uint64_t));
    memcpy(order, pos, (size_t)n * sizeof(uint64_t));
    g_sort_seg = seg;
    qsort(order, (size_t)n, sizeof(uint64_t), by_size_desc);
    uint64_t next = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        t[i].seg = seg;
        t[i].pos = order;
        t[i].n = n;
        t[i].next = &next;
        pthread_create(&th[i], NULL, dec_worker, &t[i]);
    }
    uint64_t s = 0, d = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        s += t[i].stored;
        d += t[i].decoded;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(order);
    free(t);
    free(th);
    *stored = s;
    *decoded = d;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
