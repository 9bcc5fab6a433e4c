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
 * Return 0 ok, -1 where the reference throws, -2 output capacity too small.
 */
#include <lz4.h>
#include <lz4frame.h>
#include <snappy-c.h>
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
