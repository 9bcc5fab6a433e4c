// rp_hostcodec.cpp — compression::compressor::uncompress for gzip and zstd
// (compression/compression.cc:34-55): the CPU fallback that SURVEY.md §8(b)
// puts behind the same surface (LZ4 and snappy decode on the GPU).  The
// reference's own loops over the reference's own libraries, loaded with
// dlopen (zlib 1.2.11 / libzstd 1.4.8, the system libraries of this image;
// compression/CMakeLists.txt links the system ones):
//   * gzip: gzip_compressor::uncompress / do_uncompress / buffer_for_input /
//     gzip_decompression_codec::inflate_to
//     (compression/internal/gzip_compressor.cc:161-230);
//   * zstd: stream_zstd::do_uncompress (compression/stream_zstd.cc:152-178)
//     with a static DCtx over ZSTD_estimateDStreamSize(8 MiB) of workspace
//     (zstd_decompress_workspace_bytes, config/configuration.cc:911-916) and
//     its 64 KiB output buffer (stream_zstd.cc:43-53).
// And compressor::compress for the same two codecs (compression.cc:17-33):
//   * gzip: gzip_compressor::compress (gzip_compressor.cc:126-161) with
//     gzip_compression_codec::reset's deflateInit2(Z_DEFAULT_COMPRESSION,
//     Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) (:51-62), one deflate
//     (Z_NO_FLUSH) per iobuf fragment into a deflateBound buffer, Z_FINISH;
//   * zstd: stream_zstd::do_compress (stream_zstd.cc:84-104): a fresh CCtx,
//     pledged source size, one ZSTD_compressStream2(ZSTD_e_flush) per
//     fragment into a ZSTD_compressBound buffer, ZSTD_endStream.
// Host code only; no device work.  Status: 0 ok, kHostCodecError where the
// reference throws std::runtime_error, kHostCodecMissing when the library is
// absent, kHostCodecOverflow when cap is too small (*out_len = size needed).
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include <memory>
#include <mutex>
#include <new>

#include "rp_hostcodec.h"

namespace rp {
namespace {

// ---------------------------------------------------------------------------
// zlib
// ---------------------------------------------------------------------------
struct ZApi {
    int (*inflateInit2_)(z_streamp, int, const char*, int);
    int (*inflateGetHeader)(z_streamp, gz_headerp);
    int (*inflate)(z_streamp, int);
    int (*inflateEnd)(z_streamp);
    int (*deflateInit2_)(z_streamp, int, int, int, int, int, const char*, int);
    uLong (*deflateBound)(z_streamp, uLong);
    int (*deflate)(z_streamp, int);
    int (*deflateEnd)(z_streamp);
};

const ZApi* zapi() {
    static ZApi a;
    static bool ok = [] {
        void* h = dlopen("libz.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return false;
        a.inflateInit2_ = (int (*)(z_streamp, int, const char*, int))dlsym(h, "inflateInit2_");
        a.inflateGetHeader = (int (*)(z_streamp, gz_headerp))dlsym(h, "inflateGetHeader");
        a.inflate = (int (*)(z_streamp, int))dlsym(h, "inflate");
        a.inflateEnd = (int (*)(z_streamp))dlsym(h, "inflateEnd");
        a.deflateInit2_ = (int (*)(z_streamp, int, int, int, int, int, const char*, int))dlsym(h, "deflateInit2_");
        a.deflateBound = (uLong(*)(z_streamp, uLong))dlsym(h, "deflateBound");
        a.deflate = (int (*)(z_streamp, int))dlsym(h, "deflate");
        a.deflateEnd = (int (*)(z_streamp))dlsym(h, "deflateEnd");
        return a.inflateInit2_ && a.inflateGetHeader && a.inflate && a.inflateEnd && a.deflateInit2_ &&
               a.deflateBound && a.deflate && a.deflateEnd;
    }();
    return ok ? &a : nullptr;
}

// gzip_decompression_codec (gzip_compressor.cc:64-104)
struct GzDec {
    const ZApi* z;
    z_stream s;
    gz_header hdr;
    bool init = false;
    GzDec(const ZApi* api) : z(api) {}
    ~GzDec() {
        if (init) z->inflateEnd(&s);
    }
    // reset(): inflateInit2(15 + 32) then inflateGetHeader; false = throw.
    // The header struct is zeroed: the reference hands zlib an uninitialised
    // gz_header, whose extra / name / comment pointers zlib then writes
    // through for FEXTRA / FNAME / FCOMMENT members (undefined behaviour
    // there; with null pointers zlib skips the copies, output unchanged)
    bool reset(const uint8_t* src, size_t n) {
        memset(&s, 0, sizeof(s));
        memset(&hdr, 0, sizeof(hdr));
        s.zalloc = Z_NULL;
        s.zfree = Z_NULL;
        s.opaque = Z_NULL;
        s.next_in = (unsigned char*)src;
        s.avail_in = (uInt)n;
        if (z->inflateInit2_(&s, 15 + 32, ZLIB_VERSION, (int)sizeof(z_stream)) != Z_OK) return false;
        init = true;
        return z->inflateGetHeader(&s, &hdr) == Z_OK;
    }
    // inflate_to (gzip_compressor.cc:161-182), its bookkeeping kept as is:
    // after a full buffer the next call gets avail_out 0, the one after
    // that the buffer from its start again
    bool inflate_to(unsigned char* out, size_t out_size) {
        size_t consumed = 0;
        int code = 0;
        int calls = 0;
        do {
            s.next_out = out + consumed;
            s.avail_out = (uInt)(out_size - consumed);
            code = z->inflate(&s, Z_NO_FLUSH);
            switch (code) {
            case Z_STREAM_ERROR:
            case Z_NEED_DICT:
            case Z_DATA_ERROR:
            case Z_MEM_ERROR:
                return false;
            default:
                break;
            }
            consumed = out_size - s.avail_out - consumed;
            // a guard the reference does not have: with no output room at
            // all (a zero-length result whose stream does not end at once)
            // its loop would not terminate
            if (out_size == 0 && ++calls > 1) break;
        } while (s.avail_out == 0 && code != Z_STREAM_END);
        return true;
    }
};

int gzip_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    const ZApi* z = zapi();
    if (!z) return kHostCodecMissing;
    if (n > 0xFFFFFFFFull) return kHostCodecError;
    size_t total;
    {
        // buffer_for_input: the whole stream through a 512-byte dummy buffer
        GzDec pass(z);
        if (!pass.reset(in, n)) return kHostCodecError;
        unsigned char dummy[512];
        if (!pass.inflate_to(dummy, sizeof(dummy))) return kHostCodecError;
        total = pass.s.total_out;
    }
    *out_len = total;
    if (total > cap) return kHostCodecOverflow;
    GzDec main(z);
    if (!main.reset(in, n)) return kHostCodecError;
    unsigned char one;  // a zero-length result still gets a non-null buffer
    if (!main.inflate_to(total ? out : &one, total)) return kHostCodecError;
    return 0;
}

// ---------------------------------------------------------------------------
// zstd (prototypes of the libzstd 1.4 API used; the structs are its ABI)
// ---------------------------------------------------------------------------
struct ZstdIn {
    const void* src;
    size_t size;
    size_t pos;
};
struct ZstdOut {
    void* dst;
    size_t size;
    size_t pos;
};
struct ZstdApi {
    size_t (*estimateDStreamSize)(size_t);
    void* (*initStaticDCtx)(void*, size_t);
    size_t (*decompressStream)(void*, ZstdOut*, ZstdIn*);
    unsigned (*isError)(size_t);
    void* (*createCCtx)();
    size_t (*freeCCtx)(void*);
    size_t (*setPledgedSrcSize)(void*, unsigned long long);
    size_t (*compressBound)(size_t);
    size_t (*compressStream2)(void*, ZstdOut*, ZstdIn*, int);
    size_t (*endStream)(void*, ZstdOut*);
};

const ZstdApi* zstdapi() {
    static ZstdApi a;
    static bool ok = [] {
        void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return false;
        a.estimateDStreamSize = (size_t(*)(size_t))dlsym(h, "ZSTD_estimateDStreamSize");
        a.initStaticDCtx = (void* (*)(void*, size_t))dlsym(h, "ZSTD_initStaticDCtx");
        a.decompressStream = (size_t(*)(void*, ZstdOut*, ZstdIn*))dlsym(h, "ZSTD_decompressStream");
        a.isError = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
        a.createCCtx = (void* (*)())dlsym(h, "ZSTD_createCCtx");
        a.freeCCtx = (size_t(*)(void*))dlsym(h, "ZSTD_freeCCtx");
        a.setPledgedSrcSize = (size_t(*)(void*, unsigned long long))dlsym(h, "ZSTD_CCtx_setPledgedSrcSize");
        a.compressBound = (size_t(*)(size_t))dlsym(h, "ZSTD_compressBound");
        a.compressStream2 = (size_t(*)(void*, ZstdOut*, ZstdIn*, int))dlsym(h, "ZSTD_compressStream2");
        a.endStream = (size_t(*)(void*, ZstdOut*))dlsym(h, "ZSTD_endStream");
        return a.estimateDStreamSize && a.initStaticDCtx && a.decompressStream && a.isError && a.createCCtx &&
               a.freeCCtx && a.setPledgedSrcSize && a.compressBound && a.compressStream2 && a.endStream;
    }();
    return ok ? &a : nullptr;
}

constexpr size_t kZstdWorkspaceWindow = 8u << 20;  // zstd_decompress_workspace_bytes default
constexpr size_t kZstdOutBuffer = 64u << 10;       // stream_zstd d_buffer

// per-thread workspace and output buffer, as the reference's thread_local ones
struct ZstdTls {
    size_t ws_size = 0;
    std::unique_ptr<uint64_t[]> ws;  // 8-byte aligned
    std::unique_ptr<uint8_t[]> obuf;
};

int zstd_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    const ZstdApi* z = zstdapi();
    if (!z) return kHostCodecMissing;
    thread_local ZstdTls t;
    if (!t.ws) {
        t.ws_size = z->estimateDStreamSize(kZstdWorkspaceWindow);
        t.ws.reset(new (std::nothrow) uint64_t[(t.ws_size + 7) / 8]);
        t.obuf.reset(new (std::nothrow) uint8_t[kZstdOutBuffer]);
        if (!t.ws || !t.obuf) {
            t.ws.reset();
            return kHostCodecError;
        }
    }
    void* dctx = z->initStaticDCtx(t.ws.get(), t.ws_size);
    if (!dctx) return kHostCodecError;
    size_t total = 0;
    auto append = [&](const uint8_t* p, size_t k) {
        if (total + k <= cap) memcpy(out + total, p, k);
        total += k;
    };
    ZstdOut o{t.obuf.get(), kZstdOutBuffer, 0};
    ZstdIn i{in, n, 0};
    while (i.pos != i.size) {
        const size_t err = z->decompressStream(dctx, &o, &i);
        if (i.pos != i.size && o.pos == o.size) {
            append(t.obuf.get(), o.size);
            o.size = kZstdOutBuffer;
            o.pos = 0;
        } else if (z->isError(err)) {
            return kHostCodecError;
        }
    }
    append(t.obuf.get(), o.pos);
    *out_len = total;
    return total > cap ? kHostCodecOverflow : 0;
}

// gzip_compressor::compress; *out_len = the stream's size (also on overflow)
int gzip_compress(const uint8_t* in, size_t n, size_t frag, uint8_t* out, size_t cap, size_t* out_len) {
    const ZApi* z = zapi();
    if (!z) return kHostCodecMissing;
    if (n > 0xFFFFFFFFull) return kHostCodecError;
    z_stream st;
    memset(&st, 0, sizeof st);
    if (z->deflateInit2_(&st, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY, ZLIB_VERSION,
                         (int)sizeof(z_stream)) != Z_OK)
        return kHostCodecError;
    const size_t bound = z->deflateBound(&st, (uLong)n);
    std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[bound ? bound : 1]);
    int rc = 0;
    if (!buf) rc = kHostCodecError;
    if (rc == 0) {
        st.next_out = buf.get();
        st.avail_out = (uInt)bound;
        if (frag == 0) frag = n ? n : 1;
        for (size_t f = 0; f < n && rc == 0; f += frag) {
            st.next_in = (unsigned char*)in + f;
            st.avail_in = (uInt)(n - f < frag ? n - f : frag);
            const int r = z->deflate(&st, Z_NO_FLUSH);
            if (r != Z_OK && r != Z_STREAM_END && r != Z_BUF_ERROR) rc = kHostCodecError;
        }
        if (rc == 0 && z->deflate(&st, Z_FINISH) != Z_STREAM_END) rc = kHostCodecError;
    }
    if (rc == 0) {
        *out_len = st.total_out;
        if (st.total_out > cap) rc = kHostCodecOverflow;
        else memcpy(out, buf.get(), st.total_out);
    }
    z->deflateEnd(&st);
    return rc;
}

// stream_zstd::do_compress
int zstd_compress(const uint8_t* in, size_t n, size_t frag, uint8_t* out, size_t cap, size_t* out_len) {
    const ZstdApi* z = zstdapi();
    if (!z) return kHostCodecMissing;
    void* ctx = z->createCCtx();
    if (!ctx) return kHostCodecError;
    int rc = 0;
    const size_t bound = z->compressBound(n);
    std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[bound ? bound : 1]);
    if (!buf || z->isError(z->setPledgedSrcSize(ctx, n))) rc = kHostCodecError;
    ZstdOut o{buf.get(), bound, 0};
    if (frag == 0) frag = n ? n : 1;
    for (size_t f = 0; f < n && rc == 0; f += frag) {
        ZstdIn i{in + f, n - f < frag ? n - f : frag, 0};
        if (z->isError(z->compressStream2(ctx, &o, &i, 1 /* ZSTD_e_flush */))) rc = kHostCodecError;
    }
    if (rc == 0) {
        z->endStream(ctx, &o);  // the reference does not check it
        *out_len = o.pos;
        if (o.pos > cap) rc = kHostCodecOverflow;
        else memcpy(out, buf.get(), o.pos);
    }
    z->freeCCtx(ctx);
    return rc;
}

}  // namespace

int host_compress(int codec, const uint8_t* in, size_t n, size_t frag, uint8_t* out, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (codec == kHostGzip) return gzip_compress(in, n, frag, out, cap, out_len);
    if (codec == kHostZstd) return zstd_compress(in, n, frag, out, cap, out_len);
    return kHostCodecMissing;
}

int host_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (codec == kHostGzip) return gzip_uncompress(in, n, out, cap, out_len);
    if (codec == kHostZstd) return zstd_uncompress(in, n, out, cap, out_len);
    return kHostCodecMissing;
}

}  // namespace rp
