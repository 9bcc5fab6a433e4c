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
        return a.inflateInit2_ && a.inflateGetHeader && a.inflate && a.inflateEnd;
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
    // reset(): inflateInit2(15 + 32) then inflateGetHeader; false = throw
    bool reset(const uint8_t* src, size_t n) {
        memset(&s, 0, sizeof(s));
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
        return a.estimateDStreamSize && a.initStaticDCtx && a.decompressStream && a.isError;
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

}  // namespace

int host_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (codec == kHostGzip) return gzip_uncompress(in, n, out, cap, out_len);
    if (codec == kHostZstd) return zstd_uncompress(in, n, out, cap, out_len);
    return kHostCodecMissing;
}

}  // namespace rp
