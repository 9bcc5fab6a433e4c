// rp_zstd_core.h — the zstd payload decoder of the device path
// (stream_zstd::do_uncompress, compression/stream_zstd.cc:152-178, over
// libzstd 1.4.8 as the reference links it), written once over an
// environment `E` that supplies input bytes, LDS-or-host tables and the
// output.  The device instantiates it with a wave environment
// (rp_inflate.hip: wave-uniform scalar state, lane-parallel copies, a 32 KiB
// LDS ring); tests/zstd_core_host.cpp instantiates it on the host only to fuzz
// the decoder logic against libzstd itself (test infrastructure).
//
// What is restated (RFC 8878 plus libzstd 1.4.8's exact acceptance rules,
// pinned against the library by tests/test_zstd_core.py):
//   * the reference's loop: one ZSTD_inBuffer over the whole payload, a
//     64 KiB ZSTD_outBuffer drained whenever it fills, a static DCtx over
//     ZSTD_estimateDStreamSize(8 MiB) of workspace (its buffer limits);
//   * ZSTD_decompressStream's two paths per frame: the single-pass shortcut
//     (content size known, fits the output room, whole frame present) and the
//     streaming path (block-size limit, ring-buffer capacity, truncation
//     yields the complete blocks and the present part of a raw block);
//   * frame / block headers, skippable frames, window and dictionary checks,
//     content-size and XXH64 content-checksum checks;
//   * literals (raw, RLE, Huffman 1 or 4 streams, treeless), Huffman weight
//     headers (direct and FSE-compressed, FSE_decompress_wksp's tail loop),
//     FSE_readNCount, ZSTD_buildFSETable, the sequence bit stream with
//     BIT_DStream_t's exact reload / overflow behaviour, repeat offsets,
//     sequence execution checks (capacity, literal overrun, reach).
// Ring-buffer mode (no content size, or larger than its window + 128 KiB),
// corrupt streams only: a match reaching past the window into the part of
// the previous ring segment that the current segment (or the up-to-32-byte
// overcopy of its copies) has already overwritten reads those newer bytes in
// libzstd.  The fast environments report it (RingDirtyHook) and turn the
// payload down; an ExactRing environment, which emulates the DCtx buffer
// write for write (ZSTD_execSequence's copies as libzstd performs them),
// decodes it as libzstd does (round 6; tests/test_zstd_core.py
// ::test_ring_mode_far_matches, tests/test_gpu_parity.py
// ::test_zstd_ring_mode_exact).  Until round 5 such payloads were rejected.
#pragma once
#include <stdint.h>

#ifndef ZS_FN
#define ZS_FN inline
#endif
#ifndef ZS_CONST
#define ZS_CONST static const
#endif
#ifndef ZS_TRACE
#define ZS_TRACE(...)
#endif
// per-phase timing hook of diagnostic builds (RPGPU_ZSTAMPS)
#ifndef ZS_PROF
#define ZS_PROF(k, stmt) stmt
#endif

namespace rp {
namespace zs {

struct SeqSym {
    uint16_t next;
    uint8_t nadd;
    uint8_t nbits;
    uint32_t base;
};
struct FseW {
    uint16_t next;
    uint8_t sym;
    uint8_t nbits;
};
struct Tabs {
    SeqSym ll[512], of[256], ml[512];
    uint16_t huf[4096];  // X1 Huffman table: symbol | bits << 8
    FseW fw[64];         // Huffman-weight FSE table
    int16_t norm[256];
    uint16_t nxt[256];
    uint8_t w[256];
    uint32_t rank[16];
};

constexpr uint64_t kUnknown = ~0ull;
constexpr uint32_t kBlockMax = 128u << 10;
constexpr uint64_t kOutRoom = 64u << 10;  // stream_zstd's ZSTD_outBuffer (stream_zstd.cc:43-53)
// ZSTD_estimateDStreamSize(8 MiB) - sizeof(ZSTD_DCtx): in + out buffers of the static DCtx
constexpr uint64_t kStaticBuffers = 131072ull + (8388608ull + 131072ull + 64ull);
constexpr uint64_t kMaxWindow = (1ull << 27) + 1;  // ZSTD_MAXWINDOWSIZE_DEFAULT
constexpr uint64_t kRingDirty = 32;                // WILDCOPY_OVERLENGTH: ZSTD_wildcopy's reach past a copy

ZS_CONST uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,   16,    18,
                                 20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
ZS_CONST uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
ZS_CONST uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,   16,    17,   18,   19,   20,
                                 21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,   34,    35,   37,   39,   41,
                                 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
ZS_CONST uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  0, 0,
                                0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
ZS_CONST uint8_t kOFBits[32] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31};
ZS_CONST uint32_t kOFBase[32] = {0,         1,         1,         5,         0xD,       0x1D,      0x3D,      0x7D,
                                 0xFD,      0x1FD,     0x3FD,     0x7FD,     0xFFD,     0x1FFD,    0x3FFD,    0x7FFD,
                                 0xFFFD,    0x1FFFD,   0x3FFFD,   0x7FFFD,   0xFFFFD,   0x1FFFFD,  0x3FFFFD,  0x7FFFFD,
                                 0xFFFFFD,  0x1FFFFFD, 0x3FFFFFD, 0x7FFFFFD, 0xFFFFFFD, 0x1FFFFFFD, 0x3FFFFFFD, 0x7FFFFFFD};
// predefined distributions (RFC 8878 3.1.1.3.2.2)
ZS_CONST int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
ZS_CONST int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,  1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
ZS_CONST int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

ZS_FN uint32_t highbit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// ---------------------------------------------------------------------------
// BIT_DStream_t (libzstd bitstream.h): a backward bit stream read through a
// 64-bit container; the reload statuses and the `used & 63` wrap of an
// overflowed stream are libzstd's (the sequence stream accepts overflow)
// ---------------------------------------------------------------------------
struct Bits {
    uint64_t c;
    uint32_t used;
    uint64_t ptr, start, limit;
    uint64_t wbase;  // the environment's read window for this stream (E::lb)
    uint32_t wreg;
};
enum { kUnfinished = 0, kEndOfBuffer = 1, kCompleted = 2, kOverflow = 3 };

template <class E>
ZS_FN bool bits_init(E& e, Bits& s, uint64_t src, uint64_t n) {
    if (n < 1) return false;
    s.start = src;
    s.limit = src + 8;
    s.wbase = kUnknown;
    s.wreg = 0;
    const uint32_t last = e.b(src + n - 1);
    if (n >= 8) {
        s.ptr = src + n - 8;
        s.c = e.lb(s, s.ptr);
        s.used = last ? 8u - highbit(last) : 0u;
        return last != 0;
    }
    s.ptr = src;
    s.c = e.le(src, (uint32_t)n);
    if (!last) return false;
    s.used = 8u - highbit(last) + (uint32_t)(8 - n) * 8u;
    return true;
}
template <class E>
ZS_FN int bits_reload(E& e, Bits& s) {
    if (s.used > 64) return kOverflow;
    if (s.ptr >= s.limit) {
        s.ptr -= s.used >> 3;
        s.used &= 7;
        s.c = e.lb(s, s.ptr);
        return kUnfinished;
    }
    if (s.ptr == s.start) return s.used < 64 ? kEndOfBuffer : kCompleted;
    uint64_t nb = s.used >> 3;
    int r = kUnfinished;
    if (s.ptr - s.start < nb) {
        nb = s.ptr - s.start;
        r = kEndOfBuffer;
    }
    s.ptr -= nb;
    s.used -= (uint32_t)nb * 8u;
    s.c = e.lb(s, s.ptr);
    return r;
}
// BIT_lookBits is BIT_getMiddleBits in 1.4.8 (an overflowed stream reads
// rotated container bits); BIT_lookBitsFast is the double shift
ZS_FN uint64_t bits_look(const Bits& s, uint32_t nb) {
    return (s.c >> ((64u - s.used - nb) & 63)) & ((1ull << nb) - 1ull);
}
ZS_FN uint64_t bits_read(Bits& s, uint32_t nb) {
    const uint64_t v = bits_look(s, nb);
    s.used += nb;
    return v;
}
ZS_FN uint64_t bits_readf(Bits& s, uint32_t nb) {  // nb >= 1
    const uint64_t v = (s.c << (s.used & 63)) >> ((64 - nb) & 63);
    s.used += nb;
    return v;
}
ZS_FN bool bits_end(const Bits& s) { return s.ptr == s.start && s.used == 64; }

// ---------------------------------------------------------------------------
// FSE_readNCount (entropy_common.c): normalized counts; bytes read or -1.
// A header shorter than 4 bytes is read from a zero-padded 4-byte copy.
// ---------------------------------------------------------------------------
template <class E>
ZS_FN int64_t read_ncount(E& e, int16_t* norm, uint32_t& maxsv, uint32_t& tlog, uint64_t src, uint64_t hbs) {
    const int64_t iend = hbs < 4 ? 4 : (int64_t)hbs;
    auto rd32 = [&](int64_t i) -> uint32_t {
        uint32_t v = 0;
        for (int k = 0; k < 4; k++)
            if (i + k < (int64_t)hbs) v |= e.b(src + (uint64_t)(i + k)) << (8 * k);
        return v;
    };
    for (uint32_t s = 0; s <= maxsv; s++) norm[s] = 0;
    int64_t ip = 0;
    uint32_t bs = rd32(0);
    int nb = (int)(bs & 15) + 5;
    if (nb > 15) return -1;
    bs >>= 4;
    int bc = 4;
    tlog = (uint32_t)nb;
    int rem = (1 << nb) + 1, thr = 1 << nb;
    nb++;
    uint32_t ch = 0;
    bool prev0 = false;
    while ((rem > 1) & (ch <= maxsv)) {
        if (prev0) {
            uint32_t n0 = ch;
            while ((bs & 0xFFFF) == 0xFFFF) {
                n0 += 24;
                if (ip < iend - 5) {
                    ip += 2;
                    bs = rd32(ip) >> (bc & 31);
                } else {
                    bs >>= 16;
                    bc += 16;
                }
            }
            while ((bs & 3) == 3) {
                n0 += 3;
                bs >>= 2;
                bc += 2;
            }
            n0 += bs & 3;
            bc += 2;
            if (n0 > maxsv) return -1;
            while (ch < n0) norm[ch++] = 0;
            if ((ip <= iend - 7) || (ip + (bc >> 3) <= iend - 4)) {
                ip += bc >> 3;
                bc &= 7;
                bs = rd32(ip) >> (bc & 31);
            } else {
                bs >>= 2;
            }
        }
        const int mx = (2 * thr - 1) - rem;
        int count;
        if ((uint32_t)(bs & (uint32_t)(thr - 1)) < (uint32_t)mx) {
            count = (int)(bs & (uint32_t)(thr - 1));
            bc += nb - 1;
        } else {
            count = (int)(bs & (uint32_t)(2 * thr - 1));
            if (count >= thr) count -= mx;
            bc += nb;
        }
        count--;
        rem -= count < 0 ? -count : count;
        norm[ch++] = (int16_t)count;
        prev0 = !count;
        while (rem < thr) {
            nb--;
            thr >>= 1;
        }
        if ((ip <= iend - 7) || (ip + (bc >> 3) <= iend - 4)) {
            ip += bc >> 3;
            bc &= 7;
        } else {
            bc -= (int)(8 * (iend - 4 - ip));
            ip = iend - 4;
        }
        bs = rd32(ip) >> (bc & 31);
    }
    if (rem != 1) return -1;
    if (bc > 32) return -1;
    maxsv = ch - 1;
    ip += (bc + 7) >> 3;
    if (hbs < 4 && ip > (int64_t)hbs) return -1;
    return ip;
}

// ZSTD_buildFSETable into t (cells 0 .. 2^tlog - 1)
ZS_FN void build_seq(SeqSym* t, const int16_t* norm, uint32_t maxsv, const uint32_t* base, const uint8_t* bits,
                     uint32_t tlog, uint16_t* nxt) {
    const uint32_t size = 1u << tlog;
    uint32_t high = size - 1;
    for (uint32_t s = 0; s <= maxsv; s++) {
        if (norm[s] == -1) {
            t[high--].base = s;
            nxt[s] = 1;
        } else {
            nxt[s] = (uint16_t)norm[s];
        }
    }
    const uint32_t mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxsv; s++)
        for (int i = 0; i < norm[s]; i++) {
            t[pos].base = s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t sym = t[u].base;
        const uint32_t ns = nxt[sym]++;
        const uint32_t nbits = tlog - highbit(ns);
        t[u].nbits = (uint8_t)nbits;
        t[u].next = (uint16_t)((ns << nbits) - size);
        t[u].nadd = bits[sym];
        t[u].base = base[sym];
    }
}

// ZSTD_buildSeqTable: bytes consumed or -1; tlog set
template <class E>
ZS_FN int64_t seq_table(E& e, Tabs* T, SeqSym* t, uint32_t& tlog, uint32_t mode, uint32_t max, uint32_t maxlog,
                        uint64_t src, uint64_t n, const uint32_t* base, const uint8_t* bits, const int16_t* dnorm,
                        uint32_t dmax, uint32_t dlog, bool repeat_ok) {
    if (mode == 0) {  // predefined
        for (uint32_t s = 0; s <= dmax; s++) T->norm[s] = dnorm[s];
        build_seq(t, T->norm, dmax, base, bits, dlog, T->nxt);
        tlog = dlog;
        return 0;
    }
    if (mode == 1) {  // RLE
        if (n == 0) return -1;
        const uint32_t sym = e.b(src);
        if (sym > max) return -1;
        t[0].next = 0;
        t[0].nbits = 0;
        t[0].nadd = bits[sym];
        t[0].base = base[sym];
        tlog = 0;
        return 1;
    }
    if (mode == 2) {  // FSE compressed
        uint32_t mx = max, tl = 0;
        const int64_t h = read_ncount(e, T->norm, mx, tl, src, n);
        if (h < 0 || tl > maxlog) return -1;
        build_seq(t, T->norm, mx, base, bits, tl, T->nxt);
        tlog = tl;
        return h;
    }
    return repeat_ok ? 0 : -1;  // repeat: the previous table of this frame
}

// ---------------------------------------------------------------------------
// Huffman table (HUF_readStats + HUF_readDTableX1): bytes of the tree
// description or -1; hlog set
// ---------------------------------------------------------------------------
template <class E>
ZS_FN int64_t fse_weights(E& e, Tabs* T, uint64_t src, uint64_t n, uint32_t& count) {
    // FSE_decompress_wksp(huffWeight, 255, src, n, ws, 6)
    uint32_t mx = 255, tl = 0;
    const int64_t h = read_ncount(e, T->norm, mx, tl, src, n);
    if (h < 0 || tl > 6) return -1;
    // FSE_buildDTable
    const uint32_t size = 1u << tl;
    uint32_t high = size - 1;
    bool fast = true;  // FSE_decodeSymbolFast (no zero-bit states) unless a count reaches half the table
    for (uint32_t s = 0; s <= mx; s++) {
        if (T->norm[s] == -1) {
            T->fw[high--].sym = (uint8_t)s;
            T->nxt[s] = 1;
        } else {
            if (T->norm[s] >= (int16_t)(1 << (tl - 1))) fast = false;
            T->nxt[s] = (uint16_t)T->norm[s];
        }
    }
    const uint32_t mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= mx; s++)
        for (int i = 0; i < T->norm[s]; i++) {
            T->fw[pos].sym = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    if (pos != 0) return -1;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t sym = T->fw[u].sym;
        const uint32_t ns = T->nxt[sym]++;
        const uint32_t nbits = tl - highbit(ns);
        T->fw[u].nbits = (uint8_t)nbits;
        T->fw[u].next = (uint16_t)((ns << nbits) - size);
    }
    // FSE_decompress_usingDTable_generic, 255 outputs at most
    Bits d;
    if (!bits_init(e, d, src + (uint64_t)h, n - (uint64_t)h)) return -1;
    uint32_t s1 = (uint32_t)bits_read(d, tl);
    bits_reload(e, d);
    uint32_t s2 = (uint32_t)bits_read(d, tl);
    bits_reload(e, d);
    uint32_t op = 0;
    const uint32_t omax = 255;
    auto sym = [&](uint32_t& st) -> uint32_t {
        const FseW f = T->fw[st];
        st = f.next + (uint32_t)(fast ? bits_readf(d, f.nbits) : bits_read(d, f.nbits));
        return f.sym;
    };
    while ((bits_reload(e, d) == kUnfinished) & (op < omax - 3)) {
        T->w[op] = (uint8_t)sym(s1);
        T->w[op + 1] = (uint8_t)sym(s2);
        T->w[op + 2] = (uint8_t)sym(s1);
        T->w[op + 3] = (uint8_t)sym(s2);
        op += 4;
    }
    for (;;) {
        if (op > omax - 2) return -1;
        T->w[op++] = (uint8_t)sym(s1);
        if (bits_reload(e, d) == kOverflow) {
            T->w[op++] = (uint8_t)sym(s2);
            break;
        }
        if (op > omax - 2) return -1;
        T->w[op++] = (uint8_t)sym(s2);
        if (bits_reload(e, d) == kOverflow) {
            T->w[op++] = (uint8_t)sym(s1);
            break;
        }
    }
    count = op;
    return 0;
}

template <class E>
ZS_FN int64_t huf_table(E& e, Tabs* T, uint64_t src, uint64_t n, uint32_t& hlog) {
    if (n == 0) return -1;
    uint32_t isz = e.b(src), osz = 0;
    if (isz >= 128) {
        osz = isz - 127;
        isz = (osz + 1) / 2;
        if (isz + 1 > n) return -1;
        if (osz >= 256) return -1;
        for (uint32_t k = 0; k < osz; k += 2) {
            const uint32_t v = e.b(src + 1 + k / 2);
            T->w[k] = (uint8_t)(v >> 4);
            T->w[k + 1] = (uint8_t)(v & 15);
        }
    } else {
        if (isz + 1 > n) return -1;
        if (fse_weights(e, T, src + 1, isz, osz) < 0) return -1;
    }
    for (int r = 0; r < 16; r++) T->rank[r] = 0;
    uint32_t total = 0;
    for (uint32_t k = 0; k < osz; k++) {
        const uint32_t w = T->w[k];
        if (w >= 12) return -1;
        T->rank[w]++;
        total += (1u << w) >> 1;
    }
    if (total == 0) return -1;
    const uint32_t tl = highbit(total) + 1;
    if (tl > 12) return -1;
    const uint32_t rest = (1u << tl) - total, lastw = highbit(rest) + 1;
    if ((1u << highbit(rest)) != rest) return -1;
    T->w[osz] = (uint8_t)lastw;
    T->rank[lastw]++;
    if (T->rank[1] < 2 || (T->rank[1] & 1)) return -1;
    const uint32_t nsym = osz + 1;
    // HUF_readDTableX1: rank starts, then each symbol's cells
    uint32_t next = 0;
    for (uint32_t r = 1; r <= tl; r++) {
        const uint32_t cur = next;
        next += T->rank[r] << (r - 1);
        T->rank[r] = cur;
    }
    for (uint32_t s = 0; s < nsym; s++) {
        const uint32_t w = T->w[s];
        const uint32_t len = (1u << w) >> 1, u0 = T->rank[w];
        const uint16_t d = (uint16_t)(s | ((tl + 1 - w) << 8));
        for (uint32_t u = 0; u < len; u++) T->huf[u0 + u] = d;
        T->rank[w] = u0 + len;
    }
    hlog = tl;
    return (int64_t)isz + 1;
}

// ---------------------------------------------------------------------------
// Literals of one block, produced lazily in consumption order (libzstd
// decodes them all first; the verdict is the same: every stream must end
// exactly once its symbols are decoded)
// ---------------------------------------------------------------------------
struct Lits {
    uint32_t kind;  // 0 raw, 1 rle, 2 huffman
    uint64_t pos;   // raw: first byte
    uint32_t rle;
    uint32_t size, used;
    uint32_t ns, seg;
    uint32_t cur, curend;  // huffman: the stream literals come from now, and where its segment ends
    Bits s[4];
    uint32_t cnt[4], dec[4];
    bool x2;           // the streams decode through libzstd's double-symbol table (HUF_decompress4X2)
    uint32_t pend[4];  // X2: code length of the symbol that opened the current step, 0 if none is open
};

// HUF_selectDecoder (huf_decompress.c): the double-symbol decoder for a
// 4-stream block when its modelled time wins
ZS_CONST uint16_t kAlgoTime[16][4] = {{0, 0, 1, 1},         {0, 0, 1, 1},         {38, 130, 1313, 74},
                                      {448, 128, 1353, 74},  {556, 128, 1353, 74},  {714, 128, 1418, 74},
                                      {883, 128, 1437, 74},  {897, 128, 1515, 75},  {926, 128, 1613, 75},
                                      {947, 128, 1729, 77},  {1107, 128, 2083, 81}, {1177, 128, 2379, 87},
                                      {1242, 128, 2415, 93}, {1349, 128, 2644, 106}, {1455, 128, 2422, 124},
                                      {722, 128, 1891, 145}};
ZS_FN bool huf_select_x2(uint32_t dsize, uint64_t csize) {
    const uint32_t q = csize >= dsize ? 15u : (uint32_t)(csize * 16 / dsize);
    const uint32_t d256 = dsize >> 8;
    const uint32_t t0 = kAlgoTime[q][0] + kAlgoTime[q][1] * d256;
    uint32_t t1 = kAlgoTime[q][2] + kAlgoTime[q][3] * d256;
    t1 += t1 >> 3;
    return t1 < t0;
}

// one literal of stream k.  X1 (single-symbol table): the symbol's code is
// consumed.  X2 (libzstd's double-symbol table, 12-bit lookups): a step
// decodes two symbols when the second code fits the 12 bits after the
// first, so the symbols are the same; only the stream's last symbol differs
// when it starts a step alone (HUF_decodeLastSymbolX2): a double entry there
// consumes both codes, clamped to the container, or nothing once the
// container is spent.
// n literals of one stream (left = the stream's symbols not yet decoded).
// X1 (single-symbol table): each symbol's code is consumed.  X2 (libzstd's
// double-symbol table, 12-bit lookups): a step decodes two symbols when the
// second code fits the 12 bits after the first, so the symbols are the same;
// only the stream's last symbol differs when it starts a step alone
// (HUF_decodeLastSymbolX2): a double entry there consumes both codes,
// clamped to the container, or nothing once the container is spent.  The
// container is refilled only when the next lookup could run past it (the
// decoded values and the end check do not depend on when libzstd refills),
// and always before a stream's last symbol (whose X2 clamp does).
template <class E>
ZS_FN uint32_t huf_one(E& e, Tabs* T, Bits& s, uint32_t& open, uint32_t left, bool x2, uint32_t hlog) {
    if (left == 1 || s.used > 64 - hlog) bits_reload(e, s);
    const uint32_t v = e.U((uint32_t)((s.c << (s.used & 63)) >> ((64 - hlog) & 63)));
    const uint32_t d = e.U(T->huf[v]);
    const uint32_t l1 = d >> 8;
    if (x2) {
        const bool paired = open && open + l1 <= 12;
        if (left == 1 && !paired) {
            const uint32_t w = e.U((uint32_t)((s.c << ((s.used + l1) & 63)) >> ((64 - hlog) & 63)));
            const uint32_t l2 = e.U(T->huf[w]) >> 8;
            if (l1 + l2 <= 12) {  // a double entry for the lone last symbol
                if (s.used < 64) s.used = s.used + l1 + l2 > 64 ? 64u : s.used + l1 + l2;
                return d & 0xFFu;
            }
        }
        open = paired ? 0u : l1;
    }
    s.used += l1;
    return d & 0xFFu;
}
template <class E>
ZS_FN void huf_run(E& e, Tabs* T, Bits& s, uint32_t& open, uint32_t left, uint32_t n, bool x2, uint32_t hlog,
                   bool emit) {
    for (uint32_t i = 0; i < n; i++, left--) {
        const uint32_t sym = huf_one(e, T, s, open, left, x2, hlog);
        if (emit) e.lit(sym);
    }
}

// An environment that keeps literals in a buffer of its own may produce a
// block's literals eagerly: Huffman ones all streams at once (E::huf_all, as
// HUF_decompress4X interleaves them), raw and RLE ones in one copy or fill
// (E::raw_ahead / E::fill_ahead); lits_emit then only takes them.  The
// symbols, and the stream states lits_finish checks, are those of the lazy
// consumption-order decode (no check happens between two symbols).
template <class E>
struct EagerLits {
    static constexpr bool value = false;
};

// stream K (a constant: the per-stream state stays in registers on the device)
#define ZS_RUN(K, N, EMIT) huf_run(e, T, L.s[K], L.pend[K], L.cnt[K] - L.dec[K], N, L.x2, hlog, EMIT)

template <class E>
ZS_FN void lits_emit(E& e, Tabs* T, Lits& L, uint32_t k, uint32_t hlog) {
    if constexpr (EagerLits<E>::value) {  // every kind already in place (raw_ahead, fill_ahead, huf_all)
        e.take(k);
        L.used += k;
    } else if (L.kind == 0) {
        e.raw(L.pos + L.used, k);
        L.used += k;
    } else if (L.kind == 1) {
        e.fill(L.rle, k);
        L.used += k;
    } else {
        while (k) {
            while (L.used == L.curend) {  // the next stream's segment
                L.cur++;
                L.curend += L.seg;
            }
            const uint32_t m = L.curend - L.used < k ? L.curend - L.used : k;
            if (L.cur == 0) {
                ZS_RUN(0, m, true);
                L.dec[0] += m;
            } else if (L.cur == 1) {
                ZS_RUN(1, m, true);
                L.dec[1] += m;
            } else if (L.cur == 2) {
                ZS_RUN(2, m, true);
                L.dec[2] += m;
            } else {
                ZS_RUN(3, m, true);
                L.dec[3] += m;
            }
            L.used += m;
            k -= m;
        }
    }
}

// every stream decoded to its libzstd count and ended exactly
template <class E>
ZS_FN bool lits_finish(E& e, Tabs* T, Lits& L, uint32_t hlog) {
    if (L.kind != 2) return true;
#define ZS_FIN(K)                                   \
    if (L.dec[K] < L.cnt[K]) {                      \
        ZS_RUN(K, L.cnt[K] - L.dec[K], false);      \
        L.dec[K] = L.cnt[K];                        \
    }                                               \
    bits_reload(e, L.s[K]);                         \
    if (!bits_end(L.s[K])) return false;
    ZS_FIN(0)
    if (L.ns == 4) {
        ZS_FIN(1)
        ZS_FIN(2)
        ZS_FIN(3)
    }
#undef ZS_FIN
    return true;
}
#undef ZS_RUN

// ---------------------------------------------------------------------------
// One sequence off the bit stream (ZSTD_decodeSequence): the offset code as
// its kind and value (the repeat offsets are applied by seq_apply), the
// literal and match lengths; the three states advanced and the container
// reloaded.  The bit reads are libzstd's, in its order.
// ---------------------------------------------------------------------------
struct RawSeq {
    uint32_t ll, ml, v, kind;  // kind 0: new offset v; 1: repeat, no offset bit; 2: repeat code v (1..4)
};
struct SeqState {
    uint32_t sll, sof, sml;
};
template <class E>
ZS_FN void seq_decode(E& e, Tabs* T, Bits& d, SeqState& q, RawSeq& r) {
    const SeqSym Ls = e.sym(T->ll[q.sll]), Ms = e.sym(T->ml[q.sml]), Os = e.sym(T->of[q.sof]);
    const uint32_t tot = (uint32_t)Ls.nadd + Ms.nadd + Os.nadd;
    if (Os.nadd > 1) {
        r.kind = 0;
        r.v = (uint32_t)(Os.base + bits_readf(d, Os.nadd));
    } else if (Os.nadd == 0) {
        r.kind = 1;
        r.v = 0;
    } else {
        r.kind = 2;
        r.v = Os.base + (Ls.base == 0 ? 1u : 0u) + (uint32_t)bits_readf(d, 1);
    }
    uint64_t ml = Ms.base;
    if (Ms.nadd) ml += bits_readf(d, Ms.nadd);
    if (tot >= 31) bits_reload(e, d);
    uint64_t ll = Ls.base;
    if (Ls.nadd) ll += bits_readf(d, Ls.nadd);
    q.sll = Ls.next + (uint32_t)bits_read(d, Ls.nbits);
    q.sml = Ms.next + (uint32_t)bits_read(d, Ms.nbits);
    q.sof = Os.next + (uint32_t)bits_read(d, Os.nbits);
    bits_reload(e, d);
    r.ll = (uint32_t)ll;
    r.ml = (uint32_t)ml;
}
// the stream's initial states (after bits_init)
template <class E>
ZS_FN void seq_begin(E& e, Bits& d, SeqState& q, uint32_t llog, uint32_t olog, uint32_t mlog) {
    q.sll = (uint32_t)bits_read(d, llog);
    bits_reload(e, d);
    q.sof = (uint32_t)bits_read(d, olog);
    bits_reload(e, d);
    q.sml = (uint32_t)bits_read(d, mlog);
    bits_reload(e, d);
}

// An environment may take a block's sequences decoded ahead (E::seqs_take:
// the same seq_decode from the same tables and stream, all of them, and the
// stream's end verdict): block() then only applies them (repeat offsets,
// the reference's checks, literals, matches).  The verdict is unchanged:
// every failure inside a block rejects the payload, whichever comes first.
template <class E>
struct EagerSeqs {
    static constexpr bool value = false;
};

// An environment may emulate the DCtx's output buffer byte for byte (round
// 6): every ZSTD_execSequence write as libzstd 1.4.x
// performs it on x86-64 (literal copy16 / wildcopy with their overcopy,
// the match's wildcopy / overlapCopy8 / extDict memmove, ZSTD_execSequenceEnd's
// safecopy near the buffer end), so that a match reaching into the
// previous ring segment where the current one has written (or overcopied)
// reads what libzstd reads.  block() then hands each sequence to
// E::exec_seq after the reference's checks (no ring rule), and payload()
// tells the environment the buffer geometry (ring_begin, ring_wrap) and
// each literal section's padding (lit_pad).
template <class E>
struct ExactRing {
    static constexpr bool value = false;
};
// An environment that is told (E::ring_dirty) when a match of a
// non-ExactRing decode reaches into the overwritten part of the previous ring
// segment, just before the payload is turned down: the device then decodes
// that payload again over an ExactRing environment (rp_inflate.hip k_zexact).
template <class E>
struct RingDirtyHook {
    static constexpr bool value = false;
};

// ---------------------------------------------------------------------------
// Frame state and one compressed block
// ---------------------------------------------------------------------------
struct Frame {
    uint64_t fo;        // frame output so far
    uint64_t seg0;      // frame position where the current output segment starts
    uint64_t prevlen;   // length of the previous segment (ring wrap), 0 if none
    uint64_t rep[3];
    uint32_t llog, olog, mlog, hlog;
    bool lit_ok, fse_ok;
    bool hx2;  // the Huffman table was last built as libzstd's double-symbol table
};

// returns the block's output length or -1
template <class E>
ZS_FN int64_t block(E& e, Tabs* T, Frame& F, uint64_t bp, uint64_t bn, uint64_t capb) {
    if (bn < 3) return -1;
    const uint64_t end = bp + bn;
    const uint32_t b0 = e.b(bp);
    const uint32_t lt = b0 & 3, lhl = (b0 >> 2) & 3;
    Lits L;
    L.kind = 0;
    L.used = 0;
    L.ns = 1;
    L.seg = 1;
    L.x2 = false;
    L.pend[0] = L.pend[1] = L.pend[2] = L.pend[3] = 0;
    uint64_t lcons = 0;
    if (lt < 2) {
        uint32_t lh, lsz;
        if (lhl == 1) {
            lh = 2;
            lsz = (uint32_t)e.le(bp, 2) >> 4;
        } else if (lhl == 3) {
            lh = 3;
            lsz = (uint32_t)e.le(bp, 3) >> 4;
        } else {
            lh = 1;
            lsz = b0 >> 3;
        }
        if (lt == 0) {
            if ((uint64_t)lh + lsz > bn) return -1;
            L.kind = 0;
            L.pos = bp + lh;
            lcons = lh + (uint64_t)lsz;
        } else {
            if (lhl == 3 && bn < 4) return -1;
            if (lsz > kBlockMax) return -1;
            L.kind = 1;
            L.rle = e.b(bp + lh);
            lcons = lh + 1u;
        }
        L.size = lsz;
        // eager: the block's raw / RLE literals in place at once
        if constexpr (EagerLits<E>::value) {
            if (L.kind == 0) e.raw_ahead(L.pos, lsz);
            else e.fill_ahead(L.rle, lsz);
        }
        // what a wildcopy reads past the literals (ZSTD_decodeLiteralsBlock):
        // raw literals are read in place from the block unless they end
        // within WILDCOPY_OVERLENGTH of it (then copied, zero padded); RLE
        // literals are memset 32 bytes long
        if constexpr (ExactRing<E>::value) {
            if (L.kind == 0) e.lit_pad(lh + (uint64_t)lsz + kRingDirty > bn ? 0 : 1, L.pos + lsz, 0u);
            else e.lit_pad(2, 0, L.rle);
        }
    } else {
        if (lt == 3 && !F.lit_ok) return -1;
        if (bn < 5) return -1;
        const uint32_t lhc = (uint32_t)e.le(bp, 4);
        uint32_t lh, lsz;
        uint64_t lcs;
        bool single = false;
        if (lhl < 2) {
            single = lhl == 0;
            lh = 3;
            lsz = (lhc >> 4) & 0x3FF;
            lcs = (lhc >> 14) & 0x3FF;
        } else if (lhl == 2) {
            lh = 4;
            lsz = (lhc >> 4) & 0x3FFF;
            lcs = lhc >> 18;
        } else {
            lh = 5;
            lsz = (lhc >> 4) & 0x3FFFF;
            lcs = (lhc >> 22) + ((uint64_t)e.b(bp + 4) << 10);
        }
        if (lsz > kBlockMax) return -1;
        if (lcs + lh > bn) return -1;
        uint64_t hs = bp + lh, hn = lcs;
        if (lt == 2) {
            if (!single && (lsz == 0 || hn == 0)) return -1;
            uint32_t hl = 0;
            const int64_t th = huf_table(e, T, hs, hn, hl);
            if (th < 0) return -1;
            if ((uint64_t)th >= hn) return -1;
            F.hlog = hl;
            F.hx2 = !single && huf_select_x2(lsz, lcs);
            hs += (uint64_t)th;
            hn -= (uint64_t)th;
        }
        L.kind = 2;
        L.size = lsz;
        if (single) {
            L.ns = 1;
            if (!bits_init(e, L.s[0], hs, hn)) return -1;
            L.cnt[0] = lsz;
            L.dec[0] = 0;
            L.cur = 0;
            L.curend = 0xFFFFFFFFu;
        } else {
            if (hn < 10) return -1;
            const uint64_t l1 = e.le(hs, 2), l2 = e.le(hs + 2, 2), l3 = e.le(hs + 4, 2);
            const uint64_t l4 = hn - (l1 + l2 + l3 + 6);
            if (l4 > hn) return -1;
            const uint64_t s1 = hs + 6, s2 = s1 + l1, s3 = s2 + l2, s4 = s3 + l3;
            if (!bits_init(e, L.s[0], s1, l1) || !bits_init(e, L.s[1], s2, l2) || !bits_init(e, L.s[2], s3, l3) ||
                !bits_init(e, L.s[3], s4, l4))
                return -1;
            L.ns = 4;
            L.x2 = F.hx2;
            L.seg = (lsz + 3) / 4;
            L.cnt[0] = L.cnt[1] = L.cnt[2] = L.seg;
            L.cnt[3] = lsz > 3 * L.seg ? lsz - 3 * L.seg : 0;
            L.dec[0] = L.dec[1] = L.dec[2] = L.dec[3] = 0;
            L.cur = 0;
            L.curend = L.seg;
        }
        F.lit_ok = true;
        lcons = lh + lcs;
        if constexpr (EagerLits<E>::value) e.huf_all(T, L, F.hlog);
        if constexpr (ExactRing<E>::value) e.lit_pad(0, 0, 0u);  // Huffman literals: zero padded
    }
    // sequences section header
    uint64_t sp = bp + lcons;
    if (end - sp < 1) return -1;
    uint32_t nseq = e.b(sp++);
    if (nseq == 0) {
        if (sp != end) return -1;
    } else if (nseq == 255) {
        if (sp + 2 > end) return -1;
        nseq = (uint32_t)e.le(sp, 2) + 0x7F00;
        sp += 2;
    } else if (nseq >= 128) {
        if (sp >= end) return -1;
        nseq = ((nseq - 128) << 8) + e.b(sp);
        sp++;
    }
    uint64_t bo = 0;
    if (nseq) {
        if (sp + 1 > end) return -1;
        const uint32_t modes = e.b(sp++);
        int64_t h = seq_table(e, T, T->ll, F.llog, modes >> 6, 35, 9, sp, end - sp, kLLBase, kLLBits, kLLNorm, 35, 6,
                              F.fse_ok);
        if (h < 0) return -1;
        sp += (uint64_t)h;
        h = seq_table(e, T, T->of, F.olog, (modes >> 4) & 3, 31, 8, sp, end - sp, kOFBase, kOFBits, kOFNorm, 28, 5,
                      F.fse_ok);
        if (h < 0) return -1;
        sp += (uint64_t)h;
        h = seq_table(e, T, T->ml, F.mlog, (modes >> 2) & 3, 52, 9, sp, end - sp, kMLBase, kMLBits, kMLNorm, 52, 6,
                      F.fse_ok);
        if (h < 0) return -1;
        sp += (uint64_t)h;
        // ZSTD_decompressSequences_body
        F.fse_ok = true;
        uint64_t r0 = F.rep[0], r1 = F.rep[1], r2 = F.rep[2];
        bool pre = false;
        if constexpr (EagerSeqs<E>::value) pre = e.seqs_take(sp, end - sp, nseq, F.llog, F.olog, F.mlog);
        Bits d;
        SeqState q;
        if (!pre) {
            if (!bits_init(e, d, sp, end - sp)) return -1;
            seq_begin(e, d, q, F.llog, F.olog, F.mlog);
        }
        // a pre-decoded section is applied by the environment in one go
        // (E::seqs_apply: the loop below, the same checks in the same
        // arithmetic, any failure rejecting the payload)
        bool applied = false;
        if constexpr (EagerSeqs<E>::value) {
            if (pre) {
                if (!e.seqs_apply(F, L, r0, r1, r2, bo, capb, nseq)) return -1;
                applied = true;
            }
        }
        for (; !applied;) {
            RawSeq rs;
            if constexpr (EagerSeqs<E>::value) {
                if (pre) e.seq_next(rs);
                else seq_decode(e, T, d, q, rs);
            } else {
                seq_decode(e, T, d, q, rs);
            }
            uint64_t off;
            if (rs.kind == 0) {
                off = rs.v;
                r2 = r1;
                r1 = r0;
                r0 = off;
            } else if (rs.kind == 1) {
                if (rs.ll != 0) {
                    off = r0;
                } else {
                    off = r1;
                    r1 = r0;
                    r0 = off;
                }
            } else {
                uint64_t t = rs.v == 3 ? r0 - 1 : (rs.v == 1 ? r1 : r2);
                t += !t;
                if (rs.v != 1) r2 = r1;
                r1 = r0;
                r0 = off = t;
            }
            const uint64_t ll = rs.ll, ml = rs.ml;
            // ZSTD_execSequence's checks, then the copies
            if (ll + ml > capb - bo) return -1;
            if (ll > (uint64_t)(L.size - L.used)) return -1;
            if constexpr (ExactRing<E>::value) {
                // the copies on the emulated buffer (reads past the window
                // into the previous segment see what libzstd sees)
                if (off > F.fo + ll - F.seg0 + F.prevlen) return -1;
                e.exec_seq(ll, off, ml);
                L.used += (uint32_t)ll;
                bo += ll + ml;
                F.fo += ll + ml;
                if (--nseq == 0) break;
                continue;
            }
            if (ll) ZS_PROF(0, lits_emit(e, T, L, (uint32_t)ll, F.hlog));
            bo += ll;
            F.fo += ll;
            if (off > F.fo - F.seg0 + F.prevlen) return -1;  // beyond the prefix and the previous segment
            // ring-buffer mode: the previous segment (libzstd's extDict) sits
            // at the start of the DCtx's buffer, where this segment's output
            // (and the up-to-32-byte overcopy of its last copies) has been
            // written over it; a source there reads those newer bytes in
            // libzstd.  Rejected here (a documented divergence on corrupt
            // streams only: a conforming encoder never reaches past its
            // window); sources further up the previous segment are the true
            // history, as here.
            if (off > F.fo - F.seg0 && F.prevlen - (off - (F.fo - F.seg0)) < F.fo - F.seg0 + kRingDirty) {
                if constexpr (RingDirtyHook<E>::value) e.ring_dirty();
                return -1;
            }
            ZS_PROF(1, e.match(off, ml));
            bo += ml;
            F.fo += ml;
            if (--nseq == 0) break;
        }
        if constexpr (EagerSeqs<E>::value) {
            if (pre ? !e.seqs_ok() : bits_reload(e, d) < kCompleted) return -1;
        } else {
            if (bits_reload(e, d) < kCompleted) return -1;
        }
        F.rep[0] = r0;
        F.rep[1] = r1;
        F.rep[2] = r2;
    }
    const uint32_t last = L.size - L.used;
    if (last > capb - bo) return -1;
    if (last) ZS_PROF(0, lits_emit(e, T, L, last, F.hlog));
    bo += last;
    F.fo += last;
    bool fin = false;
    ZS_PROF(2, fin = lits_finish(e, T, L, F.hlog));
    if (!fin) return -1;
    return (int64_t)bo;
}

// ---------------------------------------------------------------------------
// The payload: stream_zstd::do_uncompress's loop over ZSTD_decompressStream.
// 0 accepted (total = bytes the loop delivers), -1 rejected (the reference
// throws).  *unsure is set when a content checksum could not be verified
// (E::check returned 2: the output outgrew what the environment holds).
//
// The loop's ZSTD_outBuffer (`opos` of 64 KiB) is emulated because it decides
// two things: the single-pass shortcut (the frame must fit the room left in
// it) and what a truncated payload yields.  The loop stops as soon as the
// input is consumed, so output the DCtx still holds then is never drained:
// when the unit (block, or present part of a raw block) that consumes the
// last input byte does not end its frame, only the part of its output that
// fits the buffer's room arrives.  (A unit that ends its frame holds a
// "hostage" input byte until its output is drained: nothing is lost.)
// ---------------------------------------------------------------------------
template <class E>
ZS_FN int payload(E& e, Tabs* T, uint64_t n, uint64_t& total, bool& unsure) {
    total = 0;
    unsure = false;
    uint64_t ip = 0, inbuf = 0, outbuf = 0, opos = 0;
    Frame F;
    // output of a streaming unit leaving the DCtx: drained into the loop's
    // buffer, which the loop empties whenever it is full and input remains
    auto drain = [&](uint64_t r) {
        for (;;) {
            const uint64_t f = r < kOutRoom - opos ? r : kOutRoom - opos;
            opos += f;
            r -= f;
            if (!r) break;
            opos = 0;
        }
    };
    while (ip < n) {
        if (opos == kOutRoom) opos = 0;  // a frame ends a call: a full buffer is emptied before the next
        const uint64_t rem = n - ip;
        if (rem < 5) return 0;  // a header still loading
        const uint32_t magic = (uint32_t)e.le(ip, 4);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
            if (rem < 8) return 0;
            const uint64_t sz = e.le(ip + 4, 4);
            const uint64_t nin = 4, nout = sz < 2112 ? sz : 2112;
            if (inbuf < nin || outbuf < nout) {
                inbuf = nin;
                outbuf = nout;
            }
            if (rem - 8 < sz) return 0;
            ip += 8 + sz;
            continue;
        }
        if (magic != 0xFD2FB528u) return -1;
        const uint32_t fhd = e.b(ip + 4);
        const uint32_t single = (fhd >> 5) & 1, fcsid = fhd >> 6, did = fhd & 3, ck = (fhd >> 2) & 1;
        const uint32_t didsz = did == 3 ? 4 : did;
        const uint64_t hsize = 5 + (single ? 0 : 1) + didsz + (fcsid ? (fcsid == 1 ? 2 : fcsid == 2 ? 4 : 8) : 0) +
                               ((single && !fcsid) ? 1 : 0);
        if (rem < hsize) return 0;
        if (fhd & 8) return -1;
        uint64_t pos = ip + 5, W = 0;
        if (!single) {
            const uint32_t wl = e.b(pos++);
            const uint32_t wlog = (wl >> 3) + 10;
            if (wlog > 31) return -1;
            W = 1ull << wlog;
            W += (W >> 3) * (wl & 7);
        }
        uint64_t dictid = 0;
        if (didsz) {
            dictid = e.le(pos, didsz);
            pos += didsz;
        }
        uint64_t fcs = kUnknown;
        if (fcsid == 0) {
            if (single) fcs = e.b(pos++);
        } else if (fcsid == 1) {
            fcs = e.le(pos, 2) + 256;
            pos += 2;
        } else if (fcsid == 2) {
            fcs = e.le(pos, 4);
            pos += 4;
        } else {
            fcs = e.le(pos, 8);
            pos += 8;
        }
        if (single) W = fcs;
        if (dictid) return -1;
        const uint64_t bsm = W < kBlockMax ? W : kBlockMax;
        const uint64_t room = kOutRoom - opos;
        // the single-pass shortcut: content size known, fits the room, whole frame here
        bool sp = false;
        uint64_t q = ip + hsize;
        if (fcs != kUnknown && room >= fcs) {
            sp = true;
            for (;;) {
                if (n - q < 3) {
                    sp = false;
                    break;
                }
                const uint32_t bh = (uint32_t)e.le(q, 3);
                const uint32_t bt = (bh >> 1) & 3;
                if (bt == 3) {
                    sp = false;
                    break;
                }
                const uint64_t cs = bt == 1 ? 1 : (bh >> 3);
                if (3 + cs > n - q) {
                    sp = false;
                    break;
                }
                q += 3 + cs;
                if (bh & 1) break;
            }
            if (sp && ck && n - q < 4) sp = false;
        }
        if (!sp) {  // the streaming path's memory control
            const uint64_t W1 = W > 1024 ? W : 1024;
            if (W1 > kMaxWindow) return -1;
            const uint64_t nin = bsm > 4 ? bsm : 4;
            const uint64_t rb = W1 + (W1 < kBlockMax ? W1 : kBlockMax) + 64;
            const uint64_t nout = fcs < rb ? fcs : rb;
            if (inbuf < nin || outbuf < nout) {
                if (nin + nout > kStaticBuffers) return -1;
                inbuf = nin;
                outbuf = nout;
            }
        }
        F.fo = 0;
        F.seg0 = 0;
        F.prevlen = 0;
        F.rep[0] = 1;
        F.rep[1] = 4;
        F.rep[2] = 8;
        F.llog = F.olog = F.mlog = F.hlog = 0;
        F.lit_ok = F.fse_ok = F.hx2 = false;
        e.frame_begin();
        // the buffer the frame's blocks decode into: the caller's output room
        // (single pass) or the DCtx's outBuff of `outbuf` bytes (streaming)
        if constexpr (ExactRing<E>::value) e.ring_begin(sp ? room : outbuf);
        uint64_t ostart = 0;  // streaming: outStart in the DCtx's buffer
        bool empty_end = false;
        ip += hsize;
        for (;;) {
            if (n - ip < 3) return 0;  // truncated (streaming only: single-pass frames are whole)
            const uint32_t bh = (uint32_t)e.le(ip, 3);
            const uint32_t last = bh & 1, bt = (bh >> 1) & 3, bsz = bh >> 3;
            if (bt == 3) return -1;
            const uint64_t cs = bt == 1 ? 1 : bsz;
            if (!sp && cs > bsm) return -1;
            ip += 3;
            if (!sp && cs == 0) {  // an empty block: the streaming path skips it (a last one ends the
                if (last) {        // frame without the content-size check)
                    empty_end = true;
                    break;
                }
                continue;
            }
            const uint64_t avail = n - ip;
            const uint64_t capb = sp ? room - F.fo : outbuf - ostart;
            uint64_t r;
            if (bt == 0) {
                const uint64_t k = avail < bsz ? avail : bsz;
                if (k > capb) return -1;
                e.raw(ip, k);
                F.fo += k;
                r = k;
            } else if (bt == 1) {
                if (avail < 1) return 0;
                if (bsz > capb) return -1;
                e.fill(e.b(ip), bsz);
                F.fo += bsz;
                r = bsz;
            } else {
                if (avail < bsz) return 0;
                if (bsz >= kBlockMax) return -1;
                int64_t o = -1;
                ZS_PROF(3, o = block(e, T, F, ip, bsz, capb));
                if (o < 0) return -1;
                r = (uint64_t)o;
            }
            ZS_TRACE("blk bt %u bsz %u last %u r %llu total %llu opos %llu avail %llu sp %d\n", bt, bsz, last,
                     (unsigned long long)r, (unsigned long long)total, (unsigned long long)opos,
                     (unsigned long long)avail, (int)sp);
            if (!sp && r > bsm) return -1;
            const bool to_end = (bt == 0 ? r : cs) == avail;
            const bool ends_frame = last && !ck && (bt != 0 || r == bsz);
            if (!sp && to_end && !ends_frame) {
                // this unit consumes the last input byte without ending its frame
                const uint64_t f = r < kOutRoom - opos ? r : kOutRoom - opos;
                total += f;
                return 0;
            }
            total += r;
            if (sp) {
                opos += r;
            } else {
                drain(r);
            }
            ip += cs;
            if (!sp) {  // the block leaves the DCtx's buffer; the buffer wraps when the next could not fit
                ostart += r;
                if (outbuf < fcs && ostart + bsm > outbuf) {
                    ostart = 0;
                    F.prevlen = F.fo - F.seg0;
                    F.seg0 = F.fo;
                    if constexpr (ExactRing<E>::value) e.ring_wrap();
                }
            }
            if (last) break;
        }
        if (fcs != kUnknown && F.fo != fcs && !empty_end) return -1;
        if (ck) {
            if (n - ip < 4) return 0;
            const int v = e.check((uint32_t)e.le(ip, 4));
            if (v == 0) return -1;
            if (v == 2) unsure = true;
            ip += 4;
        }
    }
    return 0;
}

}  // namespace zs
}  // namespace rp
