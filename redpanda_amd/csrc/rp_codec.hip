// rp_codec.hip — compression::compressor::uncompress on the device
// (compression/compression.cc:34-55):
//   * LZ4 frames: lz4_frame_compressor::uncompress / do_uncompressed
//     (compression/internal/lz4_frame_compressor.cc:115-213) over lz4 1.9.3's
//     LZ4F state machine and LZ4_decompress_safe_usingDict;
//   * snappy: snappy_java_compressor::uncompress
//     (compression/internal/snappy_java_compressor.cc:76-129), falling back to
//     snappy_standard_compressor (compression/snappy_standard_compressor.cc:
//     43-78) over snappy 1.1.8 RawUncompress.
// The control flow (every accept/reject decision) is the oracle's
// (oracle/rp_oracle.c), which restates those libraries.
//
// Execution model (lane engine): one LANE decodes one unit — an LZ4 block of
// a block-independent frame, a snappy-java chunk, or a whole sequential
// frame (linked LZ4 blocks, raw snappy, anything the planner did not split).
// An LZ4/snappy parse is a serial chain of dependent byte reads; run on one
// lane it costs a few dozen VALU instructions per sequence, and a wave
// advances 64 such chains at once.  (The round-2 first engine parsed one
// unit per wave on the scalar unit and spent ~370 instructions and ~2900
// cycles of one wave per sequence; see DESIGN.md.)
//   * Input: every sequence starts with one unaligned 16-byte load at the
//     token; the token, short literals (<= 14 bytes, the common case) and
//     the match offset come out of those four VGPRs (v_alignbyte).
//   * Output: 16-byte stores straight into the unit's arena slot; a copy may
//     write up to 15 bytes past its end ("wild" copy, as liblz4 does) while
//     that stays inside the slot — later sequences overwrite them.  Matches
//     with offsets >= 16 copy 16 bytes at a time from the lane's own earlier
//     output (program order on one lane makes its stores visible to its
//     loads); offsets 1..15 build the 16-byte repeating pattern in registers
//     (v_perm from a selector table) and store it at steps of a multiple of
//     the offset.
// Integer/byte work only: no MFMA.
#include "rp_device.h"
// RPGPU_DSTAMPS: diagnostic build of the decode kernel (scripts/build_exp.py
// dstamps -DRPGPU_DSTAMPS --unit rp_codec.hip): per unit kind, wall-clock
// totals / maxima / finish times, printed by k_print_dstamps; never measured
#ifdef RPGPU_DSTAMPS
#include <cstdio>
__device__ unsigned long long g_dst[64];
#endif

namespace rp {

typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

// 16 bytes at any byte address (one global_load_dwordx4)
DEV uint4 gld16(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, (const g_u8*)p, 16);
    return v;
}
DEV void gst16(uint8_t* p, uint4 v) { __builtin_memcpy((g_u8*)p, &v, 16); }

// ---------------------------------------------------------------------------
// per-lane stream and output views
// ---------------------------------------------------------------------------
struct Src {
    const uint8_t* p;  // stream start
    int64_t n;         // stream bytes
    int64_t rl;        // bytes readable from p (to the end of the job's data): 16-byte loads stay below
    // optional LDS copy of stream bytes [wlo, whi) (k_lz_walk's staged walk of
    // long pieces): 16-byte reads inside it come from LDS
    const lds_u8* win = nullptr;
    int64_t wlo = 0, whi = 0;
};
struct Dst {
    uint8_t* p;        // output position 0 of this unit
    int64_t lim;       // bytes writable from p (to the end of the unit's slot): wild stores stay below
};

DEV Src sub(const Src& s, int64_t at, int64_t n) { return Src{s.p + at, n, s.rl - at}; }

// byte i of the stream (bytes past it read as zero)
DEV uint32_t b8(const Src& s, int64_t i) { return (i >= 0 && i < s.n) ? (uint32_t)s.p[i] : 0u; }
DEV uint32_t le16(const Src& s, int64_t i) { return b8(s, i) | (b8(s, i + 1) << 8); }
DEV uint32_t le32(const Src& s, int64_t i) { return le16(s, i) | (le16(s, i + 2) << 16); }

// 16 stream bytes from i; bytes past the job's data read as zero
DEV uint4 ld16(const Src& s, int64_t i) {
    if (s.win && i >= s.wlo && i + 16 <= s.whi) {
        // five aligned dwords (the window has 16 spare bytes), then funnel shifts
        typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
        const uint32_t o = (uint32_t)(i - s.wlo);
        lds_cu32* w = (lds_cu32*)s.win + (o >> 2);
        const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4], sh = o & 3;
        return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                          __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
    }
    if (i + 16 <= s.rl) return gld16(s.p + i);
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t b = (i + k < s.rl) ? (uint32_t)s.p[i + k] << (8 * (k & 3)) : 0u;
        if (k < 4) w0 |= b; else if (k < 8) w1 |= b; else if (k < 12) w2 |= b; else w3 |= b;
    }
    return make_uint4(w0, w1, w2, w3);
}

// dword i (0..3, per lane) of a 16-byte value; 0 past it
DEV uint32_t dw(const uint4& w, uint32_t i) { return i == 0 ? w.x : i == 1 ? w.y : i == 2 ? w.z : i == 3 ? w.w : 0u; }
// the 4 bytes at byte k (0..15) of a 16-byte value, zero-filled past its end
DEV uint32_t at32(const uint4& w, uint32_t k) {
    const uint32_t i = k >> 2;
    return __builtin_amdgcn_alignbyte(dw(w, i + 1), dw(w, i), k & 3);
}
// the value shifted down by one byte (bytes 1..15, then a zero byte)
DEV uint4 shr1(const uint4& w) {
    return make_uint4(__builtin_amdgcn_alignbyte(w.y, w.x, 1), __builtin_amdgcn_alignbyte(w.z, w.y, 1),
                      __builtin_amdgcn_alignbyte(w.w, w.z, 1), w.w >> 8);
}

// 16 bytes (the first len of them significant, 1..16) at output o
DEV void put(const Dst& d, int64_t o, const uint4& v, uint32_t len) {
    if (o + 16 <= d.lim) {
        gst16(d.p + o, v);
        return;
    }
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        if (k < len) d.p[o + k] = (uint8_t)(dw(v, k >> 2) >> (8 * (k & 3)));
}

// len stream bytes from ip to output o (64 bytes in flight per step)
DEV void copy_in(const Src& s, int64_t ip, const Dst& d, int64_t o, int64_t len) {
    int64_t c = 0;
    for (; c + 64 <= len && ip + c + 64 <= s.rl && o + c + 64 <= d.lim; c += 64) {
        const uint4 a = gld16(s.p + ip + c), b = gld16(s.p + ip + c + 16), e = gld16(s.p + ip + c + 32),
                    f = gld16(s.p + ip + c + 48);
        gst16(d.p + o + c, a);
        gst16(d.p + o + c + 16, b);
        gst16(d.p + o + c + 32, e);
        gst16(d.p + o + c + 48, f);
    }
    for (; c < len; c += 16) put(d, o + c, ld16(s, ip + c), (uint32_t)(len - c < 16 ? len - c : 16));
}

// ---------------------------------------------------------------------------
// match copy: ml bytes at output o from o - off (the source may start in the
// history before d.p).  off >= 16: 16-byte pieces (every byte a piece reads
// was stored before it); off 1..15: the repeating pattern in registers;
// off 0: zeros (liblz4 1.9.3's write32(op, 0) / LZ4_memcpy_using_offset_base
// produce zeros for offset 0).
// ---------------------------------------------------------------------------
struct alignas(16) PatTab {
    uint32_t a[16][4], b[16][4];  // v_perm selectors: pattern byte i = src byte i % off
};
constexpr PatTab make_pat() {
    PatTab t{};
    for (uint32_t off = 1; off < 16; off++)
        for (uint32_t d = 0; d < 4; d++) {
            uint32_t a = 0, b = 0;
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t idx = (4 * d + k) % off;
                // v_perm_b32: selector 0..3 -> S1 bytes, 4..7 -> S0 bytes, 12 -> 0x00
                a |= (idx < 8 ? idx : 12u) << (8 * k);
                b |= (idx >= 8 ? idx - 8 : 12u) << (8 * k);
            }
            t.a[off][d] = a;
            t.b[off][d] = b;
        }
    return t;
}
__constant__ PatTab kPat = make_pat();

DEV void copy_match(const Dst& d, int64_t o, uint32_t off, int64_t ml) {
    if (off >= 16) {
        const uint8_t* s = d.p + o - off;
        int64_t c = 0;
        if (off >= 64)
            for (; c + 64 <= ml && o + c + 64 <= d.lim; c += 64) {
                const uint4 a = gld16(s + c), b = gld16(s + c + 16), e = gld16(s + c + 32), f = gld16(s + c + 48);
                gst16(d.p + o + c, a);
                gst16(d.p + o + c + 16, b);
                gst16(d.p + o + c + 32, e);
                gst16(d.p + o + c + 48, f);
            }
        for (; c < ml; c += 16) {
            uint4 v;
            if (o + c + 16 <= d.lim) v = gld16(s + c);
            else {  // near the slot end: the source bytes one by one (never past o + c)
                uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t k = 0; k < 16; k++)
                    if (c + k < ml) w[k >> 2] |= (uint32_t)s[c + k] << (8 * (k & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            put(d, o + c, v, (uint32_t)(ml - c < 16 ? ml - c : 16));
        }
        return;
    }
    uint4 p = make_uint4(0, 0, 0, 0);
    uint32_t step = 16;
    if (off) {
        // the off source bytes (the rest of the 16 are not read)
        uint4 v;
        if (o + 16 <= d.lim) v = gld16(d.p + o - off);
        else {
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t k = 0; k < 16; k++)
                if (k < off) w[k >> 2] |= (uint32_t)d.p[o - off + k] << (8 * (k & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        const uint4 sa = *(const uint4*)&kPat.a[off][0], sb = *(const uint4*)&kPat.b[off][0];
        p.x = __builtin_amdgcn_perm(v.y, v.x, sa.x) | __builtin_amdgcn_perm(v.w, v.z, sb.x);
        p.y = __builtin_amdgcn_perm(v.y, v.x, sa.y) | __builtin_amdgcn_perm(v.w, v.z, sb.y);
        p.z = __builtin_amdgcn_perm(v.y, v.x, sa.z) | __builtin_amdgcn_perm(v.w, v.z, sb.z);
        p.w = __builtin_amdgcn_perm(v.y, v.x, sa.w) | __builtin_amdgcn_perm(v.w, v.z, sb.w);
        // a multiple of off: the pattern restarts in phase at every step
        // (16 / off for off 1..15, less one, in 4-bit fields)
        step = off * (((0x00000001112347F0ull >> (4 * off)) & 15u) + 1u);
    }
    for (int64_t c = 0; c < ml; c += step) put(d, o + c, p, (uint32_t)(ml - c < 16 ? ml - c : 16));
}

// ---------------------------------------------------------------------------
// XXH32 (lz4 1.9.3 xxhash.c) on one lane, four stripes in flight
// ---------------------------------------------------------------------------
DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ __attribute__((noinline)) uint32_t xxh32_lane(const uint8_t* p, uint64_t n, uint32_t seed) {
    const uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
    uint64_t i = 0;
    uint32_t h;
    if (n >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        auto round4 = [&](const uint4& q) __attribute__((always_inline)) {
            v1 = rotl32(v1 + q.x * P2, 13) * P1;
            v2 = rotl32(v2 + q.y * P2, 13) * P1;
            v3 = rotl32(v3 + q.z * P2, 13) * P1;
            v4 = rotl32(v4 + q.w * P2, 13) * P1;
        };
        for (; i + 64 <= n; i += 64) {
            const uint4 a = gld16(p + i), b = gld16(p + i + 16), c = gld16(p + i + 32), e = gld16(p + i + 48);
            round4(a);
            round4(b);
            round4(c);
            round4(e);
        }
        for (; i + 16 <= n; i += 16) round4(gld16(p + i));
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    for (; i + 4 <= n; i += 4) {
        const uint32_t wd = (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
        h = rotl32(h + wd * P3, 17) * P4;
    }
    for (; i < n; i++) h = rotl32(h + p[i] * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

// XXH32 of n bytes at p by one wave.  The wave streams the input in 1 KiB
// rows (coalesced, the next row in flight) through an LDS buffer; lanes 0..3
// run the four accumulators, lane k folding dword k of each 16-byte stripe
// (ds_read_b32, issued ahead of the serial rounds), so the serial chain is
// plain VALU.  (A scalar-unit version, one readlane per dword, serialised
// on the CU's one scalar unit across waves.)  lz4 1.9.3 xxhash.c XXH32.
DEV uint32_t xxh32_wave(const uint8_t* p, uint64_t n, uint32_t seed, lds_u8* buf) {
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    const uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
    const uint32_t l = lane();
    const uint64_t ns = n >> 4;  // whole stripes
    uint32_t h;
    if (ns) {
        uint32_t acc = l == 0 ? seed + P1 + P2 : l == 1 ? seed + P2 : l == 2 ? seed : seed - P1;
        // the row loads are unconditional (a lane past the end reads stripe
        // 0 again, unused): a select right after a load made the compiler
        // wait for it there, so the next row was never in flight
        uint4 q = gld16(p + 16 * (uint64_t)(l < ns ? l : 0u));
        lds_u32* w = (lds_u32*)buf;
        for (uint64_t r = 0; r < ns; r += 64) {
            const uint64_t k = r + 64 + l;
            const uint4 nq = gld16(p + 16 * (k < ns ? k : 0ull));
            // each stripe word's product with P2 by its own lane (a wave
            // instruction for 64 stripes): the four serial chains below are
            // then add, rotate and one multiply per stripe
            w[4 * l] = q.x * P2;
            w[4 * l + 1] = q.y * P2;
            w[4 * l + 2] = q.z * P2;
            w[4 * l + 3] = q.w * P2;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const uint32_t cnt = ns - r < 64 ? (uint32_t)(ns - r) : 64u;
            if (l < 4) {
                uint32_t i = 0;
                for (; i + 8 <= cnt; i += 8) {
                    uint32_t x[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) x[u] = w[4 * (i + u) + l];
#pragma unroll
                    for (int u = 0; u < 8; u++) acc = rotl32(acc + x[u], 13) * P1;
                }
                for (; i < cnt; i++) acc = rotl32(acc + w[4 * i + l], 13) * P1;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            q = nq;
        }
        h = rotl32(rl(acc, 0), 1) + rotl32(rl(acc, 1), 7) + rotl32(rl(acc, 2), 12) + rotl32(rl(acc, 3), 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    // the last < 16 bytes: lane k holds byte k
    uint64_t i = ns << 4;
    const uint32_t t = (uint32_t)(n - i);
    const uint32_t b = l < t ? (uint32_t)p[i + l] : 0u;
    uint32_t k = 0;
    for (; k + 4 <= t; k += 4) {
        const uint32_t wd = rl(b, (int)k) | (rl(b, (int)k + 1) << 8) | (rl(b, (int)k + 2) << 16) | (rl(b, (int)k + 3) << 24);
        h = rotl32(h + wd * P3, 17) * P4;
    }
    for (; k < t; k++) h = rotl32(h + rl(b, (int)k) * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

// ---------------------------------------------------------------------------
// LZ4 block: rpo_lz4_block_decode (oracle) = lz4 1.9.3 LZ4_decompress_generic
// for LZ4_decompress_safe_usingDict (fast loop + safe loop, every check).
// One sequence walk, two sinks: DirectSink copies on the spot (the lane
// engine), RecSink writes SeqRecs for the wave engine and may suspend the
// walk when its buffer is full (PState holds the resume point).  Every
// accept/reject decision depends on positions and lengths only, never on
// byte values, so the walk alone decides the block's verdict and length.
// H = history bytes before the block; `need` records the most history any
// match reached for (a walk run with H = 65536 then fails iff need > the
// real H: every history check of the reference fails the block).
// Positions are 32-bit: a block is at most 4 MiB in and out, and a length
// read from it at most 255x that.
// ---------------------------------------------------------------------------
constexpr int32_t kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12, kFastSafeDistance = 64;

struct PState {
    int32_t ip, op;    // resume point (stream / output position)
    int32_t need;      // max over matches of offset - match position
    int32_t st;        // 0 walking, 1 done (op = decoded length), -1 rejected
    uint32_t ulen;     // snappy: the stream's uncompressed length
    uint32_t safe;     // lz4: in the safe loop
};

// the input window: 32 stream bytes from wb (two 16-byte loads issued
// together), reloaded only when a read falls outside it; an LZ4 sequence of
// short lengths spans 3-4 bytes, so one load round trip serves several
// one 16-byte load per window (a 32-byte window, two loads, measured slower:
// C2 walk 16.4 vs 13.8 ms, more VGPRs and fewer resident waves)
constexpr int32_t kWinSpan = 16;
struct Win {
    uint4 w, x;  // bytes [wb, wb + 16), [wb + 16, wb + 32)
    int32_t wb;
};
DEV void win_init(Win& W, const Src& s, int32_t p) {
    W.w = ld16(s, p);
    W.x = kWinSpan > 16 ? ld16(s, (int64_t)p + 16) : make_uint4(0, 0, 0, 0);
    W.wb = p;
}
DEV void win_need(Win& W, const Src& s, int32_t p, int32_t nbytes) {
    if (p < W.wb || p + nbytes > W.wb + kWinSpan) win_init(W, s, p);
}
// dword i (0..7) of the window; 0 past it
DEV uint32_t win_dw(const Win& W, uint32_t i) { return i < 4 ? dw(W.w, i) : dw(W.x, i - 4); }
DEV uint32_t win_at32(const Win& W, uint32_t k) {
    const uint32_t i = k >> 2;
    return __builtin_amdgcn_alignbyte(win_dw(W, i + 1), win_dw(W, i), k & 3);
}
DEV uint32_t win_byte(Win& W, const Src& s, int32_t p) {
    win_need(W, s, p, 1);
    const uint32_t k = (uint32_t)(p - W.wb);
    return (win_dw(W, k >> 2) >> (8 * (k & 3))) & 0xFFu;
}
DEV uint32_t win_le16(Win& W, const Src& s, int32_t p) {
    win_need(W, s, p, 2);
    return win_at32(W, (uint32_t)(p - W.wb)) & 0xFFFFu;
}

DEV int32_t lz_read_var(Win& W, const Src& s, int32_t& ip, int32_t lencheck, bool loop_check, bool initial_check, int& err) {
    int32_t length = 0;
    uint32_t b;
    err = 0;
    if (initial_check && ip >= lencheck) {
        err = 1;
        return length;
    }
    do {
        b = win_byte(W, s, ip);
        ip++;
        length += (int32_t)b;
        if (loop_check && ip >= lencheck) {
            err = 2;
            return length;
        }
    } while (b == 255);
    return length;
}

DEV void lz4_begin(PState& ps, const Src& s, int32_t oend) {
    ps.ip = ps.op = ps.need = 0;
    ps.ulen = 0;
    ps.safe = oend < kFastSafeDistance;
    ps.st = 0;
    if (oend == 0) ps.st = (s.n == 1 && b8(s, 0) == 0) ? 1 : -1;
    else if (s.n == 0) ps.st = -1;
}

// sinks: seq(w, wb, lip, llen, lo, off, ml) with the input window (16 stream
// bytes from wb), the literal [lip, lip + llen) to output lo and the match
// (off, ml; ml = 0: none) at lo + llen; false = suspend after it
struct DirectSink {
    const Src& s;
    const Dst& d;
    DEV bool seq(const uint4& w, int32_t wb, int32_t lip, int32_t llen, int32_t lo, uint32_t off, int32_t ml) {
        if (llen > 0) {
            // short literals right behind a window-leading token are already in w
            if (lip == wb + 1 && llen <= 15) put(d, lo, shr1(w), (uint32_t)llen);
            else copy_in(s, lip, d, lo, llen);
        }
        if (ml > 0) copy_match(d, (int64_t)lo + llen, off, ml);
        return true;
    }
};
struct RecSink {
    SeqRec* out;
    uint32_t n, cap;
    DEV bool seq(const uint4&, int32_t, int32_t lip, int32_t llen, int32_t, uint32_t off, int32_t ml) {
        out[n] = SeqRec{(uint32_t)lip, (uint32_t)llen, (uint32_t)ml, off};
        return ++n < cap;
    }
};

// stop_ip: suspend (st stays 0) before a sequence starting at or past it
template <class Sink>
DEV void lz4_run(const Src& s, int32_t oend, int32_t H, PState& ps, Sink& sink, int32_t stop_ip = INT32_MAX) {
    if (ps.st) return;
    const int32_t iend = (int32_t)s.n;
    const int32_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    int32_t ip = ps.ip, op = ps.op, need = ps.need, length, offset = 0, cpy = 0, lip = 0, llen = 0, ml = 0;
    int err;
    bool last = false, safe = ps.safe != 0;
    Win W;
    win_init(W, s, ip);
#define LZ_FAIL() do { ps.st = -1; return; } while (0)
    // The two loops of LZ4_decompress_generic as one: `safe` is the safe
    // loop (entered for good at the first fast-loop exit); every path ends at
    // `emit` with the sequence's literal (lip, llen; op already past it) and
    // match (offset, ml).
    for (;;) {
        if (ip >= stop_ip) {
            ps.ip = ip;
            ps.op = op;
            ps.need = need;
            ps.safe = safe;
            return;
        }
        const uint32_t token = win_byte(W, s, ip);
        ip++;
        length = (int32_t)(token >> 4);
#define RD_OFFSET() ((int32_t)win_le16(W, s, ip))
        if (!safe) {
            if (length == 15) {
                length += lz_read_var(W, s, ip, iend - 15, true, true, err);
                if (err == 1) LZ_FAIL();
                cpy = op + length;
                if (cpy > oend - 32 || ip + length > iend - 32) { safe = true; goto safe_literal_copy; }
            } else {
                cpy = op + length;
                if (ip > iend - (16 + 1)) { safe = true; goto safe_literal_copy; }
            }
            lip = ip;
            llen = length;
            ip += length;
            op = cpy;
            offset = RD_OFFSET();
            ip += 2;
            length = (int32_t)(token & 15);
            if (length == 15) {
                if (offset > op + H) LZ_FAIL();
                length += lz_read_var(W, s, ip, iend - kLastLiterals + 1, true, false, err);
                if (err) LZ_FAIL();
                length += kMinMatch;
                if (op + length >= oend - kFastSafeDistance) { safe = true; goto safe_match_copy; }
            } else {
                length += kMinMatch;
                if (op + length >= oend - kFastSafeDistance) { safe = true; goto safe_match_copy; }
            }
            if (offset > op + H) LZ_FAIL();
            ml = length;
            goto emit;
        }
        if (length != 15 && ip < shortiend && op <= shortoend) {
            lip = ip;
            llen = length;
            op += length;
            ip += length;
            length = (int32_t)(token & 15);
            offset = RD_OFFSET();
            ip += 2;
            if (length != 15 && offset >= 8 && offset <= op + H) {
                ml = length + kMinMatch;
                goto emit;
            }
            goto lbl_copy_match;
        }
        if (length == 15) {
            length += lz_read_var(W, s, ip, iend - 15, true, true, err);
            if (err == 1) LZ_FAIL();
        }
        cpy = op + length;
    safe_literal_copy:
        lip = ip;
        llen = length;
        if (cpy > oend - kMfLimit || ip + length > iend - (2 + 1 + kLastLiterals)) {
            if (ip + length != iend || cpy > oend) LZ_FAIL();
            ip += length;
            op += length;
            last = true;
            goto emit;
        }
        ip += length;
        op = cpy;
        offset = RD_OFFSET();
        ip += 2;
        length = (int32_t)(token & 15);
    lbl_copy_match:
        if (length == 15) {
            length += lz_read_var(W, s, ip, iend - kLastLiterals + 1, true, false, err);
            if (err) LZ_FAIL();
        }
        length += kMinMatch;
    safe_match_copy:
        if (offset > op + H) LZ_FAIL();
        // a match starting in the history (offset > op) ends by oend - 5;
        // so does one inside the block (cpy > oend - 12 -> cpy <= oend - 5)
        if (op + length > oend - kLastLiterals) LZ_FAIL();
        ml = length;
    emit:
#undef RD_OFFSET
        if (last) {
            sink.seq(W.w, W.wb, lip, llen, op - llen, 0u, 0);
            ps.st = 1;
            ps.op = op;
            ps.need = need;
            return;
        }
        if (offset - op > need) need = offset - op;
        const bool go = sink.seq(W.w, W.wb, lip, llen, op - llen, (uint32_t)offset, ml);
        op += ml;
        if (!go) {
            ps.ip = ip;
            ps.op = op;
            ps.need = need;
            ps.safe = safe;
            return;
        }
    }
#undef LZ_FAIL
}

// the lane engine's block decode: decoded length or -1
DEV int32_t lz4_block(const Src& s, const Dst& d, int32_t oend, int64_t H64) {
    PState ps;
    lz4_begin(ps, s, oend);
    DirectSink sink{s, d};
    lz4_run(s, oend, H64 > 65536 ? 65536 : (int32_t)H64, ps, sink);  // offsets are < 65536
    return ps.st == 1 ? ps.op : -1;
}
// ---------------------------------------------------------------------------
// LZ4 frame: rpo_lz4f_uncompress (oracle) — LZ4F_getFrameInfo + the
// LZ4F_decompress loop of do_uncompressed, including its output-buffer
// estimate (contentSize, or 4x the input; grown 1.5x + 1 KiB whenever a call
// returns with it full), which decides how much of a truncated frame is
// returned.  Output at d.p, which has room for the planned capacity
// (decode_capacity_dev).  Returns 0 (out_len set) or -1 where the reference
// throws.
//
// single != 0: the stream is one planned block of a block-independent frame
// (its data, then its checksum when kBlkChecksum): the header is not read,
// the block is decoded with oend = bcap and the unit ends after it.
// ---------------------------------------------------------------------------
DEV int lz4_unit(const Src& s, const Dst& d, uint32_t single, uint32_t bcap, int64_t& out_len) {
    out_len = 0;
    const int64_t n = s.n;
    int64_t pos, bmax;
    bool linked, bcs, ccs;
    uint64_t content_size, est;
    if (single) {
        pos = 0;
        bmax = bcap;
        linked = false;
        bcs = (single & kBlkChecksum) != 0;
        ccs = false;
        content_size = 0;
        est = ~0ull >> 2;
    } else {
        if (n < 7) return -1;                                    // frameHeader_incomplete
        const uint32_t magic = le32(s, 0);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {              // skippable frame
            if (n < 8) return -1;
            pos = 4;
            if (n - pos < 4) return 0;
            const uint32_t sz = le32(s, pos);
            pos += 4;
            if (n - pos < (int64_t)sz) return 0;
            pos += sz;
            return pos < n ? -1 : 0;
        }
        if (magic != 0x184D2204u) return -1;                     // frameType_unknown
        const uint32_t flg = b8(s, 4);
        const int64_t hsize = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
        if (n < hsize) return -1;
        if ((flg >> 1) & 1) return -1;                           // reservedFlag_set
        if (((flg >> 6) & 3) != 1) return -1;                    // headerVersion_wrong
        const uint32_t bd = b8(s, 5);
        if ((bd >> 7) & 1) return -1;
        const uint32_t bsid = (bd >> 4) & 7;
        if (bsid < 4) return -1;                                 // maxBlockSize_invalid
        if (bd & 15) return -1;
        if (((xxh32_small(s.p + 4, (uint32_t)(hsize - 5)) >> 8) & 0xFFu) != b8(s, hsize - 1)) return -1;
        linked = !((flg >> 5) & 1);
        bcs = (flg >> 4) & 1;
        ccs = (flg >> 2) & 1;
        const bool csf = (flg >> 3) & 1;
        content_size = csf ? ((uint64_t)le32(s, 6) | ((uint64_t)le32(s, 10) << 32)) : 0;
        bmax = bsid == 4 ? (64 << 10) : bsid == 5 ? (256 << 10) : bsid == 6 ? (1 << 20) : (4 << 20);
        pos = hsize;
        // compute_frame_uncompressed_size (lz4_frame_compressor.cc:115-121)
        est = (content_size == 0 || content_size > (uint64_t)n * 255) ? (uint64_t)n * 4 : content_size;
    }
    uint64_t remaining = content_size;
    int64_t out = 0;
    for (uint32_t blk_no = 0;; blk_no++) {
        uint32_t bh;
        if (single) {
            if (blk_no) break;
            bh = (uint32_t)(n - (bcs ? 4 : 0)) | ((single & kBlkRaw) ? 0x80000000u : 0u);
        } else {
            if (n - pos < 4) { out_len = out; return 0; }        // waiting for a block header
            bh = le32(s, pos);
            pos += 4;
            if (bh == 0) break;                                  // end mark
        }
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
                copy_in(s, pos, d, out, k);
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
                if (le32(s, pos) != xxh32_lane(s.p + blk, (uint64_t)bsz, 0)) return -1;
                pos += 4;
            }
            continue;
        }
        if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
        if (pos == n) { out_len = out; return 0; }
        const int64_t need = bsz + (bcs ? 4 : 0);
        if (n - pos < need) { out_len = out; return 0; }         // dstage_storeCBlock: wait
        if (bcs && le32(s, pos + bsz) != xxh32_lane(s.p + pos, (uint64_t)bsz, 0)) return -1;
        const Dst bd{d.p + out, d.lim - out};
        const int64_t dd = lz4_block(sub(s, pos, bsz), bd, (int32_t)bmax, linked ? out : 0);
        if (dd < 0) return -1;                                   // decompressionFailed
        pos += need;
        if (content_size) remaining -= (uint64_t)dd;
        const int64_t space = (int64_t)(est - (uint64_t)out);
        if (space >= bmax || dd <= space) { out += dd; continue; }
        // decoded into tmpOut: `space` bytes flushed now, the rest on later
        // calls — which only happen while input remains
        int64_t pending = dd - space;
        out += space;
        while (pending) {
            if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
            if (pos == n) { out_len = out; return 0; }
            const int64_t sp = (int64_t)(est - (uint64_t)out), f = pending < sp ? pending : sp;
            out += f;
            pending -= f;
        }
    }
    if (single) { out_len = out; return 0; }
    if (remaining) return -1;                                    // frameSize_wrong
    if (ccs) {
        if (n - pos < 4) { out_len = out; return 0; }
        if (le32(s, pos) != xxh32_lane(d.p, (uint64_t)out, 0)) return -1;
        pos += 4;
    }
    out_len = out;
    return pos < n ? -1 : 0;                                     // input left over: throw
}

// ---------------------------------------------------------------------------
// snappy 1.1.8 (oracle: snappy_varint32 / snappy_decode_tags /
// snappy_raw_checked / rpo_snappy_*_uncompress)
// ---------------------------------------------------------------------------
DEV int snappy_varint(const Src& s, int64_t pos, int64_t n, uint32_t& v, int64_t& used) {
    uint32_t r = 0;
    for (int64_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        const uint32_t b = b8(s, pos + i);
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

// snappy_raw_checked: varint length, then DecompressAllTags over the rest:
// succeeds iff the tags end exactly at n and exactly ulen bytes come out.
// whole: snappy_standard_compressor semantics for a raw payload (length 0
// is an empty result, the tags are not looked at).  Positions are 32-bit:
// streams are batch payloads (< 2 GiB).
DEV void snappy_begin(PState& ps, const Src& s, bool whole) {
    ps.ip = ps.op = ps.need = 0;
    ps.safe = 0;
    ps.st = 0;
    uint32_t ulen;
    int64_t used;
    if (snappy_varint(s, 0, s.n, ulen, used)) { ps.st = -1; return; }
    ps.ulen = ulen;
    ps.ip = (int32_t)used;
    if (whole && ulen == 0) { ps.st = 1; return; }  // "empty frame"
    // no tag sequence expands more than 64/3 per input byte
    if ((uint64_t)ulen > 22ull * (uint64_t)s.n + 64) ps.st = -1;
}

template <class Sink>
DEV void snappy_run(const Src& s, PState& ps, Sink& sink, int32_t stop_ip = INT32_MAX) {
    if (ps.st) return;
    const int64_t n = s.n, ulen = ps.ulen;
    int64_t ip = ps.ip, op = ps.op;
    Win W;
    win_init(W, s, (int32_t)ip);
    while (ip < n) {
        if (ip >= stop_ip) {
            ps.ip = (int32_t)ip;
            ps.op = (int32_t)op;
            return;
        }
        const uint32_t c = win_byte(W, s, (int32_t)ip);
        const uint32_t t = c & 3;
        const int64_t extra = t == 0 ? (((c >> 2) >= 60) ? (int64_t)((c >> 2) - 59) : 0) : t == 1 ? 1 : t == 2 ? 2 : 4;
        if (n - ip < 1 + extra) { ps.st = -1; return; }
        uint32_t x = 0;  // the tag's extra bytes (at most 4)
        if (extra) {
            win_need(W, s, (int32_t)ip + 1, (int32_t)extra);
            x = win_at32(W, (uint32_t)(ip + 1 - W.wb));
        }
        bool go;
        if (t == 0) {
            int64_t lit = (int64_t)(c >> 2) + 1;
            if (lit >= 61) lit = (int64_t)(extra == 4 ? x : x & ((1u << (8 * extra)) - 1u)) + 1;
            const int64_t lip = ip + 1 + extra;
            if (n - lip < lit) { ps.st = -1; return; }      // premature end of input
            if (ulen - op < lit) { ps.st = -1; return; }    // SnappyArrayWriter::Append overflow
            go = sink.seq(W.w, W.wb, (int32_t)lip, (int32_t)lit, (int32_t)op, 0u, 0);
            op += lit;
            ip = lip + lit;
        } else {
            const int64_t len = t == 1 ? 4 + ((c >> 2) & 7) : (int64_t)(c >> 2) + 1;
            const int64_t off = t == 1 ? (int64_t)(((c >> 5) << 8) | (x & 0xFFu)) : t == 2 ? (int64_t)(x & 0xFFFFu) : (int64_t)x;
            ip += 1 + extra;
            // AppendFromSelf: Produced() <= offset - 1u || op_end > op_limit_
            if (off == 0 || op < off || ulen - op < len) { ps.st = -1; return; }
            go = sink.seq(W.w, W.wb, 0, 0, (int32_t)op, (uint32_t)off, (int32_t)len);
            op += len;
        }
        if (!go && ip < n) {
            ps.ip = (int32_t)ip;
            ps.op = (int32_t)op;
            return;
        }
    }
    ps.op = (int32_t)op;
    ps.st = op == ulen ? 1 : -1;
}

DEV int snappy_raw_checked(const Src& s, const Dst& d, int64_t& out_len) {
    PState ps;
    snappy_begin(ps, s, false);
    DirectSink sink{s, d};
    snappy_run(s, ps, sink);
    if (ps.st != 1) return -1;
    out_len = ps.ulen;
    return 0;
}
// snappy_java_compressor::uncompress: the xerial stream's chunks one after
// the other, or the raw fallback (snappy_standard_compressor: length 0 is
// an empty result, RawUncompress not called).  single: the stream is one
// planned raw chunk.
DEV int snappy_unit(const Src& s, const Dst& d, uint32_t single, int64_t& out_len) {
    out_len = 0;
    const int64_t n = s.n;
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    bool java = !single && n >= 16;
    for (int i = 0; i < 8 && java; i++) java = b8(s, i) == magic[i];
    int64_t pos = 0, out = 0;
    if (java) {
        const int32_t min_version = (int32_t)le32(s, 12);  // native little endian
        if (min_version < 1) return -1;
        pos = 16;
    } else if (!single) {
        uint32_t ulen;
        int64_t used;
        if (snappy_varint(s, 0, n, ulen, used)) return -1;
        if (ulen == 0) return 0;  // "empty frame"
    }
    for (;;) {
        Src cs = s;
        if (java) {
            if (pos == n) break;
            if (n - pos < 4) return -1;                     // consume_be_type out_of_range
            const int32_t cl = (int32_t)((b8(s, pos) << 24) | (b8(s, pos + 1) << 16) | (b8(s, pos + 2) << 8) | b8(s, pos + 3));
            pos += 4;
            if (cl < 0) return -1;
            if (n - pos < (int64_t)cl) return -1;           // consume_to out_of_range
            cs = sub(s, pos, cl);
            pos += cl;
        }
        int64_t got = 0;
        if (snappy_raw_checked(cs, Dst{d.p + out, d.lim - out}, got)) return -1;
        out += got;
        if (!java) break;
    }
    out_len = out;
    return 0;
}

// compression::compressor::uncompress dispatch (compression/compression.cc:34-55)
// for one unit of work, on this lane; output complete when it returns 0
DEV int decode_unit(int codec, const Src& s, const Dst& d, uint32_t single, uint32_t bcap, int64_t& out_len) {
    out_len = 0;
    if (s.n == 0) return -1;
    if (codec == RPGPU_CODEC_SNAPPY) return snappy_unit(s, d, single, out_len);
    if (codec == RPGPU_CODEC_LZ4) return lz4_unit(s, d, single, bcap, out_len);
    return -1;
}

// ---------------------------------------------------------------------------
// Planning (one wave per compressed batch, wave-uniform reads through a
// 512-byte window): frames whose pieces are independent and that are
// structurally complete decode to the concatenation of their pieces (or fail
// when any piece fails): that is the sequential decoder's result for such
// frames, since every flush of do_uncompressed happens while input remains.
// Those frames are split into BlockItems at the plan rule's positions
// (decode_capacity_dev); everything else (linked LZ4 blocks, truncated or
// malformed frames, raw snappy) is decoded whole by one lane.
// ---------------------------------------------------------------------------
struct In {
    const uint8_t* src;  // stream start
    int64_t n;           // stream bytes
    int64_t base;        // stream offset of the window start
    uint32_t w0, w1;     // lane l: dwords base + 4 l and base + 256 + 4 l
};

DEV uint32_t ld_dw(const uint8_t* src, int64_t n, uintptr_t a) {
    return a < (uintptr_t)(src + n) ? *(const uint32_t*)a : 0u;  // a is 4-aligned: never crosses a page
}

DEV void in_init(In& in, const uint8_t* src, int64_t n) {
    in.src = src;
    in.n = n;
    in.base = -(1ll << 60);
    in.w0 = in.w1 = 0;
}

// byte ip of the stream (uniform; bytes past the stream read as zero)
DEV uint32_t in_byte(In& in, int64_t ip) {
    int64_t o = ip - in.base;
    if (o < 0 || o >= 512) {
        const uintptr_t a = ((uintptr_t)(in.src + ip)) & ~(uintptr_t)3;
        in.base = (int64_t)(a - (uintptr_t)in.src);
        in.w0 = ld_dw(in.src, in.n, a + 4u * lane());
        in.w1 = ld_dw(in.src, in.n, a + 256u + 4u * lane());
        o = ip - in.base;
    }
    const int li = (int)((o >> 2) & 63);
    const uint32_t w = o < 256 ? rl(in.w0, li) : rl(in.w1, li);
    return (w >> (8 * (uint32_t)(o & 3))) & 0xFFu;
}
DEV uint32_t in_le16(In& in, int64_t ip) { return in_byte(in, ip) | (in_byte(in, ip + 1) << 8); }
DEV uint32_t in_le32(In& in, int64_t ip) { return in_le16(in, ip) | (in_le16(in, ip + 2) << 16); }

DEV int in_varint(In& in, int64_t pos, int64_t n, uint32_t& v) {
    uint32_t r = 0;
    for (int64_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        const uint32_t b = in_byte(in, pos + i);
        if (i < 4) {
            r |= (b & 127) << (7 * i);
            if (b < 128) { v = r; return 0; }
        } else {
            r |= (b & 127) << 28;
            if (b < 16) { v = r; return 0; }
            return -1;
        }
    }
    return -1;
}


#ifndef RPGPU_LONG_LZ4
#define RPGPU_LONG_LZ4 65536u
#endif
// dense pieces (decoded capacity >= RPGPU_DENSE_X10 / 10 x compressed, at least
// RPGPU_DENSE_MIN compressed: thousands of short sequences) are wave-walked
// too, where the window-parallel parse takes ~13 sequences per step;
// literal-heavy ones stay on the lane walk, whose 256-byte windows skip long
// literals.  Measured (step ms C2 / C5): off 65.4 / 38.4; x3 from 4 KiB
// 65.4 / 23.1; x2 from 1 KiB 64.5 / 23.1.
#ifndef RPGPU_DENSE_X10
#define RPGPU_DENSE_X10 20u
#endif
#ifndef RPGPU_DENSE_MIN
#define RPGPU_DENSE_MIN 1024u
#endif
#ifndef RPGPU_ALONE_MIN
#define RPGPU_ALONE_MIN 0u
#endif
DEV bool piece_dense(uint32_t csize, uint32_t cap) {
    return RPGPU_DENSE_X10 && csize >= RPGPU_DENSE_MIN && 10ull * cap >= (uint64_t)RPGPU_DENSE_X10 * csize;
}
// the pieces k_lz_exec runs alone (the long list): long, dense, and (with
// RPGPU_ALONE_MIN) every compressed piece of at least that many bytes
DEV bool piece_is_long(uint32_t kind, uint32_t csize, uint32_t cap) {
    return !(kind & kBlkRaw) && ((kind & kBlkWhole) || csize > RPGPU_LONG_LZ4 || piece_dense(csize, cap) ||
                                 (RPGPU_ALONE_MIN && csize >= RPGPU_ALONE_MIN));
}
// Long pieces all run alone in k_lz_exec.  Dense ones are wave-walked only
// when the job has few pieces for the lanes the walk keeps resident
// (few_pieces): with many, the lane walk does them faster in aggregate (C2,
// ~250 K pieces: step 63.7 -> 56.2 ms with its dense LZ4 blocks on the lane
// walk); with few, lanes sit idle behind the slowest ones (C5, ~55 K pieces:
// 23.1 -> 31.5 ms without the wave walk, 28.9 with only its snappy chunks on
// it).  RPGPU_DENSE_WALK 1 / 0 force it on / off (diagnostics).
#ifndef RPGPU_DENSE_WALK
#define RPGPU_DENSE_WALK 2
#endif
DEV bool piece_wave_walked(uint32_t kind, uint32_t csize, uint32_t cap, bool few_pieces) {
    const bool dense = RPGPU_DENSE_WALK == 1 || (RPGPU_DENSE_WALK == 2 && few_pieces);
    return !(kind & kBlkRaw) && ((kind & kBlkWhole) || csize > RPGPU_LONG_LZ4 || (dense && piece_dense(csize, cap)));
}

// long pieces base + i for the set bits i of m (lane 0): one atomic per 64
// blocks of a frame (one per piece cost the planner ~1 ms on C2's dense
// blocks).  k_lz_exec runs every long piece alone (long_list); k_lz_walk
// walks those of w (wlong_list: not the ones k_lzf_walk takes, which it
// would claim one wave-wide atomic apiece only to skip)
DEV void note_longs(const DeviceJob& j, uint32_t base, uint64_t m, uint64_t w) {
    if (m) {
        uint32_t at = atomicAdd(&j.counters[11], (uint32_t)__builtin_popcountll(m));
        for (; m; m &= m - 1) j.long_list[at++] = base + (uint32_t)__builtin_ctzll(m);
    }
    if (w) {
        uint32_t at = atomicAdd(&j.counters[38], (uint32_t)__builtin_popcountll(w));
        for (; w; w &= w - 1) j.wlong_list[at++] = base + (uint32_t)__builtin_ctzll(w);
    }
}
// k_lzf_walk's per-lane window (design note at k_lzf_walk)
#ifndef RPGPU_LZF_WIN
#define RPGPU_LZF_WIN 256
#endif
constexpr uint32_t kFWin = RPGPU_LZF_WIN;  // sequence starts walked per staged window
constexpr uint32_t kFSlot = kFWin + 32;    // + a 16-byte read at the last start, or the offset bytes after it
constexpr uint32_t kFMarginIn = 64, kFMarginOut = 128;
static_assert(kFWin % 32 == 0 && kFWin >= 64, "lane window");
// a planned LZ4 block k_lzf_walk takes: no raw block, no block checksum
// (independent or linked), at most 64 KiB in and out (the records' 16-bit
// fields)
DEV bool lzf_eligible(bool raw, bool bcs, int64_t bsz, int64_t bmax) {
    return !raw && !bcs && bsz >= 16 && bsz <= 65536 && bmax >= 256 && bmax <= 65536;
}
// the records an LZ4 block of csize bytes parses into at most (every
// sequence but the last takes >= 3 input bytes)
DEV uint32_t lzf_reserve(uint32_t csize) { return csize / 3 + 2; }
// eligible blocks base + i for the set bits i of m (lane 0), one atomic per
// 64 for the list and one for their frecs: each block's first_slab (pstate)
// holds its offset in the group, `res` records in all; a group frecs cannot
// hold stays with k_lz_walk.  Returns the blocks listed.
DEV uint64_t note_fast(const DeviceJob& j, uint32_t base, uint64_t m, uint32_t res) {
    if (!m || !j.lzf_list || !j.frecs) return 0;
    const uint64_t fb = atomicAdd((unsigned long long*)(j.counters + 42), (unsigned long long)res);
    if (fb + res > j.frec_cap) return 0;
    const uint64_t listed = m;
    uint32_t at = atomicAdd(&j.counters[45], (uint32_t)__builtin_popcountll(m));
    for (; m; m &= m - 1) {
        const uint32_t p = base + (uint32_t)__builtin_ctzll(m);
        j.lzf_list[at++] = p;
        j.pstate[p].first_slab += (uint32_t)fb;
        j.blocks[p].fast = kLzfListed;
    }
    return listed;
}

// blocks base + i for the set bits i of m (lane 0) that k_lz_walk's lane
// loop considers (every block but k_lzf_walk's and k_raw_copy's: C2 leaves
// it none, where its lanes had scanned all 277 K items)
DEV void note_lane(const DeviceJob& j, uint32_t base, uint64_t m) {
    if (!m) return;
    uint32_t at = atomicAdd(&j.counters[41], (uint32_t)__builtin_popcountll(m));
    for (; m; m &= m - 1) j.lane_list[at++] = base + (uint32_t)__builtin_ctzll(m);
}
// the blocks [0, (k & 63) + 1) of a group of 64
DEV uint64_t group_mask(uint32_t k) { return (k & 63) == 63 ? ~0ull : (1ull << ((k & 63) + 1)) - 1; }
// independent raw blocks without a block checksum base + i for the set bits
// i of m (lane 0): k_raw_copy copies them (BlockItem.fast = kLzfRaw)
DEV void note_raw(const DeviceJob& j, uint32_t base, uint64_t m) {
    if (!m) return;
    uint32_t at = atomicAdd(&j.counters[40], (uint32_t)__builtin_popcountll(m));
    for (; m; m &= m - 1) {
        const uint32_t p = base + (uint32_t)__builtin_ctzll(m);
        j.raw_list[at++] = p;
        j.blocks[p].fast = kLzfRaw;
    }
}

// a long piece (walked by a wave in k_lz_walk): lane 0 appends it
DEV void note_long(const DeviceJob& j, uint32_t idx) {
    const uint32_t at = atomicAdd(&j.counters[11], 1u);
    j.long_list[at] = idx;
    const uint32_t aw = atomicAdd(&j.counters[38], 1u);
    j.wlong_list[aw] = idx;
}

// reserve `nb` items (wave-uniform); UINT32_MAX when the list is full
DEV uint32_t reserve_blocks(const DeviceJob& j, uint32_t nb) {
    const uint32_t first = wave_fetch_add(&j.counters[4], nb);
    return ((uint64_t)first + nb <= j.block_capacity) ? first : 0xFFFFFFFFu;
}

// LZ4F frame (lz4_frame_compressor.cc:115-200 over lz4 1.9.3), complete in
// structure: returns true and fills the plan when eligible.  Independent
// blocks go to the block list; a linked frame's blocks (at most 64) are
// decoded in order by one wave of k_lz_exec (link_list)
DEV bool plan_lz4f(const DeviceJob& j, In& in, int64_t n, uint64_t src_abs, uint64_t dst_abs, uint32_t item,
                   FramePlan& fp) {
    if (n < 7) return false;
    if (in_le32(in, 0) != 0x184D2204u) return false;
    const uint32_t flg = in_byte(in, 4);
    const int64_t hsize = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
    if (n < hsize || ((flg >> 1) & 1) || ((flg >> 6) & 3) != 1) return false;
    const bool linked = !((flg >> 5) & 1);
    const uint32_t bd = in_byte(in, 5);
    const uint32_t bsid = (bd >> 4) & 7;
    if (((bd >> 7) & 1) || bsid < 4 || (bd & 15)) return false;
    if (((uni32(xxh32_small(in.src + 4, (uint32_t)(hsize - 5))) >> 8) & 0xFFu) != in_byte(in, hsize - 1)) return false;
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
    if (pos != n || nb == 0 || (linked && nb > 64)) return false;
    const uint32_t first = reserve_blocks(j, nb);
    if (first == 0xFFFFFFFFu) return false;
    pos = hsize;
    uint64_t plan = 0, lm = 0, fm = 0, rm = 0;
    uint32_t fres = 0;
    for (uint32_t k = 0; k < nb; k++) {
        const uint32_t bh = in_le32(in, pos);
        const int64_t bsz = bh & 0x7FFFFFFFu;
        const bool raw = (bh & 0x80000000u) != 0;
        if (lane() == 0) {
            BlockItem it;
            it.src = src_abs + (uint64_t)pos + 4;
            it.dst = dst_abs + plan;
            it.csize = (uint32_t)bsz;
            it.kind = (raw ? kBlkRaw : 0u) | (bcs ? kBlkChecksum : 0u) | (linked ? kBlkLinked : 0u);
            it.out = -1;
            it.cap = raw ? (uint32_t)bsz : (uint32_t)bmax;
            it.crc = it.fast = 0;
            j.blocks[first + k] = it;
            if (piece_is_long(it.kind, it.csize, it.cap)) lm |= 1ull << (k & 63);
            if (raw && !bcs && !linked && j.raw_list) rm |= 1ull << (k & 63);
            if (lzf_eligible(raw, bcs, bsz, bmax) && j.frecs) {
                fm |= 1ull << (k & 63);
                j.pstate[first + k].first_slab = fres;
                fres += lzf_reserve((uint32_t)bsz);
            }
            if ((k & 63) == 63 || k + 1 == nb) {
                const uint64_t listed = note_fast(j, first + (k & ~63u), fm, fres);
                note_longs(j, first + (k & ~63u), lm, lm & ~listed);
                note_raw(j, first + (k & ~63u), rm);
                note_lane(j, first + (k & ~63u), group_mask(k) & ~listed & ~rm);
                lm = 0;
                fm = 0;
                rm = 0;
                fres = 0;
            }
        }
        plan += raw ? (uint64_t)bsz : (uint64_t)bmax;
        pos += 4 + bsz + (bcs ? 4 : 0);
    }
    if (linked) {
        const uint32_t at = wave_fetch_add(&j.counters[7], 1u);
        if (lane() == 0) j.link_list[at] = item;
    }
    fp.mode = 1;
    fp.first = first;
    fp.nb = nb;
    fp.ccs = ccs;
    fp.ccs_val = ccs_val;
    fp.content_size = csf ? ((uint64_t)in_le32(in, 6) | ((uint64_t)in_le32(in, 10) << 32)) : 0;
    // a content-size field of 0 is "unknown" to LZ4F (frameRemainingSize is
    // never set, so the frameSize_wrong check never fires): found by the
    // round-6 mutation corpus, where the job rejected such a frame that
    // liblz4, the oracle and rpgpu_uncompress all accept
    fp.csf = csf && fp.content_size != 0;
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
        if (in_varint(in, pos, clen, ulen)) return false;
        if ((uint64_t)ulen > 22ull * (uint64_t)clen + 64) return false;
        pos += clen;
        nb++;
    }
    if (nb == 0) return false;
    const uint32_t first = reserve_blocks(j, nb);
    if (first == 0xFFFFFFFFu) return false;
    pos = 16;
    uint64_t plan = 0, lm = 0, fm = 0;
    for (uint32_t k = 0; k < nb; k++) {
        const int32_t clen = (int32_t)((in_byte(in, pos) << 24) | (in_byte(in, pos + 1) << 16) |
                                       (in_byte(in, pos + 2) << 8) | in_byte(in, pos + 3));
        pos += 4;
        uint32_t ulen = 0;
        in_varint(in, pos, clen, ulen);
        if (lane() == 0) {
            BlockItem it;
            it.src = src_abs + (uint64_t)pos;
            it.dst = dst_abs + plan;
            it.csize = (uint32_t)clen;
            it.kind = kBlkSnappy;
            it.out = -1;
            it.cap = ulen;
            it.crc = it.fast = 0;
            j.blocks[first + k] = it;
            if (piece_is_long(it.kind, it.csize, it.cap)) lm |= 1ull << (k & 63);
            if ((k & 63) == 63 || k + 1 == nb) {
                note_longs(j, first + (k & ~63u), lm, lm);
                note_lane(j, first + (k & ~63u), group_mask(k));
                lm = 0;
            }
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

// a raw (non-xerial) snappy payload: one item, decoded whole by one lane's
// walk and executed by the wave engine
DEV bool plan_snappy_whole(const DeviceJob& j, int64_t n, uint64_t src_abs, uint64_t dst_abs, uint64_t cap, FramePlan& fp) {
    if (cap > 0xFFFFFFFFull) return false;
    const uint32_t first = reserve_blocks(j, 1);
    if (first == 0xFFFFFFFFu) return false;
    if (lane() == 0) {
        BlockItem it;
        it.src = src_abs;
        it.dst = dst_abs;
        it.csize = (uint32_t)n;
        it.kind = kBlkSnappy | kBlkWhole;
        it.out = -1;
        it.cap = (uint32_t)cap;
        it.crc = it.fast = 0;
        j.blocks[first] = it;
        note_long(j, first);
        note_lane(j, first, 1ull);
    }
    fp.mode = 2;
    fp.first = first;
    fp.nb = 1;
    fp.ccs = 0;
    fp.ccs_val = 0;
    fp.csf = 0;
    fp.content_size = 0;
    return true;
}

// ---------------------------------------------------------------------------
// k_decode: one wave per compressed batch of the job (work list built by
// k_emit), wave-strided: the frame is planned into BlockItems, or queued
// whole on the sequential list.  Each item writes only its own plan.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_decode(DeviceJob j) {
    const uint32_t count = j.counters[2];
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6); item < count; item += nw) {
        const uint32_t b = j.decode_list[item];
        const rpgpu_batch_result* R = &j.batches[b];
        const uint32_t seg = uni32(R->segment);
        const uint64_t S = uni64(j.seg_off[seg]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
        const int64_t n = (int64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
        const int codec = (int)(uni32((uint32_t)(uint16_t)R->attrs) & 7u);
        const uint64_t doff = uni64(j.dcap[b]);
        const uint64_t cap = uni64(j.dcap[b + 1]) - doff;
        FramePlan fp;
        fp.mode = 0;
        fp.first = fp.nb = fp.ccs = fp.ccs_val = fp.csf = fp.xxh = fp.pad = 0;
        fp.content_size = 0;
        if (doff + cap > j.decoded_capacity) {
            fp.mode = 3;  // no room: DECODE_OVERFLOW
        } else {
            In in;
            in_init(in, j.data + S, n);
            bool planned = false;
            if (n > 0 && j.block_capacity) {
                if (codec == RPGPU_CODEC_LZ4) {
                    planned = plan_lz4f(j, in, n, S, doff, item, fp);
                } else if (codec == RPGPU_CODEC_SNAPPY) {
                    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
                    bool java = n >= 16;
                    for (int i = 0; i < 8 && java; i++) java = in_byte(in, i) == magic[i];
                    planned = java ? plan_snappy_java(j, in, n, S, doff, fp) : plan_snappy_whole(j, n, S, doff, cap, fp);
                }
            }
            if (!planned) {
                fp.mode = 0;
                const uint32_t at = wave_fetch_add(&j.counters[6], 1u);
                if (lane() == 0) j.seq_list[at] = item;
            }
        }
        if (lane() == 0) j.plans[item] = fp;
    }
}

// ---------------------------------------------------------------------------
// Wave engine (k_lz_exec).  Lanes first walk up to 64 pieces in parallel
// (lz4_run / snappy_run into RecSink: kRecsPerLane SeqRecs each); then the
// wave executes the pieces in order against a 64 KiB LDS ring holding the
// last 64 KiB of output (every LZ4 offset, and every snappy offset of a
// piece up to 64 KiB, lands in it), storing whole 1 KiB chunks to the arena
// with coalesced 16-byte-per-lane stores.
//   * Records run 64 at a time, one per lane: a prefix sum places them, the
//     literals are copied lane-parallel, then the matches in rounds: in each
//     round every match whose source ends before the first unexecuted
//     match's output (all bytes there are final), plus that first match
//     itself (whose source may overlap its own output), copies at once.
//   * Records longer than kBig run alone, wave-cooperatively.
//   * Linked frames keep the ring across blocks (positions count from the
//     frame start); a batch's writes may then overwrite ring slots 64 KiB
//     back, so a match whose source lies before (batch end - 64 KiB) reads
//     it back from the arena (sc1 loads of bytes stored long before).
//   * Raw blocks are plain 16-byte-per-lane copies (through the ring in a
//     linked frame, whose later blocks may copy from them).
// ---------------------------------------------------------------------------
// The ring is small so that many waves share a CU: the execution is a chain
// of LDS and load latencies per wave, and throughput scales with the waves
// resident (16 KiB: 10 per CU; the 64 KiB ring of the first wave engine
// allowed 2).  Matches reaching further back than the ring read the arena.
#ifndef RPGPU_XRING_KIB
#define RPGPU_XRING_KIB 16
#endif
constexpr uint32_t kXRing = RPGPU_XRING_KIB * 1024u, kXM = kXRing - 1;
static_assert((kXRing & kXM) == 0 && kXRing >= 16384, "ring: a power of two >= 16 KiB");
// longer literals / matches run wave-cooperatively (a 64-record batch then
// writes at most 128 kBig bytes)
constexpr uint32_t kBig = kXRing >= 32768 ? 128 : 64;
// ring stores are deferred: unflushed output stays below kFlushLag (+ the
// 1 KiB flush granule + one batch), so most batches issue no global store
// and the loads they wait on are counted exactly (gfx9's vmcnt also counts
// stores)
constexpr uint32_t kFlushLag = kXRing >= 65536 ? (24u << 10) : kXRing / 4;

// a batch overwrites ring slots up to 128 kBig bytes behind the front, and
// its far matches read up to kBig bytes past (front - ring): both must lie
// below the flushed position; xbig's far reads need ring >= lag + 2 KiB + 64
static_assert(kFlushLag + 1024 + 128 * kBig + kBig <= kXRing, "ring too small for the flush lag and a batch");
static_assert(kXRing >= kFlushLag + 2048 + 128, "ring too small for xbig's far reads");
// Workgroup layout: kExecWaves independent waves (each claims its own work)
// share one LDS image: their rings, then the CRC tables of the streaming
// decoded-payload CRC (braid T1023..T1020 and slice T3..T0, 1 KiB each, a
// single copy) and the short-offset pattern selectors.  (One wave per
// workgroup left no room for shared tables; 9 rings + 8.5 KiB fit 160 KiB,
// as many waves per CU as the 10 one-wave workgroups that were resident.)
#ifdef RPGPU_EXEC_WAVES
constexpr uint32_t kExecWaves = RPGPU_EXEC_WAVES;  // (experiment builds)
#else
constexpr uint32_t kExecWaves = (160u * 1024u - 8704u) / kXRing;
#endif
constexpr uint32_t kXCrcOff = kExecWaves * kXRing;
constexpr uint32_t kXPatOff = kXCrcOff + 8192u;
constexpr uint32_t kXLds = kXPatOff + 512u;
static_assert(kExecWaves >= 1 && kXLds <= 160u * 1024u, "k_lz_exec LDS image exceeds 160 KiB");
constexpr uint32_t kBufFlags = 0x00020000u;    // buffer resource word 3 (raw, 32-bit data format)
constexpr int kSc1 = 16;                       // cache policy: sc1 (L2-coherent, bypasses the vector L1)

typedef const __attribute__((address_space(3))) uint32_t lds_cu32;

struct CrcState {
    uint32_t bp[4], bq[4];  // braid k's state is bp[k] ^ bq[k]
    uint4 pend;             // the pending row
    uint32_t crow;          // end of the rows taken in
    uint32_t hp;            // a row is pending
};

struct XRing {
    lds_u8* r;
    uint8_t* dst;           // arena address of position 0
    uint32_t op;            // next output position (uniform)
    uint32_t flushed;       // positions below are stored to dst
    // streaming CRC of the output (reset_size_checksum_metadata's new crc,
    // computed as flushed rows pass instead of re-reading the arena): rows
    // of 1 KiB from position 0, lane l holding bytes [16 l, +16); braid k of
    // a lane accumulates its dword k of every row (state bp ^ bq); the last
    // row seen stays pending (un-braided) until the next one arrives or the
    // output ends, where it is folded (crc_finish)
    lds_cu32* ct;           // T1023..T1020 (4 x 256), then T3..T0
    CrcState cs;
    bool linked;            // positions may pass the ring size (the ring wraps)
    bool hist;              // later pieces copy from this output (a linked frame): raw pieces go through the ring
    bool fpend;             // flush stores issued since the last full wait
    uint32_t safe;          // positions below are stored and the stores complete
    const __attribute__((address_space(3))) uint32_t* pat;  // kPat.a then kPat.b in LDS (a constant-memory
                                                          // load per short-offset match waited on HBM latency)
    __amdgpu_buffer_rsrc_t rs;  // dst window for far read-backs (linked)
#ifdef RPGPU_DSTAMPS
    uint64_t ds[10];            // per-piece phase cycles / counts (diagnostic build), see ds_flush
#endif
};

DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// one braid step of braid k with word w: the CRC of (state ^ w) over the
// word and the 1020 bytes of the other braids of the row
DEV void xbraid(CrcState& c, lds_cu32* ct, int k, uint32_t w) {
    const uint32_t v = xor3(c.bp[k], c.bq[k], w);
    const uint32_t a = ct[v & 255u], b = ct[256u + ((v >> 8) & 255u)], d = ct[512u + ((v >> 16) & 255u)];
    c.bq[k] = ct[768u + (v >> 24)];
    c.bp[k] = xor3(a, b, d);
}
// slice-by-4 word step from v = state ^ word, xored with e
DEV uint32_t xword(lds_cu32* ct, uint32_t v, uint32_t e) {
    return xor3(xor3(ct[1024u + (v & 255u)], ct[1280u + ((v >> 8) & 255u)], ct[1536u + ((v >> 16) & 255u)]),
                ct[1792u + (v >> 24)], e);
}
DEV void crc_init(CrcState& c) {
#pragma unroll
    for (int k = 0; k < 4; k++) c.bp[k] = c.bq[k] = 0u;
    c.pend = make_uint4(0u, 0u, 0u, 0u);
    c.crow = 0;
    c.hp = 0;
}
// the next 1 KiB row of the output (this lane's 16 bytes; zero past the end)
DEV void crc_row(CrcState& c, lds_cu32* ct, const uint4& v) {
#if defined(RPGPU_XABL) && RPGPU_XABL == 3
    return;  // ablation (diagnostic build only): no streaming CRC
#endif
    if (c.hp) {
        xbraid(c, ct, 0, c.pend.x);
        xbraid(c, ct, 1, c.pend.y);
        xbraid(c, ct, 2, c.pend.z);
        xbraid(c, ct, 3, c.pend.w);
    }
    c.pend = v;
    c.hp = 1;
    c.crow += 1024u;
}
DEV void crc_row(XRing& x, const uint4& v) { crc_row(x.cs, x.ct, v); }
// linear CRC (zero state, no final xor) of output [0, n), every row up to n
// taken in: the pending row folded with word steps, the lane states moved
// to the row end (x^(8 * 16 (63 - l))) and merged, then moved back over the
// zero padding of the last row (x^(-8 z))
DEV uint32_t crc_finish(const XRing& x, const Tables* __restrict__ T, uint32_t n) {
    const CrcState& c = x.cs;
    if (!c.hp) return 0u;
    uint32_t w = xword(x.ct, xor3(c.bp[0], c.bq[0], c.pend.x), c.bp[1] ^ c.bq[1]);
    w = xword(x.ct, w ^ c.pend.y, c.bp[2] ^ c.bq[2]);
    w = xword(x.ct, w ^ c.pend.z, c.bp[3] ^ c.bq[3]);
    const uint32_t s0 = xword(x.ct, w ^ c.pend.w, 0u);
    const uint32_t acc = wave_xor(multmodp(T->lane_rowend[lane()], s0));
    return multmodp(uni32(T->inv_shift[(c.crow - n) & 1023u]), uni32(acc));
}

// 16 ring bytes at position p (wrapping).  (Three aligned 8-byte reads
// funnel-shifted instead of one unaligned 16-byte read: C2 decode 26.1 ->
// 27.8 ms, the extra instructions cost more than the LDS pipe's unaligned
// stalls saved.)
DEV uint4 xld16(const lds_u8* r, uint32_t p) {
    const uint32_t sl = p & kXM;
    if (sl <= kXRing - 16) {
        uint4 v;
        __builtin_memcpy(&v, r + sl, 16);
        return v;
    }
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) w[k >> 2] |= (uint32_t)r[(p + k) & kXM] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
// the first len (1..16) bytes of v to ring position p (wrapping), exactly
DEV void xst(lds_u8* r, uint32_t p, const uint4& v, uint32_t len) {
    const uint32_t sl = p & kXM;
    if (sl <= kXRing - 16) {
        lds_u8* q = r + sl;
        if (len == 16) {
            __builtin_memcpy(q, &v, 16);
            return;
        }
        uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32), hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
        if (len & 8) { __builtin_memcpy(q, &lo, 8); q += 8; lo = hi; }
        if (len & 4) { const uint32_t t = (uint32_t)lo; __builtin_memcpy(q, &t, 4); q += 4; lo >>= 32; }
        if (len & 2) { const uint16_t t = (uint16_t)lo; __builtin_memcpy(q, &t, 2); q += 2; lo >>= 16; }
        if (len & 1) *q = (uint8_t)lo;
        return;
    }
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        if (k < len) r[(p + k) & kXM] = (uint8_t)(dw(v, k >> 2) >> (8 * (k & 3)));
}

// store ring positions [x.flushed, upto) to the arena: whole 16-byte pieces
// as one ds_read_b128 + global_store_dwordx4 per lane, edge pieces byte by
// byte.  Uniform trip count.
// Every flush but a piece's last one ends on a 1 KiB boundary, so each
// flushed row is taken into the streaming CRC whole, in order, once.
DEV void xflush(XRing& x, uint32_t upto) {
    const uint32_t f = x.flushed;
    if (f >= upto) return;
    const uint32_t l = lane();
    const uint32_t c0 = f & ~1023u;
    const uint32_t nch = (((upto + 1023u) & ~1023u) - c0) >> 10;
    for (uint32_t i = 0; i < nch; i++) {
        const uint32_t a = c0 + (i << 10) + 16u * l;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (a >= f && a + 16 <= upto) {
            v = xld16(x.r, a);
            gst16(x.dst + a, v);
        } else if (a + 16 > f && a < upto) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (uint32_t b = 0; b < 16; b++)
                if (a + b >= f && a + b < upto) {
                    const uint32_t y = x.r[(a + b) & kXM];
                    x.dst[a + b] = (uint8_t)y;
                    w[b >> 2] |= y << (8 * (b & 3));
                }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        crc_row(x, v);
    }
    x.flushed = upto;
    x.fpend = true;
}
DEV void xflush_chunks(XRing& x) { xflush(x, x.op & ~1023u); }

// inclusive prefix sum over the wave on the DPP network (no LDS round
// trips): row_shr 1/2/4/8 within each 16-lane row, then row_bcast:15 and
// row_bcast:31 carry the row totals upward
DEV uint32_t wave_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
    return v;
}

// one lane's match: ml bytes at d from d - off (every source byte final or
// this match's own earlier output)
// RPGPU_XMATCH_BATCH: 3 (default) = a source that does not overlap its
// destination read 32 bytes at a time, both reads before the stores (C2
// decode 24.4 -> 23.9 ms); 0 = 16 bytes at a time; experiment builds: 1 = a
// non-overlapping match's source loaded whole before its stores (1632 VGPR
// spills: C2 decode 26 -> 47 ms); 2 = far sources two 16-byte loads at a time
#ifndef RPGPU_XMATCH_BATCH
#define RPGPU_XMATCH_BATCH 3
#endif
DEV void xmatch(XRing& x, uint32_t d, uint32_t off, uint32_t ml, bool far) {
    const uint32_t s = d - off;
#if RPGPU_XMATCH_BATCH == 3
    // a source that does not overlap the destination (off >= ml: C2 99.96 %
    // of matches; every far one) is read 32 bytes at a time, both loads in
    // flight before the stores: one LDS (or arena) latency per 32 bytes
    // instead of one per 16 (the round's chain is these latencies)
    if (far || off >= ml) {
        for (uint32_t c = 0; c < ml; c += 32) {
            uint4 v0, v1;
            if (far) {
                const auto t0 = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + c, 0, kSc1);
                const auto t1 = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + c + 16, 0, kSc1);
                v0 = make_uint4(t0[0], t0[1], t0[2], t0[3]);
                v1 = make_uint4(t1[0], t1[1], t1[2], t1[3]);
            } else {
                v0 = xld16(x.r, s + c);
                v1 = c + 16 < ml ? xld16(x.r, s + c + 16) : v0;
            }
            xst(x.r, d + c, v0, ml - c < 16 ? ml - c : 16);
            if (c + 16 < ml) xst(x.r, d + c + 16, v1, ml - c - 16 < 16 ? ml - c - 16 : 16);
        }
        return;
    }
#endif
#if RPGPU_XMATCH_BATCH == 2
    if (far) {
        for (uint32_t c = 0; c < ml; c += 32) {
            const auto t0 = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + c, 0, kSc1);
            const auto t1 = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + c + 16, 0, kSc1);
            xst(x.r, d + c, make_uint4(t0[0], t0[1], t0[2], t0[3]), ml - c < 16 ? ml - c : 16);
            if (c + 16 < ml) xst(x.r, d + c + 16, make_uint4(t1[0], t1[1], t1[2], t1[3]), ml - c - 16 < 16 ? ml - c - 16 : 16);
        }
        return;
    }
#endif
#if RPGPU_XMATCH_BATCH == 1
    // ml <= kBig here (xbatch).  A source that does not overlap the
    // destination (every far one: off > ring - 1 KiB) is read whole before
    // anything is stored: one load latency per match instead of one per 16
    // bytes
    if (far || off >= ml) {
        uint4 t[kBig / 16];
#pragma unroll
        for (uint32_t k = 0; k < kBig / 16; k++) {
            t[k] = make_uint4(0u, 0u, 0u, 0u);
            if (16 * k < ml) {
                if (far) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + 16 * k, 0, kSc1);
                    t[k] = make_uint4(v[0], v[1], v[2], v[3]);
                } else {
                    t[k] = xld16(x.r, s + 16 * k);
                }
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kBig / 16; k++)
            if (16 * k < ml) xst(x.r, d + 16 * k, t[k], ml - 16 * k < 16 ? ml - 16 * k : 16);
        return;
    }
#endif
    if (far) {
        for (uint32_t c = 0; c < ml; c += 16) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(x.rs, s + c, 0, kSc1);
            xst(x.r, d + c, make_uint4(t[0], t[1], t[2], t[3]), ml - c < 16 ? ml - c : 16);
        }
        return;
    }
    if (off >= 16) {
        for (uint32_t c = 0; c < ml; c += 16) xst(x.r, d + c, xld16(x.r, s + c), ml - c < 16 ? ml - c : 16);
        return;
    }
    uint4 p = make_uint4(0, 0, 0, 0);
    uint32_t step = 16;
    if (off) {
        const uint4 v = xld16(x.r, s);  // bytes [s, s + off) are the pattern
        const uint4 sa = make_uint4(x.pat[4 * off], x.pat[4 * off + 1], x.pat[4 * off + 2], x.pat[4 * off + 3]);
        const uint4 sb = make_uint4(x.pat[64 + 4 * off], x.pat[64 + 4 * off + 1], x.pat[64 + 4 * off + 2],
                                    x.pat[64 + 4 * off + 3]);
        p.x = __builtin_amdgcn_perm(v.y, v.x, sa.x) | __builtin_amdgcn_perm(v.w, v.z, sb.x);
        p.y = __builtin_amdgcn_perm(v.y, v.x, sa.y) | __builtin_amdgcn_perm(v.w, v.z, sb.y);
        p.z = __builtin_amdgcn_perm(v.y, v.x, sa.z) | __builtin_amdgcn_perm(v.w, v.z, sb.z);
        p.w = __builtin_amdgcn_perm(v.y, v.x, sa.w) | __builtin_amdgcn_perm(v.w, v.z, sb.w);
        step = off * (((0x00000001112347F0ull >> (4 * off)) & 15u) + 1u);
    }
    for (uint32_t c = 0; c < ml; c += step) xst(x.r, d + c, p, ml - c < 16 ? ml - c : 16);
}

// a lane's literal bytes (up to kBig), loaded a window ahead of its batch:
// every load of a batch is then in flight before the batch starts.
// The loads are unconditional and land straight in the registers the batch
// reads (no select or copy after them: a value moved or masked right after
// its load makes the compiler wait for that load there, which drained the
// prefetch).  A chunk that would read past the job's data (the stream's
// last 16 bytes) is loaded from 16 bytes before that end instead and
// shifted into place once it has arrived (lit_fix): sh packs each chunk's
// shift, 4 bits per chunk.  Reads start at most 16 bytes before the stream
// (s.p - 16 lies inside the job's data: a payload follows its 61-byte
// header).
struct Lit {
    uint4 v[kBig / 16];
    uint32_t sh;
};
DEV Lit lit_load(const Src& s, const SeqRec& r) {
    Lit L;
    L.sh = 0;
    const int64_t top = s.rl - 16;
#pragma unroll
    for (uint32_t k = 0; k < kBig / 16; k++) {
        const bool want = r.ll > 16 * k && r.ll <= kBig;
        const int64_t q = (int64_t)r.lip + 16 * k;
        const int64_t a = want ? (q < top ? q : top) : (top < 0 ? top : 0);
        L.sh |= (uint32_t)(want ? q - a : 0) << (4 * k);
        L.v[k] = gld16(s.p + a);
    }
    return L;
}
// bytes [sh, 16) of v to [0, 16 - sh)
DEV uint4 shr16(const uint4& v, uint32_t sh) {
    const uint32_t d = sh >> 2, b = sh & 3;
    return make_uint4(__builtin_amdgcn_alignbyte(dw(v, d + 1), dw(v, d), b),
                      __builtin_amdgcn_alignbyte(dw(v, d + 2), dw(v, d + 1), b),
                      __builtin_amdgcn_alignbyte(dw(v, d + 3), dw(v, d + 2), b),
                      __builtin_amdgcn_alignbyte(dw(v, d + 4), dw(v, d + 3), b));
}
DEV void lit_fix(Lit& L) {
    if (!__ballot(L.sh != 0)) return;
#pragma unroll
    for (uint32_t k = 0; k < kBig / 16; k++) {
        const uint32_t sh = (L.sh >> (4 * k)) & 15u;
        if (sh) L.v[k] = shr16(L.v[k], sh);
    }
}

// the records of lanes [lo, hi) (none longer than kBig); lit = each lane's
// literal bytes (loaded a window ahead)
DEV void xbatch(XRing& x, const Src& s, const SeqRec& r, uint32_t lo, uint32_t hi_lane, const Lit& lit) {
    const uint32_t l = lane();
#ifdef RPGPU_DSTAMPS
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
    const bool v = l >= lo && l < hi_lane;
    const uint32_t len = v ? r.ll + r.ml : 0u;
    const uint32_t incl = wave_scan(len);
#ifdef RPGPU_DSTAMPS
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t o = x.op + incl - len;
    const uint32_t hi = x.op + rl(incl, (int)hi_lane - 1);
    if (v && r.ll) {
#pragma unroll
        for (uint32_t k = 0; k < kBig / 16; k++)
            if (r.ll > 16 * k) xst(x.r, o + 16 * k, lit.v[k], r.ll - 16 * k < 16 ? r.ll - 16 * k : 16);
    }
    const uint32_t d = o + r.ll, src = d - r.off;
    bool pend = v && r.ml > 0;
#ifdef RPGPU_DSTAMPS
    const uint64_t c2 = __builtin_amdgcn_s_memtime();
    uint32_t rounds = 0;
#endif
    // sources before (batch end - 64 KiB): their ring slots may be rewritten by this batch
#if defined(RPGPU_XABL) && RPGPU_XABL == 2
    const bool far = false;  // ablation (diagnostic build only): far sources read the ring
#else
    const bool far = x.linked && pend && hi > kXRing && src < hi - kXRing;
#endif
#if defined(RPGPU_XABL) && RPGPU_XABL == 1
    pend = false;  // ablation (diagnostic build only): no match copies
#endif
    // a far source was stored by an earlier flush: wait only while a flush
    // may still be in flight (a wait drains every earlier memory op)
#ifdef RPGPU_DSTAMPS
    const uint64_t farm = __ballot(far), mm = __ballot(pend);
    x.ds[6] += farm ? 1u : 0u;
    x.ds[7] += (uint64_t)__builtin_popcountll(farm);
    x.ds[9] += (uint64_t)__builtin_popcountll(mm);
#endif
    if (__ballot(far && src + r.ml > x.safe) && x.fpend) {
#ifdef RPGPU_DSTAMPS
        if (l == 0) atomicAdd(&g_dst[54], 1ull);
#endif
        wait_vm();
        x.fpend = false;
        x.safe = x.flushed;
    }
    for (;;) {
        const uint64_t pm = __ballot(pend);
        if (!pm) break;
#ifdef RPGPU_DSTAMPS
        rounds++;
#endif
        const int first = __builtin_ctzll(pm);
        const uint32_t f = rl(d, first);
#if defined(RPGPU_XABL) && RPGPU_XABL == 4
        const bool ready = pend;  // ablation (diagnostic build only): every match in one round, no dependencies
#else
        const bool ready = pend && (src + r.ml <= f || l == (uint32_t)first);
#endif
        if (ready) xmatch(x, d, r.off, r.ml, far);
        pend = pend && !ready;
    }
#ifdef RPGPU_DSTAMPS
    const uint64_t c3 = __builtin_amdgcn_s_memtime();
#endif
    x.op = hi;
#ifdef RPGPU_DSTAMPS
    const uint64_t c4 = __builtin_amdgcn_s_memtime();
    // accumulated per piece, added to g_dst once per piece (ds_flush): an
    // atomic per batch from every wave perturbed the kernel it measured
    x.ds[0] += c1 - c0;  // scan (waits for the batch's records / literals)
    x.ds[1] += c2 - c1;  // literals
    x.ds[2] += c3 - c2;  // rounds
    x.ds[3] += c4 - c3;  // flush
    x.ds[4] += 1u;       // batches
    x.ds[5] += rounds;
    x.ds[8] += farm ? c3 - c2 : 0u;  // rounds of batches with far lanes
#endif
}

#ifdef RPGPU_DSTAMPS
DEV void ds_flush(const XRing& x) {
    if (lane() != 0) return;
    const int slot[10] = {16, 17, 18, 19, 20, 21, 52, 53, 56, 55};
    for (int i = 0; i < 10; i++) atomicAdd(&g_dst[slot[i]], (unsigned long long)x.ds[i]);
}
#endif

// one long record, wave-cooperatively
DEV void xbig(XRing& x, const Src& s, uint32_t lip, uint32_t ll, uint32_t ml, uint32_t off) {
    const uint32_t l = lane();
    for (uint32_t c = 0; c < ll; c += 1024) {
        const uint32_t k = c + 16 * l;
        if (k < ll) xst(x.r, x.op + k, ld16(s, (int64_t)lip + k), ll - k < 16 ? ll - k : 16);
        const uint32_t e = x.op + (c + 1024 < ll ? c + 1024 : ll);
        if (e - x.flushed > kFlushLag) xflush(x, e & ~1023u);
    }
    x.op += ll;
    if (ml == 0) return;
    const uint32_t d = x.op, sp = d - off;
    if (off == 0 || off >= 64) {
        // 64 bytes per step, one per lane; a step never reads what it
        // writes (off >= 64).  Sources more than ring - 1 KiB back are read
        // from the arena (stored: the flush lags at most kFlushLag + 1 KiB),
        // as the ring may no longer hold them
        const bool far = x.linked && off > kXRing - 1024;
        for (uint32_t c = 0; c < 64 * ((ml + 63) / 64); c += 64) {
            if (far && x.fpend && sp + c + 64 > x.safe) {
                wait_vm();
                x.fpend = false;
                x.safe = x.flushed;
            }
            uint32_t v = 0;
            if (off && c + l < ml)
                v = far ? __builtin_amdgcn_raw_buffer_load_b8(x.rs, sp + c + l, 0, kSc1) : (uint32_t)x.r[(sp + c + l) & kXM];
            if (c + l < ml) x.r[(d + c + l) & kXM] = (uint8_t)v;
            const uint32_t e = d + (c + 64 < ml ? c + 64 : ml);
            if (e - x.flushed > kFlushLag) xflush(x, e & ~1023u);
        }
    } else {
        // period off: lanes k < L = off * floor(64 / off) hold the pattern
        // once; every L output bytes repeat it
        const uint32_t L = off * (64u / off);
        const uint32_t k = l < L ? l : 0u;
        const uint32_t inv = 65536u / off + 1u;  // (k * inv) >> 16 = k / off for k < 64, off < 64
        const uint32_t v = x.r[(sp + (k - off * ((k * inv) >> 16))) & kXM];
        for (uint32_t c = 0; c < ml; c += L) {
            if (l < L && c + l < ml) x.r[(d + c + l) & kXM] = (uint8_t)v;
            const uint32_t e = d + (c + L < ml ? c + L : ml);
            if (e - x.flushed > kFlushLag) xflush(x, e & ~1023u);
        }
    }
    x.op += ml;
    if (x.op - x.flushed > kFlushLag) xflush_chunks(x);
}

// Record sources of the window pipeline: load(k) reads record k (an index
// past the end reads record 0: unconditional, see Lit) and unpack() makes
// it a SeqRec once it has arrived (zero for an index past the end).
struct SeqRecs {  // k_lz_walk's 16-byte records
    const SeqRec* recs;
    typedef SeqRec Raw;
    DEV Raw load(uint32_t k, uint32_t cnt) const { return recs[k < cnt ? k : 0u]; }
    DEV SeqRec unpack(const Raw& v, bool ok) const {
        return ok ? v : SeqRec{0u, 0u, 0u, 0u};
    }
};
struct FRecs {  // k_lzf_walk's 8-byte records {lip | ll << 16, ml | off << 16}
    const uint2* recs;
    typedef uint2 Raw;
    DEV Raw load(uint32_t k, uint32_t cnt) const { return recs[k < cnt ? k : 0u]; }
    DEV SeqRec unpack(const Raw& v, bool ok) const {
        return ok ? SeqRec{v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16} : SeqRec{0u, 0u, 0u, 0u};
    }
};

// records [0, cnt) in windows of 64 (lane k = record 64 w + k): records are
// loaded two windows ahead and literal heads one window ahead, so the
// global-load latency hides behind the previous window's LDS work; a record
// longer than kBig splits its window and runs alone.  The window's deferred
// flush is issued at its top, before its prefetch loads: the waits the
// register rotation needs at the window's end then find the stores and the
// loads a window old.
#ifndef RPGPU_XSPLIT
#define RPGPU_XSPLIT 1
#endif
template <class RS>
DEV void xwindows(XRing& x, const Src& s, const RS& rs, uint32_t cnt) {
    if (cnt == 0) return;
    const uint32_t l = lane();
    typename RS::Raw q0 = rs.load(l, cnt), q1 = rs.load(64 + l, cnt);
    SeqRec r1 = rs.unpack(q1, 64 + l < cnt);
    SeqRec r0 = rs.unpack(q0, l < cnt);
    Lit lit0 = lit_load(s, r0);
    // vmcnt drains in issue order: once a batch has waited for its records
    // (loaded two windows back), every flush issued before that load is
    // complete, so far matches below that flush position need no wait
    uint32_t fh0 = x.safe, fh1 = x.safe;
    for (uint32_t b = 0; b < cnt; b += 64) {
        x.safe = fh1 > x.safe ? fh1 : x.safe;
        fh1 = fh0;
        if (x.op - x.flushed > kFlushLag) xflush_chunks(x);
        fh0 = x.flushed;  // (stores issued before this window's record loads)
        const typename RS::Raw q2 = rs.load(b + 128 + l, cnt);
        const Lit lit1 = lit_load(s, r1);
        lit_fix(lit0);
        const uint32_t nb = cnt - b < 64 ? cnt - b : 64;
        const uint64_t bigm = __ballot(l < nb && (r0.ll > kBig || r0.ml > kBig));
        if (RPGPU_XSPLIT && !bigm) {
            xbatch(x, s, r0, 0, nb, lit0);
        } else {
            uint32_t lo = 0;
            for (;;) {
                const uint64_t bm = bigm & (~0ull << lo);
                const uint32_t e = bm ? (uint32_t)__builtin_ctzll(bm) : nb;
                if (e > lo) xbatch(x, s, r0, lo, e, lit0);
                if (!bm) break;
                xbig(x, s, rl(r0.lip, (int)e), rl(r0.ll, (int)e), rl(r0.ml, (int)e), rl(r0.off, (int)e));
                lo = e + 1;
                if (lo >= nb) break;
            }
        }
        r0 = r1;
        r1 = rs.unpack(q2, b + 128 + l < cnt);
        lit0 = lit1;
    }
}
DEV void xrecords(XRing& x, const Src& s, const SeqRec* recs, uint32_t cnt) { xwindows(x, s, SeqRecs{recs}, cnt); }
DEV void frecords(XRing& x, const Src& s, const uint2* recs, uint32_t cnt) { xwindows(x, s, FRecs{recs}, cnt); }

// raw bytes straight from the stream to the arena (an independent raw
// block): 16 bytes per lane, U KiB per step (U loads in flight per lane)
// (the rows also feed the streaming CRC)
template <int U>
DEV CrcState raw_copy_rows(uint8_t* dst, const uint8_t* src, int64_t rl, uint32_t len, lds_cu32* ct, CrcState c) {
    const Src s{src, (int64_t)len, rl};
    const uint32_t l = lane();
    uint32_t k = 0;
    for (; k + 1024 * U <= len; k += 1024 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ld16(s, (int64_t)k + 1024 * u + 16 * l);
#pragma unroll
        for (int u = 0; u < U; u++) gst16(dst + k + 1024 * u + 16 * l, v[u]);
#pragma unroll
        for (int u = 0; u < U; u++) crc_row(c, ct, v[u]);
    }
    for (; k < len; k += 1024) {
        const uint32_t q = k + 16 * l;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q + 16 <= len) {
            v = ld16(s, q);
            gst16(dst + q, v);
        } else if (q < len) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (uint32_t b = q; b < len; b++) {
                const uint32_t y = src[b];
                dst[b] = (uint8_t)y;
                w[(b - q) >> 2] |= y << (8 * ((b - q) & 3));
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        crc_row(c, ct, v);
    }
    return c;
}
// k_lz_exec's copy (raw blocks of linked frames' neighbours, checksummed
// ones).  Not inlined: inlined into k_lz_exec, its unrolled rows of CRC
// table loads pushed the kernel past the 168 VGPRs its 9-wave workgroups
// allow; a call per raw piece is cheap.
__device__ __noinline__ CrcState raw_copy(uint8_t* dst, const uint8_t* src, int64_t rl, uint32_t len, lds_cu32* ct,
                                          CrcState c) {
    return raw_copy_rows<4>(dst, src, rl, len, ct, c);
}
DEV void xcopy_raw(XRing& x, const Src& s, uint32_t len) { x.cs = raw_copy(x.dst, s.p, s.rl, len, x.ct, x.cs); }

// A piece's stream and walk state (one lane)
struct Piece {
    Src s;
    PState ps;
    uint32_t kind, cap;
};

// a piece's stream, block checksum and walk start (per lane; wave: the whole
// wave works on this one piece and hashes the checksum together)
DEV void piece_begin(Piece& pc, const DeviceJob& j, const BlockItem& it, lds_u8* xbuf = nullptr) {
    const uint64_t n = it.csize;
    pc.s = Src{j.data + it.src, (int64_t)n, (int64_t)(j.data_len - it.src)};
    pc.kind = it.kind;
    pc.cap = it.cap;
    pc.ps.ip = pc.ps.op = pc.ps.need = 0;
    pc.ps.ulen = 0;
    pc.ps.safe = 0;
    pc.ps.st = 0;
    if ((it.kind & kBlkChecksum) &&
        le32(Src{pc.s.p, (int64_t)n + 4, pc.s.rl}, (int64_t)n) != (xbuf ? xxh32_wave(pc.s.p, n, 0, xbuf) : xxh32_lane(pc.s.p, n, 0))) {
        pc.ps.st = -1;  // block checksum mismatch (LZ4F_decompress, checked before the block decodes)
        return;
    }
    if (it.kind & kBlkRaw) {
        pc.ps.st = 1;
        pc.ps.op = (int32_t)n;
        return;
    }
    if (it.kind & kBlkSnappy) snappy_begin(pc.ps, pc.s, (it.kind & kBlkWhole) != 0);
    else lz4_begin(pc.ps, pc.s, (int32_t)it.cap);
}

template <class Sink>
DEV void piece_run(const Src& s, uint32_t kind, uint32_t cap, PState& ps, Sink& sink, int32_t stop_ip = INT32_MAX) {
    if (kind & kBlkSnappy) snappy_run(s, ps, sink, stop_ip);
    else lz4_run(s, (int32_t)cap, 65536, ps, sink, stop_ip);  // H = 64 KiB: the history check is `need` (see lz4_run)
}

// records into slabs of the pool; false (suspend) once the pool is exhausted
// records into slabs of the pool; false (suspend) once the pool is
// exhausted.  Records are stored four at a time (64 contiguous bytes, one
// store burst per line half): a lane storing one 16-byte record per
// sequence left the L2 with partial lines of some 300 M scattered records.
struct SlabSink {
    SeqRec* pool;
    uint32_t* slab_next;
    uint32_t* cursor;
    uint32_t pool_slabs;
    uint32_t slab, pos, n;
    uint32_t cut;      // the pool ran out: the walk was suspended for good
    uint4 r0, r1, r2;  // records (pos & ~3) .. pos - 1, not stored yet
    DEV bool seq(const uint4&, int32_t, int32_t lip, int32_t llen, int32_t, uint32_t off, int32_t ml) {
        const uint4 r = make_uint4((uint32_t)lip, (uint32_t)llen, (uint32_t)ml, off);
        const uint32_t k = pos & 3;
        if (k == 3) {
            uint4* q = (uint4*)(pool + (size_t)slab * kSlabRecs + pos - 3);
            q[0] = r0;
            q[1] = r1;
            q[2] = r2;
            q[3] = r;
        } else if (k == 0) {
            r0 = r;
        } else if (k == 1) {
            r1 = r;
        } else {
            r2 = r;
        }
        n++;
        if (++pos < kSlabRecs) return true;
        const uint32_t ns = atomicAdd(cursor, 1u);
        if (ns >= pool_slabs) {
            cut = 1;
            return false;
        }
        slab_next[slab] = ns;
        slab = ns;
        pos = 0;
        return true;
    }
    // store the records still held (when the walk returns)
    DEV void finish() {
        const uint32_t k = pos & 3;
        uint4* q = (uint4*)(pool + (size_t)slab * kSlabRecs + (pos - k));
        if (k > 0) q[0] = r0;
        if (k > 1) q[1] = r1;
        if (k > 2) q[2] = r2;
    }
};

// ---------------------------------------------------------------------------
// k_lz_walk: every planned BlockItem (linked or not) is walked into slab
// records.  Long pieces (a raw snappy payload, an LZ4 block above 64 KiB
// compressed: one serial chain of up to ~10^5 sequences) go first, one WAVE
// each: the wave stages 4 KiB of the stream at a time in LDS (16 bytes per
// lane per load, one memory latency per window) and lane 0 walks it from
// there, where a lane walking the stream in HBM waits a memory latency per
// sequence.  Then one LANE per remaining piece, taken off counters[10]:
// block checksum, then the walk.  High occupancy: the lane walk is a chain
// of dependent loads per lane.
// ---------------------------------------------------------------------------
#ifndef RPGPU_WALK_PRIO
#define RPGPU_WALK_PRIO 0  // s_setprio of a wave walking a long piece (experiment builds)
#endif
constexpr uint32_t kWalkWin = 4096;  // staged stream bytes per wave (long pieces)


namespace {
DEV uint64_t rl64(uint64_t v, int l) {
    return (uint64_t)rl((uint32_t)v, l) | ((uint64_t)rl((uint32_t)(v >> 32), l) << 32);
}
DEV uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_up((uint32_t)(v >> 32), d, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
}  // namespace

// The walk of one long raw snappy stream by a whole wave, window-parallel:
// with the stream staged in LDS, lane l decodes the tags that WOULD start at
// ip + l and at ip + 64 + l (one 8-byte LDS read each: type, lengths, offset
// and the position of the tag after it).  The true tags among those 128 are
// found by pointer doubling in each 64-position half at once (two
// independent chains of shuffles: the second costs no latency), the first
// half's chain from ip, the second's from where the first leaves its half;
// the output positions of the chain tags are a prefix sum, which is all the
// op-dependent checks need; their records are stored by the lanes in chain
// order.  The checks are DecompressAllTags' over the stream,
// SnappyArrayWriter's limits and AppendFromSelf's offset rule, in tag order
// (the first failing tag on the chain fails the stream).  A lane walking
// the stream alone took ~1 us per tag (62 K tags: 65 ms on C5); one 64-position
// window per round ~19.5 tags per ~2.7 K cycles (the round's latency chain),
// two windows ~39.
struct SnapCand {
    uint32_t nxt, lip, t;  // next tag position (0xFFFFFFFF: none), literal position, tag type
    uint64_t out, off;     // output bytes, copy offset
    bool bad;              // cut short by the stream's end, or offset 0
};
DEV SnapCand snappy_cand(const __attribute__((address_space(3))) uint32_t* w32, int64_t w0, uint32_t p, uint32_t n) {
    SnapCand r{0xFFFFFFFFu, 0u, 0u, 0u, 0u, false};
    if (p >= n) return r;
    const uint32_t o = (uint32_t)((int64_t)p - w0);
    const uint64_t q = (((uint64_t)w32[(o >> 2) + 1] << 32) | w32[o >> 2]) >> (8 * (o & 3));
    const uint32_t c = (uint32_t)q & 0xFFu, x = (uint32_t)(q >> 8);
    r.t = c & 3;
    const uint32_t extra = r.t == 0 ? (((c >> 2) >= 60) ? (c >> 2) - 59 : 0u) : r.t == 1 ? 1u : r.t == 2 ? 2u : 4u;
    if (n - p < 1 + extra) {
        r.bad = true;
    } else if (r.t == 0) {
        uint64_t lit = (uint64_t)(c >> 2) + 1;
        if (lit >= 61) lit = (uint64_t)(extra == 4 ? x : x & ((1u << (8 * extra)) - 1u)) + 1;
        r.lip = p + 1 + extra;
        if ((uint64_t)(n - r.lip) < lit) r.bad = true;
        else {
            r.out = lit;
            r.nxt = r.lip + (uint32_t)lit;
        }
    } else {
        r.out = r.t == 1 ? 4 + ((c >> 2) & 7) : (c >> 2) + 1;
        r.off = r.t == 1 ? (((c >> 5) << 8) | (x & 0xFFu)) : r.t == 2 ? (x & 0xFFFFu) : x;
        r.nxt = p + 1 + extra;
        if (r.off == 0) r.bad = true;
    }
    return r;
}

DEV void walk_snappy_long(const DeviceJob& j, Piece& pc, SlabSink& sink, lds_u8* win) {
    typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
    const uint32_t l = lane();
    // the walk state is wave-uniform: kept in SGPRs (readfirstlane), or the
    // compiler runs the loop as a divergent VGPR loop
    const uint32_t n = uni32((uint32_t)pc.s.n);
    const uint64_t ulen = uni32(pc.ps.ulen);
    uint32_t ip = uni32((uint32_t)pc.ps.ip);
    uint64_t op = uni32((uint32_t)pc.ps.op);
    int32_t st = 0;
    uint32_t slab = sink.slab, pos = sink.pos, nrec = sink.n;
    bool cut = false;
    int64_t w0 = -1;
    lds_cu32* w32 = (lds_cu32*)win;
    const uint64_t below = (1ull << l) - 1;
#ifdef RPGPU_DSTAMPS
    uint64_t ds_it = 0, ds_hops = 0, ds_c0 = 0, ds_c1 = 0, ds_c2 = 0;
#endif
    while (st == 0 && !cut) {
        ip = uni32(ip);
        op = uni64(op);
#ifdef RPGPU_DSTAMPS
        const uint64_t q0 = __builtin_amdgcn_s_memtime();
        ds_it++;
#endif
        if (ip >= n) {
            st = op == ulen ? 1 : -1;
            break;
        }
        if (w0 < 0 || (int64_t)ip + 136 > w0 + kWalkWin) {
            w0 = (int64_t)ip & ~15ll;
#pragma unroll
            for (uint32_t k = 0; k < kWalkWin / 1024; k++) {
                const uint4 v = ld16(pc.s, w0 + 1024 * k + 16 * l);
                __builtin_memcpy(win + 1024 * k + 16 * l, &v, 16);
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        // the tags that would start at ip + l (a) and ip + 64 + l (b)
        const uint32_t ib = ip + 64;
        const SnapCand a = snappy_cand(w32, w0, ip + l, n);
        const SnapCand b = snappy_cand(w32, w0, ib + l, n);
#ifdef RPGPU_DSTAMPS
        const uint64_t q1 = __builtin_amdgcn_s_memtime();
#endif
        // the true tags of each half by pointer doubling: J = the lane of the
        // next tag in the half (itself where the chain leaves the half, ends
        // the stream or meets a bad tag), F = the lanes visited from here;
        // after six rounds (F, J) <- (F | F[J], J[J]) lane e's F is the chain
        // from e.  (A scalar hop per tag, readlane -> SALU -> branch, cost
        // ~130 cycles each.)
        uint32_t Ja = l, Jb = l;
        if (!a.bad && a.nxt != 0xFFFFFFFFu && a.nxt - ip < 64u && a.nxt < n) Ja = a.nxt - ip;
        if (!b.bad && b.nxt != 0xFFFFFFFFu && b.nxt - ib < 64u && b.nxt < n) Jb = b.nxt - ib;
        uint64_t Fa = 1ull << l, Fb = 1ull << l;
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const uint32_t Jao = (uint32_t)__shfl((int)Ja, (int)Ja, 64);
            const uint32_t Jbo = (uint32_t)__shfl((int)Jb, (int)Jb, 64);
            const uint32_t alo = (uint32_t)__shfl((int)(uint32_t)Fa, (int)Ja, 64);
            const uint32_t blo = (uint32_t)__shfl((int)(uint32_t)Fb, (int)Jb, 64);
            const uint32_t ahi = (uint32_t)__shfl((int)(uint32_t)(Fa >> 32), (int)Ja, 64);
            const uint32_t bhi = (uint32_t)__shfl((int)(uint32_t)(Fb >> 32), (int)Jb, 64);
            Fa |= (uint64_t)alo | ((uint64_t)ahi << 32);
            Fb |= (uint64_t)blo | ((uint64_t)bhi << 32);
            Ja = Jao;
            Jb = Jbo;
        }
        const uint64_t ca = (uint64_t)uni32(rl((uint32_t)Fa, 0)) | ((uint64_t)uni32(rl((uint32_t)(Fa >> 32), 0)) << 32);
        // where the first half's chain leaves it: the second half's entry
        const uint32_t qa = uni32(rl(a.nxt, 63 - __builtin_clzll(ca)));
        const uint32_t e = qa - ib;  // (a good chain tag's successor is >= ib or the stream's end)
        uint64_t cb = 0;
        if (qa < n && e < 64u)
            cb = (uint64_t)uni32(rl((uint32_t)Fb, (int)e)) | ((uint64_t)uni32(rl((uint32_t)(Fb >> 32), (int)e)) << 32);
        const uint32_t qn = cb ? uni32(rl(b.nxt, 63 - __builtin_clzll(cb))) : qa;
#ifdef RPGPU_DSTAMPS
        ds_hops += (uint64_t)(__builtin_popcountll(ca) + __builtin_popcountll(cb));
        const uint64_t q2 = __builtin_amdgcn_s_memtime();
        ds_c0 += q1 - q0;
        ds_c1 += q2 - q1;
#endif
        const bool ona = (ca >> l) & 1, onb = (cb >> l) & 1;
        // output before each chain tag: 32-bit DPP scans (a good chain tag's
        // output is a literal inside the stream or a copy of <= 64 bytes)
        const uint32_t oa = ona ? (uint32_t)a.out : 0u, ob = onb ? (uint32_t)b.out : 0u;
        const uint32_t ia = wave_scan(oa), ibn = wave_scan(ob);
        const uint32_t ta = uni32(rl(ia, 63));
        const uint64_t opa = op + (ia - oa), opb = op + ta + (ibn - ob);
        const bool fail = (ona && (a.bad || (int64_t)(ulen - opa) < (int64_t)a.out || (a.t != 0 && opa < a.off))) ||
                          (onb && (b.bad || (int64_t)(ulen - opb) < (int64_t)b.out || (b.t != 0 && opb < b.off)));
        if (__ballot(fail)) {
            st = -1;
            break;
        }
        // records in chain order: the first half's, then the second's
        const uint32_t na = (uint32_t)__builtin_popcountll(ca);
        const uint32_t cnt = na + (uint32_t)__builtin_popcountll(cb);
        const uint32_t room = kSlabRecs - pos;
        uint32_t ns = 0xFFFFFFFFu, emit = cnt;
        if (cnt >= room) {
            ns = wave_fetch_add(&j.counters[9], 1u);
            if (ns >= j.pool_slabs) {
                emit = room;  // the pool ran out: the walk stops after the slab's last record
                cut = true;
            } else if (l == 0) {
                j.slab_next[slab] = ns;
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const bool on = h ? onb : ona;
            const SnapCand& c = h ? b : a;
            const uint32_t rank = h ? na + (uint32_t)__builtin_popcountll(cb & below)
                                    : (uint32_t)__builtin_popcountll(ca & below);
            if (on && rank < emit) {
                const SeqRec r = c.t == 0 ? SeqRec{c.lip, (uint32_t)c.out, 0u, 0u} : SeqRec{0u, 0u, (uint32_t)c.out, (uint32_t)c.off};
                if (rank < room) j.pool[(size_t)slab * kSlabRecs + pos + rank] = r;
                else j.pool[(size_t)ns * kSlabRecs + (rank - room)] = r;
            }
        }
        nrec += emit;
        if (cnt >= room && !cut) {
            slab = ns;
            pos = cnt - room;
        } else {
            pos += emit;
        }
        if (emit < cnt) {
            // resume after the last stored record (the emit-th chain tag)
            const bool inb = emit > na;
            uint64_t m = inb ? cb : ca;
            const uint32_t k = inb ? emit - na : emit;
            uint32_t kk = 0;
            for (uint32_t x = 0; x < k; x++) {
                kk = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
            }
            ip = inb ? rl(b.nxt, (int)kk) : rl(a.nxt, (int)kk);
            op = inb ? op + ta + rl(ibn, (int)kk) : op + rl(ia, (int)kk);
            break;
        }
        op += ta + rl(ibn, 63);
        ip = qn;
#ifdef RPGPU_DSTAMPS
        ds_c2 += __builtin_amdgcn_s_memtime() - q2;
#endif
    }
#ifdef RPGPU_DSTAMPS
    if (lane() == 0) {
        atomicAdd(&g_dst[40], ds_it);
        atomicAdd(&g_dst[41], ds_hops);
        atomicAdd(&g_dst[42], ds_c0);
        atomicAdd(&g_dst[43], ds_c1);
        atomicAdd(&g_dst[44], ds_c2);
    }
#endif
    pc.ps.ip = (int32_t)ip;
    pc.ps.op = (int32_t)(uint32_t)op;
    pc.ps.st = st;
    sink.slab = slab;
    sink.pos = pos;
    sink.n = nrec;
    sink.cut = cut;
}

// a stream byte for a lane of the window-parallel walks: from the staged
// window when inside it, else from memory (0 past the job's data)
DEV uint32_t wbyte(const Src& s, const lds_u8* win, int64_t w0, int64_t q) {
    if (q >= w0 && q < w0 + (int64_t)kWalkWin) return win[q - w0];
    return (q >= 0 && q < s.rl) ? (uint32_t)s.p[q] : 0u;
}

// the stored records [pos & ~3, pos) back into the sink's registers (the
// window-parallel walks store records directly; the serial walk then goes on
// through the sink's four-record buffer)
DEV void sink_resync(SlabSink& sink) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t k = sink.pos & 3;
    const uint4* q = (const uint4*)(sink.pool + (size_t)sink.slab * kSlabRecs + (sink.pos - k));
    if (k > 0) sink.r0 = q[0];
    if (k > 1) sink.r1 = q[1];
    if (k > 2) sink.r2 = q[2];
}

// Window-parallel LZ4 block walk (the wave's own piece): lane l decodes the
// sequence that would start at ip + l the way LZ4_decompress_generic's fast
// loop does (token, literal length, offset, match length, next token); the
// true sequences are found by readlane hops from ip, their output positions
// by a prefix sum.  Only sequences the fast loop would take without
// leaving it are handled here (every condition that sends the reference to
// its safe loop, or could fail the block, hands the rest of the block to
// the serial walk: the block's last ~64 output bytes and ~32 input bytes,
// and anything unusual).  The history check is the walk's `need` bound, as
// in lz4_run.  Advances pc.ps and the sink.
DEV void walk_lz4_wave(const DeviceJob& j, Piece& pc, SlabSink& sink, lds_u8* win) {
    typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
    const uint32_t l = lane();
    const int64_t iend = (int64_t)uni64((uint64_t)pc.s.n), oend = (int64_t)uni32(pc.cap);
    if (pc.ps.st != 0 || pc.ps.safe) return;
    // wave-uniform walk state in SGPRs (see walk_snappy_long)
    int64_t ip = (int32_t)uni32((uint32_t)pc.ps.ip), op = (int32_t)uni32((uint32_t)pc.ps.op);
    int32_t need = pc.ps.need;
    uint32_t slab = sink.slab, pos = sink.pos, nrec = sink.n;
    bool cut = false;
    int64_t w0 = -1;
    lds_cu32* w32 = (lds_cu32*)win;
    for (;;) {
        ip = (int64_t)uni64((uint64_t)ip);
        op = (int64_t)uni64((uint64_t)op);
        if (w0 < 0 || ip + 72 > w0 + kWalkWin) {
            w0 = ip & ~15ll;
#pragma unroll
            for (uint32_t k = 0; k < kWalkWin / 1024; k++) {
                const uint4 v = ld16(pc.s, w0 + 1024 * k + 16 * l);
                __builtin_memcpy(win + 1024 * k + 16 * l, &v, 16);
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        // the sequence that would start at ip + l (fast-loop rules)
        const int64_t p = ip + l;
        bool ok = p < iend;
        int64_t ll = 0, ml = 0, lip = 0, nxt = -1;
        uint32_t off = 0;
        if (ok) {
            const uint32_t o = (uint32_t)(p - w0);
            const uint32_t token = (w32[o >> 2] >> (8 * (o & 3))) & 0xFFu;
            int64_t q = p + 1;
            ll = token >> 4;
            if (ll == 15) {
                if (q >= iend - 15) ok = false;  // initial error / near the end: serial
                uint32_t b = 255;
                while (ok && b == 255) {
                    b = wbyte(pc.s, win, w0, q);
                    q++;
                    ll += b;
                    if (q >= iend - 15) ok = false;
                }
                if (ok && q + ll > iend - 32) ok = false;  // the fast loop would go safe
            } else if (q > iend - 17) {
                ok = false;
            }
            if (ok) {
                lip = q;
                q += ll;
                off = wbyte(pc.s, win, w0, q) | (wbyte(pc.s, win, w0, q + 1) << 8);
                q += 2;
                ml = token & 15;
                if (ml == 15) {
                    uint32_t b = 255;
                    while (ok && b == 255) {
                        b = wbyte(pc.s, win, w0, q);
                        q++;
                        ml += b;
                        if (q >= iend - kLastLiterals + 1) ok = false;
                    }
                }
                ml += kMinMatch;
                nxt = q;
            }
        }
        // the true sequences among the 64, up to the first one not handled here
        // chain by pointer doubling (walk_snappy_long): J = the lane of the
        // next sequence, itself where the chain leaves the window or at a
        // sequence not handled here; the chain ends before the first such one
        const uint64_t okm = __ballot(ok);
        uint32_t J = l;
        if (ok && nxt - ip < 64) J = (uint32_t)(nxt - ip);
        uint64_t F = 1ull << l;
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const uint32_t Jo = (uint32_t)__shfl((int)J, (int)J, 64);
            const uint32_t flo = (uint32_t)__shfl((int)(uint32_t)F, (int)J, 64);
            const uint32_t fhi = (uint32_t)__shfl((int)(uint32_t)(F >> 32), (int)J, 64);
            F |= (uint64_t)flo | ((uint64_t)fhi << 32);
            J = Jo;
        }
        uint64_t chain = (uint64_t)uni32(rl((uint32_t)F, 0)) | ((uint64_t)uni32(rl((uint32_t)(F >> 32), 0)) << 32);
        const uint64_t nok = chain & ~okm;
        bool stop = false;
        if (nok) {
            chain &= (1ull << __builtin_ctzll(nok)) - 1;
            stop = true;
        }
        // output positions (32-bit DPP scan: chain sequences lie inside the
        // block); the op-dependent fast-loop conditions
        const bool on = (chain >> l) & 1;
        const uint32_t len = on ? (uint32_t)(ll + ml) : 0u;
        const uint32_t incl = wave_scan(len);
        const int64_t opt = op + (int64_t)(incl - len);  // output at the sequence start
        const bool go_safe = on && ((ll >= 15 && opt + ll > oend - 32) || opt + ll + ml >= oend - kFastSafeDistance);
        const uint64_t gm = __ballot(go_safe);
        if (gm) {
            chain &= (1ull << __builtin_ctzll(gm)) - 1;  // the sequences before it
            stop = true;
        }
        const bool mine = (chain >> l) & 1;
        // records in chain order (the sink's slab rules)
        const uint32_t cnt = (uint32_t)__builtin_popcountll(chain);
        const uint32_t rank = (uint32_t)__builtin_popcountll(chain & ((1ull << l) - 1));
        const uint32_t room = kSlabRecs - pos;
        uint32_t ns = 0xFFFFFFFFu, emit = cnt;
        if (cnt && cnt >= room) {
            ns = wave_fetch_add(&j.counters[9], 1u);
            if (ns >= j.pool_slabs) {
                emit = room;
                cut = true;
            } else if (l == 0) {
                j.slab_next[slab] = ns;
            }
        }
        int32_t d = INT32_MIN;
        if (mine && rank < emit) {
            const SeqRec r{(uint32_t)lip, (uint32_t)ll, (uint32_t)ml, off};
            if (rank < room) j.pool[(size_t)slab * kSlabRecs + pos + rank] = r;
            else j.pool[(size_t)ns * kSlabRecs + (rank - room)] = r;
            d = (int32_t)off - (int32_t)(opt + ll);  // offset - match position
        }
        for (int m = 32; m > 0; m >>= 1) {
            const int32_t v = __shfl_xor(d, m, 64);
            d = v > d ? v : d;
        }
        need = d > need ? d : need;
        nrec += emit;
        if (cnt && cnt >= room && !cut) {
            slab = ns;
            pos = cnt - room;
        } else {
            pos += emit;
        }
        if (emit == 0) break;  // nothing handled here: the serial walk takes over at ip
        // state after the last stored sequence
        uint64_t m2 = chain;
        uint32_t kk = 0;
        for (uint32_t e = 0; e < emit; e++) {
            kk = (uint32_t)__builtin_ctzll(m2);
            m2 &= m2 - 1;
        }
        op += (int64_t)rl(incl, (int)kk);
        ip = (int64_t)rl64((uint64_t)nxt, (int)kk);
        if (stop || cut || emit < cnt) break;
    }
    pc.ps.ip = (int32_t)ip;
    pc.ps.op = (int32_t)op;
    pc.ps.need = need;
    sink.slab = slab;
    sink.pos = pos;
    sink.n = nrec;
    sink.cut = cut;
    sink_resync(sink);
}

DEV void walk_long(const DeviceJob& j, uint32_t p, lds_u8* win) {
    const uint32_t l = lane();
#ifdef RPGPU_DSTAMPS
    const uint64_t t0 = wall_clock64();
#endif
    BlockItem it;
    it.src = uni64(j.blocks[p].src);
    it.dst = 0;
    it.csize = uni32(j.blocks[p].csize);
    it.kind = uni32(j.blocks[p].kind);
    it.out = -1;
    it.cap = uni32(j.blocks[p].cap);
    it.crc = it.fast = 0;
    Piece pc;
    piece_begin(pc, j, it, win);  // (the window buffer hashes the block checksum first)
    PieceState out;
    out.nrec = 0;
    out.first_slab = 0xFFFFFFFFu;
    if (pc.ps.st == 0) {
        const uint32_t fs = wave_fetch_add(&j.counters[9], 1u);
        if (fs < j.pool_slabs) {
            out.first_slab = fs;
            SlabSink sink{j.pool, j.slab_next, &j.counters[9], j.pool_slabs, fs, 0, 0, 0, {}, {}, {}};
            const int64_t n = pc.s.n;
            const bool lanes_store = (pc.kind & kBlkSnappy) != 0;  // records already stored by the lanes
            if (lanes_store) walk_snappy_long(j, pc, sink, win);
            else if (!sink.cut && (walk_lz4_wave(j, pc, sink, win), !sink.cut)) for (;;) {
                // stage [w0, w0 + 4 KiB) of the stream (w0 16-aligned below ip)
                const int64_t w0 = (int64_t)pc.ps.ip & ~15ll;
#pragma unroll
                for (uint32_t k = 0; k < kWalkWin / 1024; k++) {
                    const int64_t at = w0 + 1024 * k + 16 * l;
                    const uint4 v = ld16(pc.s, at);
                    __builtin_memcpy(win + 1024 * k + 16 * l, &v, 16);
                }
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                Src ws = pc.s;
                ws.win = win;
                ws.wlo = w0;
                ws.whi = w0 + kWalkWin;
                // suspend before a sequence within 32 bytes of the window end
                const int32_t stop = w0 + kWalkWin < n ? (int32_t)(w0 + kWalkWin - 32) : INT32_MAX;
                if (l == 0) piece_run(ws, pc.kind, pc.cap, pc.ps, sink, stop);
                // lane 0's walk state to every lane
                pc.ps.ip = (int32_t)rl((uint32_t)pc.ps.ip, 0);
                pc.ps.op = (int32_t)rl((uint32_t)pc.ps.op, 0);
                pc.ps.need = (int32_t)rl((uint32_t)pc.ps.need, 0);
                pc.ps.st = (int32_t)rl((uint32_t)pc.ps.st, 0);
                pc.ps.safe = rl(pc.ps.safe, 0);
                sink.slab = rl(sink.slab, 0);
                sink.pos = rl(sink.pos, 0);
                sink.n = rl(sink.n, 0);
                sink.cut = rl(sink.cut, 0);
                if (pc.ps.st != 0 || sink.cut) break;
            }
            if (l == 0 && !lanes_store) sink.finish();
            out.nrec = sink.n;
        }
    }
    if (l == 0) {
        out.ip = pc.ps.ip;
        out.op = pc.ps.op;
        out.need = pc.ps.need;
        out.st = pc.ps.st;
        out.ulen = pc.ps.ulen;
        out.safe = pc.ps.safe;
        j.pstate[p] = out;
#ifdef RPGPU_DSTAMPS
        const uint64_t dt = wall_clock64() - t0;
        atomicAdd(&g_dst[24], dt);
        atomicAdd(&g_dst[25], 1ull);
        if (dt > atomicMax(&g_dst[26], dt)) { g_dst[32] = out.nrec; g_dst[33] = it.csize; }
#endif
    }
}

// a piece's walk result to the job (one lane)
DEV void put_pstate(const DeviceJob& j, uint32_t p, const PState& ps, uint32_t nrec, uint32_t first_slab) {
    PieceState out;
    out.ip = ps.ip;
    out.op = ps.op;
    out.need = ps.need;
    out.st = ps.st;
    out.ulen = ps.ulen;
    out.safe = ps.safe;
    out.nrec = nrec;
    out.first_slab = first_slab;
    j.pstate[p] = out;
}

// Lane walk in rounds.  Every round, each lane with a piece stages the
// kLaneWin stream bytes at its parse position in its LDS slot (16-byte
// loads issued by all lanes together: one memory latency per round for the
// whole wave), then walks as many sequences as start within the first
// kLaneWin - 16 of them.  A lane walking straight from HBM made the whole
// wave wait a memory latency at nearly every sequence (some lane always
// needed a new window), ~4 us per sequence on C2's JSON blocks.  Window
// size measured (C2 / C5 decode ms): 64 B 47.7 / 45.6, 192 B 44.4 / 43.9,
// 256 B 43.4 / 40.4, 512 B 46.6 / 35.8 (fewer resident waves).
#ifndef RPGPU_LANE_WIN
#define RPGPU_LANE_WIN 256
#endif
constexpr uint32_t kLaneWin = RPGPU_LANE_WIN, kLaneSlot = kLaneWin + 16;  // + the spare bytes ld16's window reads need

__global__ __launch_bounds__(256) void k_lz_walk(DeviceJob j) {
    constexpr uint32_t kWaveLds = 64 * kLaneSlot > kWalkWin + 16 ? 64 * kLaneSlot : kWalkWin + 16;
    __shared__ __attribute__((aligned(16))) uint8_t wwin[4][kWaveLds];
    const uint32_t reserved = j.counters[4];
    const uint32_t nblk = reserved < j.block_capacity ? reserved : j.block_capacity;
    const uint32_t nlong = j.counters[38];
    const uint32_t nlane = j.counters[41] < j.block_capacity ? j.counters[41] : j.block_capacity;
    // few pieces: fewer than 512 per CU (the grid is 16 workgroups per CU, 2
    // resident: 512 lanes)
    const bool few = nblk < gridDim.x * 32u;
    lds_u8* wl = (lds_u8*)wwin[threadIdx.x >> 6];
    for (;;) {
        const uint32_t k = wave_fetch_add(&j.counters[39], 1u);
        if (k >= nlong) break;
        const uint32_t p = uni32(j.wlong_list[k]);
        if (uni32(j.blocks[p].fast) != kLzfNone) continue;  // the fast path has it
        if (!piece_wave_walked(uni32(j.blocks[p].kind), uni32(j.blocks[p].csize), uni32(j.blocks[p].cap), few))
            continue;  // a dense piece: the lane walk takes it
#if RPGPU_WALK_PRIO
        __builtin_amdgcn_s_setprio(RPGPU_WALK_PRIO);
#endif
        walk_long(j, p, wl);
#if RPGPU_WALK_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
    }
    lds_u8* slot = wl + kLaneSlot * lane();
    bool active = false, drained = false;
    uint32_t p = 0, first_slab = 0;
    Piece pc;
    SlabSink sink{j.pool, j.slab_next, &j.counters[9], j.pool_slabs, 0, 0, 0, 0, {}, {}, {}};
    for (;;) {
        // lanes without a piece take the next ones, one claim per wave (a
        // claim per lane serialised ~277K atomics on C2: 1.5 ms); pieces that
        // end at their begin, raw ones or a failed block checksum, are
        // written at once
        for (;;) {
            const bool want = !active && !drained;
            const uint64_t wm = __ballot(want);
            if (!wm) break;
            const int lead = __builtin_ctzll(wm);
            uint32_t u0 = 0;
            if (lane() == (uint32_t)lead) u0 = atomicAdd(&j.counters[10], (uint32_t)__builtin_popcountll(wm));
            const uint32_t u = rl(u0, lead) + (uint32_t)__builtin_popcountll(wm & ((1ull << lane()) - 1));
            if (!want) continue;
            if (u >= nlane) {
                drained = true;
                continue;
            }
            p = j.lane_list[u];
            const BlockItem it = j.blocks[p];
            if (it.fast != kLzfNone) continue;                               // the fast path has it
            if (piece_wave_walked(it.kind, it.csize, it.cap, few)) continue;  // walked above
            piece_begin(pc, j, it);
            first_slab = 0xFFFFFFFFu;
            if (pc.ps.st == 0) {
                const uint32_t fs = atomicAdd(&j.counters[9], 1u);
                if (fs < j.pool_slabs) {
                    first_slab = fs;
                    sink.slab = fs;
                    sink.pos = sink.n = sink.cut = 0;
                    active = true;
                    continue;
                }
            }
            put_pstate(j, p, pc.ps, 0, first_slab);
        }
        if (!__ballot(active)) break;
        // stage the window
        const int64_t wb = (int64_t)pc.ps.ip & ~15ll;
        if (active) {
            uint4 v[kLaneWin / 16];
#pragma unroll
            for (uint32_t k = 0; k < kLaneWin / 16; k++) v[k] = ld16(pc.s, wb + 16 * k);
#pragma unroll
            for (uint32_t k = 0; k < kLaneWin / 16; k++) __builtin_memcpy(slot + 16 * k, &v[k], 16);
        }
        if (active) {
            Src ws = pc.s;
            ws.win = slot;
            ws.wlo = wb;
            ws.whi = wb + kLaneWin;
            const int32_t stop = wb + kLaneWin < pc.s.n ? (int32_t)(wb + kLaneWin - 16) : INT32_MAX;
            piece_run(ws, pc.kind, pc.cap, pc.ps, sink, stop);
            if (pc.ps.st != 0 || sink.cut) {
                sink.finish();
                put_pstate(j, p, pc.ps, sink.n, first_slab);
                active = false;
            }
        }
    }
}

// execute piece p at x.op (its walk stored by k_lz_walk); returns its decoded
// length or -1.  `hist` = output bytes before it that its matches may reach.
// A walk the pool cut short continues here, on lane 0, kRecsPerLane records
// at a time through the wave's own buffer.
DEV int32_t exec_piece(XRing& x, const DeviceJob& j, uint32_t p, uint32_t hist, SeqRec* buf) {
    const uint32_t l = lane();
    const BlockItem& itr = j.blocks[p];
    const uint64_t src = uni64(itr.src);
    const uint32_t csize = uni32(itr.csize), kind = uni32(itr.kind), cap = uni32(itr.cap);
    const PieceState& psr = j.pstate[p];
    const uint32_t fast = uni32(itr.fast);
    if (fast == kLzfReject) return -1;
    int32_t st = (int32_t)uni32((uint32_t)psr.st);
    if (st < 0) return -1;
    const Src s{j.data + src, (int64_t)csize, (int64_t)(j.data_len - src)};
    if (fast == kLzfReady) {
        // walked by k_lzf_walk: its 8-byte records; a linked block's matches
        // reach at most `need` before it (checked against the real history)
        const uint32_t start = x.op;
        frecords(x, s, j.frecs + uni32(psr.first_slab), uni32(psr.nrec));
        if ((int32_t)uni32((uint32_t)psr.need) > (int32_t)hist) return -1;
        return (int32_t)(x.op - start);
    }
    if (kind & kBlkRaw) {
        if (x.hist) xbig(x, s, 0, csize, 0, 0);
        else {
            xcopy_raw(x, s, csize);
            x.op += csize;
            x.flushed = x.op;
            x.fpend = true;
        }
        return (int32_t)csize;
    }
    const uint32_t start = x.op;
    uint32_t nrec = uni32(psr.nrec), slab = uni32(psr.first_slab);
    int32_t need = (int32_t)uni32((uint32_t)psr.need);
    while (nrec) {
        const uint32_t c = nrec < kSlabRecs ? nrec : kSlabRecs;
        const uint32_t next = c == kSlabRecs ? uni32(j.slab_next[slab]) : 0u;
        xrecords(x, s, j.pool + (size_t)slab * kSlabRecs, c);
        nrec -= c;
        slab = next;
    }
    if (st == 0) {
        PState ps;
        ps.ip = (int32_t)uni32((uint32_t)psr.ip);
        ps.op = (int32_t)uni32((uint32_t)psr.op);
        ps.need = need;
        ps.st = 0;
        ps.ulen = uni32(psr.ulen);
        ps.safe = uni32(psr.safe);
        for (;;) {
            uint32_t n = 0;
            if (l == 0) {
                RecSink sink{buf, 0, kRecsPerLane};
                piece_run(s, kind, cap, ps, sink);
                n = sink.n;
            }
            wait_vm();  // lane 0's records, stored through this CU's L1, are then seen by every lane
            n = rl(n, 0);
            st = (int32_t)rl((uint32_t)ps.st, 0);
            xrecords(x, s, buf, n);
            if (st != 0) break;
        }
        if (st < 0) return -1;
        need = (int32_t)rl((uint32_t)ps.need, 0);
    }
    // history check of the walk (run with H = 64 KiB)
    if (need > (int32_t)hist) return -1;
    return (int32_t)(x.op - start);
}

DEV void xring_init(XRing& x, const DeviceJob& j, lds_u8* ring, uint64_t dst, bool linked, bool hist,
                    const __attribute__((address_space(3))) uint32_t* pat, lds_cu32* ct) {
    x.r = ring;
    x.pat = pat;
    x.ct = ct;
    crc_init(x.cs);
    x.dst = j.decoded + dst;
    x.op = 0;
    x.flushed = 0;
    x.linked = linked;
    x.hist = hist;
    x.fpend = false;
    x.safe = 0;
    const uint64_t room = j.decoded_capacity - dst;
    x.rs = __builtin_amdgcn_make_buffer_rsrc(x.dst, 0, (int)(room < 0x7FFFFFFFull ? room : 0x7FFFFFFFull), kBufFlags);
#ifdef RPGPU_DSTAMPS
    for (int i = 0; i < 10; i++) x.ds[i] = 0;
#endif
}

// the blocks of one linked LZ4F frame, in order, one position space
DEV void exec_linked(const DeviceJob& j, lds_u8* ring, SeqRec* buf, uint32_t item,
                     const __attribute__((address_space(3))) uint32_t* pat, lds_cu32* ct) {
    const uint32_t first = uni32(j.plans[item].first), nb = uni32(j.plans[item].nb);
    const uint64_t fdst = uni64(j.dcap[uni32(j.decode_list[item])]);
    XRing x;
    xring_init(x, j, ring, fdst, true, true, pat, ct);
#ifdef RPGPU_DSTAMPS
    const uint64_t t1 = wall_clock64();
#endif
    bool ok = true;
    for (uint32_t k = 0; k < nb; k++) {
        const uint32_t at = x.op;
        const int32_t dd = ok ? exec_piece(x, j, first + k, at, buf) : -1;
        if (dd < 0) ok = false;
        if (lane() == 0) {
            j.blocks[first + k].dst = fdst + at;
            j.blocks[first + k].out = dd;
        }
    }
    xflush(x, x.op);
    // the frame's whole output, one stream (its blocks are contiguous)
    const uint32_t fcrc = ok ? crc_finish(x, j.tables, x.op) : 0u;
    if (lane() == 0) j.blocks[first].crc = fcrc;
#ifdef RPGPU_DSTAMPS
    if (lane() == 0) { atomicAdd(&g_dst[10], wall_clock64() - t1); atomicAdd(&g_dst[9], 1ull); }
    ds_flush(x);
#endif
}

// one independent piece
DEV void exec_one(const DeviceJob& j, lds_u8* ring, SeqRec* buf, uint32_t p, uint32_t kind,
                  const __attribute__((address_space(3))) uint32_t* pat, lds_cu32* ct) {
    const uint32_t fast = uni32(j.blocks[p].fast);
    if (fast == kLzfRaw) return;  // k_raw_copy did it
    if (fast == kLzfReject) {
        if (lane() == 0) j.blocks[p].out = -1;  // (k_lzf_walk wrote it; kept here for clarity)
        return;
    }
    {
        const uint64_t dst = uni64(j.blocks[p].dst);
        XRing x;
        // a piece longer than the ring wraps it: wrap-aware like a linked frame
        xring_init(x, j, ring, dst, uni32(j.blocks[p].cap) > kXRing, false, pat, ct);
#ifdef RPGPU_DSTAMPS
        const uint64_t e0 = wall_clock64();
#endif
        const int32_t dd = exec_piece(x, j, p, 0, buf);
        if (dd >= 0) xflush(x, x.op);
        const uint32_t pcrc = dd >= 0 ? crc_finish(x, j.tables, x.op) : 0u;
        if (lane() == 0) {
            j.blocks[p].out = dd;
            j.blocks[p].crc = pcrc;
        }
#ifdef RPGPU_DSTAMPS
        if (lane() == 0) {
            const int k = (kind & kBlkRaw) ? 4 : (kind & kBlkSnappy) ? 6 : 2;
            atomicAdd(&g_dst[k], wall_clock64() - e0);
            atomicAdd(&g_dst[k + 1], 1ull);
            atomicAdd(&g_dst[11], (unsigned long long)j.pstate[p].nrec);
            if (j.pstate[p].st == 0) atomicAdd(&g_dst[12], 1ull);
        }
        ds_flush(x);
#endif
    }
}

// up to 64 consecutive block items (independent pieces; linked ones and the
// long ones, run first on their own, skipped)
DEV void exec_chunk(const DeviceJob& j, lds_u8* ring, SeqRec* buf, uint32_t base, uint32_t nblk,
                    const __attribute__((address_space(3))) uint32_t* pat, lds_cu32* ct) {
    const uint32_t end = base + 64 < nblk ? base + 64 : nblk;
    for (uint32_t p = base; p < end; p++) {
        const uint32_t kind = uni32(j.blocks[p].kind);
        if ((kind & kBlkLinked) || piece_is_long(kind, uni32(j.blocks[p].csize), uni32(j.blocks[p].cap))) continue;
        exec_one(j, ring, buf, p, kind, pat, ct);
    }
}

// ---------------------------------------------------------------------------
// k_lz_exec: persistent, kExecWaves independent waves per workgroup (a
// 16 KiB LDS ring each), one workgroup per CU; units by one agent-scope
// counter (counters[8]):
// first the linked frames, then the long pieces one unit each (a 1 MiB raw
// snappy payload is ~1000 record batches: taken first, and alone, it no
// longer ends the kernel behind 63 other pieces of its chunk), then the
// block list in chunks of 64.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64 * kExecWaves) void k_lz_exec(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xlds[];
    const uint32_t wi = threadIdx.x >> 6;
    lds_u8* ring = (lds_u8*)(xlds + wi * kXRing);
    uint32_t* ct_w = (uint32_t*)(xlds + kXCrcOff);
    uint32_t* pat_w = (uint32_t*)(xlds + kXPatOff);
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) {
        ct_w[i] = j.tables->braid[i >> 8][i & 255u];               // T1023, T1022, T1021, T1020
        ct_w[1024u + i] = j.tables->hdr[3u - (i >> 8)][i & 255u];  // T3, T2, T1, T0
    }
    for (uint32_t i = threadIdx.x; i < 128u; i += blockDim.x)
        pat_w[i] = i < 64u ? (&kPat.a[0][0])[i] : (&kPat.b[0][0])[i - 64u];
    __syncthreads();
    const __attribute__((address_space(3))) uint32_t* pat = (const __attribute__((address_space(3))) uint32_t*)pat_w;
    lds_cu32* ct = (lds_cu32*)ct_w;
    SeqRec* buf = j.seqs + ((size_t)blockIdx.x * kExecWaves + wi) * kRecsPerLane;
    const uint32_t nlink = j.counters[7];
    const uint32_t reserved = j.counters[4];
    const uint32_t nblk = reserved < j.block_capacity ? reserved : j.block_capacity;
    const uint32_t nlong = j.counters[11];
    const uint32_t total = nlink + nlong + (nblk + 63) / 64;
    for (;;) {
        const uint32_t u = wave_fetch_add(&j.counters[8], 1u);
        if (u >= total) break;
        if (u < nlink) {
            exec_linked(j, ring, buf, uni32(j.link_list[u]), pat, ct);
        } else if (u < nlink + nlong) {
            const uint32_t p = uni32(j.long_list[u - nlink]);
            const uint32_t kind = uni32(j.blocks[p].kind);
            if (!(kind & kBlkLinked)) exec_one(j, ring, buf, p, kind, pat, ct);
        } else {
            exec_chunk(j, ring, buf, (u - nlink - nlong) * 64, nblk, pat, ct);
        }
    }
}

// ---------------------------------------------------------------------------
// k_raw_copy: the independent raw LZ4F blocks without a block checksum
// (note_raw; C2: 183 K of its 277 K blocks, 12 GB), copied to their arena
// slots with their streaming CRC exactly as exec_one would (raw_copy,
// crc_finish), a static stride of waves, 16 waves per CU.  It runs while
// k_lzf_walk (latency-bound, on the side stream) parses the LZ4 blocks, so
// the copy's HBM traffic hides behind the parse instead of holding k_lz_exec's
// ring waves through 16 dependent load rounds per block.
// ---------------------------------------------------------------------------
#ifndef RPGPU_RAW_THREADS
#define RPGPU_RAW_THREADS 1024
#endif
__global__ __launch_bounds__(RPGPU_RAW_THREADS) void k_raw_copy(DeviceJob j) {
    __shared__ uint32_t ct_w[2048];
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) {
        ct_w[i] = j.tables->braid[i >> 8][i & 255u];
        ct_w[1024u + i] = j.tables->hdr[3u - (i >> 8)][i & 255u];
    }
    __syncthreads();
    lds_cu32* ct = (lds_cu32*)ct_w;
    const uint32_t nraw = j.counters[40];
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t u = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < nraw; u += waves) {
        const uint32_t p = uni32(j.raw_list[u]);
        const uint64_t src = uni64(j.blocks[p].src), dst = uni64(j.blocks[p].dst);
        const uint32_t n = uni32(j.blocks[p].csize);
        XRing x;
        xring_init(x, j, nullptr, dst, false, false, nullptr, ct);
        x.cs = raw_copy_rows<8>(x.dst, j.data + src, (int64_t)(j.data_len - src), n, ct, x.cs);
        const uint32_t pcrc = crc_finish(x, j.tables, n);
        if (lane() == 0) {
            j.blocks[p].out = (int32_t)n;
            j.blocks[p].crc = pcrc;
            atomicAdd((unsigned long long*)(j.counters + 24), (unsigned long long)n);  // k_crc_compose's gate
        }
    }
}

// ---------------------------------------------------------------------------
// k_zexec: the zstd members the member pass parsed into records
// (rp_inflate.hip zstd_fast_item, inf_state kZsFast), one wave each, claimed
// in member-list order, through the same ring executor as LZ4 pieces: literals from the
// member's literal buffer, matches from the ring or, further back, from the
// slot itself (linked mode).  The decoded crc is k_validate_decoded's.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64 * kExecWaves) void k_zexec(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xlds[];
    const uint32_t wi = threadIdx.x >> 6;
    lds_u8* ring = (lds_u8*)(xlds + wi * kXRing);
    uint32_t* ct_w = (uint32_t*)(xlds + kXCrcOff);
    uint32_t* pat_w = (uint32_t*)(xlds + kXPatOff);
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) {
        ct_w[i] = j.tables->braid[i >> 8][i & 255u];
        ct_w[1024u + i] = j.tables->hdr[3u - (i >> 8)][i & 255u];
    }
    for (uint32_t i = threadIdx.x; i < 128u; i += blockDim.x)
        pat_w[i] = i < 64u ? (&kPat.a[0][0])[i] : (&kPat.b[0][0])[i - 64u];
    __syncthreads();
    const __attribute__((address_space(3))) uint32_t* pat = (const __attribute__((address_space(3))) uint32_t*)pat_w;
    lds_cu32* ct = (lds_cu32*)ct_w;
    const uint32_t count = j.counters[16];
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[21], 1u);
        if (i >= count) break;
        if (uni32(j.inf_state[i]) != kZsFast) continue;
        const uint32_t b = uni32(j.inf_list[i]);
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t dst = uni64(j.dcap[b]), cap = uni64(j.dcap[b + 1]) - dst, total = uni64(j.inf_total[i]);
        if (dst + cap > j.decoded_capacity) {
            if (lane() == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
            continue;
        }
        const uint8_t* base = j.inf_scratch + uni64(j.inf_off[i]);
        const ZsFastDesc* d = (const ZsFastDesc*)base;
        const uint64_t nlit = uni64(d->nlit), nrec = uni64(d->nrec);
        const uint8_t* lits = base + uni64(d->lit_off);
        const SeqRec* recs = (const SeqRec*)(base + uni64(d->rec_off));
        // the literal buffer has 16 spare bytes: 16-byte loads stay inside
        const Src s{lits, (int64_t)nlit, (int64_t)nlit + 16};
        XRing x;
        xring_init(x, j, ring, dst, total > kXRing, false, pat, ct);
        xrecords(x, s, recs, (uint32_t)nrec);
        xflush(x, x.op);
        if (lane() == 0) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
            R->reserved0 = 0;  // k_validate_decoded computes the decoded crc
        }
    }
}

// ---------------------------------------------------------------------------
// k_decode_blocks: the sequential frames (what the planner did not split:
// truncated or malformed frames, linked frames of more than 64 blocks,
// unplannable snappy-java streams), one per lane through the lane engine,
// taken off counters[5].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_decode_blocks(DeviceJob j) {
    const uint32_t nseq = j.counters[6];
    const int64_t data_len = (int64_t)j.data_len;
    for (;;) {
        const uint32_t item = atomicAdd(&j.counters[5], 1u);
        if (item >= nseq) break;
        const uint32_t b = j.decode_list[j.seq_list[item]];
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t src = j.seg_off[R->segment] + R->file_pos + RPGPU_HEADER_SIZE;
        const int64_t n = (int64_t)(uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE);
        const int codec = (int)((uint32_t)(uint16_t)R->attrs & 7u);
        const uint64_t dst = j.dcap[b], cap = j.dcap[b + 1] - dst;
        int64_t got = 0;
        const int rc = decode_unit(codec, Src{j.data + src, n, data_len - (int64_t)src}, Dst{j.decoded + dst, (int64_t)cap},
                                   0, 0, got);
        if (rc == 0) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)got;
        }
    }
}

// one wave per block-parallel frame: all pieces decoded, moved together
// when an earlier one came out short (ascending 1 KiB steps, each loaded
// whole before it is stored: safe for any gap), content size / checksum
// checked
// defer (round 6): the content checksum of a frame whose pieces all came out
// where the planner put them (no move) is k_content_xxh's, which runs beside
// this kernel from k_lz_exec's end; such a frame gets its verdict here as if
// it matched, and k_content_apply takes it back after the join if it did not.
// A frame whose pieces move is hashed here, after its move, as without defer.
__global__ __launch_bounds__(256) void k_decode_finish(DeviceJob j, int defer) {
    __shared__ __attribute__((aligned(16))) uint8_t xb[4][1024];
    lds_u8* xbuf = (lds_u8*)xb[threadIdx.x >> 6];
    const uint32_t count = j.counters[2];
    const uint32_t l = lane();
    // frames claimed one at a time: the content checksums are long serial
    // chains (~1 ms per MiB: XXH32's four accumulators, one lane each) and
    // only some frames carry one, so those are claimed first (counters[44])
    // and all start at once; the rest after them (counters[14]).  (In item
    // order a wave could meet two 1 MiB checksummed frames in a row: C2's
    // k_decode_finish 2.5-3.1 ms.)
    for (uint32_t phase = defer ? 1u : 0u; phase < 2; phase++)
    for (;;) {
        const uint32_t item = wave_fetch_add(&j.counters[phase == 0 ? 44 : 14], 1u);
        if (item >= count) break;
        const uint32_t mode = uni32(j.plans[item].mode);
        const bool xxh_first = mode == 1 && uni32(j.plans[item].ccs) != 0;
        if (!defer && xxh_first != (phase == 0)) continue;
        const uint32_t b = uni32(j.decode_list[item]);
        rpgpu_batch_result* R = &j.batches[b];
        if (mode == 3) {
            if (l == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
            continue;
        }
        if (mode == 0) continue;
        const uint32_t first = uni32(j.plans[item].first), nb = uni32(j.plans[item].nb);
        const uint64_t d0 = uni64(j.dcap[b]);
        bool ok = true, moved = false;
        uint64_t run = d0;  // where the next piece belongs
        for (uint32_t k = 0; k < nb; k++) {
            const int32_t out = (int32_t)uni32((uint32_t)j.blocks[first + k].out);
            if (out < 0) { ok = false; break; }
            const uint64_t at = uni64(j.blocks[first + k].dst);
            if (at < run) { ok = false; break; }  // a piece longer than planned (cannot happen: out <= cap)
            if (at != run) {
                moved = true;
                uint8_t* dd = j.decoded;
                for (uint32_t o = 0; o < (uint32_t)out; o += 1024) {
                    const uint32_t c = o + 16 * l;
                    if (c + 16 <= (uint32_t)out) {
                        const uint4 v = gld16(dd + at + c);
                        gst16(dd + run + c, v);
                    }
                }
                wait_vm();
                // the last < 16 bytes, forward byte by byte (dst below src)
                if (l == 0)
                    for (uint32_t e = (uint32_t)out & ~15u; e < (uint32_t)out; e++) dd[run + e] = dd[at + e];
                wait_vm();
            }
            run += (uint64_t)out;
        }
        const uint64_t total = run - d0;
        if (ok && mode == 1) {
            if (uni32(j.plans[item].csf) && total != uni64(j.plans[item].content_size)) ok = false;  // frameSize_wrong
            if (ok && !(defer && !moved) && uni32(j.plans[item].ccs) &&
                xxh32_wave(j.decoded + d0, total, 0, xbuf) != uni32(j.plans[item].ccs_val))
                ok = false;
        }
        uint32_t dcrc = 0;
        if (ok) {
            // reset_size_checksum_metadata's new crc (storage/parser_utils.cc:
            // 114-120) from the streaming CRCs k_lz_exec took of each piece:
            // the BE40 prefix with the codec bits of attrs cleared (BE byte
            // 1), then the pieces in order, each moved to the payload end by
            // GF(2) shifts (a linked frame is one stream already)
            const uint32_t codec = uni32((uint32_t)(uint16_t)R->attrs) & 7u;
            const uint32_t S0 = uni32((uint32_t)R->reserved1) ^ j.tables->hdr[38][codec] ^ j.tables->c40;
            uint32_t acc = 0;
            if (uni32(j.blocks[first].kind) & kBlkLinked) {
                if (l == 0) acc = j.blocks[first].crc;
            } else {
                uint64_t carry = 0;
                for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
                    const uint32_t k = b0 + l;
                    const uint32_t o = k < nb ? (uint32_t)j.blocks[first + k].out : 0u;
                    const uint32_t incl = wave_scan(o);
                    if (k < nb) acc ^= crc_shift(j.blocks[first + k].crc, total - (carry + incl));
                    carry += rl(incl, 63);
                }
            }
            dcrc = ~(crc_shift(S0, total) ^ wave_xor(acc));
        }
        if (ok && l == 0) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
            R->decoded_crc = dcrc;
            // decoded crc done (k_validate_decoded skips its CRC pass); OR'd:
            // with defer, k_crc_compose ran before and set bit 1
            R->reserved0 = (uint16_t)(R->reserved0 | 1u);
        }
    }
}

// the content checksums k_decode_finish(defer) leaves: one wave per
// checksummed frame whose pieces need no move (the same test as the
// finish's: every piece decoded, each where the previous one ended), from
// k_lz_exec's end, beside the rest of the decode stage.  The verdict goes to
// FramePlan.xxh only (k_decode_finish writes the result beside it);
// k_content_apply applies it after the join.  Four waves per workgroup, one
// per SIMD: with one-wave workgroups two hashing waves could share a SIMD,
// each at half speed (the longest hash 2.0 -> 2.95 ms).
#ifndef RPGPU_XXH_PRIO
#define RPGPU_XXH_PRIO 1
#endif
__global__ __launch_bounds__(256) void k_content_xxh(DeviceJob j) {
    __shared__ __attribute__((aligned(16))) uint8_t xb[4][1024];
    lds_u8* xbuf = (lds_u8*)xb[threadIdx.x >> 6];
    const uint32_t count = j.counters[2];
    const uint32_t l = lane();
    // first in issue on a shared SIMD (k_dchain, which waits on memory, is
    // above it): beside k_decode_finish's waves at equal priority the chains
    // ran ~1.4x their time alone
    __builtin_amdgcn_s_setprio(RPGPU_XXH_PRIO);
    for (;;) {
        const uint32_t item = wave_fetch_add(&j.counters[44], 1u);
        if (item >= count) break;
        if (uni32(j.plans[item].mode) != 1u || uni32(j.plans[item].ccs) == 0u) continue;
        const uint32_t b = uni32(j.decode_list[item]);
        const uint32_t first = uni32(j.plans[item].first), nb = uni32(j.plans[item].nb);
        const uint64_t d0 = uni64(j.dcap[b]);
        uint64_t carry = 0;
        uint32_t bad = 0;
        for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
            const uint32_t k = b0 + l;
            const int32_t out = k < nb ? (int32_t)j.blocks[first + k].out : 0;
            const uint32_t o = out > 0 ? (uint32_t)out : 0u;
            const uint32_t incl = wave_scan(o);
            if (k < nb && (out < 0 || j.blocks[first + k].dst != d0 + carry + (incl - o))) bad = 1;
            carry += rl(incl, 63);
        }
        if (wave_or(bad)) continue;  // moved (or failed): k_decode_finish's
        if (uni32(j.plans[item].csf) && carry != uni64(j.plans[item].content_size)) continue;  // fails there
        const uint32_t v = xxh32_wave(j.decoded + d0, carry, 0, xbuf) == uni32(j.plans[item].ccs_val) ? 1u : 2u;
        if (l == 0) j.plans[item].xxh = v;
    }
}

// after the join: a mismatched checksum restores what k_emit left in the
// result (no CODEC_OK, decoded_len / decoded_crc 0, reserved0 bit 0 clear),
// which is what k_decode_finish writes for such a frame without defer.
// (k_dchain may have chained the frame's payload meanwhile: never read, its
// verdict now fails dchain_ok.)
__global__ __launch_bounds__(256) void k_content_apply(DeviceJob j) {
    const uint32_t count = j.counters[2];
    for (uint32_t item = blockIdx.x * blockDim.x + threadIdx.x; item < count; item += gridDim.x * blockDim.x) {
        if (j.plans[item].xxh != 2u) continue;
        rpgpu_batch_result* R = &j.batches[j.decode_list[item]];
        R->flags = R->flags & ~(uint32_t)RPGPU_F_CODEC_OK;
        R->decoded_len = 0;
        R->decoded_crc = 0;
        atomicAnd(reserved0_word(R), ~(1u << 16));
    }
}

__global__ __launch_bounds__(64) void k_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst,
                                                       uint64_t cap, int64_t* res) {
    if (threadIdx.x != 0) return;
    int64_t got = 0;
    // src has at least 16 readable bytes past n (rpgpu_uncompress pads it)
    const int rc = decode_unit(codec, Src{src, (int64_t)n, (int64_t)n + 16}, Dst{dst, (int64_t)cap}, 0, 0, got);
    res[0] = rc;
    res[1] = got;
}

// rpgpu_uncompress_batch: one lane per payload (staged inputs, planned
// output slots), res[2 i] = rc, res[2 i + 1] = decoded length
__global__ __launch_bounds__(256) void k_uncompress_many(const UncItem* __restrict__ items, uint32_t count,
                                                         const uint8_t* in, uint64_t in_total, uint8_t* out,
                                                         int64_t* res) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const UncItem it = items[i];
    int64_t got = 0;
    const int rc = decode_unit(it.codec, Src{in + it.src, (int64_t)it.n, (int64_t)(in_total - it.src)},
                               Dst{out + it.dst, (int64_t)it.cap}, 0, 0, got);
    res[2 * i] = rc;
    res[2 * i + 1] = got;
}

#ifdef RPGPU_DSTAMPS
__global__ void k_print_dstamps() {
    const unsigned long long* g = g_dst;
    printf("RPGPU_DSTAMPS lz4 pieces=%llu exec_ms=%.1f | raw=%llu exec_ms=%.1f | snappy=%llu exec_ms=%.1f | "
           "linked=%llu exec_ms=%.1f | records=%llu pool-cut=%llu (wave-summed ms)\n",
           g[3], g[2] / 1e5, g[5], g[4] / 1e5, g[7], g[6] / 1e5, g[9], g[10] / 1e5, g[11], g[12]);
    printf("RPGPU_DSTAMPS batches=%llu rounds=%llu | per batch clk: scan=%.0f lit=%.0f rounds=%.0f flush=%.0f\n", g[20], g[21],
           (double)g[16] / g[20], (double)g[17] / g[20], (double)g[18] / g[20], (double)g[19] / g[20]);
    printf("RPGPU_DSTAMPS walk long=%llu sum_ms=%.1f max_ms=%.2f (nrec %llu csize %llu) | lane pieces=%llu sum_ms=%.1f "
           "max_ms=%.2f (nrec %llu csize %llu kind %llu) | wave end spread ms=%.2f\n",
           g[25], g[24] / 1e5, g[26] / 1e5, g[32], g[33], g[28], g[27] / 1e5, g[29] / 1e5, g[30], g[31] & 0xFFFFFFFFull,
           g[31] >> 32, (double)(g[34] - g[35]) / 1e5);
    printf("RPGPU_DSTAMPS snappy-long iterations=%llu hops=%llu | per iteration clk: decode=%.0f hops=%.0f rest=%.0f\n",
           g[40], g[41], (double)g[42] / (g[40] ? g[40] : 1), (double)g[43] / (g[40] ? g[40] : 1),
           (double)g[44] / (g[40] ? g[40] : 1));
    printf("RPGPU_DSTAMPS lzf walk rounds=%llu wave-steps=%llu | tails=%llu tail records=%llu\n", g[48], g[49], g[50],
           g[51]);
    printf("RPGPU_DSTAMPS exec batches with far lanes=%llu far lanes=%llu far drains=%llu match lanes=%llu | rounds clk "
           "in batches with far lanes=%.0f per batch (all batches %.0f)\n", g[52], g[53], g[54], g[55],
           (double)g[56] / (g[52] ? g[52] : 1), (double)g[18] / (g[20] ? g[20] : 1));
    for (int i = 0; i < 64; i++) g_dst[i] = 0;
}
__global__ void k_init_dstamps() {
    for (int i = 0; i < 46; i++) g_dst[i] = 0;  // [46, 64): k_lzf_walk / k_lzf_tail, which run before it
    g_dst[35] = ~0ull;
}
#endif

// ===========================================================================
// LZ4 block walk for k_lz_exec: k_lzf_walk + k_lzf_tail.
//
// The frames Redpanda writes are LZ4F with independent 64 KiB blocks
// (compression/internal/lz4_frame_compressor.cc:70-76: LZ4F_blockIndependent,
// default block size), decoded by LZ4F_decompress -> LZ4_decompress_safe per
// block (lz4_frame_compressor.cc:123-200).  A block is one serial chain of
// sequences (C2's JSON blocks: ~3200 of ~20 decoded bytes each).
//
// k_lzf_walk walks one block per LANE, 64 blocks per wave, from the
// planner's list (k_decode_blocks, lzf_eligible).  Every round each lane
// stages the kFSlot stream bytes at its parse position in its own LDS slot
// (all lanes' 16-byte loads in flight together: one memory latency per
// round for the wave) and walks the sequences that start in the first kFWin
// of them with a straight-line step (fseq_w: three aligned 8-byte LDS reads
// funnel-shifted, ~60 instructions, no per-sequence branches), writing each as an 8-byte
// record {lip | ll << 16, ml | off << 16} to frecs (a block reserves
// csize / 3 + 2 records: every sequence but the last takes >= 3 input bytes).
// Verdicts follow LZ4_decompress_generic (liblz4 1.9.3, lz4_run above): a
// sequence far from both ends (kFMarginIn input bytes, kFMarginOut output
// bytes) is one the reference's fast loop takes, whose only failure is an
// offset reaching before the block (H = 0 for an independent block; a
// linked block's reach is kept as `need` and checked against its real
// history when its frame executes).  At the first sequence that is not such
// an ordinary one (the block's last ones, offset 0, a length of more than
// one extension byte) the lane files the block for k_lzf_tail, which runs
// lz4_run itself from that exact state to the block's end, one lane per
// block, all tails in lock step; then takes its next block.  A block with no
// room in frecs stays with k_lz_walk (BlockItem.fast stays kLzfNone).
// k_lz_exec executes the records (exec_piece -> frecords) like the walk's.
//
// (Round 5 first tried one WAVE per block: the block staged whole in LDS,
// lanes parsing 1/64 of it each from speculative starts that resynchronise
// with the true chain, a visited-position bitmap to chain them.  Four
// passes over every lane's segment plus the resynchronisation wait cost
// ~160 us per block, 9.2 ms on C2, against ~2 wave-steps per sequence here.)
// ===========================================================================

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// one sequence at ip: literal [lip, lip + ll), match (off, ml; ml = 0: the
// stream ends in this literal run), next token at nxt (> n when the lengths
// run past the block)
struct FSeq {
    uint32_t lip, ll, ml, off, nxt;
};
// fseq_w: the sequence at ip of a lane window: slot holds stream bytes
// [wb, wb + kFSlot), zero past the block's n bytes; ip - wb < kFWin.  Three
// aligned 8-byte LDS reads (24 bytes from ip rounded down to 8) funnel-shifted
// to the 16 bytes at ip cover the token, a literal-length byte, literals up
// to 11 bytes, the offset and a match-length byte (C2: 98 % of sequences);
// otherwise two aligned dwords at the literals' end.  (Unaligned LDS reads
// stalled the LDS pipe: SQ_LDS_UNALIGNED_STALL was 87 % of its active
// cycles.)  st: 0 parsed; 1 a length needs more than one extension byte; 2
// the offset bytes lie too close to the window's end.  (Byte for byte the
// parse of LZ4_decompress_generic's length reads; checked against a
// byte-wise parse on adversarial streams.)
DEV FSeq fseq_w(const lds_u8* slot, uint32_t wb, uint32_t ip, uint32_t n, uint32_t& st) {
    typedef const __attribute__((address_space(3))) uint64_t lds_cu64;
    typedef const __attribute__((address_space(3))) uint32_t lds_cu32w;
    const uint32_t rel = ip - wb, a = rel >> 3, sh = 8 * (rel & 7);
    const uint64_t w0 = ((lds_cu64*)slot)[a], w1 = ((lds_cu64*)slot)[a + 1], w2 = ((lds_cu64*)slot)[a + 2];
    const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
    const uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
    const uint32_t tok = (uint32_t)lo & 0xFFu, b1 = ((uint32_t)lo >> 8) & 0xFFu;
    const uint32_t l4 = tok >> 4, m4 = tok & 15u;
    const bool e = l4 == 15;
    const uint32_t ll = l4 + (e ? b1 : 0u);
    const uint32_t lip = ip + (e ? 2u : 1u);
    const uint32_t pe = lip + ll;
    // the literals reach the end (ll > n - lip || n - lip - ll < 2): the last sequence
    const bool last = pe + 2 > n;
    const uint32_t k = pe - ip;
    // bytes [k, k + 4) of the 16 for k <= 12 (a per-lane dword select
    // compiles to branches)
    const uint32_t fs = 8 * (k & 7);
    const uint64_t fa = (k & 8) ? hi : lo, fb = (k & 8) ? 0ull : hi;
    uint32_t t = (uint32_t)(fa >> fs) | (uint32_t)((fb << 1) << (63 - fs));
    const uint32_t rp = pe - wb;
    const bool rd = k > 12 && !last;
    const bool past = rd && rp + 8 > kFSlot;
    if (rd && !past) {
        const uint32_t d0 = ((lds_cu32w*)slot)[rp >> 2], d1 = ((lds_cu32w*)slot)[(rp >> 2) + 1];
        t = __builtin_amdgcn_alignbyte(d1, d0, rp & 3);
    }
    const bool me = m4 == 15;
    const uint32_t b2 = (t >> 16) & 0xFFu;
    FSeq q;
    q.lip = lip;
    q.ll = ll;
    q.off = last ? 0u : t & 0xFFFFu;
    q.ml = last ? 0u : m4 + (me ? b2 : 0u) + 4;
    q.nxt = last ? pe : pe + (me ? 3u : 2u);
    st = (e && b1 == 255) ? 1u : past ? 2u : (!last && me && b2 == 255) ? 1u : 0u;
    return q;
}

// lz4_run's sink for a block's tail: 8-byte records
struct FRecSink {
    uint2* out;
    uint32_t n, cap;
    DEV bool seq(const uint4&, int32_t, int32_t lip, int32_t llen, int32_t, uint32_t off, int32_t ml) {
        if (n < cap) out[n] = make_uint2((uint32_t)lip | ((uint32_t)llen << 16), (uint32_t)ml | (off << 16));
        n++;
        return true;
    }
};

constexpr uint32_t kFLaneWgs = (160u * 1024u) / (256u * kFSlot);  // resident 256-lane workgroups per CU
static_assert(kFLaneWgs >= 1, "lane windows");

__global__ __launch_bounds__(256) void k_lzf_walk(DeviceJob j) {
    __shared__ __attribute__((aligned(16))) uint8_t fwin[256 * kFSlot];
    lds_u8* slot = (lds_u8*)fwin + kFSlot * threadIdx.x;
    const uint32_t cnt_list = j.counters[45];
    const uint32_t nlist = cnt_list < j.block_capacity ? cnt_list : j.block_capacity;
    bool active = false, drained = false;
    uint32_t p = 0, n = 0, cap = 0, ip = 0, op = 0, r = 0, resv = 0, base = 0;
    int32_t need = 0;
    bool linked = false;
    Src s{nullptr, 0, 0};
#ifdef RPGPU_DSTAMPS
    uint64_t d_rounds = 0, d_steps = 0;
#endif
    for (;;) {
        // lanes without a block take the next ones: one claim per wave
        for (;;) {
            const bool want = !active && !drained;
            const uint64_t wm = __ballot(want);
            if (!wm) break;
            const int lead = __builtin_ctzll(wm);
            uint32_t u0 = 0;
            if (lane() == (uint32_t)lead) u0 = atomicAdd(&j.counters[46], (uint32_t)__builtin_popcountll(wm));
            const uint32_t u = rl(u0, lead) + (uint32_t)__builtin_popcountll(wm & ((1ull << lane()) - 1));
            if (!want) continue;
            if (u >= nlist) {
                drained = true;
                continue;
            }
            p = j.lzf_list[u];
            const BlockItem it = j.blocks[p];
            resv = lzf_reserve(it.csize);
            base = j.pstate[p].first_slab;  // reserved by the planner (note_fast)
            n = it.csize;
            cap = it.cap;
            linked = (it.kind & kBlkLinked) != 0;
            s = Src{j.data + it.src, (int64_t)n, (int64_t)(j.data_len - it.src)};
            ip = op = r = 0;
            need = 0;
            active = true;
        }
        if (!__ballot(active)) break;
        // stage stream bytes [wb, wb + kFSlot), zero past the block
        const uint32_t wb = ip;
        // (in two halves: 9 loads in flight per lane, ~36 fewer VGPRs, so two
        // workgroups per CU stay resident beside k_raw_copy's)
#pragma unroll
        for (uint32_t h = 0; h < 2; h++)
        if (active) {
            constexpr uint32_t kH = kFSlot / 32;
            uint4 v[kH];
#pragma unroll
            for (uint32_t c0 = 0; c0 < kH; c0++) v[c0] = ld16(s, (int64_t)wb + 16 * (h * kH + c0));
#pragma unroll
            for (uint32_t c0 = 0; c0 < kH; c0++) {
                const uint32_t c = h * kH + c0;
                const int32_t keep = (int32_t)n - (int32_t)(wb + 16 * c);  // bytes of this chunk inside the block
                if (keep < 16) {
                    uint32_t w[4] = {v[c0].x, v[c0].y, v[c0].z, v[c0].w};
#pragma unroll
                    for (uint32_t d = 0; d < 4; d++) {
                        const int32_t kd = keep - 4 * (int32_t)d;
                        w[d] = kd >= 4 ? w[d] : kd <= 0 ? 0u : (w[d] & ((1u << (8 * kd)) - 1u));
                    }
                    v[c0] = make_uint4(w[0], w[1], w[2], w[3]);
                }
                __builtin_memcpy(slot + 16 * c, &v[c0], 16);
            }
        }
        // walk the window: 0 on, 1 the tail, 2 reject, 3 restage
        bool go = active;
        uint32_t outcome = 0;
#ifdef RPGPU_DSTAMPS
        d_rounds++;
#endif
        while (__ballot(go)) {
#ifdef RPGPU_DSTAMPS
            d_steps++;
#endif
            uint32_t st;
            const FSeq q = fseq_w(slot, wb, go ? ip : wb, n, st);
            const uint32_t opl = op + q.ll, ope = opl + q.ml;
            const bool ord = st == 0 && q.ml != 0 && q.nxt + kFMarginIn <= n && ope + kFMarginOut <= cap && q.off != 0;
            // before the block (LZ4_decompress_safe: offset outside buffers)
            const bool rej = ord && !linked && q.off > opl;
            if (go && ord && linked) {
                const int32_t d = (int32_t)q.off - (int32_t)opl;
                need = d > need ? d : need;
            }
            const bool ok = go && ord && !rej;
            if (ok) j.frecs[(size_t)base + r] = make_uint2(q.lip | (q.ll << 16), q.ml | (q.off << 16));
            if (go && !ok) outcome = (st == 2 && ip > wb) ? 3u : rej ? 2u : 1u;
            r += ok ? 1u : 0u;
            op = ok ? ope : op;
            ip = ok ? q.nxt : ip;
            go = ok && ip < wb + kFWin;
        }
        if (active && outcome == 1) {
            // the rest is the reference loop's: k_lzf_tail
            const uint32_t t = atomicAdd(&j.counters[47], 1u);
            j.lzf_tail[t] = p;
            PieceState ps;
            ps.ip = (int32_t)ip;
            ps.op = (int32_t)op;
            ps.need = need;
            ps.st = 0;
            ps.ulen = (int32_t)resv;  // (the reservation, for k_lzf_tail)
            ps.safe = 0;
            ps.nrec = r;
            ps.first_slab = base;
            j.pstate[p] = ps;
            active = false;
        } else if (active && outcome == 2) {
            j.blocks[p].out = -1;
            j.blocks[p].crc = 0u;
            j.blocks[p].fast = kLzfReject;
            active = false;
        }
    }
#ifdef RPGPU_DSTAMPS
    if (lane() == 0) {
        atomicAdd(&g_dst[48], d_rounds);
        atomicAdd(&g_dst[49], d_steps);
    }
#endif
}

// the tails k_lzf_walk filed: lz4_run from the first sequence that is not an
// ordinary one (the reference's fast loop, every earlier sequence having been
// one) to the block's end, one lane per block
__global__ __launch_bounds__(256) void k_lzf_tail(DeviceJob j) {
    const uint32_t nt = j.counters[47];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
        const uint32_t p = j.lzf_tail[t];
        const BlockItem it = j.blocks[p];
        PieceState pst = j.pstate[p];
        const bool linked = (it.kind & kBlkLinked) != 0;
        const Src s{j.data + it.src, (int64_t)it.csize, (int64_t)(j.data_len - it.src)};
        PState ps;
        ps.ip = pst.ip;
        ps.op = pst.op;
        ps.need = 0;
        ps.st = 0;
        ps.ulen = 0;
        ps.safe = it.cap < (uint32_t)kFastSafeDistance;
        const uint32_t resv = (uint32_t)pst.ulen;
        FRecSink fs{j.frecs + pst.first_slab, pst.nrec, resv};
        lz4_run(s, (int32_t)it.cap, linked ? 65536 : 0, ps, fs);
#ifdef RPGPU_DSTAMPS
        atomicAdd(&g_dst[50], 1ull);
        atomicAdd(&g_dst[51], (unsigned long long)(fs.n - pst.nrec));
#endif
        if (ps.st != 1) {
            j.blocks[p].out = -1;
            j.blocks[p].crc = 0u;
            j.blocks[p].fast = kLzfReject;
            continue;
        }
        if (fs.n > resv) {  // (cannot happen: the reservation bounds any parse)
            j.blocks[p].out = -1;
            j.blocks[p].fast = kLzfReject;
            continue;
        }
        const int32_t need = ps.need > pst.need ? ps.need : pst.need;
        pst.ip = 0;
        pst.op = ps.op;
        pst.need = need > 0 ? need : 0;
        pst.st = 1;
        pst.ulen = 0;
        pst.safe = 0;
        pst.nrec = fs.n;
        j.pstate[p] = pst;
        j.blocks[p].fast = kLzfReady;
    }
}

uint32_t lz_exec_wgs_per_cu() { return kExecWaves; }

hipError_t launch_decode(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_decode_blocks(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode_blocks, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_lz_walk(const DeviceJob& j, hipStream_t s, uint32_t grid) {
#ifdef RPGPU_DSTAMPS
    hipLaunchKernelGGL(k_init_dstamps, dim3(1), dim3(1), 0, s);
#endif
    hipLaunchKernelGGL(k_lz_walk, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_raw_copy(const DeviceJob& j, hipStream_t s, uint32_t cus) {
    if (!j.raw_list) return hipSuccess;
    // one 16-wave workgroup per CU (one 8 KiB CRC table copy: k_lzf_walk's
    // two 74 KiB workgroups per CU still fit beside it)
    hipLaunchKernelGGL(k_raw_copy, dim3(cus), dim3(RPGPU_RAW_THREADS), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_lz_exec(const DeviceJob& j, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_lz_exec, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kXLds);
        attr = true;
    }
    if (!j.exec_waves) return hipSuccess;
    hipLaunchKernelGGL(k_lz_exec, dim3(j.exec_waves / kExecWaves), dim3(64 * kExecWaves), kXLds, s, j);
#ifdef RPGPU_DSTAMPS
    hipLaunchKernelGGL(k_print_dstamps, dim3(1), dim3(1), 0, s);
#endif
    return hipGetLastError();
}

hipError_t launch_lzf_walk(const DeviceJob& j, hipStream_t s, uint32_t cus) {
    if (!j.frecs || !j.lzf_list || !j.lzf_tail) return hipSuccess;
    // persistent lane walkers, as many as the windows allow per CU; then the tails
    hipLaunchKernelGGL(k_lzf_walk, dim3(cus * kFLaneWgs), dim3(256), 0, s, j);
    hipLaunchKernelGGL(k_lzf_tail, dim3(cus * 2), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_zexec(const DeviceJob& j, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_zexec, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kXLds);
        attr = true;
    }
    if (!j.exec_waves || !j.inf_scratch) return hipSuccess;
    hipLaunchKernelGGL(k_zexec, dim3(j.exec_waves / kExecWaves), dim3(64 * kExecWaves), kXLds, s, j);
    return hipGetLastError();
}

hipError_t launch_decode_finish(const DeviceJob& j, hipStream_t s, uint32_t grid, bool defer) {
    hipLaunchKernelGGL(k_decode_finish, dim3(grid), dim3(256), 0, s, j, defer ? 1 : 0);
    return hipGetLastError();
}
hipError_t launch_content_xxh(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_content_xxh, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_content_apply(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_content_apply, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_uncompress_many(const UncItem* items, uint32_t count, const uint8_t* in, uint64_t in_total,
                                  uint8_t* out, int64_t* res, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_uncompress_many, dim3((count + 255) / 256), dim3(256), 0, s, items, count, in, in_total, out, res);
    return hipGetLastError();
}

hipError_t launch_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, int64_t* res,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_uncompress_one, dim3(1), dim3(64), 0, s, codec, src, n, dst, cap, res);
    return hipGetLastError();
}

}  // namespace rp
