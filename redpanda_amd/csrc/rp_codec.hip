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
// Execution model: one wave decodes one piece (an LZ4 block of a
// block-independent frame, a snappy-java chunk, or a whole sequential frame).
//   * Parsing is wave-uniform: token / tag bytes come out of a 512-byte input
//     window held one dword per lane (two VGPRs), read with v_readlane.
//   * Output goes through a per-wave LDS ring (kRing bytes, indexed by the
//     absolute arena address) and leaves for HBM in coalesced 16-byte-per-lane
//     stores of whole 1 KiB chunks.
//   * Literals up to 64 bytes are copied at once, one byte per lane, from the
//     input window (ds_bpermute); longer ones stream from global memory.
//   * Matches are queued, one per lane, into a group covering at most kSpan
//     output bytes.  When the group closes, every match whose source ends
//     before the group's first match is final and is copied lane-parallel:
//     from the ring when the source is still in it, else from HBM (the
//     wave's own earlier stores, read back with sc1 loads).  The rest
//     (sources inside the group) are copied in order, one match per step,
//     64 bytes per lane-parallel LDS round trip.
//   * Long matches (> 64 bytes), zero offsets and long literals run on the
//     spot, flushing the ring as they go.
// Integer/byte work only: no MFMA.
#include "rp_device.h"
#if defined(RPGPU_CHECKED) || defined(RPGPU_TRACE)
#include <cstdio>
#endif
// RPGPU_TRACE: diagnostic build (scripts/build_exp.py trace -DRPGPU_TRACE
// --unit rp_codec.hip) printing the decode engine's steps; never measured
#ifdef RPGPU_TRACE
#define TRACE(...) do { if (lane() == 0) printf(__VA_ARGS__); } while (0)
#else
#define TRACE(...) do { } while (0)
#endif
// RPGPU_DSTAMPS: diagnostic build of the decode kernel (scripts/build_exp.py
// dstamps -DRPGPU_DSTAMPS --unit rp_codec.hip): s_memtime cycle totals per
// item kind and per engine phase, printed by k_print_dstamps; never measured
#ifdef RPGPU_DSTAMPS
#include <cstdio>
__device__ unsigned long long g_dst[32];
#define DST(d, i, x) ((d).st[i] += (uint64_t)(x))
#define DCLK() __builtin_amdgcn_s_memtime()
#else
#define DST(d, i, x) do { } while (0)
#define DCLK() 0ull
#endif
#if defined(RPGPU_TRACE_ITEMS)
#include <cstdio>
#define TRACE_ITEM(...) do { if (lane() == 0) printf(__VA_ARGS__); } while (0)
#else
#define TRACE_ITEM(...) do { } while (0)
#endif

namespace rp {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u32 lds_v4;

#ifndef RPGPU_RING_KIB
#define RPGPU_RING_KIB 16
#endif
constexpr uint32_t kRing = RPGPU_RING_KIB * 1024u;  // per-wave output ring
constexpr uint32_t kRM = kRing - 1u;
static_assert((kRing & kRM) == 0 && kRing >= 8192, "ring must be a power of two >= 8 KiB");
constexpr uint32_t kDecWaves = 4;      // waves per workgroup of the decode kernels
constexpr int64_t kSpan = 2048;        // output bytes one match group may cover
constexpr uint32_t kFarMax = 48;       // far matches up to this length are copied lane-parallel
constexpr uint32_t kBufFlags = 0x00020000u;  // buffer resource word 3 (raw, 32-bit data format)
constexpr int kSc1 = 16;               // cache policy: sc1 (L2-coherent, bypasses the vector L1)

// ---------------------------------------------------------------------------
// input window: 512 bytes, lane l holds dwords base + 4 l (w0) and base + 256
// + 4 l (w1); base is 4-aligned in absolute address
// ---------------------------------------------------------------------------
struct In {
    const uint8_t* src;  // stream start
    int64_t n;           // stream bytes
    int64_t base;        // stream offset of the window start
    uint32_t w0, w1;
#ifdef RPGPU_DSTAMPS
    uint64_t loads;      // window (re)loads
#endif
};

DEV uint32_t ld_dw(const uint8_t* src, int64_t n, uintptr_t a) {
    return a < (uintptr_t)(src + n) ? *(const uint32_t*)a : 0u;  // a is 4-aligned: never crosses a page
}

DEV void in_init(In& in, const uint8_t* src, int64_t n) {
    in.src = src;
    in.n = n;
    in.base = -(1ll << 60);
    in.w0 = in.w1 = 0;
#ifdef RPGPU_DSTAMPS
    in.loads = 0;
#endif
}

DEV void in_load(In& in, int64_t ip) {
#ifdef RPGPU_DSTAMPS
    in.loads++;
#endif
    const uintptr_t a = ((uintptr_t)(in.src + ip)) & ~(uintptr_t)3;
    in.base = (int64_t)(a - (uintptr_t)in.src);
    const uintptr_t mine = a + 4u * lane();
    in.w0 = ld_dw(in.src, in.n, mine);
    in.w1 = ld_dw(in.src, in.n, mine + 256u);
}

// byte ip of the stream (uniform; bytes past the stream read as zero)
DEV uint32_t in_byte(In& in, int64_t ip) {
    int64_t o = ip - in.base;
    if (o < 0 || o >= 512) {
        in_load(in, ip);
        o = ip - in.base;
    }
    const int li = (int)((o >> 2) & 63);
    const uint32_t w = o < 256 ? rl(in.w0, li) : rl(in.w1, li);
    return (w >> (8 * (uint32_t)(o & 3))) & 0xFFu;
}
DEV uint32_t in_le16(In& in, int64_t ip) { return in_byte(in, ip) | (in_byte(in, ip + 1) << 8); }
DEV uint32_t in_le32(In& in, int64_t ip) { return in_le16(in, ip) | (in_le16(in, ip + 2) << 16); }

// ---------------------------------------------------------------------------
// output state.  Positions are absolute arena offsets (uniform, 64-bit).
// ---------------------------------------------------------------------------
struct Dec {
    uint8_t* arena;           // decoded arena (global)
    lds_u8* ring;             // this wave's kRing bytes
    __amdgpu_buffer_rsrc_t rs;  // arena window for sc1 read-backs, based at `lo`
    uint64_t lo;              // lowest position this decode may read (frame start)
    uint64_t base;            // position of relative output 0
    uint64_t op;              // next output position
    uint64_t flushed;         // bytes below are stored to the arena
    uint64_t confirmed;       // bytes below are visible to sc1 loads (vmcnt drained)
    uint64_t ring_lo;         // the ring holds [max(ring_lo, op - kRing), op)
#ifdef RPGPU_DSTAMPS
    uint64_t st[8];           // 0 sequences, 1 groups, 2 group cycles, 3 serial matches, 4 far groups,
                              // 5 flush cycles, 6 ring-parallel lanes, 7 far-parallel lanes
#endif
};

// matches waiting in the open group, lane j = j-th match
struct Group {
    uint32_t rop, off, ml;    // per lane: output position - m0, offset, length
    uint32_t n;               // queued matches
    uint64_t m0;              // output position of the first queued match
};

DEV void dec_init(Dec& d, uint8_t* arena, uint64_t arena_cap, lds_u8* ring, uint64_t at) {
    d.arena = arena;
    d.ring = ring;
    d.lo = at;
    d.base = at;
    d.op = at;
    d.flushed = at;
    d.confirmed = at;
    d.ring_lo = at;
    // read-backs past the arena's end return zeros instead of faulting
    const uint64_t room = arena_cap > at ? arena_cap - at : 0;
    d.rs = __builtin_amdgcn_make_buffer_rsrc(arena + at, 0, (int)(room < 0x7FFFFFFFull ? room : 0x7FFFFFFFull), kBufFlags);
#ifdef RPGPU_DSTAMPS
    for (int i = 0; i < 8; i++) d.st[i] = 0;
#endif
}

DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// make every stored byte below `upto` visible to the sc1 read-backs
DEV void confirm(Dec& d, uint64_t upto) {
    if (upto > d.confirmed) {
        wait_vm();
        d.confirmed = d.flushed;
    }
}

DEV uint32_t rd_back8(const Dec& d, uint64_t at) {
    return __builtin_amdgcn_raw_buffer_load_b8(d.rs, (uint32_t)(at - d.lo), 0, kSc1);
}

// store ring bytes [d.flushed, upto) to the arena: whole 16-byte pieces as
// one ds_read_b128 + global_store_dwordx4 per lane (1 KiB per wave
// instruction), ragged edge pieces byte by byte.  The trip count is made
// uniform up front: a loop whose exit the compiler treats per lane left
// chunks unstored (lanes dropped from EXEC) when it was written as
// while (flushed < upto).
DEV void flush(Dec& d, uint64_t upto) {
    const uint64_t f = uni64(d.flushed);
    upto = uni64(upto);
    if (f >= upto) return;
    const uint64_t t0 = DCLK();
    TRACE("flush %llu..%llu\n", (unsigned long long)f, (unsigned long long)upto);
    const uint32_t l = lane();
    const uint64_t c_first = f & ~1023ull;
    const uint32_t nchunks = uni32((uint32_t)((((upto + 1023) & ~1023ull) - c_first) >> 10));
    for (uint32_t i = 0; i < nchunks; i++) {
        const uint64_t a = c_first + ((uint64_t)i << 10) + 16u * l;
        const uint32_t r = (uint32_t)a & kRM;
        if (a >= f && a + 16 <= upto) {
            *(v4u32*)(d.arena + a) = *(const lds_v4*)(d.ring + r);
        } else if (a + 16 > f && a < upto) {
#pragma unroll
            for (uint32_t b = 0; b < 16; b++)
                if (a + b >= f && a + b < upto) d.arena[a + b] = d.ring[r + b];
        }
    }
    d.flushed = upto;
    (void)t0;
}

// flush whole chunks only (the ragged tail stays in the ring until the end)
DEV void flush_chunks(Dec& d) { flush(d, d.op & ~1023ull); }

// ---------------------------------------------------------------------------
// match groups
// ---------------------------------------------------------------------------
DEV void group_init(Group& g) {
    g.rop = g.off = g.ml = 0;
    g.n = 0;
    g.m0 = 0;
}

DEV uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// one match, uniform, sources final (written or in the arena): each source
// byte from the ring when the ring still holds it, else read back from the
// arena.  `top` = the highest position written so far.  Handles overlap
// (off < ml) and off == 0 (zeros, as liblz4's write32(op, 0) /
// LZ4_memcpy_using_offset_base produce).  Long copies flush as they go so
// the ring never overwrites unstored bytes.
DEV uint64_t ring_bound(const Dec& d, uint64_t top) {
    const uint64_t r = top > kRing ? top - kRing : 0;
    return r > d.ring_lo ? r : d.ring_lo;
}

DEV void match_serial(Dec& d, uint64_t op, uint32_t off, uint32_t ml, uint64_t top) {
    const uint32_t l = lane();
    TRACE("serial op=%llu off=%u ml=%u top=%llu\n", (unsigned long long)op, off, ml, (unsigned long long)top);
    const uint32_t o32 = (uint32_t)op;
    if (off == 0) {
        for (uint32_t c = 0; c < ml; c += 64) {
            if (c + l < ml) d.ring[(o32 + c + l) & kRM] = 0;
            d.op = op + (c + 64 < ml ? c + 64 : ml);
            if ((d.op & ~1023ull) > d.flushed + 2048) flush_chunks(d);
        }
        return;
    }
    const uint64_t s = op - off;
    const uint32_t s32 = (uint32_t)s;
    if (off < 64 && off < ml) {
        // period off: lanes k < L = off * floor(64 / off) hold the pattern
        // once; every chunk of L output bytes repeats it
        const uint32_t L = off * (64u / off);
        const uint32_t k = l < L ? l : 0u;
        // k mod off: with inv = floor(2^16 / off) + 1 the quotient
        // (k * inv) >> 16 is exact for k < 64, off < 64
        const uint32_t inv = 65536u / off + 1u;
        const uint32_t kmod = k - off * ((k * inv) >> 16);
        const uint64_t bnd = ring_bound(d, top > op + 64 ? top : op + 64);
        if (s < bnd) confirm(d, bnd);
        const uint32_t v = s + kmod >= bnd ? (uint32_t)d.ring[(s32 + kmod) & kRM] : rd_back8(d, s + kmod);
        for (uint32_t c = 0; c < ml; c += L) {
            if (l < L && c + l < ml) d.ring[(o32 + c + l) & kRM] = (uint8_t)v;
            d.op = op + (c + L < ml ? c + L : ml);
            if ((d.op & ~1023ull) > d.flushed + 2048) flush_chunks(d);
        }
        return;
    }
    // 64-byte steps; with off >= 64 every source byte is final before it is read
    for (uint32_t c = 0; c < ml; c += 64) {
        const uint64_t wt = op + c + 64;
        const uint64_t bnd = ring_bound(d, top > wt ? top : wt);
        if (s + c < bnd) confirm(d, bnd);
        const bool act = c + l < ml;
        const uint32_t cut = s + c >= bnd ? 0u : (uint32_t)(bnd - (s + c) < 64 ? bnd - (s + c) : 64);
        uint32_t v = d.ring[(s32 + c + l) & kRM];
        if (act && l < cut) v = rd_back8(d, s + c + l);
        if (act) d.ring[(o32 + c + l) & kRM] = (uint8_t)v;
        d.op = op + (c + 64 < ml ? c + 64 : ml);
        if ((d.op & ~1023ull) > d.flushed + 2048) flush_chunks(d);
    }
}

// run the open group (see the header).  Every byte below d.op other than
// the queued matches' outputs is already in the ring.  Per-lane arithmetic
// is 32-bit: ring slots only need the low bits of a position, and every
// source lies within 4 GiB above d.lo.
DEV void group_exec(Dec& d, Group& g) {
    if (g.n == 0) return;
    const uint64_t t0 = DCLK();
    DST(d, 1, 1);
    const uint32_t l = lane();
    const bool mine = l < g.n;
    const uint64_t end = d.op;
    const uint64_t near_lo = ring_bound(d, end);
    // relative to d.lo (all sources are at or above it)
    const uint32_t m0r = (uint32_t)(g.m0 - d.lo);
    const uint32_t opr = m0r + g.rop;
    const uint32_t sr = opr - g.off;
    const uint32_t nlr = (uint32_t)(near_lo - d.lo);
    const uint32_t lo32 = (uint32_t)d.lo;  // ring slot of relative position p: (lo32 + p) & kRM
    const bool indep = mine && sr + g.ml <= m0r;
    const bool near = sr >= nlr;
    const bool ring_par = indep && near;
    const bool far_par = indep && !near && g.ml <= kFarMax;
    DST(d, 6, __builtin_popcountll(__ballot(ring_par)));

    DST(d, 4, __ballot(far_par) ? 1 : 0);
    TRACE("group n=%u m0=%llu end=%llu ring=%llx far=%llx\n", g.n, (unsigned long long)g.m0, (unsigned long long)end,
          (unsigned long long)__ballot(ring_par), (unsigned long long)__ballot(far_par));
    // lane-parallel, sources in the ring
    if (__ballot(ring_par)) {
        const uint32_t kmax = wave_max(ring_par ? g.ml : 0u);
        const uint32_t rs = lo32 + sr, ro = lo32 + opr;
        for (uint32_t k = 0; k < kmax; k += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = d.ring[(rs + k + i) & kRM];
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (ring_par && k + i < g.ml) d.ring[(ro + k + i) & kRM] = (uint8_t)v[i];
        }
    }
    // lane-parallel, sources read back from the arena: 64 bytes from the
    // 16-aligned address at or below the source, each byte placed by its
    // window offset; bytes at or above near_lo (a source straddling a direct
    // copy's end) come from the ring, where they may not be stored yet
    if (__ballot(far_par)) {
        confirm(d, d.lo + wave_max(far_par ? sr + g.ml : 0u));
        const uint32_t sa = sr & 15u;
        // unconditional: lanes outside far_par read harmless bytes (the
        // resource returns zeros past its range)
        uint32_t qa[16];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            auto t = __builtin_amdgcn_raw_buffer_load_b128(d.rs, far_par ? (sr & ~15u) + 16 * i : 0u, 0, kSc1);
            qa[4 * i] = t[0];
            qa[4 * i + 1] = t[1];
            qa[4 * i + 2] = t[2];
            qa[4 * i + 3] = t[3];
        }
        const uint32_t cut = (far_par && sr + g.ml > nlr) ? nlr - sr : 0xFFFFFFFFu;
        const uint32_t ws = lo32 + sr - sa, wo = lo32 + opr - sa;  // ring slots of window byte 0
        const uint32_t kend = far_par ? sa + g.ml : 0u;            // window bytes [sa, kend) are the source
        const uint32_t tmax = (wave_max(kend) + 3) >> 2;
#pragma unroll 1
        for (uint32_t t = 0; t < tmax; t++) {
            const uint32_t dw = qa[t];  // uniform index: v_movrels
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t w = 4 * t + b;
                if (w >= sa && w < kend) {
                    uint32_t byte = (dw >> (8 * b)) & 0xFFu;
                    if (w - sa >= cut) byte = d.ring[(ws + w) & kRM];
                    d.ring[(wo + w) & kRM] = (uint8_t)byte;
                }
            }
        }
    }
    // in order: matches whose sources lie inside the group (or that are too
    // long for the lane-parallel read-back)
    const uint64_t serial = __ballot(mine && !ring_par && !far_par);
    DST(d, 3, __builtin_popcountll(serial));
    if (serial) {
        const uint64_t keep = d.op;
        uint64_t m = serial;
        while (m) {
            const int j = __builtin_ctzll(m);
            m &= m - 1;
            const uint64_t o = g.m0 + rl(g.rop, j);
            match_serial(d, o, rl(g.off, j), rl(g.ml, j), keep);
        }
        d.op = keep;
    }
    g.n = 0;
    flush_chunks(d);
    DST(d, 2, DCLK() - t0);
}

// One sequence at d.op: the literal bytes [lip, lip + llen) of the stream,
// then (has_match) a match (off, ml).  The open group closes first when it
// cannot take the sequence (one group_exec call site per parser).  Literals
// up to 64 bytes are one byte per lane from the input window (ds_bpermute);
// longer ones stream 16 bytes per lane from global memory.  Matches join
// the group unless they are long or have offset 0.
DEV void emit_seq(Dec& d, Group& g, In& in, int64_t lip, int64_t llen, uint32_t off, uint32_t ml, bool has_match) {
    const uint32_t l = lane();
    DST(d, 0, 1);
    const bool big_lit = llen > 64;
    const bool big_match = has_match && (off == 0 || ml > 64);
    const uint64_t mend = d.op + (uint64_t)llen + (has_match ? ml : 0u);
    if (g.n && (big_lit || big_match || g.n == 64 || mend - g.m0 > (uint64_t)kSpan)) group_exec(d, g);
    const uint64_t op = d.op;
    if (llen > 0 && !big_lit) {
        if (lip < in.base || lip + llen > in.base + 512) in_load(in, lip);
        const int64_t o = lip + (int64_t)l - in.base;  // lanes < llen: inside the window
        const int li = (int)((o >> 2) & 63);
        const uint32_t v0 = (uint32_t)__shfl((int)in.w0, li, 64);
        const uint32_t v1 = (uint32_t)__shfl((int)in.w1, li, 64);
        const uint32_t w = o < 256 ? v0 : v1;
        if ((int64_t)l < llen) d.ring[((uint32_t)op + l) & kRM] = (uint8_t)(w >> (8 * (uint32_t)(o & 3)));
        d.op = op + (uint64_t)llen;
    } else if (big_lit) {
        const uint8_t* src = in.src + lip;
        const uint32_t o32 = (uint32_t)op;
        for (int64_t c = 0; c < llen; c += 1024) {
            const int64_t k = c + 16 * (int64_t)l;
            const uint32_t r = o32 + (uint32_t)k;
            if (k + 16 <= llen) {
                const uint4 v = ld16u(src + k);
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int bb = 0; bb < 16; bb++) d.ring[(r + bb) & kRM] = (uint8_t)(wv[bb >> 2] >> (8 * (bb & 3)));
            } else {
                for (int64_t bb = k; bb < llen && bb < k + 16; bb++) d.ring[(o32 + (uint32_t)bb) & kRM] = src[bb];
            }
            d.op = op + (uint64_t)(c + 1024 < llen ? c + 1024 : llen);
            flush_chunks(d);
        }
    }
    if (!has_match) return;
    const uint64_t mo = d.op;
    if (big_match) {
        match_serial(d, mo, off, ml, mo);
        d.op = mo + ml;
        flush_chunks(d);
        return;
    }
    if (g.n == 0) g.m0 = mo;
    const uint32_t j = g.n;
    const bool me = l == j;
    g.rop = me ? (uint32_t)(mo - g.m0) : g.rop;
    g.off = me ? off : g.off;
    g.ml = me ? ml : g.ml;
    g.n = j + 1;
    d.op = mo + ml;
}

// end of a decode: everything queued is run and stored
DEV void dec_finish(Dec& d, Group& g) {
    group_exec(d, g);
    flush(d, d.op);
}

// a run of raw bytes straight to the arena (stored LZ4 blocks): 16 bytes per
// lane, 4 KiB per step, then the ring no longer covers what lies below
DEV void copy_direct(Dec& d, Group& g, const uint8_t* src, int64_t len) {
    if (len <= 0) return;
    TRACE_ITEM("  cd enter op %llu len %lld\n", (unsigned long long)d.op, (long long)len);
    dec_finish(d, g);
    TRACE_ITEM("  cd finished\n");
    const int64_t l = lane();
    uint8_t* dst = d.arena + d.op;
    int64_t head = (int64_t)((16u - ((uintptr_t)dst & 15u)) & 15u);
    if (head > len) head = len;
    if (l < head) dst[l] = src[l];
    const int64_t mid = head + ((len - head) & ~15ll);
    for (int64_t c = head; c < mid; c += 4096) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t k = c + 1024 * u + 16 * l;
            if (k < mid) v[u] = ld16u(src + k);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t k = c + 1024 * u + 16 * l;
            if (k < mid) *(uint4*)(dst + k) = v[u];
        }
    }
    if (l < len - mid) dst[mid + l] = src[mid + l];
    TRACE_ITEM("  cd copied\n");
    d.op += (uint64_t)len;
    d.flushed = d.op;
    d.ring_lo = d.op;
}

// ---------------------------------------------------------------------------
// XXH32 (lz4 1.9.3 xxhash.c): stripes streamed 1 KiB per row (lane l holds
// stripe 64 r + l, pre-multiplied by PRIME2), the four accumulators advance
// on the scalar unit, one readlane per word.  Read with sc1 loads so bytes
// this kernel stored are seen.
// ---------------------------------------------------------------------------
DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ __attribute__((noinline)) uint32_t xxh32_wave(const uint8_t* p, uint64_t n, uint32_t seed) {
    const uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, 0x7FFFFFFF, kBufFlags);
    const uint32_t l = lane();
    uint64_t i = 0;
    uint32_t h;
    if (n >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint64_t nst = n / 16;
        auto row = [&](uint64_t r) __attribute__((always_inline)) {
            uint4 q = make_uint4(0, 0, 0, 0);
            if (r * 64 + l < nst) {
                auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(16 * (r * 64 + l)), 0, kSc1);
                q = make_uint4(t[0], t[1], t[2], t[3]);
            }
            return q;
        };
        uint4 cur = row(0);
        for (uint64_t r = 0; r * 64 < nst; r++) {
            const uint4 nxt = row(r + 1);
            const uint32_t x = cur.x * P2, y = cur.y * P2, z = cur.z * P2, w = cur.w * P2;
            const uint32_t cnt = (uint32_t)(nst - r * 64 < 64 ? nst - r * 64 : 64);
            for (uint32_t k = 0; k < cnt; k++) {
                v1 = rotl32(v1 + rl(x, (int)k), 13) * P1;
                v2 = rotl32(v2 + rl(y, (int)k), 13) * P1;
                v3 = rotl32(v3 + rl(z, (int)k), 13) * P1;
                v4 = rotl32(v4 + rl(w, (int)k), 13) * P1;
            }
            cur = nxt;
        }
        i = nst * 16;
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    // the last < 16 bytes: lane k < 16 holds byte i + k
    const uint32_t rem = (uint32_t)(n - i);
    const uint32_t b = l < rem ? __builtin_amdgcn_raw_buffer_load_b8(rs, (uint32_t)(i + l), 0, kSc1) : 0u;
    uint32_t k = 0;
    for (; k + 4 <= rem; k += 4) {
        const uint32_t wd = rl(b, (int)k) | (rl(b, (int)k + 1) << 8) | (rl(b, (int)k + 2) << 16) | (rl(b, (int)k + 3) << 24);
        h = rotl32(h + wd * P3, 17) * P4;
    }
    for (; k < rem; k++) h = rotl32(h + rl(b, (int)k) * P5, 11) * P1;
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
// Output starts at d.op; H = history bytes before it.  Returns the decoded
// length or -1.
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

DEV int64_t lz4_block(In& in, int64_t n, Dec& d, Group& g, int64_t oend, int64_t H) {
    const int64_t iend = n;
    int64_t ip = 0, op = 0;
    const int64_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    uint32_t token;
    int64_t length, offset = 0, cpy = 0, lip = 0, llen = 0, ml = 0;
    int err;
    bool last = false;

    if (oend == 0) return (n == 1 && in_byte(in, 0) == 0) ? 0 : -1;
    if (n == 0) return -1;

    // The two loops of LZ4_decompress_generic as one: `safe` is the safe
    // loop (entered for good at the first fast-loop exit); every path ends at
    // `emit` with the sequence's literal (lip, llen) and match (offset, ml).
    bool safe = oend - op < kFastSafeDistance;
    for (;;) {
        token = in_byte(in, ip++);
        length = token >> 4;
        if (!safe) {
            if (length == 15) {
                length += lz_read_var(in, ip, iend - 15, true, true, err);
                if (err == 1) return -1;
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
            offset = in_le16(in, ip);
            ip += 2;
            length = token & 15;
            if (length == 15) {
                if (offset > op + H) return -1;
                length += lz_read_var(in, ip, iend - kLastLiterals + 1, true, false, err);
                if (err) return -1;
                length += kMinMatch;
                if (op + length >= oend - kFastSafeDistance) { safe = true; goto safe_match_copy; }
            } else {
                length += kMinMatch;
                if (op + length >= oend - kFastSafeDistance) { safe = true; goto safe_match_copy; }
            }
            if (offset > op + H) return -1;
            ml = length;
            goto emit;
        }
        if (length != 15 && ip < shortiend && op <= shortoend) {
            lip = ip;
            llen = length;
            op += length;
            ip += length;
            length = token & 15;
            offset = in_le16(in, ip);
            ip += 2;
            if (length != 15 && offset >= 8 && offset <= op + H) {
                ml = length + kMinMatch;
                goto emit;
            }
            goto lbl_copy_match;
        }
        if (length == 15) {
            length += lz_read_var(in, ip, iend - 15, true, true, err);
            if (err == 1) return -1;
        }
        cpy = op + length;
    safe_literal_copy:
        lip = ip;
        llen = length;
        if (cpy > oend - kMfLimit || ip + length > iend - (2 + 1 + kLastLiterals)) {
            if (ip + length != iend || cpy > oend) return -1;
            ip += length;
            op += length;
            last = true;
            goto emit;
        }
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
        // a match starting in the history (offset > op) ends by oend - 5;
        // so does one inside the block (cpy > oend - 12 -> cpy <= oend - 5)
        if (op + length > oend - kLastLiterals) return -1;
        ml = length;
    emit:
        emit_seq(d, g, in, lip, llen, (uint32_t)offset, (uint32_t)ml, !last);
        if (last) break;
        op += ml;
    }
    return op;
}

// ---------------------------------------------------------------------------
// LZ4 frame: rpo_lz4f_uncompress (oracle) — LZ4F_getFrameInfo + the
// LZ4F_decompress loop of do_uncompressed, including its output-buffer
// estimate (contentSize, or 4x the input; grown 1.5x + 1 KiB whenever a call
// returns with it full), which decides how much of a truncated frame is
// returned.  Output at d.op, which has room for the planned capacity
// (decode_capacity_dev).  Returns 0 (out_len set) or -1 where the reference
// throws.
//
// single != 0: the stream is one planned block of a block-independent frame
// (its data, then its checksum when kBlkChecksum): the header is not read,
// the block is decoded with oend = bcap and the unit ends after it.
// ---------------------------------------------------------------------------
DEV int lz4_unit(In& in, const uint8_t* s, int64_t n, Dec& d, Group& g, uint32_t single, uint32_t bcap,
                 int64_t& out_len) {
    out_len = 0;
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
        const uint32_t magic = in_le32(in, 0);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {              // skippable frame
            if (n < 8) return -1;
            pos = 4;
            if (n - pos < 4) return 0;
            const uint32_t sz = in_le32(in, pos);
            pos += 4;
            if (n - pos < (int64_t)sz) return 0;
            pos += sz;
            return pos < n ? -1 : 0;
        }
        if (magic != 0x184D2204u) return -1;                     // frameType_unknown
        const uint32_t flg = in_byte(in, 4);
        const int64_t hsize = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
        if (n < hsize) return -1;
        if ((flg >> 1) & 1) return -1;                           // reservedFlag_set
        if (((flg >> 6) & 3) != 1) return -1;                    // headerVersion_wrong
        const uint32_t bd = in_byte(in, 5);
        if ((bd >> 7) & 1) return -1;
        const uint32_t bsid = (bd >> 4) & 7;
        if (bsid < 4) return -1;                                 // maxBlockSize_invalid
        if (bd & 15) return -1;
        if (((xxh32_wave(s + 4, (uint64_t)(hsize - 5), 0) >> 8) & 0xFFu) != in_byte(in, hsize - 1)) return -1;
        linked = !((flg >> 5) & 1);
        bcs = (flg >> 4) & 1;
        ccs = (flg >> 2) & 1;
        const bool csf = (flg >> 3) & 1;
        content_size = csf ? ((uint64_t)in_le32(in, 6) | ((uint64_t)in_le32(in, 10) << 32)) : 0;
        bmax = bsid == 4 ? (64 << 10) : bsid == 5 ? (256 << 10) : bsid == 6 ? (1 << 20) : (4 << 20);
        pos = hsize;
        // compute_frame_uncompressed_size (lz4_frame_compressor.cc:115-121)
        est = (content_size == 0 || content_size > (uint64_t)n * 255) ? (uint64_t)n * 4 : content_size;
    }
    uint64_t remaining = content_size;
    int64_t out = 0;
    const uint64_t start = d.op;
    for (uint32_t blk_no = 0;; blk_no++) {
        uint32_t bh;
        if (single) {
            if (blk_no) break;
            bh = (uint32_t)(n - (bcs ? 4 : 0)) | ((single & kBlkRaw) ? 0x80000000u : 0u);
        } else {
            if (n - pos < 4) { out_len = out; return 0; }        // waiting for a block header
            bh = in_le32(in, pos);
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
                copy_direct(d, g, s + pos, k);
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
                if (in_le32(in, pos) != xxh32_wave(s + blk, (uint64_t)bsz, 0)) return -1;
                pos += 4;
            }
            continue;
        }
        if ((uint64_t)out == est) est = 1024 + ((est * 3) + 1) / 2;
        if (pos == n) { out_len = out; return 0; }
        const int64_t need = bsz + (bcs ? 4 : 0);
        if (n - pos < need) { out_len = out; return 0; }         // dstage_storeCBlock: wait
        if (bcs && in_le32(in, pos + bsz) != xxh32_wave(s + pos, (uint64_t)bsz, 0)) return -1;
        In bin;
        in_init(bin, s + pos, bsz);
        d.op = start + (uint64_t)out;
        const uint64_t tb0 = DCLK();
        const int64_t dd = lz4_block(bin, bsz, d, g, bmax, linked ? out : 0);
        DST(d, 1, 0);
#ifdef RPGPU_DSTAMPS
        d.st[5] += bin.loads;  // (reuses the flush slot: window loads)
        d.st[7] += DCLK() - tb0;  // (reuses the far-lanes slot: block cycles)
#endif
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
        dec_finish(d, g);
        wait_vm();
        if (in_le32(in, pos) != xxh32_wave(d.arena + start, (uint64_t)out, 0)) return -1;
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

// snappy_raw_checked: varint length, then DecompressAllTags over the rest:
// succeeds iff the tags end exactly at n and exactly ulen bytes come out
// (output from d.op)
DEV int snappy_raw_checked(In& in, int64_t n, Dec& d, Group& g, int64_t& out_len) {
    uint32_t ulen32;
    int64_t ip;
    if (snappy_varint_in(in, 0, n, ulen32, ip)) return -1;
    // no tag sequence expands more than 64/3 per input byte
    if ((uint64_t)ulen32 > 22ull * (uint64_t)n + 64) return -1;
    const int64_t ulen = ulen32;
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
        int64_t lip = 0, lit = 0, len = 0, off = 0;
        if ((c & 3) == 0) {
            lit = (int64_t)(c >> 2) + 1;
            if (lit >= 61) {
                const int64_t ll = lit - 60;
                uint32_t v = 0;
                for (int64_t k = 0; k < ll; k++) v |= in_byte(in, ip + k) << (8 * k);
                lit = (int64_t)v + 1;
                ip += ll;
            }
            if (n - ip < lit) return -1;       // premature end of input
            if (ulen - op < lit) return -1;    // SnappyArrayWriter::Append overflow
            lip = ip;
            ip += lit;
        } else {
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
        }
        emit_seq(d, g, in, lip, lit, (uint32_t)off, (uint32_t)len, (c & 3) != 0);
        op += lit + len;
    }
    if (op != ulen) return -1;
    out_len = ulen;
    return 0;
}

// snappy_java_compressor::uncompress: the xerial stream's chunks one after
// the other, or the raw fallback (snappy_standard_compressor: length 0 is
// an empty result, RawUncompress not called).  single: the stream is one
// planned raw chunk.
DEV int snappy_unit(In& in, const uint8_t* s, int64_t n, Dec& d, Group& g, uint32_t single, int64_t& out_len) {
    out_len = 0;
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    bool java = !single && n >= 16;
    for (int i = 0; i < 8 && java; i++) java = in_byte(in, i) == magic[i];
    int64_t pos = 0, out = 0;
    if (java) {
        const int32_t min_version = (int32_t)in_le32(in, 12);  // native little endian
        if (min_version < 1) return -1;
        pos = 16;
    } else if (!single) {
        uint32_t ulen;
        int64_t used;
        if (snappy_varint_in(in, 0, n, ulen, used)) return -1;
        if (ulen == 0) return 0;  // "empty frame"
    }
    const uint64_t start = d.op;
    for (;;) {
        const uint8_t* cs = s;
        int64_t clen = n;
        if (java) {
            if (pos == n) break;
            if (n - pos < 4) return -1;                     // consume_be_type out_of_range
            const int32_t cl = (int32_t)((in_byte(in, pos) << 24) | (in_byte(in, pos + 1) << 16) |
                                         (in_byte(in, pos + 2) << 8) | in_byte(in, pos + 3));
            pos += 4;
            if (cl < 0) return -1;
            if (n - pos < (int64_t)cl) return -1;           // consume_to out_of_range
            cs = s + pos;
            clen = cl;
            pos += cl;
        }
        In cin;
        in_init(cin, cs, clen);
        int64_t got = 0;
        d.op = start + (uint64_t)out;
        if (snappy_raw_checked(cin, clen, d, g, got)) return -1;
        out += got;
        if (!java) break;
    }
    out_len = out;
    return 0;
}

// compression::compressor::uncompress dispatch (compression/compression.cc:34-55)
// for one unit of work; output at d.op, complete and stored when it returns 0
DEV int decode_unit(int codec, const uint8_t* s, int64_t n, Dec& d, uint32_t single, uint32_t bcap,
                    int64_t& out_len) {
    out_len = 0;
    if (n == 0) return -1;
    In in;
    in_init(in, s, n);
    Group g;
    group_init(g);
    int rc = -1;
    TRACE_ITEM("  unit codec %d\n", codec);
    if (codec == RPGPU_CODEC_SNAPPY) rc = snappy_unit(in, s, n, d, g, single, out_len);
    else if (codec == RPGPU_CODEC_LZ4) rc = lz4_unit(in, s, n, d, g, single, bcap, out_len);
    TRACE_ITEM("  unit rc %d\n", rc);
    if (rc == 0) dec_finish(d, g);  // a truncated frame may have decoded past out_len: harmless
    TRACE_ITEM("  unit finished\n");
    return rc;
}

// ---------------------------------------------------------------------------
// Planning: frames whose pieces are independent and that are structurally
// complete decode to the concatenation of their pieces (or fail when any
// piece fails): that is the sequential decoder's result for such frames,
// since every flush of do_uncompressed happens while input remains.  Those
// frames are split into BlockItems at the plan rule's positions
// (decode_capacity_dev); everything else (linked LZ4 blocks, truncated or
// malformed frames, raw snappy) is decoded whole by one wave.
// ---------------------------------------------------------------------------

// Wave-uniform atomic fetch-add of `v` (lane 0's contribution; the other
// lanes add 0).  Every lane executes the atomic: written as
// `if (lane() == 0) x = atomicAdd(..)` followed by readfirstlane, the
// compiler's divergence analysis took the claimed value for a per-lane one
// and built the claim loop of k_decode_blocks with a per-lane exit whose
// lanes never all left (the decode kernel did not terminate).
DEV uint32_t wave_fetch_add(uint32_t* p, uint32_t v) {
    return uni32(atomicAdd(p, lane() == 0 ? v : 0u));
}

// reserve `nb` items (wave-uniform); UINT32_MAX when the list is full
DEV uint32_t reserve_blocks(const DeviceJob& j, uint32_t nb) {
    const uint32_t first = wave_fetch_add(&j.counters[4], nb);
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
    if (((xxh32_wave(in.src + 4, (uint64_t)(hsize - 5), 0) >> 8) & 0xFFu) != in_byte(in, hsize - 1)) return false;
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
        fp.first = fp.nb = fp.ccs = fp.ccs_val = fp.csf = 0;
        fp.content_size = 0;
        if (doff + cap > j.decoded_capacity) {
            fp.mode = 3;  // no room: DECODE_OVERFLOW
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
                const uint32_t at = wave_fetch_add(&j.counters[6], 1u);
                if (lane() == 0) j.seq_list[at] = item;
            }
        }
        if (lane() == 0) j.plans[item] = fp;
    }
}

// ---------------------------------------------------------------------------
// k_decode_blocks: persistent waves take work by one agent-scope counter:
// first the sequential frames (the longest items), then the BlockItems.
// The claim is one lane-0 atomicAdd whose result is made uniform by
// readfirstlane; `total` is read once, before the loop, so every wave
// leaves the loop when its claim passes it.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_decode_blocks(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
    // the wave's ring; readfirstlane makes its base provably wave-uniform
    lds_u8* ring = (lds_u8*)(dlds + uni32(threadIdx.x >> 6) * kRing);
    const uint32_t nseq = j.counters[6];
    const uint32_t reserved = j.counters[4];
    const uint32_t nblk = reserved < j.block_capacity ? reserved : j.block_capacity;
    const uint32_t total = nseq + nblk;
    for (;;) {
        const uint32_t item = wave_fetch_add(&j.counters[5], 1u);
        if (item >= total) break;
        // the unit: a whole frame (sequential list) or one planned piece
        uint32_t b = 0, single = 0, bcap = 0, blk = 0;
        int codec;
        uint64_t src, dst;
        int64_t n;
        if (item < nseq) {
            b = uni32(j.decode_list[uni32(j.seq_list[item])]);
            const rpgpu_batch_result* R = &j.batches[b];
            src = uni64(j.seg_off[uni32(R->segment)]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
            n = (int64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
            codec = (int)(uni32((uint32_t)(uint16_t)R->attrs) & 7u);
            dst = uni64(j.dcap[b]);
        } else {
            blk = item - nseq;
            const BlockItem it = j.blocks[blk];
            const uint32_t kind = uni32(it.kind);
            src = uni64(it.src);
            dst = uni64(it.dst);
            bcap = uni32(it.cap);
            codec = (kind & kBlkSnappy) ? RPGPU_CODEC_SNAPPY : RPGPU_CODEC_LZ4;
            single = kind | 0x100u;
            n = (int64_t)uni32(it.csize) + ((kind & kBlkChecksum) ? 4 : 0);
        }
        Dec d;
        dec_init(d, j.decoded, j.decoded_capacity, ring, dst);
        int64_t got = 0;
        TRACE_ITEM("item %u/%u wg %u w %u codec %d single %x n %lld src %llu dst %llu cap %u\n", item, total, blockIdx.x,
                   threadIdx.x >> 6, codec, single, (long long)n, (unsigned long long)src, (unsigned long long)dst, bcap);
        const uint64_t it0 = DCLK();
        const int rc = decode_unit(codec, j.data + src, n, d, single, bcap, got);
        TRACE_ITEM("done %u rc %d got %lld\n", item, rc, (long long)got);
#ifdef RPGPU_DSTAMPS
        {
            const uint64_t dt = DCLK() - it0;
            // kinds: 0 whole frames, 1 LZ4 blocks, 2 raw blocks, 3 snappy chunks
            const int kind = item < nseq ? 0 : (codec == RPGPU_CODEC_SNAPPY ? 3 : ((single & kBlkRaw) ? 2 : 1));
            if (lane() == 0) {
                atomicAdd(&g_dst[2 * kind], (unsigned long long)dt);
                atomicAdd(&g_dst[2 * kind + 1], 1ull);
                atomicMax(&g_dst[8 + kind], (unsigned long long)dt);
                for (int i = 0; i < 8; i++) atomicAdd(&g_dst[16 + i], (unsigned long long)d.st[i]);
                atomicAdd(&g_dst[24 + kind], (unsigned long long)got);
            }
        }
#endif
        if (lane() == 0) {
            if (item < nseq) {
                if (rc == 0) {
                    rpgpu_batch_result* R = &j.batches[b];
                    R->flags = R->flags | RPGPU_F_CODEC_OK;
                    R->decoded_len = (uint32_t)got;
                }
            } else {
                j.blocks[blk].out = (int32_t)(rc == 0 ? got : -1);
            }
        }
    }
}

#ifdef RPGPU_DSTAMPS
__global__ void k_print_dstamps() {
    const char* kn[4] = {"frames", "lz4 blocks", "raw blocks", "snappy chunks"};
    for (int k = 0; k < 4; k++)
        printf("RPGPU_DSTAMPS %s: n=%llu cycles=%llu avg=%.0f max=%llu bytes=%llu\n", kn[k], g_dst[2 * k + 1], g_dst[2 * k],
               g_dst[2 * k + 1] ? (double)g_dst[2 * k] / (double)g_dst[2 * k + 1] : 0.0, g_dst[8 + k], g_dst[24 + k]);
    printf("RPGPU_DSTAMPS seqs=%llu groups=%llu group_cycles=%llu serial=%llu far_groups=%llu window_loads=%llu "
           "ring_lanes=%llu lz4_block_cycles=%llu\n", g_dst[16], g_dst[17], g_dst[18], g_dst[19], g_dst[20], g_dst[21], g_dst[22],
           g_dst[23]);
    for (int i = 0; i < 32; i++) g_dst[i] = 0;
}
#endif

// one wave per block-parallel frame: all pieces decoded, moved together
// when an earlier one came out short, content size / checksum checked
__global__ __launch_bounds__(256) void k_decode_finish(DeviceJob j) {
    const uint32_t count = j.counters[2];
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + uni32(threadIdx.x >> 6); item < count; item += nw) {
        const FramePlan fp = j.plans[item];
        const uint32_t mode = uni32(fp.mode);
        const uint32_t b = uni32(j.decode_list[item]);
        rpgpu_batch_result* R = &j.batches[b];
        if (mode == 3) {
            if (lane() == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
            continue;
        }
        if (mode == 0) continue;
        const uint32_t first = uni32(fp.first), nb = uni32(fp.nb);
        const uint64_t d0 = uni64(j.dcap[b]);
        bool ok = true;
        uint64_t run = d0;  // where the next piece belongs
        for (uint32_t k = 0; k < nb; k++) {
            const BlockItem it = j.blocks[first + k];
            const int32_t out = (int32_t)uni32((uint32_t)it.out);
            if (out < 0) { ok = false; break; }
            const uint64_t at = uni64(it.dst);
            if (at < run) { ok = false; break; }  // a piece longer than planned (cannot happen: out <= cap)
            if (at != run) {
                // forward move to a lower address in 1 KiB steps (each step
                // loads before it stores; the gap is at least the shortfall)
                uint8_t* dd = j.decoded;
                const int64_t gap = (int64_t)(at - run);
                const int64_t step = gap < 64 ? gap : 64;
                for (int64_t o = 0; o < out; o += step) {
                    const int64_t k2 = o + lane();
                    uint8_t v = 0;
                    if (lane() < step && k2 < out) v = dd[at + k2];
                    wait_vm();
                    if (lane() < step && k2 < out) dd[run + k2] = v;
                    wait_vm();
                }
            }
            run += (uint64_t)out;
        }
        const uint64_t total = run - d0;
        if (ok && mode == 1) {
            if (uni32(fp.csf) && total != uni64(fp.content_size)) ok = false;  // frameSize_wrong
            if (ok && uni32(fp.ccs)) {
                wait_vm();
                if (xxh32_wave(j.decoded + d0, total, 0) != uni32(fp.ccs_val)) ok = false;
            }
        }
        if (lane() == 0 && ok) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
        }
    }
}

__global__ __launch_bounds__(64) void k_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst,
                                                       uint64_t cap, int64_t* res) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
    Dec d;
    dec_init(d, dst, cap, (lds_u8*)dlds, 0);
    int64_t got = 0;
    const int rc = decode_unit(codec, src, (int64_t)n, d, 0, 0, got);
    if (lane() == 0) {
        res[0] = rc;
        res[1] = got;
    }
}

static void set_lds_attrs() {
    static bool done = false;
    if (done) return;
    (void)hipFuncSetAttribute((const void*)k_decode_blocks, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kDecWaves * kRing));
    (void)hipFuncSetAttribute((const void*)k_uncompress_one, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRing);
    done = true;
}

hipError_t launch_decode(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_decode_blocks(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    set_lds_attrs();
    hipLaunchKernelGGL(k_decode_blocks, dim3(grid), dim3(64 * kDecWaves), kDecWaves * kRing, s, j);
#ifdef RPGPU_DSTAMPS
    hipLaunchKernelGGL(k_print_dstamps, dim3(1), dim3(1), 0, s);
#endif
    return hipGetLastError();
}

hipError_t launch_decode_finish(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    hipLaunchKernelGGL(k_decode_finish, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, int64_t* res,
                                 hipStream_t s) {
    set_lds_attrs();
    hipLaunchKernelGGL(k_uncompress_one, dim3(1), dim3(64), kRing, s, codec, src, n, dst, cap, res);
    return hipGetLastError();
}

}  // namespace rp
