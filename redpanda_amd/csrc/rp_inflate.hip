// rp_inflate.hip — gzip_compressor::uncompress on the device
// (compression/internal/gzip_compressor.cc:161-230): zlib 1.2.11 inflate
// with inflateInit2(15 + 32) (a gzip member or a zlib stream), as the
// reference's loop drives it.  The accept/reject rules are the oracle's
// restatement (oracle/rp_oracle.c rpo_gzip_uncompress), which is pinned
// against zlib itself:
//   * an error anywhere before the end of the first member rejects;
//   * input that runs out is not an error: the output is what inflate could
//     decode from the bytes present (a code decodes once all its bits are
//     there; stored blocks byte by byte);
//   * bytes after the first member are ignored.
//
// The reference decodes every payload twice (buffer_for_input sizes the
// output with a pass through a 512-byte buffer, then decodes into a buffer of
// exactly that size).  The engine does the same: k_inflate_plan runs the
// decoder without output to size each member's arena slot before the slot
// scan, and k_inflate decodes into the slot.
//
// Execution model: one wave per member.  Deflate is a serial bit stream, so
// the decoder state is wave-uniform (scalar registers); the wave's lanes
// build the Huffman codes (ballots over the code lengths), find a code's
// length with one compare per lane (lane L holds the left-justified limit of
// the length-L codes: canonical codes make that the whole decode), copy
// matches 64 bytes per step, and flush, CRC32 and Adler-32 1 KiB of output
// per step.  Output goes through a 32 KiB LDS ring (deflate distances reach
// 32768 back) and leaves in coalesced 16-byte stores.
// Integer work only: no MFMA.
//
// zstd (stream_zstd::do_uncompress, compression/stream_zstd.cc:152-178) runs
// here too, on the same member list, scratch slots and passes: the decoder
// logic is rp_zstd_core.h (libzstd 1.4.8's acceptance rules as the
// reference's loop sees them), instantiated over ZDev below.
#include "rp_device.h"

#define ZS_FN DEV
#define ZS_CONST static __constant__
#ifdef RPGPU_ZSTAMPS  // diagnostic build: wall-clock totals per decoder phase (scripts/build_exp.py)
#define ZS_PROF(k, stmt)                        \
    {                                           \
        const uint64_t t0_ = wall_clock64();    \
        stmt;                                   \
        e.prof[k] += wall_clock64() - t0_;      \
    }
__device__ unsigned long long g_zst[16];  // [0..7] the wave decoder, [8..15] the lane parse
#endif
#include "rp_zstd_core.h"

namespace rp {

typedef __attribute__((address_space(3))) uint8_t inf_lds_u8;

constexpr uint32_t kInfRing = 32768, kInfMask = kInfRing - 1;
// per-wave LDS: the code tables (symbols in canonical order, code lengths of
// a dynamic header) and, for the decode pass, the output ring
struct InfTabs {
    uint16_t lsym[288];
    uint16_t dsym[32];
    uint16_t csym[19];
    uint16_t pad0;
    uint8_t lens[320];
    uint32_t crc_tab[256];  // CRC32 (IEEE, reflected 0xEDB88320) byte table
    // root tables of the literal/length and distance codes: the next 9
    // stream bits -> symbol | length << 9 for codes of at most 9 bits, 0 for
    // a longer (or invalid) code
    uint16_t lroot[512], droot[512];
};
constexpr uint32_t kInfTabBytes = (sizeof(InfTabs) + 15u) & ~15u;
constexpr uint32_t kInfLdsDecode = kInfRing + kInfTabBytes;

// x^(2^k) mod the reflected CRC32 polynomial 0xEDB88320 (period 32)
static __constant__ uint32_t kX2nIeee[32] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0xEDB88320u, 0xB1E6B092u, 0xA06A2517u,
    0xED627DAEu, 0x88D14467u, 0xD7BBFE6Au, 0xEC447F11u, 0x8E7EA170u, 0x6427800Eu, 0x4D47BAE0u, 0x09FE548Fu,
    0x83852D0Fu, 0x30362F1Au, 0x7B5A9CC3u, 0x31FEC169u, 0x9FEC022Au, 0x6C8DEDC4u, 0x15D6874Du, 0x5FDE7A4Eu,
    0xBAD90E37u, 0x2E4E5EEFu, 0x4EABA214u, 0xA8A472C0u, 0x429A969Eu, 0x148D302Au, 0xC40BA6D0u, 0xC4E22C3Cu};

DEV uint32_t ieee_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
// x^(8 n) mod P; x2n = kX2nIeee held one entry per lane (lane k: x^(2^k)):
// a constant-memory table read per step is a vector load and a wait each
// n may differ per lane: the loop runs wave-uniformly (a lane that has
// finished its bits must still be there when the table is read across lanes)
DEV uint32_t ieee_xpow8(uint32_t n, uint32_t x2n) {
    uint32_t p = 1u << 31;
    for (uint32_t i = 0; i < 32; i++) {
        if (__ballot((n >> i) != 0) == 0) break;
        const uint32_t f = rl(x2n, (int)((3 + i) & 31u));
        if ((n >> i) & 1) p = ieee_mulmod(f, p);
    }
    return p;
}

// deflate's length / distance bases and extra bits (RFC 1951 3.2.5)
static __constant__ uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                              35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static __constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                              3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static __constant__ uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                               193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
                                               6145, 8193, 12289, 16385, 24577};
static __constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                               6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static __constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ---------------------------------------------------------------------------
// Input: the member's bytes through a 512-byte window held one dword per
// lane (two rows); reads are wave-uniform.  Bytes past the member read as 0.
// ---------------------------------------------------------------------------
struct InfIn {
    const uint8_t* src;  // the member's first byte
    const uint8_t* al;   // src rounded down to 4 bytes: window dwords are read from here
    uint64_t n, nphys;   // member bytes; n + mis
    uint32_t mis;        // src & 3
    uint64_t base;       // window start (4-aligned offset from al)
    uint32_t w0, w1;     // lane l: dwords base + 4 l, base + 256 + 4 l
};

DEV InfIn inf_in(const uint8_t* src, uint64_t n) {
    InfIn in;
    in.src = src;
    in.mis = (uint32_t)((uintptr_t)src & 3);
    in.al = src - in.mis;
    in.n = n;
    in.nphys = n + in.mis;
    in.base = ~0ull >> 1;
    in.w0 = in.w1 = 0;
    return in;
}
// an aligned dword that starts inside the member never crosses a page, so
// reading its bytes past the member end is safe (they are masked)
DEV uint32_t inf_ld(const InfIn& in, uint64_t a) { return a < in.nphys ? *(const uint32_t*)(in.al + a) : 0u; }
DEV uint32_t inf_dw(InfIn& in, uint64_t a) {  // a: 4-aligned, wave-uniform
    uint64_t o = a - in.base;
    if (a < in.base || o >= 512) {
        in.base = a;
        in.w0 = inf_ld(in, a + 4u * lane());
        in.w1 = inf_ld(in, a + 256u + 4u * lane());
        o = 0;
    }
    const int li = (int)((o >> 2) & 63);
    return o < 256 ? rl(in.w0, li) : rl(in.w1, li);
}
DEV uint32_t inf_byte(InfIn& in, uint64_t i) {
    if (i >= in.n) return 0u;
    const uint64_t p = i + in.mis;
    return (inf_dw(in, p & ~3ull) >> (8u * (uint32_t)(p & 3))) & 0xFFu;
}
// 32 bits of the stream from bit position bp (LSB first), zero past the end
DEV uint32_t inf_peek(InfIn& in, uint64_t bp) {
    const uint64_t pb = bp + 8ull * in.mis, b = pb >> 3, a = b & ~3ull;
    const uint32_t sh = (uint32_t)(((b & 3) << 3) | (pb & 7));
    const uint32_t d0 = inf_dw(in, a), d1 = inf_dw(in, a + 4);
    const uint32_t v = sh ? __builtin_amdgcn_alignbit(d1, d0, sh) : d0;
    const uint64_t avail = in.n * 8 - bp;
    return avail < 32 ? v & ((1u << avail) - 1u) : v;
}
// 64 bits from bp (two peeks)
DEV uint64_t inf_peek64(InfIn& in, uint64_t bp) {
    return (uint64_t)inf_peek(in, bp) | ((uint64_t)(bp + 32 < in.n * 8 ? inf_peek(in, bp + 32) : 0u) << 32);
}

// ---------------------------------------------------------------------------
// Canonical Huffman code: lane L (1..15) holds the left-justified 15-bit
// limit of the codes of length <= L, the first code of length L and the
// canonical index of that code; symbols in LDS in canonical order.
// ---------------------------------------------------------------------------
struct InfCode {
    uint32_t lim, first, offs;  // lane L
};

// inflate_table acceptance (zlib 1.2.11 inftrees.c, the oracle's
// huff_build): over-subscribed -> error; incomplete -> error unless a single
// 1-bit literal/length or distance code; no codes at all -> an empty code
// (any decode reports an invalid code after one bit).  type: 0 code-length
// code, 1 literal/length, 2 distance.  Returns 0 ok, -1 error.
DEV int inf_build(const inf_lds_u8* lens, uint32_t m, int type, uint16_t* syms, InfCode& c) {
    const uint32_t l = lane();
    uint32_t cnt = 0;
    for (uint32_t ch = 0; ch < m; ch += 64) {
        const uint32_t s = ch + l;
        const uint32_t len = s < m ? (uint32_t)lens[s] : 0u;
#pragma unroll
        for (uint32_t L = 1; L <= 15; L++) {
            const uint32_t k = (uint32_t)__builtin_popcountll(__ballot(len == L));
            if (l == L) cnt += k;
        }
    }
    int left = 1;
    uint32_t code = 0, offs = 0, max = 0;
    c.lim = c.first = c.offs = 0;
    for (uint32_t L = 1; L <= 15; L++) {
        const uint32_t cL = rl(cnt, (int)L);
        left = 2 * left - (int)cL;
        if (left < 0) return -1;  // over-subscribed
        if (l == L) {
            c.first = code;
            c.offs = offs;
            c.lim = (code + cL) << (15 - L);
        }
        code = (code + cL) << 1;
        offs += cL;
        if (cL) max = L;
    }
    if (max == 0) {  // no codes: every lookup is the invalid entry
        c.lim = 0;
        return 0;
    }
    if (left > 0 && (type == 0 || max != 1)) return -1;  // incomplete
    // symbols in canonical order: (length, value), ranks by ballot
    uint32_t next = c.offs;  // lane L: next slot for length L
    for (uint32_t ch = 0; ch < m; ch += 64) {
        const uint32_t s = ch + l;
        const uint32_t len = s < m ? (uint32_t)lens[s] : 0u;
        uint32_t pos = 0;
#pragma unroll
        for (uint32_t L = 1; L <= 15; L++) {
            const uint64_t mask = __ballot(len == L);
            if (len == L) pos = rl(next, (int)L) + (uint32_t)__builtin_popcountll(mask & ((1ull << l) - 1ull));
            if (l == L) next += (uint32_t)__builtin_popcountll(mask);
        }
        if (len) syms[pos] = (uint16_t)s;
    }
    return 0;
}

// One symbol from the 32 peeked bits v, `avail` bits left in the stream:
// 1 decoded (sym, len), 0 the code needs bits past the end (truncated), -1
// an invalid code (one bit).  The shortest code matching the zero-extended
// bits decodes once all its bits are present: zlib's table lookup.
DEV int inf_decode(uint32_t v, uint64_t avail, const InfCode& c, const uint16_t* syms, uint32_t& sym, uint32_t& len) {
    const uint32_t r = __builtin_bitreverse32(v) >> 17;  // next 15 bits, first bit most significant
    const uint64_t m = __ballot(r < c.lim);
    if (m == 0) return avail >= 1 ? -1 : 0;
    const uint32_t L = (uint32_t)__builtin_ctzll(m);
    if (L > avail) return 0;
    const uint32_t idx = rl(c.offs, (int)L) + (r >> (15 - L)) - rl(c.first, (int)L);
    sym = uni32((uint32_t)syms[idx]);
    len = L;
    return 1;
}

// the root table of a built code (lanes fill 8 entries each): entry idx =
// the next 9 stream bits; the shortest length L <= 9 whose left-justified
// limit exceeds them gives the symbol (inf_decode's rule on a prefix)
DEV void inf_root(const InfCode& c, const uint16_t* syms, uint16_t* root) {
    const uint32_t l = lane();
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t idx = 64u * k + l;
        const uint32_t r9 = __builtin_bitreverse32(idx) >> 23;  // first stream bit most significant
        const uint32_t r15 = r9 << 6;
        uint32_t e = 0;
        for (uint32_t L = 1; L <= 9; L++) {
            const uint32_t lim = rl(c.lim, (int)L);
            if (e == 0 && r15 < lim) {
                const uint32_t sidx = rl(c.offs, (int)L) + (r9 >> (9 - L)) - rl(c.first, (int)L);
                e = (uint32_t)syms[sidx] | (L << 9);
            }
        }
        root[idx] = (uint16_t)e;
    }
}

// ---------------------------------------------------------------------------
// Output (decode pass): ring in LDS, 1 KiB chunks flushed to the slot with
// their CRC32 / Adler-32 folded into the running check.
// ---------------------------------------------------------------------------
struct InfOut {
    inf_lds_u8* ring;
    const uint32_t* tab;  // CRC32 byte table (LDS)
    uint8_t* dst;         // slot start (16-byte aligned)
    uint64_t flushed;     // bytes flushed (multiple of 1024 until the end)
    uint32_t crc;         // raw register (init 0xFFFFFFFF)
    uint32_t ada, adb;    // Adler-32 sums
    bool gz;
    uint32_t x2n;         // lane k: x^(2^k) mod P
    uint32_t lane_mul;    // lane l: x^(8 (1024 - 16 (l + 1))): its 16 bytes moved to a full chunk's end
    uint32_t chunk_mul;   // x^(8 * 1024)
    uint64_t cap;         // bytes dst holds (16-byte multiple); past it the pass only counts
    bool over;            // the output outgrew dst: no more stores, no check
};

// flush output bytes [o.flushed, o.flushed + len) (len <= 1024, the start
// 1 KiB aligned) from the ring and fold them into the check
DEV void inf_flush(InfOut& o, uint32_t len) {
    // the slot is full: the bytes are no longer stored, but the check still
    // folds them in (a member whose check then fails is rejected by this pass
    // and needs no second one)
    if (o.over || o.flushed + len > o.cap) o.over = true;
    const uint32_t l = lane();
    const uint32_t at = (uint32_t)(o.flushed & kInfMask) + 16u * l;
    const uint32_t t = 16u * l < len ? min(16u, len - 16u * l) : 0u;  // this lane's bytes
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t) {
        v = *(const uint4*)(o.ring + at);
        if (!o.over) *(uint4*)(o.dst + o.flushed + 16u * l) = v;  // the slot is rounded up to 16: a whole piece fits
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (o.gz) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++)
            if (k < t) c = o.tab[(c ^ (w[k >> 2] >> (8 * (k & 3)))) & 0xFFu] ^ (c >> 8);
        // lane l's raw CRC moved to the end of the piece: x^(8 (len - 16 l - t))
        const bool full = len == 1024u;
        uint32_t x = t ? ieee_mulmod(full ? o.lane_mul : ieee_xpow8(len - 16u * l - t, o.x2n), c) : 0u;
        x = wave_xor(x);
        o.crc = ieee_mulmod(full ? o.chunk_mul : ieee_xpow8(len, o.x2n), o.crc) ^ uni32(x);
    } else {
        uint32_t s1 = 0, s2 = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++)
            if (k < t) {
                const uint32_t d = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
                s1 += d;
                s2 += (len - 16u * l - k) * d;  // weight: bytes from it to the chunk end
            }
        for (int off = 32; off > 0; off >>= 1) {
            s1 += __shfl_xor(s1, off, 64);
            s2 += __shfl_xor(s2, off, 64);
        }
        s1 = uni32(s1);
        s2 = uni32(s2);
        o.adb = (uint32_t)(((uint64_t)o.adb + (uint64_t)len * o.ada + s2) % 65521u);
        o.ada = (o.ada + s1) % 65521u;
    }
    o.flushed += len;
}

// every complete 1 KiB chunk below op
DEV void inf_flush_upto(InfOut& o, uint64_t op) {
    while ((op >> 10) > (o.flushed >> 10)) inf_flush(o, 1024u);
}

// match: ml bytes from dist back (dist <= op, checked).  A match overlapping
// its own output (dist < ml) repeats the dist bytes before it: byte k is
// k mod dist into them, by a multiply with the rounded-up reciprocal (exact
// for k < 2^32 / dist); every read is issued before any write.
DEV void inf_copy(InfOut& o, uint64_t op, uint32_t dist, uint32_t ml) {
    const uint32_t l = lane();
    const bool rep = dist < ml;
    const uint64_t mg = rep ? 0xFFFFFFFFull / dist + 1ull : 0ull;
    const uint32_t n = (ml + 63) >> 6;  // deflate: ml <= 258, at most 5 rows
    uint32_t b[5];
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t k = 64u * i + l;
        const uint32_t x = rep ? k - (uint32_t)(((uint64_t)k * mg) >> 32) * dist : k;
        b[i] = (i < n && k < ml) ? (uint32_t)o.ring[((uint32_t)(op - dist) + x) & kInfMask] : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t k = 64u * i + l;
        if (i < n && k < ml) o.ring[(uint32_t)(op + k) & kInfMask] = (uint8_t)b[i];
    }
}

// ---------------------------------------------------------------------------
// The member decoder.  kWrite = false: the sizing pass (no output, no data
// check); true: the decode pass into `o`.  Returns -1 rejected, 0 accepted;
// `total` = bytes produced.
// ---------------------------------------------------------------------------
// deflate's length / distance tables held one symbol per lane (base | extra
// << 16): a v_readlane per symbol instead of a vector load and its wait
struct InfSymTabs {
    uint32_t len, dist;
};
DEV InfSymTabs inf_sym_tabs() {
    const uint32_t l = lane();
    InfSymTabs t;
    t.len = l < 29 ? (uint32_t)kLenBase[l] | ((uint32_t)kLenExtra[l] << 16) : 0u;
    t.dist = l < 30 ? (uint32_t)kDistBase[l] | ((uint32_t)kDistExtra[l] << 16) : 0u;
    return t;
}

template <bool kWrite>
DEV int inflate_member(InfIn& in, InfTabs* T, InfOut& o, const InfSymTabs& ST, uint64_t& total) {
    const uint32_t l = lane();
    const uint64_t nbits = in.n * 8;
    uint64_t bp = 0, op = 0;
    total = 0;
    bool gz = false;
    uint32_t v, sym, len;
    InfCode LC, DC, CC;
#define NEED(k) \
    if (nbits - bp < (uint64_t)(k)) goto done
    // HEAD
    NEED(16);
    v = inf_peek(in, bp);
    if ((v & 0xFFFFu) == 0x8b1fu) {
        gz = true;
        // FLAGS, TIME, OS, EXLEN, EXTRA, NAME, COMMENT, HCRC
        uint32_t hc = 0xFFFFFFFFu;  // header CRC register (FHCRC)
        auto hcrc = [&](uint64_t from, uint64_t cnt) __attribute__((always_inline)) {
            for (uint64_t i = 0; i < cnt; i++) hc = T->crc_tab[(hc ^ inf_byte(in, from + i)) & 0xFFu] ^ (hc >> 8);
        };
        hcrc(0, 2);
        bp = 16;
        NEED(16);
        const uint32_t flags = inf_peek(in, bp) & 0xFFFFu;
        if ((flags & 0xFFu) != 8u) return -1;  // unknown compression method
        if (flags & 0xe000u) return -1;        // unknown header flags set
        const bool fh = (flags & 0x0200u) != 0;
        if (fh) hcrc(2, 2);
        bp = 32;
        NEED(32);
        if (fh) hcrc(4, 4);
        bp = 64;
        NEED(16);
        if (fh) hcrc(8, 2);
        bp = 80;
        if (flags & 0x0400u) {
            NEED(16);
            const uint64_t xlen = inf_peek(in, bp) & 0xFFFFu;
            if (fh) hcrc(10, 2);
            bp += 16;
            const uint64_t have = in.n - (bp >> 3), copy = xlen < have ? xlen : have;
            if (fh) hcrc(bp >> 3, copy);
            bp += 8 * copy;
            if (copy < xlen) goto done;
        }
        for (uint32_t f = 0x0800u; f <= 0x1000u; f <<= 1) {
            if (!(flags & f)) continue;
            uint64_t p = bp >> 3;
            if (p >= in.n) goto done;
            const uint64_t start = p;
            uint32_t c;
            do c = inf_byte(in, p++); while (c && p < in.n);
            if (fh) hcrc(start, p - start);
            bp = 8 * p;
            if (c) goto done;
        }
        if (fh) {
            NEED(16);
            if ((inf_peek(in, bp) & 0xFFFFu) != (~hc & 0xFFFFu)) return -1;  // header crc mismatch
            bp += 16;
        }
    } else {
        const uint32_t hold = v & 0xFFFFu;
        if ((((hold & 0xFFu) << 8) + (hold >> 8)) % 31u) return -1;  // incorrect header check
        if ((hold & 0x0Fu) != 8u) return -1;                         // unknown compression method
        if (((hold >> 4) & 0x0Fu) + 8u > 15u) return -1;             // invalid window size
        bp = 16;
        if (hold & 0x2000u) {  // FDICT: DICTID, then Z_NEED_DICT
            NEED(32);
            return -1;
        }
    }
    if (kWrite) {
        o.gz = gz;
        o.crc = 0xFFFFFFFFu;
        o.ada = 1;
        o.adb = 0;
    }
    // blocks
    for (;;) {
        NEED(3);
        v = inf_peek(in, bp);
        const uint32_t last = v & 1u, type = (v >> 1) & 3u;
        bp += 3;
        if (type == 0) {  // STORED
            bp = (bp + 7) & ~7ull;
            NEED(32);
            v = inf_peek(in, bp);
            if ((v & 0xFFFFu) != ((v >> 16) ^ 0xFFFFu)) return -1;  // invalid stored block lengths
            bp += 32;
            uint64_t length = v & 0xFFFFu;
            const uint64_t p = bp >> 3, have = in.n - p, copy = length < have ? length : have;
            if (kWrite) {
                // 1 KiB per step: lane l's 16 bytes, byte loads (any alignment)
                for (uint64_t c = 0; c < copy; c += 1024) {
                    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t k = 0; k < 16; k++) {
                        const uint64_t i = c + 16u * l + k;
                        if (i < copy) w[k >> 2] |= (uint32_t)in.src[p + i] << (8 * (k & 3));
                    }
#pragma unroll
                    for (uint32_t k = 0; k < 16; k++) {
                        const uint64_t i = c + 16u * l + k;
                        if (i < copy) o.ring[(uint32_t)(op + i - c) & kInfMask] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
                    }
                    const uint64_t step = copy - c < 1024 ? copy - c : 1024;
                    op += step;
                    inf_flush_upto(o, op);
                }
            } else {
                op += copy;
            }
            bp += 8 * copy;
            if (copy < length) goto done;
        } else if (type == 3) {
            return -1;  // invalid block type
        } else {
            inf_lds_u8* lens = (inf_lds_u8*)T->lens;
            if (type == 1) {  // fixed codes
                for (uint32_t s = l; s < 288; s += 64) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                inf_build(lens, 288, 1, T->lsym, LC);
                if (l < 32) lens[l] = 5;
                inf_build(lens, 32, 2, T->dsym, DC);
                inf_root(LC, T->lsym, T->lroot);
                inf_root(DC, T->dsym, T->droot);
            } else {  // TABLE
                NEED(14);
                v = inf_peek(in, bp);
                const uint32_t nlen = (v & 31u) + 257, ndist = ((v >> 5) & 31u) + 1, ncode = ((v >> 10) & 15u) + 4;
                bp += 14;
                if (nlen > 286 || ndist > 30) return -1;  // too many length or distance symbols
                // code-length code lengths (3 bits each, permuted)
                const uint64_t need = 3ull * ncode;
                const bool all = nbits - bp >= need;
                const uint32_t got = all ? ncode : (uint32_t)((nbits - bp) / 3);
                // lane i < 19: its code length (0 when past ncode); 57 bits at most
                const uint64_t w57 = inf_peek64(in, bp);
                const uint32_t cl = l < got ? (uint32_t)(w57 >> (3 * (l < 19 ? l : 0))) & 7u : 0u;
                if (!all) goto done;
                bp += need;
                if (l < 19) lens[kClenOrder[l]] = (uint8_t)(l < ncode ? cl : 0u);
                if (inf_build(lens, 19, 0, T->csym, CC)) return -1;  // invalid code lengths set
                uint32_t have = 0;
                while (have < nlen + ndist) {
                    v = inf_peek(in, bp);
                    const int r = inf_decode(v, nbits - bp, CC, T->csym, sym, len);
                    if (r == 0) goto done;
                    if (r < 0) { sym = 0; len = 1; }  // zlib's CODELENS reads an invalid entry as length 0
                    bp += len;
                    if (sym < 16) {
                        if (l == 0) lens[have] = (uint8_t)sym;
                        have++;
                        continue;
                    }
                    uint32_t rep = 0, cnt;
                    v = inf_peek(in, bp);
                    if (sym == 16) {
                        NEED(2);
                        if (have == 0) return -1;  // invalid bit length repeat
                        rep = uni32((uint32_t)lens[have - 1]);
                        cnt = 3 + (v & 3u);
                        bp += 2;
                    } else if (sym == 17) {
                        NEED(3);
                        cnt = 3 + (v & 7u);
                        bp += 3;
                    } else {
                        NEED(7);
                        cnt = 11 + (v & 127u);
                        bp += 7;
                    }
                    if (have + cnt > nlen + ndist) return -1;  // invalid bit length repeat
                    if (l < cnt) lens[have + l] = (uint8_t)rep;  // cnt <= 138: lanes, twice
                    if (l + 64 < cnt) lens[have + l + 64] = (uint8_t)rep;
                    if (l + 128 < cnt) lens[have + l + 128] = (uint8_t)rep;
                    have += cnt;
                }
                if (lens[256] == 0) return -1;                             // invalid code -- missing end-of-block
                if (inf_build(lens, nlen, 1, T->lsym, LC)) return -1;      // invalid literal/lengths set
                if (inf_build(lens + nlen, ndist, 2, T->dsym, DC)) return -1;  // invalid distances set
                inf_root(LC, T->lsym, T->lroot);
                inf_root(DC, T->dsym, T->droot);
            }
            // fast loop: far from the end of the member every code's bits are
            // present, so no truncation test; a 64-bit bit buffer refilled a
            // dword at a time from the window, codes of <= 9 bits from the
            // root tables, longer ones by the limit compare.  It hands over to
            // the exact loop below near the end (and at the block end).
            if (kWrite) {
                const uint64_t pb = bp + 8ull * in.mis;
                uint64_t pq = (pb >> 5) << 2;                 // next dword to load (physical byte offset)
                uint32_t sh = (uint32_t)(pb & 31);
                uint64_t bb = (uint64_t)(inf_dw(in, pq) >> sh);
                uint32_t bc = 32 - sh;
                pq += 4;
                bool eob = false;
                // literals gathered one per lane, written to the ring 64 at a
                // time (a single-lane LDS store per literal was an exec-mask
                // round trip each)
                uint32_t lb = 0, nl = 0;
                auto spill = [&]() __attribute__((always_inline)) {
                    if (nl) {
                        if (l < nl) o.ring[(uint32_t)(op + l) & kInfMask] = (uint8_t)lb;
                        op += nl;
                        nl = 0;
                        inf_flush_upto(o, op);
                    }
                };
                // safe while the next two refills stay inside the member
                while (pq + 12 <= in.nphys) {
                    while (bc <= 32) {
                        bb |= (uint64_t)inf_dw(in, pq) << bc;
                        bc += 32;
                        pq += 4;
                    }
                    uint32_t e = uni32((uint32_t)T->lroot[(uint32_t)bb & 511u]);
                    if (e == 0) {  // a code longer than 9 bits
                        const int r = inf_decode((uint32_t)bb, 64, LC, T->lsym, sym, len);
                        if (r < 0) return -1;  // invalid literal/length code
                        e = sym | (len << 9);
                    }
                    sym = e & 511u;
                    len = e >> 9;
                    bb >>= len;
                    bc -= len;
                    if (sym < 256) {
#ifdef RPGPU_GZ_NOOUT  // diagnostic variant: decode only (the check then fails), to time the symbol chain
                        op++;
                        continue;
#endif
                        lb = l == nl ? sym : lb;
                        if (++nl == 64) spill();
                        continue;
                    }
                    spill();
                    if (sym == 256) { eob = true; break; }
                    if (sym > 285) return -1;  // invalid literal/length code
                    const uint32_t lt = rl(ST.len, (int)(sym - 257));
                    const uint32_t le = lt >> 16;
                    const uint32_t ml = (lt & 0xFFFFu) + ((uint32_t)bb & ((1u << le) - 1u));
                    bb >>= le;
                    bc -= le;
                    if (bc <= 32) {  // the distance code and its extra bits need <= 28
                        bb |= (uint64_t)inf_dw(in, pq) << bc;
                        bc += 32;
                        pq += 4;
                    }
                    e = uni32((uint32_t)T->droot[(uint32_t)bb & 511u]);
                    if (e == 0) {
                        const int r = inf_decode((uint32_t)bb, 64, DC, T->dsym, sym, len);
                        if (r < 0) return -1;  // invalid distance code
                        e = sym | (len << 9);
                    }
                    sym = e & 511u;
                    len = e >> 9;
                    if (sym > 29) return -1;  // invalid distance code
                    bb >>= len;
                    bc -= len;
                    const uint32_t dt = rl(ST.dist, (int)sym);
                    const uint32_t de = dt >> 16;
                    const uint32_t dist = (dt & 0xFFFFu) + ((uint32_t)bb & ((1u << de) - 1u));
                    bb >>= de;
                    bc -= de;
                    if (dist > op) return -1;  // invalid distance too far back
#ifdef RPGPU_GZ_NOOUT
                    op += ml;
                    continue;
#endif
                    inf_copy(o, op, dist, ml);
                    op += ml;
                    inf_flush_upto(o, op);
                }
                spill();
                bp = 8 * (pq - in.mis) - bc;  // the bits consumed
                if (eob) {
                    if (last) break;
                    continue;
                }
            }
            // LEN .. MATCH
            for (;;) {
                v = inf_peek(in, bp);
                int r = inf_decode(v, nbits - bp, LC, T->lsym, sym, len);
                if (r == 0) goto done;
                if (r < 0 || sym > 285) return -1;  // invalid literal/length code
                bp += len;
                if (sym < 256) {
                    if (kWrite) {
                        if (l == 0) o.ring[(uint32_t)op & kInfMask] = (uint8_t)sym;
                        op++;
                        if ((op & 1023) == 0) inf_flush(o, 1024u);
                    } else {
                        op++;
                    }
                    continue;
                }
                if (sym == 256) break;
                sym -= 257;
                const uint32_t lt = rl(ST.len, (int)sym);
                uint32_t ml = lt & 0xFFFFu;
                const uint32_t le = lt >> 16;
                v >>= len;  // the extra bits follow the code (len + le <= 20 < 32)
                if (le) {
                    NEED(le);
                    ml += v & ((1u << le) - 1u);
                    bp += le;
                }
                v = inf_peek(in, bp);
                r = inf_decode(v, nbits - bp, DC, T->dsym, sym, len);
                if (r == 0) goto done;
                if (r < 0 || sym > 29) return -1;  // invalid distance code
                bp += len;
                const uint32_t dt = rl(ST.dist, (int)sym);
                uint32_t dist = dt & 0xFFFFu;
                const uint32_t de = dt >> 16;
                if (de) {
                    NEED(de);
                    dist += (v >> len) & ((1u << de) - 1u);  // len + de <= 28
                    bp += de;
                }
                if (dist > op) return -1;  // invalid distance too far back
                if (kWrite) {
                    inf_copy(o, op, dist, ml);
                    op += ml;
                    inf_flush_upto(o, op);
                } else {
                    op += ml;
                }
            }
        }
        if (last) break;
    }
    // CHECK, LENGTH (the sizing pass stops before them: it holds no bytes to
    // check, and the plan depends only on what decodes)
    // a check that fails returns -2: the stream decoded (its plan stands),
    // the reference still throws
    if (kWrite) {
        bp = (bp + 7) & ~7ull;
        NEED(32);
        if (op > o.flushed) inf_flush(o, (uint32_t)(op - o.flushed));
        total = op;
        // (an outgrown slot holds no bytes, but the check was folded: a
        // failing one rejects here, a passing one leaves the member to the
        // second pass, which writes its bytes into the arena)
        const uint32_t w = inf_peek(in, bp);
        if (gz) {
            if (w != ~o.crc) return -2;  // incorrect data check
        } else {
            const uint32_t be = __builtin_bswap32(w);
            if (be != ((o.adb << 16) | o.ada)) return -2;
        }
        bp += 32;
        if (gz) {
            NEED(32);
            if (inf_peek(in, bp) != (uint32_t)op) return -2;  // incorrect length check
        }
        return 0;
    }
done:
    if (kWrite && op > o.flushed) inf_flush(o, (uint32_t)(op - o.flushed));
    total = op;
    return 0;
#undef NEED
}

// ---------------------------------------------------------------------------
// Job passes.  k_emit lists the gzip and zstd batches of RPGPU_JOB_DECODE
// jobs (inf_list, counters[16] items).
//   first pass (k_members_first, after k_emit, before the slot scans): one
//     wave per member decodes it into a scratch slot of the context's pool,
//     sized from the member's ISIZE trailer (gzip, capped by deflate's 1032:1
//     ratio) or first frame's content size (zstd); it sets the member's arena
//     reservation (dcap: the output rounded up to 16, 0 when the stream is
//     rejected, the plan rule of the reference's sizing pass: for gzip a
//     failed data / length check still reserves) and index slots, and its
//     state: 0 decoded and checked (the bytes wait in scratch), 1 rejected,
//     2 the output outgrew the scratch slot (or the pool ran out): decoded
//     again by the second pass;
//   k_inflate_copy: state 0 members from scratch into their arena slots;
//   second pass (k_members): state 2 members, into the slot.
// The reference decodes every gzip payload twice (buffer_for_input, then the
// real pass); here a well-formed member is decoded once.
// k_validate_decoded then computes the new crc / header_crc and walks it.
// ---------------------------------------------------------------------------
DEV void inf_load_tab(uint32_t* tab) {
    for (uint32_t i = lane(); i < 256; i += 64) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        tab[i] = c;
    }
}

DEV InfIn inf_batch(const DeviceJob& j, const rpgpu_batch_result* R) {
    const uint64_t S = uni64(j.seg_off[uni32(R->segment)]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
    const uint64_t n = (uint64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
    return inf_in(j.data + S, n);
}

// per-wave constants of the decode passes
struct InfWave {
    InfSymTabs ST;
    uint32_t x2n, lane_mul, chunk_mul;
};
DEV InfWave inf_wave() {
    InfWave w;
    w.ST = inf_sym_tabs();
    const uint32_t l = lane();
    w.x2n = l < 32 ? kX2nIeee[l] : 0u;
    w.lane_mul = ieee_xpow8(1024u - 16u * (l + 1), w.x2n);
    w.chunk_mul = ieee_xpow8(1024u, w.x2n);
    return w;
}
DEV InfOut inf_out(uint8_t* lds, const InfTabs* T, const InfWave& w, uint8_t* dst, uint64_t cap) {
    InfOut o;
    o.ring = (inf_lds_u8*)lds;
    o.tab = T->crc_tab;
    o.dst = dst;
    o.flushed = 0;
    o.x2n = w.x2n;
    o.lane_mul = w.lane_mul;
    o.chunk_mul = w.chunk_mul;
    o.cap = cap;
    o.over = false;
    return o;
}

// a member's first-pass scratch slot: the size its trailer / frame header
// claims (payload-controlled), capped by deflate's 1032:1 expansion limit, by
// 64x the input (above that a member is decoded again by the second pass) and
// by 1/8 of the pool, so one hostile trailer cannot starve the members
// claimed after it
DEV uint64_t scratch_guess(const DeviceJob& j, uint64_t claimed, uint64_t n) {
    uint64_t g = claimed;
    g = g < 1032ull * n + 64 ? g : 1032ull * n + 64;
    const uint64_t ratio = 64ull * n > (64ull << 10) ? 64ull * n : (64ull << 10);
    g = g < ratio ? g : ratio;
    g = g < j.inf_scratch_bytes / 8 ? g : j.inf_scratch_bytes / 8;
    return (g + 15) & ~15ull;
}

// first pass of gzip member i (batch b): decode into a scratch slot sized
// from the ISIZE trailer, set the plan and the state
DEV void gzip_first_item(const DeviceJob& j, uint8_t* lds, InfTabs* T, const InfWave& W, uint32_t i, uint32_t b,
                         const rpgpu_batch_result* R) {
    InfIn in = inf_batch(j, R);
    uint64_t total = 0;
    int rc = -1;  // compressor::uncompress throws on an empty payload (compression/compression.cc:34-55)
    bool over = true;
    uint64_t soff = 0;
    if (in.n) {
        // scratch slot from the ISIZE trailer (a guess: a truncated or
        // padded member's last bytes are something else)
        const uint64_t isize = in.n >= 4 ? (uint64_t)(inf_byte(in, in.n - 4) | (inf_byte(in, in.n - 3) << 8) |
                                                      (inf_byte(in, in.n - 2) << 16) | (inf_byte(in, in.n - 1) << 24))
                                         : 0;
        const uint64_t guess = scratch_guess(j, isize, in.n);
        soff = uni64(atomicAdd((unsigned long long*)j.inf_scratch_used, lane() == 0 ? (unsigned long long)guess : 0ull));
        const uint64_t cap = soff + guess <= j.inf_scratch_bytes ? guess : 0;
        InfOut o = inf_out(lds, T, W, j.inf_scratch + soff, cap);
        rc = inflate_member<true>(in, T, o, W.ST, total);
        over = o.over;
    }
    // the plan: the output rounded up to 16 unless the stream is rejected
    const uint64_t cap = rc == -1 ? 0 : (total + 15) & ~15ull;
    if (lane() == 0) {
        const int32_t rcount = R->record_count;
        j.dcap[b] = cap;
        j.slots[b] = ((j.flags & RPGPU_JOB_PARSE) && rcount > 0 && (uint64_t)rcount <= cap) ? (uint64_t)rcount : 0;
        j.inf_state[i] = rc != 0 ? 1u : over ? 2u : 0u;
        j.inf_off[i] = soff;
        j.inf_total[i] = total;
    }
}

// decoded members from scratch into their arena slots (one wave per member)
__global__ __launch_bounds__(256) void k_inflate_copy(DeviceJob j) {
    const uint32_t count = j.counters[16];
    const uint32_t l = lane();
    for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < count; i += gridDim.x * 4) {
        if (uni32(j.inf_state[i]) != 0) continue;
        const uint32_t b = uni32(j.inf_list[i]);
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t dst = uni64(j.dcap[b]), cap = uni64(j.dcap[b + 1]) - dst, total = uni64(j.inf_total[i]);
        if (dst + cap > j.decoded_capacity) {
            if (l == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
            continue;
        }
        const uint8_t* src = j.inf_scratch + uni64(j.inf_off[i]);
        for (uint64_t c = 16ull * l; c < total; c += 1024) *(uint4*)(j.decoded + dst + c) = *(const uint4*)(src + c);
        if (l == 0) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
            R->reserved0 = 0;  // k_validate_decoded computes the decoded crc
        }
    }
}

// the second pass of gzip member i (its output outgrew the scratch slot)
DEV void gzip_item(const DeviceJob& j, uint8_t* lds, InfTabs* T, const InfWave& W, rpgpu_batch_result* R,
                   uint64_t dst, uint64_t cap) {
    InfIn in = inf_batch(j, R);
    InfOut o = inf_out(lds, T, W, j.decoded + dst, cap);
    uint64_t total = 0;
    const int rc = inflate_member<true>(in, T, o, W.ST, total);
    if (rc == 0 && !o.over && lane() == 0) {
        R->flags = R->flags | RPGPU_F_CODEC_OK;
        R->decoded_len = (uint32_t)total;
        R->reserved0 = 0;
    }
}

// ---------------------------------------------------------------------------
// Split decode of large gzip members.  A member decodes serially on one wave
// (above), so a job's member pass is as long as its largest member.  A gzip
// member of >= kGzsMin stored bytes is cut instead into chunks of kGzsChunk
// deflate bytes, one wave each:
//   k_gzsplan    parses the gzip header (FHCRC members stay serial) and lists
//                the member's chunks (GzsItem);
//   k_gzsfind    finds the first dynamic-block header in each chunk k >= 1:
//                lanes test 64 bit offsets at a time (block type, HLIT, HDIST
//                and a complete code-length code), survivors are queued and
//                each lane decodes one survivor's code lengths through its own
//                7-bit table (complete literal/length and distance codes,
//                end-of-block present: what a valid header satisfies);
//   k_gzsdecode  decodes each chunk from its block start until the block
//                boundary where the next chunk's start lies, into a 16-bit
//                symbol region (a byte, or 256 + a position in the 32 KiB
//                before the chunk: a match reaching before the chunk's start
//                copies those placeholders -- the ring is primed with them);
//   k_gzsresolve walks the chain from chunk 0 (each chunk must end where the
//                next one begins, so a false start is never used), writes the
//                bytes into a scratch slot with the placeholders replaced from
//                the bytes before each chunk, computes the CRC32 in 256 pieces
//                and sets the member's plan and state as gzip_first_item does.
// The verdicts are those of inflate_member: a stream error in a chained chunk
// (or a placeholder before the member's start: a distance too far back)
// rejects; running out of input accepts what decoded; the CRC32 / ISIZE rules
// of the CHECK section.  A member whose chain does not close (a false start, a
// stored or fixed block at a chunk seam, a region outgrown) is left to
// k_members_first, which decodes it serially as before.
// ---------------------------------------------------------------------------
constexpr int kBufFlagsZs = 0x00020000;  // buffer resource word 3 (raw, 32-bit data format)
DEV void zs_wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
constexpr int kZsSc1 = 16;  // cache policy sc1: L2-coherent, bypasses the vector L1
typedef __attribute__((address_space(3))) uint16_t gzs_lds_u16;
// the chunk's ring holds its last 4 K symbols (8 KiB of LDS: eight 12 KiB
// workgroups leave a CU ~64 KiB for the zstd kernels beside them; an 8 K
// ring filled the CU, C6 resolve+plan 64.4 -> 60.3 ms); a match from farther
// back reads the chunk's region in the pool (its flushed symbols) or, before
// the chunk's start, is a placeholder
#ifndef RPGPU_GZS_RING
#define RPGPU_GZS_RING 4096
#endif
#ifndef RPGPU_GZS_WGS
#define RPGPU_GZS_WGS 8  // k_gzsdecode workgroups (one wave) per CU
#endif
constexpr uint32_t kGzsRing = RPGPU_GZS_RING, kGzsMask = kGzsRing - 1;
static_assert((kGzsRing & kGzsMask) == 0 && kGzsRing >= 2048, "split-decode ring: a power of two >= 2 K symbols");
constexpr uint32_t kGzsLds = 2 * kGzsRing + kInfTabBytes;

struct GzsOut {
    gzs_lds_u16* ring;  // kGzsRing symbols
    uint16_t* dst;      // the chunk's region in the pool
    __amdgpu_buffer_rsrc_t rs;  // dst as a buffer (L2-coherent reads of flushed symbols)
    uint64_t flushed, cap;
    bool over;
};

// symbols [flushed, flushed + len) (len <= 1024, the start 1 K aligned) to
// the region: 16 per lane (32 bytes)
DEV void gzs_flush(GzsOut& o, uint32_t len) {
    if (o.over || o.flushed + len > o.cap) {
        o.over = true;
    } else {
        const uint32_t l = lane();
        if (16u * l < len) {
            const uint32_t at = (uint32_t)(o.flushed & kGzsMask) + 16u * l;
            const uint4 a = *(const uint4*)(o.ring + at), b = *(const uint4*)(o.ring + at + 8);
            uint4* d = (uint4*)(o.dst + o.flushed + 16u * l);  // the region is a whole number of 1 K pieces
            d[0] = a;
            d[1] = b;
        }
    }
    o.flushed += len;
}
DEV void gzs_flush_upto(GzsOut& o, uint64_t op) {
    while ((op >> 10) > (o.flushed >> 10)) gzs_flush(o, 1024u);
}
// inf_copy over 16-bit symbols; dist > kGzsRing: the source lies before the
// ring (dist > ml, no overlap): the region's flushed symbols, or before the
// chunk's start its placeholders (256 + 32768 + position)
DEV void gzs_copy(GzsOut& o, uint64_t op, uint32_t dist, uint32_t ml) {
    const uint32_t l = lane();
    gzs_lds_u16* ring = o.ring;
    const uint32_t n = (ml + 63) >> 6;
    uint32_t b[5];
    if (dist > kGzsRing) {
        if (o.over) {
#pragma unroll
            for (uint32_t i = 0; i < 5; i++) b[i] = 0;
        } else {
            zs_wait_vm();  // the symbols read below were stored by this wave's flushes
#pragma unroll
            for (uint32_t i = 0; i < 5; i++) {
                const uint32_t k = 64u * i + l;
                const int64_t src = (int64_t)op - (int64_t)dist + (int64_t)k;
                b[i] = 0;
                if (i < n && k < ml)
                    b[i] = src < 0 ? (uint32_t)(256 + 32768 + src)
                                   : (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(o.rs, (int)(2 * src), 0, kZsSc1);
            }
        }
    } else {
        const bool rep = dist < ml;
        const uint64_t mg = rep ? 0xFFFFFFFFull / dist + 1ull : 0ull;
#pragma unroll
        for (uint32_t i = 0; i < 5; i++) {
            const uint32_t k = 64u * i + l;
            const uint32_t x = rep ? k - (uint32_t)(((uint64_t)k * mg) >> 32) * dist : k;
            b[i] = (i < n && k < ml) ? (uint32_t)ring[((uint32_t)(op - dist) + x) & kGzsMask] : 0u;
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t k = 64u * i + l;
        if (i < n && k < ml) ring[(uint32_t)(op + k) & kGzsMask] = (uint16_t)b[i];
    }
}

// Decode blocks from bit bp (a block header) until a block boundary at
// `stop`.  marks: matches may reach before the start (placeholders), else
// such a distance is the stream error it is.  Returns 1 stopped at `stop`, 2
// the final block ended (bp: its end), 3 the input ran out (inflate_member's
// `done`), -1 a stream error, -3 the region was outgrown, -4 passed `stop`
// (a false start); `total` = symbols decoded.
DEV int gzs_run(InfIn& in, InfTabs* T, GzsOut& o, const InfSymTabs& ST, uint64_t& bp, uint64_t stop, bool marks,
                uint64_t& total) {
    const uint32_t l = lane();
    const uint64_t nbits = in.n * 8;
    uint64_t op = 0;
    uint32_t v, sym, len;
    InfCode LC, DC, CC;
    int st = 0;
#define GNEED(k)                          \
    if (nbits - bp < (uint64_t)(k)) {     \
        st = 3;                           \
        goto out;                         \
    }
#define GFAIL  \
    {          \
        st = -1; \
        goto out; \
    }
    for (;;) {
        if (bp == stop) { st = 1; break; }
        if (bp > stop) { st = -4; break; }
        GNEED(3);
        v = inf_peek(in, bp);
        const uint32_t last = v & 1u, type = (v >> 1) & 3u;
        bp += 3;
        if (type == 0) {  // STORED
            bp = (bp + 7) & ~7ull;
            GNEED(32);
            v = inf_peek(in, bp);
            if ((v & 0xFFFFu) != ((v >> 16) ^ 0xFFFFu)) GFAIL;
            bp += 32;
            const uint64_t length = v & 0xFFFFu;
            const uint64_t p = bp >> 3, have = in.n - p, copy = length < have ? length : have;
            for (uint64_t c = 0; c < copy; c += 1024) {
#pragma unroll
                for (uint32_t k = 0; k < 16; k++) {
                    const uint64_t i = c + 16u * l + k;
                    if (i < copy) o.ring[(uint32_t)(op + i - c) & kGzsMask] = (uint16_t)in.src[p + i];
                }
                op += copy - c < 1024 ? copy - c : 1024;
                gzs_flush_upto(o, op);
            }
            bp += 8 * copy;
            if (copy < length) { st = 3; goto out; }
        } else if (type == 3) {
            GFAIL;
        } else {
            inf_lds_u8* lens = (inf_lds_u8*)T->lens;
            if (type == 1) {
                for (uint32_t s = l; s < 288; s += 64) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                inf_build(lens, 288, 1, T->lsym, LC);
                if (l < 32) lens[l] = 5;
                inf_build(lens, 32, 2, T->dsym, DC);
            } else {
                GNEED(14);
                v = inf_peek(in, bp);
                const uint32_t nlen = (v & 31u) + 257, ndist = ((v >> 5) & 31u) + 1, ncode = ((v >> 10) & 15u) + 4;
                bp += 14;
                if (nlen > 286 || ndist > 30) GFAIL;
                const uint64_t need = 3ull * ncode;
                const bool all = nbits - bp >= need;
                const uint32_t got = all ? ncode : (uint32_t)((nbits - bp) / 3);
                const uint64_t w57 = inf_peek64(in, bp);
                const uint32_t cl = l < got ? (uint32_t)(w57 >> (3 * (l < 19 ? l : 0))) & 7u : 0u;
                if (!all) { st = 3; goto out; }
                bp += need;
                if (l < 19) lens[kClenOrder[l]] = (uint8_t)(l < ncode ? cl : 0u);
                if (inf_build(lens, 19, 0, T->csym, CC)) GFAIL;
                uint32_t have = 0;
                while (have < nlen + ndist) {
                    v = inf_peek(in, bp);
                    const int r = inf_decode(v, nbits - bp, CC, T->csym, sym, len);
                    if (r == 0) { st = 3; goto out; }
                    if (r < 0) { sym = 0; len = 1; }
                    bp += len;
                    if (sym < 16) {
                        if (l == 0) lens[have] = (uint8_t)sym;
                        have++;
                        continue;
                    }
                    uint32_t rep = 0, cnt;
                    v = inf_peek(in, bp);
                    if (sym == 16) {
                        GNEED(2);
                        if (have == 0) GFAIL;
                        rep = uni32((uint32_t)lens[have - 1]);
                        cnt = 3 + (v & 3u);
                        bp += 2;
                    } else if (sym == 17) {
                        GNEED(3);
                        cnt = 3 + (v & 7u);
                        bp += 3;
                    } else {
                        GNEED(7);
                        cnt = 11 + (v & 127u);
                        bp += 7;
                    }
                    if (have + cnt > nlen + ndist) GFAIL;
                    if (l < cnt) lens[have + l] = (uint8_t)rep;
                    if (l + 64 < cnt) lens[have + l + 64] = (uint8_t)rep;
                    if (l + 128 < cnt) lens[have + l + 128] = (uint8_t)rep;
                    have += cnt;
                }
                if (lens[256] == 0) GFAIL;
                if (inf_build(lens, nlen, 1, T->lsym, LC)) GFAIL;
                if (inf_build(lens + nlen, ndist, 2, T->dsym, DC)) GFAIL;
            }
            inf_root(LC, T->lsym, T->lroot);
            inf_root(DC, T->dsym, T->droot);
            // fast loop (inflate_member's, over 16-bit symbols)
            {
                const uint64_t pb = bp + 8ull * in.mis;
                uint64_t pq = (pb >> 5) << 2;
                uint32_t sh = (uint32_t)(pb & 31);
                uint64_t bb = (uint64_t)(inf_dw(in, pq) >> sh);
                uint32_t bc = 32 - sh;
                pq += 4;
                bool eob = false, bad = false;
                uint32_t lb = 0, nl = 0;
                auto spill = [&]() __attribute__((always_inline)) {
                    if (nl) {
                        if (l < nl) o.ring[(uint32_t)(op + l) & kGzsMask] = (uint16_t)lb;
                        op += nl;
                        nl = 0;
                        gzs_flush_upto(o, op);
                    }
                };
                while (pq + 12 <= in.nphys) {
                    while (bc <= 32) {
                        bb |= (uint64_t)inf_dw(in, pq) << bc;
                        bc += 32;
                        pq += 4;
                    }
                    uint32_t e = uni32((uint32_t)T->lroot[(uint32_t)bb & 511u]);
                    if (e == 0) {
                        const int r = inf_decode((uint32_t)bb, 64, LC, T->lsym, sym, len);
                        if (r < 0) { bad = true; break; }
                        e = sym | (len << 9);
                    }
                    sym = e & 511u;
                    len = e >> 9;
                    bb >>= len;
                    bc -= len;
                    if (sym < 256) {
                        lb = l == nl ? sym : lb;
                        if (++nl == 64) spill();
                        continue;
                    }
                    spill();
                    if (sym == 256) { eob = true; break; }
                    if (sym > 285) { bad = true; break; }
                    const uint32_t lt = rl(ST.len, (int)(sym - 257));
                    const uint32_t le = lt >> 16;
                    const uint32_t ml = (lt & 0xFFFFu) + ((uint32_t)bb & ((1u << le) - 1u));
                    bb >>= le;
                    bc -= le;
                    if (bc <= 32) {
                        bb |= (uint64_t)inf_dw(in, pq) << bc;
                        bc += 32;
                        pq += 4;
                    }
                    e = uni32((uint32_t)T->droot[(uint32_t)bb & 511u]);
                    if (e == 0) {
                        const int r = inf_decode((uint32_t)bb, 64, DC, T->dsym, sym, len);
                        if (r < 0) { bad = true; break; }
                        e = sym | (len << 9);
                    }
                    sym = e & 511u;
                    len = e >> 9;
                    if (sym > 29) { bad = true; break; }
                    bb >>= len;
                    bc -= len;
                    const uint32_t dt = rl(ST.dist, (int)sym);
                    const uint32_t de = dt >> 16;
                    const uint32_t dist = (dt & 0xFFFFu) + ((uint32_t)bb & ((1u << de) - 1u));
                    bb >>= de;
                    bc -= de;
                    if (dist > op && !marks) { bad = true; break; }
                    gzs_copy(o, op, dist, ml);
                    op += ml;
                    gzs_flush_upto(o, op);
                }
                spill();
                if (bad) GFAIL;
                bp = 8 * (pq - in.mis) - bc;
                if (eob) {
                    if (last) { st = 2; break; }
                    continue;
                }
            }
            // exact loop near the end of the member
            for (;;) {
                v = inf_peek(in, bp);
                int r = inf_decode(v, nbits - bp, LC, T->lsym, sym, len);
                if (r == 0) { st = 3; goto out; }
                if (r < 0 || sym > 285) GFAIL;
                bp += len;
                if (sym < 256) {
                    if (l == 0) o.ring[(uint32_t)op & kGzsMask] = (uint16_t)sym;
                    op++;
                    if ((op & 1023) == 0) gzs_flush(o, 1024u);
                    continue;
                }
                if (sym == 256) break;
                sym -= 257;
                const uint32_t lt = rl(ST.len, (int)sym);
                uint32_t ml = lt & 0xFFFFu;
                const uint32_t le = lt >> 16;
                v >>= len;
                if (le) {
                    GNEED(le);
                    ml += v & ((1u << le) - 1u);
                    bp += le;
                }
                v = inf_peek(in, bp);
                r = inf_decode(v, nbits - bp, DC, T->dsym, sym, len);
                if (r == 0) { st = 3; goto out; }
                if (r < 0 || sym > 29) GFAIL;
                bp += len;
                const uint32_t dt = rl(ST.dist, (int)sym);
                uint32_t dist = dt & 0xFFFFu;
                const uint32_t de = dt >> 16;
                if (de) {
                    GNEED(de);
                    dist += (v >> len) & ((1u << de) - 1u);
                    bp += de;
                }
                if (dist > op && !marks) GFAIL;
                gzs_copy(o, op, dist, ml);
                op += ml;
                gzs_flush_upto(o, op);
            }
        }
        if (last) { st = 2; break; }
    }
out:
    if (op > o.flushed) gzs_flush(o, (uint32_t)(op - o.flushed));
    total = op;
    if (st > 0 && o.over) st = -3;
    return st;
#undef GNEED
#undef GFAIL
}

// 32 stream bits from bit q, lane-private (bytes past the member: whatever
// the member's last dword holds, or 0): from the LDS copy of the chunk's
// bytes (w: dwords from physical offset wa, kGzsWin bytes) when it holds them
typedef __attribute__((address_space(3))) uint32_t gzs_lds_u32;
constexpr uint32_t kGzsWin = 18432;
DEV uint32_t gzs_bits(const InfIn& in, uint64_t q, const gzs_lds_u32* w, uint64_t wa) {
    const uint64_t pb = q + 8ull * in.mis, a = (pb >> 3) & ~3ull;
    const uint32_t sh = (uint32_t)(pb - 8 * a);
    uint32_t d0, d1;
    if (a >= wa && a + 8 <= wa + kGzsWin) {
        d0 = w[(a - wa) >> 2];
        d1 = w[((a - wa) >> 2) + 1];
    } else {
        d0 = inf_ld(in, a);
        d1 = inf_ld(in, a + 4);
    }
    return sh ? __builtin_amdgcn_alignbit(d1, d0, sh) : d0;
}

// the dword at 4-aligned physical byte a: from the LDS window when it holds it
DEV uint32_t gzs_dw(const InfIn& in, uint64_t a, const gzs_lds_u32* w, uint64_t wa) {
    return (a >= wa && a + 4 <= wa + kGzsWin) ? w[(a - wa) >> 2] : inf_ld(in, a);
}

// stage 2 of the block-header search, one candidate per lane: decode the
// code lengths at bit p through the lane's own table tb (128 entries: the
// next 7 stream bits -> symbol | length << 5) and require what a valid
// dynamic header has (inflate_member's TABLE checks)
DEV bool gzs_check(const InfIn& in, uint64_t p, inf_lds_u8* tb, uint64_t nbits, const gzs_lds_u32* w, uint64_t wa) {
    constexpr uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    const uint32_t a = gzs_bits(in, p, w, wa), b = gzs_bits(in, p + 32, w, wa), c = gzs_bits(in, p + 64, w, wa);
    const uint32_t nlen = ((a >> 3) & 31u) + 257, ndist = ((a >> 8) & 31u) + 1, ncode = ((a >> 13) & 15u) + 4;
    const uint64_t x = (((uint64_t)b << 32 | a) >> 17) | ((uint64_t)c << 47);
    uint64_t Ls = 0;
#pragma unroll
    for (uint32_t q = 0; q < 19; q++)
        if (q < ncode) Ls |= ((x >> (3 * q)) & 7ull) << (3 * ord[q]);
    uint32_t code = 0;
    for (uint32_t L = 1; L <= 7; L++) {
#pragma unroll
        for (uint32_t s = 0; s < 19; s++) {
            if (((uint32_t)(Ls >> (3 * s)) & 7u) == L) {
                const uint32_t r = __builtin_bitreverse32(code) >> (32 - L);
                for (uint32_t e = r; e < 128; e += 1u << L) tb[e] = (uint8_t)(s | (L << 5));
                code++;
            }
        }
        code <<= 1;
    }
    uint64_t q = p + 17 + 3 * ncode;
    const uint32_t tot = nlen + ndist;
    uint32_t have = 0, prev = 0, kl = 0, kd = 0, lmax = 0, dmax = 0;
    bool ok = true, eob = false;
    while (ok && have < tot) {
        if (q + 32 > nbits) { ok = false; break; }
        const uint32_t v = gzs_bits(in, q, w, wa);
        const uint32_t e = tb[v & 127u];
        const uint32_t s = e & 31u, L = e >> 5;
        uint32_t val = s, cnt = 1;
        q += L;
        if (s == 16) {
            ok = have > 0;
            val = prev;
            cnt = 3 + ((v >> L) & 3u);
            q += 2;
        } else if (s == 17) {
            val = 0;
            cnt = 3 + ((v >> L) & 7u);
            q += 3;
        } else if (s == 18) {
            val = 0;
            cnt = 11 + ((v >> L) & 127u);
            q += 7;
        }
        if (have + cnt > tot) ok = false;
        if (kl > 32768u || kd > 32768u) ok = false;  // over-subscribed already
        if (ok && val) {
            const uint32_t e1 = have + cnt;
            const uint32_t nl = (e1 < nlen ? e1 : nlen) - (have < nlen ? have : nlen);
            kl += nl * (32768u >> val);
            kd += (cnt - nl) * (32768u >> val);
            if (nl) lmax = lmax > val ? lmax : val;
            if (cnt > nl) dmax = dmax > val ? dmax : val;
            if (have <= 256 && 256 < e1) eob = true;
        }
        prev = val;
        have += cnt;
    }
    return ok && eob && kl <= 32768u && kd <= 32768u && (kl == 32768u || lmax == 1) &&
           (kd == 32768u || dmax <= 1);
}

// ---------------------------------------------------------------------------
// zstd: the decoder of rp_zstd_core.h over a wave environment.  State is
// wave-uniform (every lane runs the same scalar logic; table reads are made
// uniform with readfirstlane); the input is read through the member's 512-byte
// window (headers, tables) and a 256-byte register window per backward bit
// stream (the sequence stream and each Huffman stream: one load per ~248
// bytes consumed); output goes through the 32 KiB LDS ring in 256-byte
// lane-parallel pieces and leaves in 1 KiB flushes (16 bytes per lane), as
// the inflate output does.  Matches reaching past the ring read the slot
// (L2-coherent loads once the flushes have completed).  A frame's XXH64
// content checksum is computed by the wave over its bytes (slot + ring).
// ---------------------------------------------------------------------------
constexpr uint32_t kZsTabBytes = (sizeof(zs::Tabs) + 15u) & ~15u;
constexpr uint32_t kZsLds = kInfRing + kZsTabBytes;
constexpr uint64_t kZsFarOff = kInfRing - 1024 - 256;  // offsets up to this read the ring

constexpr uint64_t kXP1 = 0x9E3779B185EBCA87ull, kXP2 = 0xC2B2AE3D27D4EB4Full, kXP3 = 0x165667B19E3779F9ull,
                   kXP4 = 0x85EBCA77C2B2AE63ull, kXP5 = 0x27D4EB2F165667C5ull;
DEV uint64_t xrotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
DEV uint64_t xround(uint64_t acc, uint64_t in) { return xrotl(acc + in * kXP2, 31) * kXP1; }

struct ZDev {
    InfIn in;
    bool dirty;  // a match reached into the overwritten previous ring segment (zs::RingDirtyHook)
    DEV void ring_dirty() { dirty = true; }
    inf_lds_u8* ring;
    uint8_t* dst;
    // output positions are 32-bit (SALU compares; the slot is < 2 GiB, and
    // output past 2^32 only counts: the core's totals are 64-bit)
    uint32_t cap;      // bytes the slot holds (a multiple of 16)
    uint32_t op;       // output position
    uint32_t flushed;  // output below left the ring (1 KiB aligned until the end)
    uint32_t stored;   // output below is in the slot
    bool over;         // the output outgrew the slot: only counted from then on
    uint32_t fstart;   // the current frame's first output byte
    uint32_t lbuf;     // Huffman literals gathered one per lane before they go to the ring
    uint32_t nlit;
    __amdgpu_buffer_rsrc_t rs;
#ifdef RPGPU_ZSTAMPS
    uint64_t prof[4];  // literals, matches, stream ends, whole compressed blocks
#endif

    DEV uint32_t b(uint64_t i) { return inf_byte(in, i); }
    DEV uint64_t le(uint64_t i, uint32_t k) {  // k (<= 8) bytes at i, inside the member
        const uint64_t p = i + in.mis, a = p & ~3ull;
        const uint32_t sh = (uint32_t)(p & 3) * 8u;
        const uint32_t d0 = inf_dw(in, a), d1 = inf_dw(in, a + 4);
        const uint64_t lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
        uint64_t v = lo;
        if (sh) v = (lo >> sh) | ((uint64_t)inf_dw(in, a + 8) << (64 - sh));
        return k >= 8 ? v : v & ((1ull << (8 * k)) - 1ull);
    }
    // 8 bytes at pos for backward bit stream s: its own register window,
    // placed to end just past the read (the stream moves down)
    DEV uint64_t lb(zs::Bits& s, uint64_t pos) {
        const uint64_t p = pos + in.mis;
        if (p < s.wbase || p + 12 > s.wbase + 256) {
            const uint64_t nb = (p + 12 > 256 ? p + 12 - 256 : 0) & ~3ull;
            s.wbase = nb;
            s.wreg = inf_ld(in, nb + 4u * lane());
        }
        const uint32_t o = (uint32_t)(p - s.wbase), li = o >> 2, sh = (o & 3) * 8u;
        const uint64_t lo = (uint64_t)rl(s.wreg, (int)li) | ((uint64_t)rl(s.wreg, (int)li + 1) << 32);
        return sh ? (lo >> sh) | ((uint64_t)rl(s.wreg, (int)li + 2) << (64 - sh)) : lo;
    }
    DEV uint32_t U(uint32_t x) { return uni32(x); }
    DEV zs::SeqSym sym(const zs::SeqSym& t) {
        uint64_t v;
        __builtin_memcpy(&v, &t, 8);
        v = uni64(v);
        zs::SeqSym r;
        __builtin_memcpy(&r, &v, 8);
        return r;
    }
    // [flushed, flushed + len) out of the ring (flushed 1 KiB aligned, len <= 1 KiB)
    DEV void flush(uint32_t len) {
        if (!over) {
            const uint32_t room = cap > flushed ? cap - flushed : 0u;
            const uint32_t at = 16u * lane();
            if (at < len && at < room) {
                const uint4 v = *(const uint4*)(ring + ((uint32_t)(flushed + at) & kInfMask));
                *(uint4*)(dst + flushed + at) = v;
            }
            const uint64_t end = (uint64_t)flushed + len;
            stored = end < cap ? (uint32_t)end : cap;
            if (end > cap) over = true;
        }
        flushed += len;
    }
    DEV void flush_upto(uint32_t p) {
        while ((p >> 10) > (flushed >> 10)) flush(1024u);
    }
    DEV void lit_spill() {
        if (!nlit) return;
        if (!over && lane() < nlit) ring[(uint32_t)(op + lane()) & kInfMask] = (uint8_t)lbuf;
        op += nlit;
        nlit = 0;
        flush_upto(op);
    }
    DEV void flush_all() {
        lit_spill();
        flush_upto(op);
        if (op > flushed) flush((uint32_t)(op - flushed));
    }
    DEV void raw(uint64_t pos, uint64_t k) {
        lit_spill();
        const uint32_t l = lane();
        for (uint64_t c = 0; c < k; c += 256) {
            const uint32_t m = k - c < 256 ? (uint32_t)(k - c) : 256u;
            if (!over) {
#pragma unroll
                for (uint32_t t = 0; t < 4; t++) {
                    const uint32_t x = 4u * l + t;
                    if (x < m) ring[(uint32_t)(op + x) & kInfMask] = in.src[pos + c + x];
                }
            }
            op += m;
            flush_upto(op);
        }
    }
    DEV void fill(uint32_t v, uint64_t k) {
        lit_spill();
        const uint32_t l = lane();
        for (uint64_t c = 0; c < k; c += 256) {
            const uint32_t m = k - c < 256 ? (uint32_t)(k - c) : 256u;
            if (!over) {
#pragma unroll
                for (uint32_t t = 0; t < 4; t++) {
                    const uint32_t x = 4u * l + t;
                    if (x < m) ring[(uint32_t)(op + x) & kInfMask] = (uint8_t)v;
                }
            }
            op += m;
            flush_upto(op);
        }
    }
    DEV void lit(uint32_t v) {
        lbuf = lane() == nlit ? v : lbuf;
        if (++nlit == 64) lit_spill();
    }
    DEV void match(uint64_t off, uint64_t ml) {
        lit_spill();
        const uint32_t l = lane();
        if (over) {
            op += (uint32_t)ml;
            flush_upto(op);
            return;
        }
        const bool far = off > kZsFarOff;
        // a match overlapping its own output repeats the off bytes before it:
        // byte x of a piece is x mod off into them (off < 256: a multiply by
        // the rounded-up reciprocal is exact for x < 256)
        const bool rep = off < 256 && off < ml;
        const uint64_t mg = rep ? 0xFFFFFFFFull / off + 1ull : 0ull;  // 2^32 for off = 1
        for (uint64_t c = 0; c < ml; c += 256) {
            const uint32_t m = ml - c < 256 ? (uint32_t)(ml - c) : 256u;
            uint32_t v[4];
            if (far) zs_wait_vm();  // the slot bytes read below were stored by this wave's flushes
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                const uint32_t x = 4u * l + t;
                v[t] = 0;
                if (x < m) {
                    if (far) {
                        v[t] = __builtin_amdgcn_raw_buffer_load_b8(rs, (int)(op + x - (uint32_t)off), 0, kZsSc1);
                    } else {
                        const uint64_t sx = rep ? x - (((uint64_t)x * mg) >> 32) * off : (uint64_t)x;
                        v[t] = ring[(op - (uint32_t)off + (uint32_t)sx) & kInfMask];
                    }
                }
            }
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                const uint32_t x = 4u * l + t;
                if (x < m) ring[(uint32_t)(op + x) & kInfMask] = (uint8_t)v[t];
            }
            op += m;
            flush_upto(op);
        }
    }
    DEV void frame_begin() {
        lit_spill();
        fstart = op;
    }
    // output byte q of this member (the slot below `flushed`, else the ring)
    DEV uint32_t byte_at(uint32_t q) {
        return q < flushed ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)q, 0, kZsSc1)
                           : (uint32_t)ring[q & kInfMask];
    }
    // XXH64 of the frame's output [fstart, op) vs the trailer's low 32 bits:
    // 1 equal, 0 not, 2 unknown (the bytes outgrew the slot)
    DEV int check(uint32_t want) {
        lit_spill();
        if (over || stored < flushed) return 2;
        zs_wait_vm();
        const uint32_t l = lane();
        const uint32_t len = op - fstart, body = len & ~31u;
        uint64_t h;
        if (len >= 32) {
            // lanes 0..3 hold the four accumulators; a 1 KiB piece at a time
            uint64_t acc = l == 0 ? kXP1 + kXP2 : l == 1 ? kXP2 : l == 2 ? 0ull : 0ull - kXP1;
            for (uint32_t c = 0; c < body; c += 1024) {
                const uint32_t m = body - c < 1024 ? body - c : 1024u;
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                if (16u * l < m) {
#pragma unroll
                    for (uint32_t t = 0; t < 16; t++) w[t >> 2] |= byte_at(fstart + c + 16u * l + t) << (8 * (t & 3));
                }
                for (uint32_t i = 0; i < m / 32; i++) {
                    // accumulator k takes bytes [32 i + 8 k, +8): lane 2 i + k / 2, half k & 1
                    const int src = (int)(2 * i + ((l & 3) >> 1));
                    const uint32_t x0 = (uint32_t)__shfl((int)w[0], src, 64), x1 = (uint32_t)__shfl((int)w[1], src, 64);
                    const uint32_t x2 = (uint32_t)__shfl((int)w[2], src, 64), x3 = (uint32_t)__shfl((int)w[3], src, 64);
                    const uint64_t word = (l & 1) ? ((uint64_t)x2 | ((uint64_t)x3 << 32)) : ((uint64_t)x0 | ((uint64_t)x1 << 32));
                    if (l < 4) acc = xround(acc, word);
                }
            }
            const uint64_t v1 = (uint64_t)rl((uint32_t)acc, 0) | ((uint64_t)rl((uint32_t)(acc >> 32), 0) << 32);
            const uint64_t v2 = (uint64_t)rl((uint32_t)acc, 1) | ((uint64_t)rl((uint32_t)(acc >> 32), 1) << 32);
            const uint64_t v3 = (uint64_t)rl((uint32_t)acc, 2) | ((uint64_t)rl((uint32_t)(acc >> 32), 2) << 32);
            const uint64_t v4 = (uint64_t)rl((uint32_t)acc, 3) | ((uint64_t)rl((uint32_t)(acc >> 32), 3) << 32);
            h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
            h = (h ^ xround(0, v1)) * kXP1 + kXP4;
            h = (h ^ xround(0, v2)) * kXP1 + kXP4;
            h = (h ^ xround(0, v3)) * kXP1 + kXP4;
            h = (h ^ xround(0, v4)) * kXP1 + kXP4;
        } else {
            h = kXP5;
        }
        h += len;
        uint32_t q = fstart + body;
        const uint32_t e = op;
        while (q + 8 <= e) {
            uint64_t k = 0;
            for (uint32_t t = 0; t < 8; t++) k |= (uint64_t)uni32(byte_at(q + t)) << (8 * t);
            h ^= xround(0, k);
            h = xrotl(h, 27) * kXP1 + kXP4;
            q += 8;
        }
        if (q + 4 <= e) {
            uint64_t k = 0;
            for (uint32_t t = 0; t < 4; t++) k |= (uint64_t)uni32(byte_at(q + t)) << (8 * t);
            h ^= k * kXP1;
            h = xrotl(h, 23) * kXP2 + kXP3;
            q += 4;
        }
        while (q < e) {
            h ^= (uint64_t)uni32(byte_at(q)) * kXP5;
            h = xrotl(h, 11) * kXP1;
            q++;
        }
        h ^= h >> 33;
        h *= kXP2;
        h ^= h >> 29;
        h *= kXP3;
        h ^= h >> 32;
        return (uint32_t)h == want ? 1 : 0;
    }
};

template <>
struct zs::RingDirtyHook<ZDev> {
    static constexpr bool value = true;
};

DEV ZDev zdev(const InfIn& in, uint8_t* lds, uint8_t* dst, uint64_t cap) {
    ZDev e;
    e.in = in;
    e.dirty = false;
    e.ring = (inf_lds_u8*)lds;
    e.dst = dst;
    e.cap = cap < (1ull << 31) ? (uint32_t)cap : 0u;  // a slot past 2 GiB: count only (never one real batch)
    e.op = e.flushed = e.stored = 0;
    e.over = false;
    e.fstart = 0;
    e.lbuf = 0;
    e.nlit = 0;
#ifdef RPGPU_ZSTAMPS
    e.prof[0] = e.prof[1] = e.prof[2] = e.prof[3] = 0;
#endif
    e.rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(cap < 0x7FFFFFFFull ? cap : 0x7FFFFFFFull), kBufFlagsZs);
    return e;
}

// the scratch slot of the first pass: the first frame's content size when
// its header carries one (exact for a one-frame payload), else 8 x the input
template <class Rd>
DEV uint64_t zs_guess_at(uint64_t n, Rd byte) {
    uint64_t g = 8 * n + 4096;
    if (n >= 6 && (byte(0) | (byte(1) << 8) | (byte(2) << 16) | (byte(3) << 24)) == 0xFD2FB528u) {
        const uint32_t fhd = byte(4);
        const uint32_t single = (fhd >> 5) & 1, fcsid = fhd >> 6, did = fhd & 3;
        const uint64_t at = 5 + (single ? 0 : 1) + (did == 3 ? 4 : did);
        const uint32_t sz = fcsid == 0 ? (single ? 1 : 0) : fcsid == 1 ? 2 : fcsid == 2 ? 4 : 8;
        if (sz && at + sz <= n) {
            uint64_t f = 0;
            for (uint32_t k = 0; k < sz; k++) f |= (uint64_t)byte(at + k) << (8 * k);
            if (fcsid == 1) f += 256;
            if (f < (1ull << 32)) g = f + 64;
        }
    }
    return (g + 15) & ~15ull;
}
DEV uint64_t zs_guess(InfIn& in) {
    return zs_guess_at(in.n, [&](uint64_t i) { return inf_byte(in, i); });
}

// ---------------------------------------------------------------------------
// zstd parse / execute split (the first pass's fast path).  ZDev keeps the
// decoder's state in SGPRs (readfirstlane on every value, spilled to VGPR
// lanes) and pushes each literal and match through the LDS ring: ~1200
// instructions per literal or sequence (profiles/r03_member_pass_sq.json).
// ZLane runs the same decoder (zs::payload: the same acceptance rules) with
// its state in VGPRs, every lane computing the same values, and produces no
// output bytes: literals go to a literal buffer and each match becomes a
// 16-byte record {literal start, literal count, match length, offset}.
// k_zexec (rp_codec.hip) executes the records with the LZ4 engine's wave
// executor straight into the arena slot once the plan is scanned.
//   A member takes this path when zs_fast_size's header walk finds only
// zstd frames without a content checksum, whole blocks and no skippable
// frame, and the scratch pool holds its literal buffer and records (sized
// exactly by that walk: literal section, raw and RLE bytes; sequence counts
// + 1).  A payload the decoder rejects is rejected (state 1, as the wave
// decoder would); one it accepts must deliver exactly the bytes its records
// describe (state 3); anything else is decoded by ZDev as before.
// ---------------------------------------------------------------------------
// a ZLane stream window: the 4 KiB of the member ending at or just past the
// 8-byte read at pos, 16 bytes per lane; returns the window start (not
// inlined: a refill is rare, and its code kept out of the literal loop)
__device__ __noinline__ uint64_t zl_fill(const uint8_t* src, uint64_t n, inf_lds_u8* w, uint64_t pos) {
    constexpr uint32_t kWin = 4096;
    // nb <= pos and nb + kWin >= pos + 8 (16-byte aligned start)
    const uint64_t nb = (pos + 8 + 15 > kWin ? pos + 8 + 15 - kWin : 0) & ~15ull;
    const uint32_t l = lane();
#pragma unroll
    for (uint32_t k = 0; k < kWin / 1024; k++) {
        const uint64_t o = nb + 1024u * k + 16u * l;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (o + 16 <= n) {
            __builtin_memcpy(&v, (const __attribute__((address_space(1))) uint8_t*)(src + o), 16);
        } else if (o < n) {
            uint32_t t[4] = {0u, 0u, 0u, 0u};
            for (uint32_t q = 0; q < 16; q++)
                if (o + q < n) t[q >> 2] |= (uint32_t)src[o + q] << (8 * (q & 3));
            v = make_uint4(t[0], t[1], t[2], t[3]);
        }
        __attribute__((address_space(3))) uint32_t* q = (__attribute__((address_space(3))) uint32_t*)(w + 1024u * k + 16u * l);
        q[0] = v.x;
        q[1] = v.y;
        q[2] = v.z;
        q[3] = v.w;
    }
    return nb;
}

struct ZLane {
    const uint8_t* src;
    uint64_t n;
    DEV void ring_dirty();  // (defined after `bad`: the wave decoder takes the member)
    uint8_t* lits;
    const ZsLitItem* items;  // the member's Huffman literal blocks k_zlits decoded ahead (k_zparse), in order
    uint32_t nitems, hidx;
    const ZsSeqItem* sitems;  // its sequence sections k_zlits decoded ahead, in order
    uint32_t nsitems, sidx;
    const zs::RawSeq* rseq;   // the taken section's raw sequences
    uint32_t rpos, rok;
    uint4 rbuf;               // 64 of them, lane k holding sequence 64 c + k
    uint64_t lits_at;        // scratch offset of lits (matches ZsLitItem::lits)
    SeqRec* recs;
    uint64_t lcap, rcap;
    uint64_t nlit, nrec, pend, mlsum;
    bool bad;
#ifdef RPGPU_ZSTAMPS
    uint64_t prof[4];
#endif
#ifdef RPGPU_ZL_UNI  // (A/B: header bytes and table reads wave-uniform)
    DEV uint32_t b(uint64_t i) { return uni32(i < n ? (uint32_t)src[i] : 0u); }
#else
    DEV uint32_t b(uint64_t i) { return i < n ? (uint32_t)src[i] : 0u; }
#endif
    DEV uint64_t le(uint64_t i, uint32_t k) {
        uint64_t v = 0;
        for (uint32_t t = 0; t < k; t++) v |= (uint64_t)b(i + t) << (8 * t);
        return v;
    }
    // 8 bytes at pos (pos + 8 <= n: the bit streams read inside the member)
    // for bit stream s from its LDS window: kZlWin bytes ending at or just past
    // the read (the streams move down), loaded by the wave 16 bytes per lane
    // when a read leaves it; each live stream has its own slot (round robin
    // over kZlSlots at bits_init, more than the streams live at once: four
    // literal streams and the sequence stream, or a weight stream)
    inf_lds_u8* win;
    uint32_t rr;
    static constexpr uint32_t kZlWin = 4096, kZlSlots = 8;
    DEV uint64_t lb(zs::Bits& s, uint64_t pos) {
        if (s.wbase == zs::kUnknown) {
            s.wreg = rr++ % kZlSlots;
            s.wbase = zs::kUnknown - 1;
        }
        inf_lds_u8* w = win + s.wreg * kZlWin;
        if (pos < s.wbase || pos + 8 > s.wbase + kZlWin) s.wbase = zl_fill(src, n, w, pos);
        const uint32_t o = (uint32_t)(pos - s.wbase), a = o & ~3u, sh = o & 3u;
        typedef const __attribute__((address_space(3))) uint32_t lds_cu32_t;
        const uint32_t d0 = *(lds_cu32_t*)(w + a), d1 = *(lds_cu32_t*)(w + a + 4);
        const uint32_t d2 = a + 8 < kZlWin ? *(lds_cu32_t*)(w + a + 8) : 0u;
        const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) |
                           ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
        return v;
    }
    // (values stay in VGPRs: making the table reads wave-uniform, so that the
    // state moves to SGPRs and branches on SCC, measured 140 -> 159 ms per
    // 1 MiB member)
#ifdef RPGPU_ZL_UNI
    DEV uint32_t U(uint32_t x) { return uni32(x); }
    DEV zs::SeqSym sym(const zs::SeqSym& t) {
        uint64_t v;
        __builtin_memcpy(&v, &t, 8);
        v = uni64(v);
        zs::SeqSym r;
        __builtin_memcpy(&r, &v, 8);
        return r;
    }
#else
    DEV uint32_t U(uint32_t x) { return x; }
    DEV zs::SeqSym sym(const zs::SeqSym& t) { return t; }
#endif
    DEV void lit(uint32_t v) {
        if (nlit >= lcap) bad = true;
        else if (lane() == 0) lits[nlit] = (uint8_t)v;
        nlit++;
        pend++;
    }
    DEV void raw(uint64_t pos, uint64_t k) {
        typedef __attribute__((address_space(1))) uint8_t g8;
        if (nlit + k > lcap) {
            bad = true;
        } else {
            // 16 bytes per lane, 1 KiB per step (any alignment); the tail bytewise
            const uint64_t body = k & ~1023ull;
            for (uint64_t c = 16u * lane(); c < body; c += 1024) {
                uint4 v;
                __builtin_memcpy(&v, (const g8*)(src + pos + c), 16);
                __builtin_memcpy((g8*)(lits + nlit + c), &v, 16);
            }
            for (uint64_t c = body + lane(); c < k; c += 64) lits[nlit + c] = src[pos + c];
        }
        nlit += k;
        pend += k;
    }
    DEV void fill(uint32_t v, uint64_t k) {
        if (nlit + k > lcap) bad = true;
        else
            for (uint64_t c = lane(); c < k; c += 64) lits[nlit + c] = (uint8_t)v;
        nlit += k;
        pend += k;
    }
    DEV void match(uint64_t off, uint64_t ml) {
        if (nrec >= rcap) bad = true;
        else if (lane() == 0)
            recs[nrec] = SeqRec{(uint32_t)(nlit - pend), (uint32_t)pend, (uint32_t)ml, (uint32_t)off};
        nrec++;
        pend = 0;
        mlsum += ml;
    }
    DEV void frame_begin() {}
    DEV int check(uint32_t) { return 2; }  // (never called: zs_fast_size admits no checksummed frame)
    // eager literals (zs::EagerLits): the block's Huffman literals are already
    // in the buffer, in consumption order
    DEV void take(uint64_t k) {
        nlit += k;
        pend += k;
    }
    // a raw / RLE literal section in place at nlit, at once (16 bytes per lane)
    DEV void raw_ahead(uint64_t pos, uint64_t k) {
        typedef __attribute__((address_space(1))) uint8_t g8;
        if (nlit + k > lcap) {
            bad = true;
            return;
        }
        const uint64_t body = k & ~1023ull;
        for (uint64_t c = 16u * lane(); c < body; c += 1024) {
            uint4 v;
            __builtin_memcpy(&v, (const g8*)(src + pos + c), 16);
            __builtin_memcpy((g8*)(lits + nlit + c), &v, 16);
        }
        for (uint64_t c = body + lane(); c < k; c += 64) lits[nlit + c] = src[pos + c];
    }
    DEV void fill_ahead(uint32_t v, uint64_t k) {
        if (nlit + k > lcap) {
            bad = true;
            return;
        }
        for (uint64_t c = lane(); c < k; c += 64) lits[nlit + c] = (uint8_t)v;
    }
    DEV uint32_t hbits(const zs::Bits& s, uint32_t hlog) {
        return (uint32_t)((s.c << (s.used & 63)) >> ((64 - hlog) & 63));
    }
    DEV void hstep(zs::Tabs* T, zs::Bits& s, uint32_t& open, bool x2, uint32_t hlog, uint64_t at) {
        const uint32_t d = U(T->huf[hbits(s, hlog)]);
        const uint32_t l1 = d >> 8;
        if (x2) open = (open && open + l1 <= 12) ? 0u : l1;
        s.used += l1;
        if (lane() == 0) lits[at] = (uint8_t)d;
    }
    // every symbol of the block's streams into the buffer at nlit (stream k's
    // segment at k * seg): the four streams advance together, their table
    // lookups issued back to back (one LDS latency per four symbols); each
    // stream's last symbol (the X2 last-symbol rule) by zs::huf_one
    DEV void huf_all(zs::Tabs* T, zs::Lits& L, uint32_t hlog) {
#ifdef RPGPU_ZSTAMPS
        const uint64_t t0 = wall_clock64();
#endif
        huf_all_(T, L, hlog);
#ifdef RPGPU_ZSTAMPS
        prof[2] += wall_clock64() - t0;
#endif
    }
    // a block k_zlits decoded ahead: its bytes are in place; the streams are
    // set to the end states lits_finish then reads (ended exactly, or
    // overflowed: the verdict k_zlits found)
    DEV bool take_planned(zs::Lits& L, uint32_t hlog) {
        if (hidx >= nitems) return false;
        const ZsLitItem* it = items + hidx++;
        const uint32_t st = it->status;
        bool same = st != 0 && it->lits == lits_at + nlit && it->lsz == L.size && it->ns == L.ns && it->hlog == hlog &&
                    it->x2 == (uint32_t)L.x2;
        for (uint32_t k = 0; k < 4; k++)
            if (k < L.ns) same = same && it->s0[k] == L.s[k].start && it->cnt[k] == L.cnt[k];
        if (!same) return false;
        for (uint32_t k = 0; k < 4; k++) {
            L.s[k].ptr = L.s[k].start;
            L.s[k].used = st == 1 ? 64u : 65u;
            L.dec[k] = L.cnt[k];
        }
        return true;
    }
    // zs::EagerSeqs: the block's sequence section decoded ahead by k_zlits
    // (same stream, same logs, all of it), read 64 at a time
    DEV bool seqs_take(uint64_t sp, uint64_t sn, uint32_t nseq, uint32_t llog, uint32_t olog, uint32_t mlog) {
        if (sidx >= nsitems) return false;
        const ZsSeqItem* it = sitems + sidx++;
        const uint32_t st = it->status;
        if (st == 0 || it->sp != sp || it->sn != sn || it->nseq != nseq || it->llog != llog || it->olog != olog ||
            it->mlog != mlog)
            return false;
        rseq = (const zs::RawSeq*)(scratch + it->seqs);
        rpos = 0;
        rok = st == 1;
        return true;
    }
    uint8_t* scratch;
    DEV void seq_next(zs::RawSeq& r) {
        const uint32_t k = rpos & 63u;
        if (k == 0) rbuf = *(const uint4*)(rseq + rpos + lane());  // (16 bytes past the section: inside the scratch region)
        r.ll = (uint32_t)__builtin_amdgcn_readlane((int)rbuf.x, (int)k);
        r.ml = (uint32_t)__builtin_amdgcn_readlane((int)rbuf.y, (int)k);
        r.v = (uint32_t)__builtin_amdgcn_readlane((int)rbuf.z, (int)k);
        r.kind = (uint32_t)__builtin_amdgcn_readlane((int)rbuf.w, (int)k);
        rpos++;
    }
    DEV bool seqs_ok() { return rok != 0; }
    // inclusive prefix sum over the wave (DPP row shifts, then the row
    // broadcasts; as rp_codec.hip's wave_scan)
    static DEV uint32_t scan(uint32_t v) {
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
        return v;
    }
    // zs::EagerSeqs: block()'s loop over a taken section, 64 sequences per
    // step, lane k holding sequence 64 c + k: the repeat offsets resolved in
    // order (a scalar pass over the 64), the positions before each sequence
    // by prefix sums of its lengths, every check of the loop per lane (any
    // lane failing rejects, as the first failure in order would), then the
    // 16-byte records written together
    DEV bool seqs_apply(zs::Frame& F, zs::Lits& L, uint64_t& r0, uint64_t& r1, uint64_t& r2, uint64_t& bo,
                        uint64_t capb, uint32_t nseq) {
        const uint32_t l = lane();
        for (uint32_t c = 0; c < nseq; c += 64) {
            const uint32_t m = nseq - c < 64 ? nseq - c : 64u;
            const bool on = l < m;
            uint4 q = make_uint4(0u, 0u, 0u, 0u);
            if (on) q = *(const uint4*)(rseq + c + l);
            const uint32_t ll = q.x, ml = q.y;
            // the repeat offsets, in order
            uint64_t myoff = 0;
            for (uint32_t k = 0; k < m; k++) {
                const uint32_t kind = (uint32_t)__builtin_amdgcn_readlane((int)q.w, (int)k);
                const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)q.z, (int)k);
                const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)q.x, (int)k);
                uint64_t off;
                if (kind == 0) {
                    off = v;
                    r2 = r1;
                    r1 = r0;
                    r0 = off;
                } else if (kind == 1) {
                    if (lk != 0) {
                        off = r0;
                    } else {
                        off = r1;
                        r1 = r0;
                        r0 = off;
                    }
                } else {
                    uint64_t t = v == 3 ? r0 - 1 : (v == 1 ? r1 : r2);
                    t += !t;
                    if (v != 1) r2 = r1;
                    r1 = r0;
                    r0 = off = t;
                }
                if (l == k) myoff = off;
            }
            // positions before this lane's sequence
            const uint32_t lli = scan(ll), mli = scan(ml);
            const uint64_t lle = lli - ll, mle = mli - ml;
            const uint64_t bok = bo + lle + mle;
            const uint64_t usedk = (uint64_t)L.used + lle;
            const uint64_t fok = F.fo + lle + ll + mle;  // after this sequence's literals
            bool fail = (uint64_t)ll + ml > capb - bok;
            fail = fail || (uint64_t)ll > (uint64_t)L.size - usedk;
            fail = fail || myoff > fok - F.seg0 + F.prevlen;
            // a reach into the overwritten previous ring segment: the wave
            // decoder (then the exact path) takes the member
            const bool dirty = myoff > fok - F.seg0 && F.prevlen - (myoff - (fok - F.seg0)) < fok - F.seg0 + zs::kRingDirty;
            if (__ballot(on && (fail || dirty))) {
                if (__ballot(on && dirty)) bad = true;
                return false;
            }
            if (nrec + m > rcap) {
                bad = true;
            } else if (on) {
                const uint32_t lip = l == 0 ? (uint32_t)(nlit - pend) : (uint32_t)(nlit + lle);
                const uint32_t lln = l == 0 ? (uint32_t)(pend + ll) : ll;
                recs[nrec + l] = SeqRec{lip, lln, ml, (uint32_t)myoff};
            }
            const uint64_t lt = (uint32_t)__builtin_amdgcn_readlane((int)lli, (int)(m - 1));
            const uint64_t mt = (uint32_t)__builtin_amdgcn_readlane((int)mli, (int)(m - 1));
            bo += lt + mt;
            F.fo += lt + mt;
            L.used += (uint32_t)lt;
            nlit += lt;
            pend = 0;
            nrec += m;
            mlsum += mt;
        }
        return true;
    }
    DEV void huf_all_(zs::Tabs* T, zs::Lits& L, uint32_t hlog) {
        const uint64_t at = nlit;
        if (at + L.size > lcap) {
            bad = true;
            return;
        }
        if (take_planned(L, hlog)) return;
        const bool x2 = L.x2;
        if (L.ns == 1) {
            const uint32_t c = L.cnt[0];
            for (uint32_t i = 0; i + 1 < c; i++) {
                if (L.s[0].used > 64 - hlog) zs::bits_reload(*this, L.s[0]);
                hstep(T, L.s[0], L.pend[0], x2, hlog, at + i);
            }
            if (c) {
                const uint32_t v = zs::huf_one(*this, T, L.s[0], L.pend[0], 1, x2, hlog);
                if (lane() == 0) lits[at + c - 1] = (uint8_t)v;
            }
        } else {
            const uint32_t seg = L.seg, c3 = L.cnt[3];
            for (uint32_t i = 0; i + 1 < seg; i++) {
                const bool s3 = i + 1 < c3;
                if (L.s[0].used > 64 - hlog) zs::bits_reload(*this, L.s[0]);
                if (L.s[1].used > 64 - hlog) zs::bits_reload(*this, L.s[1]);
                if (L.s[2].used > 64 - hlog) zs::bits_reload(*this, L.s[2]);
                if (s3 && L.s[3].used > 64 - hlog) zs::bits_reload(*this, L.s[3]);
                const uint32_t d0 = U(T->huf[hbits(L.s[0], hlog)]), d1 = U(T->huf[hbits(L.s[1], hlog)]),
                               d2 = U(T->huf[hbits(L.s[2], hlog)]), d3 = s3 ? U(T->huf[hbits(L.s[3], hlog)]) : 0u;
                const uint32_t l0 = d0 >> 8, l1 = d1 >> 8, l2 = d2 >> 8, l3 = d3 >> 8;
                if (x2) {
                    L.pend[0] = (L.pend[0] && L.pend[0] + l0 <= 12) ? 0u : l0;
                    L.pend[1] = (L.pend[1] && L.pend[1] + l1 <= 12) ? 0u : l1;
                    L.pend[2] = (L.pend[2] && L.pend[2] + l2 <= 12) ? 0u : l2;
                    if (s3) L.pend[3] = (L.pend[3] && L.pend[3] + l3 <= 12) ? 0u : l3;
                }
                L.s[0].used += l0;
                L.s[1].used += l1;
                L.s[2].used += l2;
                if (s3) L.s[3].used += l3;
                if (lane() == 0) {
                    lits[at + i] = (uint8_t)d0;
                    lits[at + seg + i] = (uint8_t)d1;
                    lits[at + 2 * seg + i] = (uint8_t)d2;
                    if (s3) lits[at + 3 * seg + i] = (uint8_t)d3;
                }
            }
            // the last symbol of streams 0..2 and whatever stream 3 has left
            // (c3 <= seg: one symbol at most)
#pragma unroll
            for (uint32_t k = 0; k < 3; k++) {
                const uint32_t v = zs::huf_one(*this, T, L.s[k], L.pend[k], 1, x2, hlog);
                if (lane() == 0) lits[at + k * seg + seg - 1] = (uint8_t)v;
            }
            if (c3) {
                const uint32_t v = zs::huf_one(*this, T, L.s[3], L.pend[3], 1, x2, hlog);
                if (lane() == 0) lits[at + 3 * seg + c3 - 1] = (uint8_t)v;
            }
        }
        L.dec[0] = L.cnt[0];
        L.dec[1] = L.cnt[1];
        L.dec[2] = L.cnt[2];
        L.dec[3] = L.cnt[3];
    }
};
static_assert(ZLane::kZlWin * ZLane::kZlSlots <= kInfRing, "ZLane's stream windows use the ring's LDS");
DEV void ZLane::ring_dirty() { bad = true; }
template <>
struct zs::EagerLits<ZLane> {
    static constexpr bool value = true;
};
template <>
struct zs::RingDirtyHook<ZLane> {
    static constexpr bool value = true;
};
template <>
struct zs::EagerSeqs<ZLane> {
    static constexpr bool value = true;
};

// The fast path's header walk: every frame a zstd frame without a content
// checksum or dictionary, every block whole; sums the literal bytes the
// decoder can emit and the sequences it can decode.  False sends the member to
// the wave decoder (which also rules on anything malformed here).
DEV bool zs_fast_size(const uint8_t* src, uint64_t n, uint64_t& nlit, uint64_t& nseq, uint32_t& nhuf, uint32_t& nsb) {
    auto b = [&](uint64_t i) -> uint32_t { return i < n ? (uint32_t)src[i] : 0u; };
    nlit = nseq = 0;
    nhuf = nsb = 0;
    uint64_t ip = 0;
    if (n == 0) return false;
    while (ip < n) {
        if (n - ip < 6) return false;
        const uint32_t magic = b(ip) | (b(ip + 1) << 8) | (b(ip + 2) << 16) | (b(ip + 3) << 24);
        if (magic != 0xFD2FB528u) return false;
        const uint32_t fhd = b(ip + 4);
        const uint32_t single = (fhd >> 5) & 1, fcsid = fhd >> 6, did = fhd & 3, ck = (fhd >> 2) & 1;
        if (ck || did || (fhd & 8)) return false;
        const uint64_t hsize = 5 + (single ? 0 : 1) + (fcsid ? (fcsid == 1 ? 2 : fcsid == 2 ? 4 : 8) : 0) +
                               ((single && !fcsid) ? 1 : 0);
        if (n - ip < hsize) return false;
        ip += hsize;
        for (;;) {
            if (n - ip < 3) return false;
            const uint32_t bh = b(ip) | (b(ip + 1) << 8) | (b(ip + 2) << 16);
            const uint32_t last = bh & 1, bt = (bh >> 1) & 3, bsz = bh >> 3;
            ip += 3;
            if (bt == 3) return false;
            // a raw / RLE block larger than Block_Maximum_Size is corrupt
            // (libzstd rejects it): the wave decoder rules on it, and its
            // payload-controlled size never reserves scratch here
            if (bt < 2 && bsz > zs::kBlockMax) return false;
            if (bt == 0) {
                if (n - ip < bsz) return false;
                nlit += bsz;
                ip += bsz;
            } else if (bt == 1) {
                if (n - ip < 1) return false;
                nlit += bsz;
                ip += 1;
            } else {
                if (n - ip < bsz || bsz < 3) return false;
                const uint32_t b0 = b(ip), lt = b0 & 3, lhl = (b0 >> 2) & 3;
                uint64_t lsz, lcons;
                if (lt < 2) {
                    uint32_t lh;
                    if (lhl == 1) {
                        lh = 2;
                        lsz = (b0 | (b(ip + 1) << 8)) >> 4;
                    } else if (lhl == 3) {
                        lh = 3;
                        lsz = (b0 | (b(ip + 1) << 8) | (b(ip + 2) << 16)) >> 4;
                    } else {
                        lh = 1;
                        lsz = b0 >> 3;
                    }
                    lcons = lt == 0 ? lh + lsz : lh + 1;
                } else {
                    if (bsz < 5) return false;
                    const uint32_t lhc = b0 | (b(ip + 1) << 8) | (b(ip + 2) << 16) | (b(ip + 3) << 24);
                    uint32_t lh;
                    uint64_t lcs;
                    if (lhl < 2) {
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
                        lcs = (lhc >> 22) + ((uint64_t)b(ip + 4) << 10);
                    }
                    lcons = lh + lcs;
                }
                if (lsz > zs::kBlockMax || lcons >= bsz) return false;
                if (lt >= 2) nhuf++;
                nlit += lsz;
                uint64_t sp = ip + lcons;
                uint32_t ns = b(sp);
                if (ns == 255) ns = (b(sp + 1) | (b(sp + 2) << 8)) + 0x7F00;
                else if (ns >= 128) ns = ((ns - 128) << 8) + b(sp + 1);
                nseq += ns;
                if (ns) nsb++;
                ip += bsz;
            }
            if (last) break;
        }
    }
    return ip == n;
}

// k_zplan's second walk over a member zs_fast_size admitted, block() step
// by step without decoding a symbol: each compressed block's Huffman literal
// section becomes a ZsLitItem (its stream bounds and literal destination;
// its table built by the decoder's own huf_table and snapshot for a new
// tree, the frame's last one for a treeless block) and its sequence section
// a ZsSeqItem (its stream and the three FSE tables seq_table builds, the
// repeat modes taking the frame's previous ones, snapshot).  It stops at
// anything block() would reject there: the blocks after it have no items
// and decode in place (or never: the member is rejected at that block).
struct ZsPlan {
    ZsLitItem* li;
    uint32_t lcap, nl;
    ZsSeqItem* si;
    uint32_t scap, ns;
    uint64_t tabs_off;   // scratch offset of the table snapshots (8 KiB Huffman, 10 KiB FSE each)
    uint64_t seqs_off;   // scratch offset of the raw sequences
};
DEV void zs_plan_items(ZLane& e, zs::Tabs* T, const DeviceJob& j, uint64_t src_off, uint64_t soff, ZsPlan& P) {
    const uint64_t n = e.n;
    uint64_t ip = 0, nlit = 0, tab = 0, tabs = P.tabs_off, seqs = P.seqs_off;
    uint32_t hlog = 0, hx2 = 0, llog = 0, olog = 0, mlog = 0;
    bool have = false, fse_ok = false;
    P.nl = P.ns = 0;
    while (ip < n) {
        if (n - ip < 6) return;
        const uint32_t fhd = e.b(ip + 4);
        const uint32_t single = (fhd >> 5) & 1, fcsid = fhd >> 6;
        ip += 5 + (single ? 0 : 1) + (fcsid ? (fcsid == 1 ? 2 : fcsid == 2 ? 4 : 8) : 0) + ((single && !fcsid) ? 1 : 0);
        have = fse_ok = false;  // a frame's first blocks must carry their tables
        for (;;) {
            if (n - ip < 3) return;
            const uint32_t bh = (uint32_t)e.le(ip, 3);
            const uint32_t last = bh & 1, bt = (bh >> 1) & 3, bsz = bh >> 3;
            ip += 3;
            const uint64_t adv = bt == 1 ? 1u : bsz;  // an RLE block occupies one byte
            if (bt == 0 || bt == 1) {
                nlit += bsz;
            } else {
                const uint64_t bp = ip, end = ip + bsz;
                const uint32_t b0 = e.b(bp), lt = b0 & 3, lhl = (b0 >> 2) & 3;
                uint64_t lcons;
                if (lt < 2) {
                    uint32_t lh, lsz;
                    if (lhl == 1) lh = 2, lsz = (uint32_t)e.le(bp, 2) >> 4;
                    else if (lhl == 3) lh = 3, lsz = (uint32_t)e.le(bp, 3) >> 4;
                    else lh = 1, lsz = b0 >> 3;
                    lcons = lt == 0 ? (uint64_t)lh + lsz : (uint64_t)lh + 1;
                    nlit += lsz;
                } else {
                    const uint32_t lhc = (uint32_t)e.le(bp, 4);
                    uint32_t lh, lsz;
                    uint64_t lcs;
                    bool one = false;
                    if (lhl < 2) {
                        one = lhl == 0;
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
                    if (lcs + lh > bsz || P.nl >= P.lcap) return;
                    uint64_t hs = bp + lh, hn = lcs;
                    if (lt == 2) {
                        if (!one && (lsz == 0 || hn == 0)) return;
                        uint32_t hl = 0;
                        const int64_t th = zs::huf_table(e, T, hs, hn, hl);
                        if (th < 0 || (uint64_t)th >= hn) return;
                        hlog = hl;
                        hx2 = !one && zs::huf_select_x2(lsz, lcs) ? 1u : 0u;
                        hs += (uint64_t)th;
                        hn -= (uint64_t)th;
                        tab = tabs;
                        tabs += 8192;
                        uint16_t* dst = (uint16_t*)(j.inf_scratch + tab);
                        for (uint32_t u = lane(); u < (1u << hl); u += 64) dst[u] = T->huf[u];
                        have = true;
                    } else if (!have) {
                        return;  // treeless without a tree: block() rejects
                    }
                    ZsLitItem it;
                    it.src = src_off;
                    it.n = n;
                    it.lits = soff + kZsFastHdr + nlit;
                    it.tab = tab;
                    it.lsz = lsz;
                    it.hlog = hlog;
                    it.status = 0;
                    for (uint32_t k = 0; k < 4; k++) it.s0[k] = 0, it.sn[k] = 0, it.cnt[k] = 0;
                    if (one) {
                        it.ns = 1;
                        it.seg = 1;
                        it.x2 = 0;
                        it.s0[0] = hs;
                        it.sn[0] = (uint32_t)hn;
                        it.cnt[0] = lsz;
                    } else {
                        if (hn < 10) return;
                        const uint64_t l1 = e.le(hs, 2), l2 = e.le(hs + 2, 2), l3 = e.le(hs + 4, 2);
                        const uint64_t l4 = hn - (l1 + l2 + l3 + 6);
                        if (l4 > hn) return;
                        it.ns = 4;
                        it.x2 = hx2;
                        it.seg = (lsz + 3) / 4;
                        it.s0[0] = hs + 6;
                        it.s0[1] = hs + 6 + l1;
                        it.s0[2] = hs + 6 + l1 + l2;
                        it.s0[3] = hs + 6 + l1 + l2 + l3;
                        it.sn[0] = (uint32_t)l1;
                        it.sn[1] = (uint32_t)l2;
                        it.sn[2] = (uint32_t)l3;
                        it.sn[3] = (uint32_t)l4;
                        it.cnt[0] = it.cnt[1] = it.cnt[2] = it.seg;
                        it.cnt[3] = lsz > 3 * it.seg ? lsz - 3 * it.seg : 0;
                    }
                    if (lane() == 0) P.li[P.nl] = it;
                    P.nl++;
                    nlit += lsz;
                    lcons = lh + lcs;
                }
                // the sequences section header and tables (block() order)
                uint64_t sp = bp + lcons;
                if (sp >= end) return;
                uint32_t nseq = e.b(sp++);
                if (nseq == 255) {
                    if (sp + 2 > end) return;
                    nseq = (uint32_t)e.le(sp, 2) + 0x7F00;
                    sp += 2;
                } else if (nseq >= 128) {
                    if (sp >= end) return;
                    nseq = ((nseq - 128) << 8) + e.b(sp);
                    sp++;
                }
                if (nseq) {
                    if (sp + 1 > end || P.ns >= P.scap) return;
                    const uint32_t modes = e.b(sp++);
                    int64_t h = zs::seq_table(e, T, T->ll, llog, modes >> 6, 35, 9, sp, end - sp, zs::kLLBase,
                                              zs::kLLBits, zs::kLLNorm, 35, 6, fse_ok);
                    if (h < 0) return;
                    sp += (uint64_t)h;
                    h = zs::seq_table(e, T, T->of, olog, (modes >> 4) & 3, 31, 8, sp, end - sp, zs::kOFBase,
                                      zs::kOFBits, zs::kOFNorm, 28, 5, fse_ok);
                    if (h < 0) return;
                    sp += (uint64_t)h;
                    h = zs::seq_table(e, T, T->ml, mlog, (modes >> 2) & 3, 52, 9, sp, end - sp, zs::kMLBase,
                                      zs::kMLBits, zs::kMLNorm, 52, 6, fse_ok);
                    if (h < 0) return;
                    sp += (uint64_t)h;
                    fse_ok = true;
                    // snapshot ll / of / ml (SeqSym, 8 bytes each) as dwords
                    uint32_t* dst = (uint32_t*)(j.inf_scratch + tabs);
                    const uint32_t* srct = (const uint32_t*)T->ll;
                    for (uint32_t u = lane(); u < (uint32_t)(kZsSeqTab / 4); u += 64) dst[u] = srct[u];
                    ZsSeqItem q;
                    q.src = src_off;
                    q.n = n;
                    q.seqs = seqs;
                    q.tab = tabs;
                    q.sp = sp;
                    q.sn = end - sp;
                    q.nseq = nseq;
                    q.llog = llog;
                    q.olog = olog;
                    q.mlog = mlog;
                    q.status = 0;
                    q.pad = 0;
                    if (lane() == 0) P.si[P.ns] = q;
                    P.ns++;
                    tabs += kZsSeqTab;
                    seqs += (uint64_t)nseq * sizeof(zs::RawSeq);
                }
            }
            ip += adv;
            if (last) break;
        }
    }
}

// the fast path of zstd member i: 0 not taken (the wave decoder runs), else
// the state set (1 rejected, kZsFast parsed)
DEV uint32_t zstd_fast_item(const DeviceJob& j, uint8_t* lds, uint32_t i, uint32_t b, const rpgpu_batch_result* R) {
    // k_zplan sized the member's buffers (ZsFastDesc at inf_off[i]) and
    // k_zlits decoded its Huffman literal blocks ahead
    const uint64_t S = uni64(j.seg_off[uni32(R->segment)]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
    const uint64_t n = (uint64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
    const uint8_t* src = j.data + S;
    const uint64_t soff = uni64(j.inf_off[i]);
    uint8_t* base = j.inf_scratch + soff;
    ZsFastDesc* D = (ZsFastDesc*)base;
    ZLane e;
    e.src = src;
    e.n = n;
    e.lits = base + uni64(D->lit_off);
    e.lits_at = soff + uni64(D->lit_off);
    e.recs = (SeqRec*)(base + uni64(D->rec_off));
    e.lcap = uni64(D->lcap);
    e.rcap = uni64(D->rcap);
    e.items = (const ZsLitItem*)(base + uni64(D->items));
    e.nitems = uni32((uint32_t)D->nitems);
    e.hidx = 0;
    e.sitems = (const ZsSeqItem*)(base + uni64(D->sitems));
    e.nsitems = uni32((uint32_t)D->nsitems);
    e.sidx = 0;
    e.scratch = j.inf_scratch;
    e.rpos = e.rok = 0;
    e.nlit = e.nrec = e.pend = e.mlsum = 0;
    e.bad = false;
    e.win = (inf_lds_u8*)lds;  // the ring's LDS (the wave decoder's, unused here)
    e.rr = 0;
#ifdef RPGPU_ZSTAMPS
    e.prof[0] = e.prof[1] = e.prof[2] = e.prof[3] = 0;
#endif
    zs::Tabs* T = (zs::Tabs*)(lds + kInfRing);
    uint64_t total = 0;
    bool unsure = false;
#ifdef RPGPU_ZSTAMPS
    const uint64_t t0 = wall_clock64();
#endif
    const int rc = zs::payload(e, T, n, total, unsure);
#ifdef RPGPU_ZSTAMPS
    if (lane() == 0) {
        for (int k = 0; k < 4; k++) atomicAdd(&g_zst[8 + k], (unsigned long long)e.prof[k]);
        atomicAdd(&g_zst[12], (unsigned long long)(wall_clock64() - t0));
        atomicAdd(&g_zst[13], 1ull);
        atomicAdd(&g_zst[14], (unsigned long long)(e.nrec + (e.nlit << 32)));
        atomicMax(&g_zst[15], (unsigned long long)(wall_clock64() - t0));
    }
#endif
    if (e.bad) return 0;  // (the header walk's sizes should always hold: the wave decoder then rules)
    if (rc != 0) {
        if (lane() == 0) {
            j.dcap[b] = 0;
            j.slots[b] = 0;
            j.inf_state[i] = 1;
            j.inf_off[i] = 0;
            j.inf_total[i] = 0;
        }
        return 1;
    }
    if (e.pend) e.match(0, 0);  // the literals after the last match
    if (unsure || e.bad || e.nlit + e.mlsum != total || total >= (1ull << 31)) return 0;
    const uint64_t cap = (total + 15) & ~15ull;
    if (lane() == 0) {
        D->nlit = e.nlit;
        D->nrec = e.nrec;
        const int32_t rcount = R->record_count;
        j.dcap[b] = cap;
        j.slots[b] = ((j.flags & RPGPU_JOB_PARSE) && rcount > 0 && (uint64_t)rcount <= cap) ? (uint64_t)rcount : 0;
        j.inf_state[i] = kZsFast;
        j.inf_off[i] = soff;
        j.inf_total[i] = total;
    }
    return kZsFast;
}

// first pass of zstd member i: the same plan / state rules as gzip's; a
// payload whose content checksum could not be checked in the slot (it
// outgrew it) is decoded again by the second pass
DEV void zstd_first_item(const DeviceJob& j, uint8_t* lds, uint32_t i, uint32_t b, const rpgpu_batch_result* R) {
    zs::Tabs* T = (zs::Tabs*)(lds + kInfRing);
    InfIn in = inf_batch(j, R);
    uint64_t total = 0, soff = 0;
    int rc = -1;  // compressor::uncompress throws on an empty payload (compression/compression.cc:34-55)
    bool again = true, dirty = false;
    if (in.n) {
        const uint64_t guess = scratch_guess(j, zs_guess(in), in.n);
        soff = uni64(atomicAdd((unsigned long long*)j.inf_scratch_used, lane() == 0 ? (unsigned long long)guess : 0ull));
        const uint64_t cap = soff + guess <= j.inf_scratch_bytes ? guess : 0;
        ZDev e = zdev(in, lds, j.inf_scratch + soff, cap);
        bool unsure = false;
#ifdef RPGPU_ZSTAMPS
        const uint64_t t0 = wall_clock64();
#endif
        rc = zs::payload(e, T, in.n, total, unsure);
        e.flush_all();
        again = unsure || e.stored < total;
        dirty = e.dirty;
#ifdef RPGPU_ZSTAMPS
        if (lane() == 0) {
            for (int k = 0; k < 4; k++) atomicAdd(&g_zst[k], (unsigned long long)e.prof[k]);
            atomicAdd(&g_zst[4], (unsigned long long)(wall_clock64() - t0));
            atomicAdd(&g_zst[5], 1ull);
            atomicAdd(&g_zst[6], (unsigned long long)total);
            atomicMax(&g_zst[7], (unsigned long long)(wall_clock64() - t0));
        }
#endif
    }
    const uint64_t cap = rc != 0 ? 0 : (total + 15) & ~15ull;
    if (lane() == 0) {
        const int32_t rcount = R->record_count;
        j.dcap[b] = cap;
        j.slots[b] = ((j.flags & RPGPU_JOB_PARSE) && rcount > 0 && (uint64_t)rcount <= cap) ? (uint64_t)rcount : 0;
        j.inf_state[i] = dirty ? kZsExact : rc != 0 ? 1u : again ? 2u : 0u;
        if (dirty) atomicAdd(&j.counters[27], 1u);
        j.inf_off[i] = soff;
        j.inf_total[i] = total;
    }
}

// the second pass of zstd member i, into its arena slot
DEV void zstd_item(const DeviceJob& j, uint8_t* lds, rpgpu_batch_result* R, uint64_t dst, uint64_t cap) {
    zs::Tabs* T = (zs::Tabs*)(lds + kInfRing);
    InfIn in = inf_batch(j, R);
    ZDev e = zdev(in, lds, j.decoded + dst, cap);
    uint64_t total = 0;
    bool unsure = false;
    const int rc = zs::payload(e, T, in.n, total, unsure);
    e.flush_all();
    if (rc == 0 && !unsure && e.stored >= total && lane() == 0) {
        R->flags = R->flags | RPGPU_F_CODEC_OK;
        R->decoded_len = (uint32_t)total;
        R->reserved0 = 0;
    }
}

// ---------------------------------------------------------------------------
// The exact path (round 6).  In libzstd's ring-buffer
// mode a corrupt stream's match can reach past the window into the part of
// the previous ring segment (the DCtx's extDict) that the current segment,
// or the up-to-32-byte overcopy of its copies, has already written, and then
// reads those newer bytes.  The fast decoders report such a member
// (zs::RingDirtyHook: ZLane hands it to ZDev, ZDev marks it kZsExact) and
// k_zexact decodes it again over ZExact: the same decoder (zs::payload, the
// same acceptance rules) on one lane, with the DCtx's output buffer emulated
// byte for byte in scratch memory -- every ZSTD_execSequence write as
// libzstd 1.4.x performs it on x86-64 (ZSTD_copy16 of the literals and the
// x86 ZSTD_wildcopy: one COPY16, then two per turn; ZSTD_overlapCopy8; the
// extDict memmove; ZSTD_execSequenceEnd's safecopy within 32 bytes of the
// buffer end; the literal buffer's padding: zeros, the RLE byte, or the
// block's own bytes for raw literals read in place) -- so that such a match
// reads what libzstd reads.  The emulation is pinned against libzstd on the
// host by tests/test_zstd_core.py (tests/cpp/zstd_core_host.cpp ExactHostEnv,
// the same writes).  Corrupt streams only: one wave takes these members one
// after another.
// ---------------------------------------------------------------------------
constexpr uint64_t kZxBuf = zs::kStaticBuffers + 512;  // the DCtx's outBuff (its largest), + overcopy room
constexpr uint64_t kZxBlk = zs::kBlockMax + 128;       // a block's literal buffer + its padding

struct ZExact {
    const uint8_t* src;
    uint64_t n;
    uint8_t* dst;                 // the member's output slot
    uint64_t cap, out, fstart;    // slot bytes, output so far, the frame's first output byte
    bool over;                    // the output outgrew the slot (counted on)
    uint8_t* buf;                 // the emulated DCtx output buffer
    uint64_t op, oend, prevlen;   // write position, buffer end, previous segment's length (extDict)
    uint8_t* blk;                 // the block's literals, then the bytes a wildcopy reads past them
    uint64_t blkn, took;
#ifdef RPGPU_ZSTAMPS
    uint64_t prof[4];
#endif

    DEV uint32_t b(uint64_t i) { return i < n ? (uint32_t)src[i] : 0u; }
    DEV uint64_t le(uint64_t i, uint32_t k) {
        uint64_t v = 0;
        for (uint32_t q = 0; q < k; q++) v |= (uint64_t)b(i + q) << (8 * q);
        return v;
    }
    DEV uint64_t lb(zs::Bits&, uint64_t i) { return le(i, 8); }
    DEV uint32_t U(uint32_t x) { return x; }
    DEV zs::SeqSym sym(const zs::SeqSym& t) { return t; }
    DEV void frame_begin() { fstart = out; }
    // final bytes [a, a + k) of the buffer to the output
    DEV void emit(uint64_t a, uint64_t k) {
        for (uint64_t q = 0; q < k; q++)
            if (out + q < cap) dst[out + q] = buf[a + q];
        out += k;
        if (out > cap) over = true;
    }
    // exact writes: raw / RLE blocks, the literals after the last sequence
    DEV void raw(uint64_t pos, uint64_t k) {
        for (uint64_t q = 0; q < k; q++) buf[op + q] = (uint8_t)b(pos + q);
        emit(op, k);
        op += k;
    }
    DEV void fill(uint32_t v, uint64_t k) {
        for (uint64_t q = 0; q < k; q++) buf[op + q] = (uint8_t)v;
        emit(op, k);
        op += k;
    }
    DEV void lit(uint32_t v) { fill(v, 1); }
    DEV void match(uint64_t, uint64_t) {}  // (ExactRing: exec_seq does the sequence's copies)
    DEV void take(uint64_t k) {
        for (uint64_t q = 0; q < k; q++) buf[op + q] = blk[took + q];
        emit(op, k);
        op += k;
        took += k;
    }
    // zs::EagerLits: the block's literals in place before its sequences
    DEV void raw_ahead(uint64_t pos, uint64_t k) {
        for (uint64_t q = 0; q < k; q++) blk[q] = (uint8_t)b(pos + q);
        blkn = k;
        took = 0;
    }
    DEV void fill_ahead(uint32_t v, uint64_t k) {
        for (uint64_t q = 0; q < k; q++) blk[q] = (uint8_t)v;
        blkn = k;
        took = 0;
    }
    DEV void huf_all(zs::Tabs* T, zs::Lits& L, uint32_t hlog) {
        for (uint32_t k = 0; k < L.ns; k++) {
            for (uint32_t i = 0; i < L.cnt[k]; i++)
                blk[(uint64_t)k * L.seg + i] = (uint8_t)zs::huf_one(*this, T, L.s[k], L.pend[k], L.cnt[k] - i, L.x2, hlog);
            L.dec[k] = L.cnt[k];
        }
        blkn = L.size;
        took = 0;
    }
    // zs::ExactRing
    DEV void ring_begin(uint64_t size) {
        oend = size;
        op = 0;
        prevlen = 0;
    }
    DEV void ring_wrap() {
        prevlen = op;
        op = 0;
    }
    DEV void lit_pad(int mode, uint64_t pos, uint32_t rle) {
        for (uint32_t q = 0; q < 64; q++) blk[blkn + q] = mode == 1 ? (uint8_t)b(pos + q) : mode == 2 ? (uint8_t)rle : 0;
    }
    // COPY16 / COPY8 (an SSE / 8-byte load, then the store)
    DEV void copy_n(uint64_t d, uint64_t s, uint32_t k) {
        uint8_t t[16];
        for (uint32_t i = 0; i < k; i++) t[i] = buf[s + i];
        for (uint32_t i = 0; i < k; i++) buf[d + i] = t[i];
    }
    DEV void wild_buf(uint64_t d, uint64_t s, int64_t length, bool overlap) {
        const uint64_t e = d + (uint64_t)length;
        if (overlap && d - s < 16) {
            do { copy_n(d, s, 8); d += 8; s += 8; } while (d < e);
            return;
        }
        copy_n(d, s, 16);
        if (16 >= length) return;
        d += 16;
        s += 16;
        do {
            copy_n(d, s, 16); d += 16; s += 16;
            copy_n(d, s, 16); d += 16; s += 16;
        } while (d < e);
    }
    DEV void wild_lit(uint64_t d, uint64_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
        for (uint32_t i = 0; i < 16; i++) buf[d + i] = blk[s + i];
        if (16 >= length) return;
        d += 16;
        s += 16;
        do {
            for (uint32_t i = 0; i < 32; i++) buf[d + i] = blk[s + i];
            d += 32;
            s += 32;
        } while (d < e);
    }
    DEV void overlap8(uint64_t& d, uint64_t& s, uint64_t offset) {
        if (offset < 8) {
            const uint32_t dec32 = (0x44441210u >> (4 * offset)) & 15u;   // {0, 1, 2, 1, 4, 4, 4, 4}
            const int32_t sub2 = (int32_t)((0xBA987888u >> (4 * offset)) & 15u);  // {8, 8, 8, 7, 8, 9, 10, 11}
            buf[d] = buf[s];
            buf[d + 1] = buf[s + 1];
            buf[d + 2] = buf[s + 2];
            buf[d + 3] = buf[s + 3];
            s += dec32;
            copy_n(d + 4, s, 4);
            s -= (uint64_t)sub2;
        } else {
            copy_n(d, s, 8);
        }
        s += 8;
        d += 8;
    }
    DEV void memmove_buf(uint64_t d, uint64_t s, uint64_t k) {
        if (d <= s)
            for (uint64_t q = 0; q < k; q++) buf[d + q] = buf[s + q];
        else
            for (uint64_t q = k; q-- > 0;) buf[d + q] = buf[s + q];
    }
    DEV void safecopy_buf(uint64_t d, uint64_t oend_w, uint64_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
        if (length < 8) {
            while (d < e) buf[d++] = buf[s++];
            return;
        }
        overlap8(d, s, d - s);
        if (e <= oend_w) {
            wild_buf(d, s, length, true);
            return;
        }
        if (d <= oend_w) {
            wild_buf(d, s, (int64_t)(oend_w - d), true);
            s += oend_w - d;
            d = oend_w;
        }
        while (d < e) buf[d++] = buf[s++];
    }
    DEV void safecopy_lit(uint64_t d, uint64_t oend_w, uint64_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
        if (length < 8) {
            while (d < e) buf[d++] = blk[s++];
            return;
        }
        if (e <= oend_w) {
            wild_lit(d, s, length);
            return;
        }
        if (d <= oend_w) {
            wild_lit(d, s, (int64_t)(oend_w - d));
            s += oend_w - d;
            d = oend_w;
        }
        while (d < e) buf[d++] = blk[s++];
    }
    // ZSTD_execSequence / ZSTD_execSequenceEnd on the buffer (prefixStart 0,
    // the extDict the previous segment's [0, prevlen) of the same buffer)
    DEV void exec_seq(uint64_t ll, uint64_t off, uint64_t ml) {
        const uint64_t o0 = op, oLitEnd = op + ll, oMatchEnd = oLitEnd + ml, oend_w = oend - 32;
        const bool end_path = oMatchEnd > oend_w;
        if (end_path) {
            safecopy_lit(op, oend_w, took, (int64_t)ll);
        } else {
            for (uint32_t i = 0; i < 16; i++) buf[op + i] = blk[took + i];
            if (ll > 16) wild_lit(op + 16, took + 16, (int64_t)ll - 16);
        }
        took += ll;
        uint64_t d = oLitEnd, m = oLitEnd - off, rem = ml;
        if (off > oLitEnd) {
            m = prevlen - (off - oLitEnd);
            if (m + ml <= prevlen) {
                memmove_buf(oLitEnd, m, ml);
                op = oMatchEnd;
                emit(o0, ll + ml);
                return;
            }
            const uint64_t len1 = prevlen - m;
            memmove_buf(oLitEnd, m, len1);
            d = oLitEnd + len1;
            rem = ml - len1;
            m = 0;
        }
        if (end_path) {
            safecopy_buf(d, oend_w, m, (int64_t)rem);
        } else if (off >= 16) {
            wild_buf(d, m, (int64_t)rem, false);
        } else {
            overlap8(d, m, off);
            if (rem > 8) wild_buf(d, m, (int64_t)rem - 8, true);
        }
        op = oMatchEnd;
        emit(o0, ll + ml);
    }
    // the frame's XXH64 content checksum over its output (2: the output
    // outgrew the slot, not checkable here)
    DEV int check(uint32_t want) {
        if (over) return 2;
        const uint64_t len = out - fstart;
        const uint8_t* p = dst + fstart;
        uint64_t h, q = 0;
        if (len >= 32) {
            uint64_t v1 = kXP1 + kXP2, v2 = kXP2, v3 = 0, v4 = 0 - kXP1;
            for (; q + 32 <= len; q += 32) {
                uint64_t w[4];
                for (int k = 0; k < 4; k++) {
                    w[k] = 0;
                    for (int t = 0; t < 8; t++) w[k] |= (uint64_t)p[q + 8 * k + t] << (8 * t);
                }
                v1 = xround(v1, w[0]);
                v2 = xround(v2, w[1]);
                v3 = xround(v3, w[2]);
                v4 = xround(v4, w[3]);
            }
            h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
            h = (h ^ xround(0, v1)) * kXP1 + kXP4;
            h = (h ^ xround(0, v2)) * kXP1 + kXP4;
            h = (h ^ xround(0, v3)) * kXP1 + kXP4;
            h = (h ^ xround(0, v4)) * kXP1 + kXP4;
        } else {
            h = kXP5;
        }
        h += len;
        for (; q + 8 <= len; q += 8) {
            uint64_t k = 0;
            for (int t = 0; t < 8; t++) k |= (uint64_t)p[q + t] << (8 * t);
            h ^= xround(0, k);
            h = xrotl(h, 27) * kXP1 + kXP4;
        }
        if (q + 4 <= len) {
            uint64_t k = 0;
            for (int t = 0; t < 4; t++) k |= (uint64_t)p[q + t] << (8 * t);
            h ^= k * kXP1;
            h = xrotl(h, 23) * kXP2 + kXP3;
            q += 4;
        }
        for (; q < len; q++) {
            h ^= (uint64_t)p[q] * kXP5;
            h = xrotl(h, 11) * kXP1;
        }
        h ^= h >> 33;
        h *= kXP2;
        h ^= h >> 29;
        h *= kXP3;
        h ^= h >> 32;
        return (uint32_t)h == want ? 1 : 0;
    }
};
template <>
struct zs::EagerLits<ZExact> {
    static constexpr bool value = true;
};
template <>
struct zs::ExactRing<ZExact> {
    static constexpr bool value = true;
};

// k_zexact: pass 0 (after the first pass, before the slot scans) decodes the
// kZsExact members into scratch slots and sets their plan and state as
// zstd_first_item does (kZsExactAgain instead of 2); pass 1 (after
// k_members) decodes the kZsExactAgain ones into their arena slots.  One
// wave, lane 0; the buffer and the literal buffer from the scratch pool.
__global__ __launch_bounds__(64) void k_zexact(DeviceJob j, int pass) {
    extern __shared__ __attribute__((aligned(16))) uint8_t zlds[];
    if (threadIdx.x != 0 || !j.inf_scratch || j.counters[27] == 0) return;
    const uint32_t count = j.counters[16];
    zs::Tabs* T = (zs::Tabs*)zlds;
    uint8_t* work = nullptr;
    for (uint32_t i = 0; i < count; i++) {
        const uint32_t st = j.inf_state[i];
        if (st != (pass == 0 ? kZsExact : kZsExactAgain)) continue;
        const uint32_t b = j.inf_list[i];
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t S = j.seg_off[R->segment] + R->file_pos + RPGPU_HEADER_SIZE;
        const uint64_t n = (uint64_t)(uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE);
        // the buffers: taken from the pool by the first pass, kept for the
        // second ([31]: offset / 16 + 1, 0 while none)
        if (!work && j.counters[31]) work = j.inf_scratch + 16ull * (j.counters[31] - 1);
        if (!work && pass == 0) {
            const uint64_t w = atomicAdd((unsigned long long*)j.inf_scratch_used, (unsigned long long)(kZxBuf + kZxBlk));
            if (w + kZxBuf + kZxBlk <= j.inf_scratch_bytes) {
                work = j.inf_scratch + w;
                j.counters[31] = (uint32_t)(w >> 4) + 1;
            }
        }
        ZExact e;
        e.src = j.data + S;
        e.n = n;
        e.dst = nullptr;
        e.out = e.fstart = 0;
        e.over = false;
        e.op = e.oend = e.prevlen = 0;
        e.blkn = e.took = 0;
        uint64_t soff = 0, cap = 0;
        if (pass == 0) {
            const uint64_t guess = scratch_guess(j, zs_guess_at(n, [&](uint64_t q) { return e.b(q); }), n);
            soff = atomicAdd((unsigned long long*)j.inf_scratch_used, (unsigned long long)guess);
            cap = soff + guess <= j.inf_scratch_bytes ? guess : 0;
            e.dst = j.inf_scratch + soff;
        } else {
            const uint64_t dst = j.dcap[b];
            cap = j.dcap[b + 1] - dst;
            if (dst + cap > j.decoded_capacity) {
                R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
                continue;
            }
            e.dst = j.decoded + dst;
        }
        e.cap = cap;
        uint64_t total = 0;
        bool unsure = false;
        int rc = -1;
        if (work && n) {
            e.buf = work;
            e.blk = work + kZxBuf;
            rc = zs::payload(e, T, n, total, unsure);
        }
        // no scratch for the buffer (a pool too small for it): the member
        // stays turned down, as the fast decoders left it
        if (pass == 0) {
            const bool again = unsure || e.over;
            const uint64_t dcap = rc != 0 ? 0 : (total + 15) & ~15ull;
            const int32_t rcount = R->record_count;
            j.dcap[b] = dcap;
            j.slots[b] = ((j.flags & RPGPU_JOB_PARSE) && rcount > 0 && (uint64_t)rcount <= dcap) ? (uint64_t)rcount : 0;
            j.inf_state[i] = rc != 0 ? 1u : again ? kZsExactAgain : 0u;
            j.inf_off[i] = soff;
            j.inf_total[i] = total;
        } else if (rc == 0 && !unsure && !e.over) {
            R->flags = R->flags | RPGPU_F_CODEC_OK;
            R->decoded_len = (uint32_t)total;
            R->reserved0 = 0;
        }
    }
}

// ---------------------------------------------------------------------------
// The member kernels: one wave per workgroup (the ring and the tables are the
// wave's own LDS, sized for the larger decoder), members claimed one at a
// time from inf_list, gzip and zstd alike, so both codecs' members run side
// by side.  The gzip CRC table shares LDS with the zstd tables: it is
// reloaded before a gzip member that follows a zstd one.
//   k_members_first (after k_emit, before the slot scans): the first pass;
//   k_inflate_copy: state-0 members from scratch into the arena;
//   k_members: the second pass of state-2 members.
// ---------------------------------------------------------------------------
constexpr uint32_t kMemLds = kZsLds > kInfLdsDecode ? kZsLds : kInfLdsDecode;

// pass 0: every member the split decode did not close (after it); with the
// split decode, pass 1 takes the members it never planned (small, FHCRC)
// beside it on another stream, and pass 2 after it the planned ones whose
// chain did not close
__global__ __launch_bounds__(64) void k_members_first(DeviceJob j, int pass) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    InfTabs* T = (InfTabs*)(lds + kInfRing);
    const InfWave W = inf_wave();
    bool tab = false;
    const uint32_t count = j.counters[16];
    // largest first (a member decodes serially, so a big one claimed last
    // would set the pass's tail): members of >= 128 KiB stored, then the rest
    for (uint32_t phase = 0; phase < 2; phase++) {
        for (;;) {
            const uint32_t i = wave_fetch_add(&j.counters[pass == 2 ? (phase ? 49 : 48) : (phase ? 20 : 17)], 1u);
            if (i >= count) break;
            const uint32_t b = uni32(j.inf_list[i]);
            const rpgpu_batch_result* R = &j.batches[b];
            const bool big = uni32((uint32_t)R->size_bytes) >= (128u << 10);
            if (big != (phase == 0)) continue;
            const uint32_t gm = j.gzs_mem ? uni32(j.gzs_mem[2 * i + 1]) : 0u;
            if (gm >> 31) continue;  // the split decode closed it
            if (pass == 1 && gm != 0) continue;  // planned: after the split decode
            if (pass == 2 && gm == 0) continue;  // done by pass 1
            if ((uni32((uint32_t)(uint16_t)R->attrs) & 7u) == RPGPU_CODEC_GZIP) {
                if (!tab) inf_load_tab(T->crc_tab);
                tab = true;
                gzip_first_item(j, lds, T, W, i, b, R);
            } else if (!j.zs_split) {
                tab = false;
                zstd_first_item(j, lds, i, b, R);
            }
        }
    }
}

// j.zs_split: the zstd members' first pass leaves k_members_first.  k_zparse
// (on a side stream, beside k_members_first's gzip members) runs the lane
// parser on each, largest first as above, and marks the members it does not
// take kZsPending; k_zfallback (after the join, before the slot scans) runs
// the wave decoder on those.  (Separate kernels: the lane parser's VGPR state
// and the wave decoder's SGPR state in one register allocation spilled.)
constexpr uint32_t kZsPending = 4;

// k_zplan: per zstd member, zs_fast_size's header walk, the scratch region
// (descriptor, literal buffer, records, literal and sequence items, table
// snapshots, raw sequences) and the items (zs_plan_items), registered in
// zs_items for k_zlits (bit 63 marks a sequence item); kZsPlanned, or
// kZsPending for the wave decoder
__global__ __launch_bounds__(64) void k_zplan(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t count = j.counters[16];
    zs::Tabs* T = (zs::Tabs*)(lds + kInfRing);
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[30], 1u);
        if (i >= count) break;
        const uint32_t b = uni32(j.inf_list[i]);
        const rpgpu_batch_result* R = &j.batches[b];
        if ((uni32((uint32_t)(uint16_t)R->attrs) & 7u) == RPGPU_CODEC_GZIP) continue;
        const uint64_t S = uni64(j.seg_off[uni32(R->segment)]) + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
        const uint64_t n = (uint64_t)uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
        uint64_t nl = 0, nq = 0;
        uint32_t nh = 0, nsb = 0;
        uint32_t state = kZsPending;
        uint64_t soff = 0;
        if (j.zs_fast && zs_fast_size(j.data + S, n, nl, nq, nh, nsb)) {
            const uint64_t lbytes = (nl + 16 + 15) & ~15ull, rcap = nq + 1;
            const uint64_t o_rec = kZsFastHdr + lbytes;
            const uint64_t o_li = o_rec + rcap * sizeof(SeqRec);
            const uint64_t o_si = o_li + (((uint64_t)nh * sizeof(ZsLitItem) + 15) & ~15ull);
            const uint64_t o_tab = o_si + (((uint64_t)nsb * sizeof(ZsSeqItem) + 15) & ~15ull);
            const uint64_t o_seq = o_tab + 8192ull * nh + kZsSeqTab * nsb;
            const uint64_t need = o_seq + nq * sizeof(zs::RawSeq) + 64 * sizeof(zs::RawSeq);
            // at most 1/8 of the pool per member (as scratch_guess): one
            // hostile header cannot starve the members claimed after it
            const bool fits = need <= j.inf_scratch_bytes / 8;
            soff = fits ? uni64(atomicAdd((unsigned long long*)j.inf_scratch_used, lane() == 0 ? (unsigned long long)need
                                                                                                : 0ull))
                        : 0;
            if (fits && soff + need <= j.inf_scratch_bytes) {
                ZLane e;
                e.src = j.data + S;
                e.n = n;
                e.win = (inf_lds_u8*)lds;
                e.rr = 0;
                e.nitems = e.nsitems = 0;
                ZsPlan P;
                P.li = (ZsLitItem*)(j.inf_scratch + soff + o_li);
                P.lcap = nh;
                P.si = (ZsSeqItem*)(j.inf_scratch + soff + o_si);
                P.scap = nsb;
                P.tabs_off = soff + o_tab;
                P.seqs_off = soff + o_seq;
                zs_plan_items(e, T, j, S, soff, P);
                const uint32_t first = wave_fetch_add(&j.counters[28], P.nl + P.ns);
                if (lane() == 0) {
                    for (uint32_t k = 0; k < P.nl && first + k < j.zs_items_cap; k++)
                        j.zs_items[first + k] = soff + o_li + (uint64_t)k * sizeof(ZsLitItem);
                    for (uint32_t k = 0; k < P.ns && first + P.nl + k < j.zs_items_cap; k++)
                        j.zs_items[first + P.nl + k] = (soff + o_si + (uint64_t)k * sizeof(ZsSeqItem)) | (1ull << 63);
                    ZsFastDesc d{};
                    d.lit_off = kZsFastHdr;
                    d.rec_off = o_rec;
                    d.lcap = nl;
                    d.rcap = rcap;
                    d.items = o_li;
                    d.nitems = P.nl;
                    d.sitems = o_si;
                    d.nsitems = P.ns;
                    *(ZsFastDesc*)(j.inf_scratch + soff) = d;
                }
                state = kZsPlanned;
            }
        }
        if (lane() == 0) {
            j.inf_state[i] = state;
            j.inf_off[i] = soff;
        }
    }
}

// A per-lane bit-stream environment for k_zlits: each lane reads its own
// stream through its own LDS window (kW bytes ending just past the read: the
// streams move down), refilled with kW / 16 independent 16-byte loads issued
// together when a read leaves it.  (Reading each reload's 8 bytes straight
// from the payload put one global-memory latency on the chain every ~7
// literals: k_zlits was 27 ms of C6's member pass.)  uni: the whole wave
// reads one stream (a sequence section), its window filled 16 bytes per lane.
struct ZPer {
    const uint8_t* src;
    uint64_t n;
    inf_lds_u8* win;  // this stream's window: kW + 16 bytes, 16-aligned
    bool uni;
    static constexpr uint32_t kW = 256, kWU = 1024;
    DEV uint64_t fill(uint64_t pos) {
        const uint32_t W = uni ? kWU : kW;
        // [nb, nb + W) holds [pos, pos + 8) at its top (16-aligned base)
        const uint64_t nb = pos + 8 + 15 > W ? (pos + 8 + 15 - W) & ~15ull : 0;
        auto chunk = [&](uint64_t a) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (a + 16 <= n) {
                __builtin_memcpy(&v, (const __attribute__((address_space(1))) uint8_t*)(src + a), 16);
            } else {
                uint32_t w4[4] = {0u, 0u, 0u, 0u};
                for (uint32_t k = 0; k < 16; k++)
                    if (a + k < n) w4[k >> 2] |= (uint32_t)src[a + k] << (8 * (k & 3));
                v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
            return v;
        };
        if (uni) {
            const uint32_t l = lane();
            const uint4 v = chunk(nb + 16u * l);
            __builtin_memcpy(win + 16u * l, &v, 16);
            if (l == 0) {
                const uint4 t = chunk(nb + kWU);
                __builtin_memcpy(win + kWU, &t, 16);
            }
        } else {
            uint4 v[kW / 16 + 1];
#pragma unroll
            for (uint32_t c = 0; c <= kW / 16; c++) v[c] = chunk(nb + 16u * c);
#pragma unroll
            for (uint32_t c = 0; c <= kW / 16; c++) __builtin_memcpy(win + 16u * c, &v[c], 16);
        }
        __builtin_amdgcn_s_waitcnt(0);  // (the wave's LDS stores land before its reads)
        return nb;
    }
    DEV uint32_t b(uint64_t i) { return i < n ? (uint32_t)src[i] : 0u; }
    DEV uint64_t le(uint64_t i, uint32_t k) {
        uint64_t v = 0;
        for (uint32_t t = 0; t < k; t++) v |= (uint64_t)b(i + t) << (8 * t);
        return v;
    }
    DEV uint64_t lb(zs::Bits& s, uint64_t pos) {  // pos + 8 <= n
        const uint32_t W = uni ? kWU : kW;
        if (pos < s.wbase || pos + 8 > s.wbase + W) s.wbase = fill(pos);
        const uint32_t o = (uint32_t)(pos - s.wbase), a = o & ~3u, sh = o & 3u;
        typedef const __attribute__((address_space(3))) uint32_t lds_cu32_t;
        const uint32_t d0 = *(lds_cu32_t*)(win + a), d1 = *(lds_cu32_t*)(win + a + 4), d2 = *(lds_cu32_t*)(win + a + 8);
        return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
    }
    DEV uint32_t U(uint32_t x) { return x; }
    DEV zs::SeqSym sym(const zs::SeqSym& t) { return t; }
};
// k_zlits' LDS: the tables, then the sequence stream's window, then the four
// literal streams' windows
constexpr uint32_t kZlitsWinU = kZsTabBytes;
constexpr uint32_t kZlitsWinL = kZlitsWinU + ZPer::kWU + 16;
constexpr uint32_t kZlitsLds = kZlitsWinL + 4 * (ZPer::kW + 16);

// a planned sequence section: its FSE tables into LDS, its stream decoded by
// zs::seq_decode into raw sequences (every lane computes the same values,
// lane 0 stores them), then whether the stream ended exactly
DEV void zseq_item(const DeviceJob& j, zs::Tabs* T, ZsSeqItem* it, inf_lds_u8* win) {
    const uint32_t l = lane();
    const uint32_t* tab = (const uint32_t*)(j.inf_scratch + uni64(it->tab));
    uint32_t* dst = (uint32_t*)T->ll;
    for (uint32_t u = l; u < (uint32_t)(kZsSeqTab / 4); u += 64) dst[u] = tab[u];
    __builtin_amdgcn_s_waitcnt(0);
    ZPer e{j.data + uni64(it->src), uni64(it->n), win, true};
    const uint32_t nseq = uni32(it->nseq);
    zs::RawSeq* out = (zs::RawSeq*)(j.inf_scratch + uni64(it->seqs));
    zs::Bits d;
    uint32_t st = 0;
    if (zs::bits_init(e, d, uni64(it->sp), uni64(it->sn))) {
        zs::SeqState q;
        zs::seq_begin(e, d, q, uni32(it->llog), uni32(it->olog), uni32(it->mlog));
        for (uint32_t k = 0; k < nseq; k++) {
            zs::RawSeq r;
            zs::seq_decode(e, T, d, q, r);
            if (l == 0) out[k] = r;
        }
        st = zs::bits_reload(e, d) >= zs::kCompleted ? 1u : 2u;
    }
    if (l == 0) it->status = st;
}

// k_zlits: one wave per planned literal block, one LANE per Huffman stream
// (the four streams of a block are independent: lane q decodes stream q
// into its segment of the member's literal buffer, all four through the
// block's table snapshot in LDS, each lane's last symbol by zs::huf_one's
// X2 rule); then whether every stream ended exactly (what lits_finish checks)
__global__ __launch_bounds__(64) void k_zlits(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    zs::Tabs* T = (zs::Tabs*)lds;  // the tables only (no ring): kZsTabBytes of LDS, more waves per CU
    const uint32_t reg = j.counters[28];
    const uint32_t count = reg < j.zs_items_cap ? reg : j.zs_items_cap;
    const uint32_t l = lane();
    for (;;) {
        const uint32_t k = wave_fetch_add(&j.counters[29], 1u);
        if (k >= count) break;
        const uint64_t ref = uni64(j.zs_items[k]);
        if (ref >> 63) {
            zseq_item(j, T, (ZsSeqItem*)(j.inf_scratch + (ref & ~(1ull << 63))), (inf_lds_u8*)(lds + kZlitsWinU));
            continue;
        }
        ZsLitItem* it = (ZsLitItem*)(j.inf_scratch + ref);
        const uint32_t hlog = uni32(it->hlog), ns = uni32(it->ns);
        const uint16_t* tab = (const uint16_t*)(j.inf_scratch + uni64(it->tab));
        for (uint32_t u = l; u < (1u << hlog); u += 64) T->huf[u] = tab[u];
        __builtin_amdgcn_s_waitcnt(0);  // (one wave: its LDS stores land before its loads)
        bool ok = true;
        if (l < ns) {
            ZPer e{j.data + it->src, it->n, (inf_lds_u8*)(lds + kZlitsWinL + (ZPer::kW + 16) * l), false};
            const uint32_t cnt = it->cnt[l], seg = it->seg;
            const bool x2 = it->x2 != 0;
            uint8_t* dst = j.inf_scratch + it->lits + (uint64_t)l * seg;
            zs::Bits s;
            uint32_t open = 0;
            ok = zs::bits_init(e, s, it->s0[l], it->sn[l]);
            if (ok) {
                for (uint32_t i = 0; i + 1 < cnt; i++) {
                    if (s.used > 64 - hlog) zs::bits_reload(e, s);
                    const uint32_t d = T->huf[(uint32_t)((s.c << (s.used & 63)) >> ((64 - hlog) & 63))];
                    const uint32_t l1 = d >> 8;
                    if (x2) open = (open && open + l1 <= 12) ? 0u : l1;
                    s.used += l1;
                    dst[i] = (uint8_t)d;
                }
                if (cnt) dst[cnt - 1] = (uint8_t)zs::huf_one(e, T, s, open, 1, x2, hlog);
                zs::bits_reload(e, s);
                ok = zs::bits_end(s);
            }
        }
        const bool all = __ballot(!ok) == 0;
        if (l == 0) it->status = all ? 1u : 2u;
    }
}

__global__ __launch_bounds__(64) void k_zparse(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t count = j.counters[16];
    for (uint32_t phase = 0; phase < 2; phase++) {
        for (;;) {
            const uint32_t i = wave_fetch_add(&j.counters[phase ? 23 : 22], 1u);
            if (i >= count) break;
            if (uni32(j.inf_state[i]) != kZsPlanned) continue;
            const uint32_t b = uni32(j.inf_list[i]);
            const rpgpu_batch_result* R = &j.batches[b];
            const bool big = uni32((uint32_t)R->size_bytes) >= (128u << 10);
            if (big != (phase == 0)) continue;
            if (!zstd_fast_item(j, lds, i, b, R) && lane() == 0) j.inf_state[i] = kZsPending;
        }
    }
}

__global__ __launch_bounds__(64) void k_zfallback(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t count = j.counters[16];
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[26], 1u);
        if (i >= count) break;
        const uint32_t b = uni32(j.inf_list[i]);
        const rpgpu_batch_result* R = &j.batches[b];
        if ((uni32((uint32_t)(uint16_t)R->attrs) & 7u) == RPGPU_CODEC_GZIP) continue;
        if (uni32(j.inf_state[i]) != kZsPending) continue;
        zstd_first_item(j, lds, i, b, R);
    }
}

__global__ __launch_bounds__(64) void k_members(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    InfTabs* T = (InfTabs*)(lds + kInfRing);
    const InfWave W = inf_wave();
    bool tab = false;
    const uint32_t count = j.counters[16];
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[18], 1u);
        if (i >= count) break;
        if (uni32(j.inf_state[i]) != 2) continue;
        const uint32_t b = uni32(j.inf_list[i]);
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t dst = uni64(j.dcap[b]), cap = uni64(j.dcap[b + 1]) - dst;
        if (dst + cap > j.decoded_capacity) {
            if (lane() == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
            continue;
        }
        if ((uni32((uint32_t)(uint16_t)R->attrs) & 7u) == RPGPU_CODEC_GZIP) {
            if (!tab) inf_load_tab(T->crc_tab);
            tab = true;
            gzip_item(j, lds, T, W, R, dst, cap);
        } else {
            tab = false;
            zstd_item(j, lds, R, dst, cap);
        }
    }
}

#ifdef RPGPU_ZSTAMPS
__global__ void k_zstamps(int print) {
    if (print)
        printf("RPGPU_ZSTAMPS payloads=%llu out=%llu wall_ms(sum) lits=%.1f match=%.1f ends=%.1f blocks=%.1f total=%.1f max_payload_ms=%.2f\n",
               g_zst[5], g_zst[6], g_zst[0] * 1e-5, g_zst[1] * 1e-5, g_zst[2] * 1e-5, g_zst[3] * 1e-5,
               g_zst[4] * 1e-5, g_zst[7] * 1e-5);
    if (print)
        printf("RPGPU_ZSTAMPS lane-parse payloads=%llu recs=%llu lits=%llu wall_ms(sum) lits=%.1f match=%.1f ends=%.1f blocks=%.1f total=%.1f max_payload_ms=%.2f\n",
               g_zst[13], g_zst[14] & 0xFFFFFFFFull, g_zst[14] >> 32, g_zst[8] * 1e-5, g_zst[9] * 1e-5,
               g_zst[10] * 1e-5, g_zst[11] * 1e-5, g_zst[12] * 1e-5, g_zst[15] * 1e-5);
    for (int k = 0; k < 16; k++) g_zst[k] = 0;
}
#endif

hipError_t launch_zstamps(hipStream_t s, int print) {
#ifdef RPGPU_ZSTAMPS
    hipLaunchKernelGGL(k_zstamps, dim3(1), dim3(1), 0, s, print);
#else
    (void)s;
    (void)print;
#endif
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The split decode's kernels (see "Split decode of large gzip members").
// ---------------------------------------------------------------------------
DEV void gzs_null(DeviceJob& j, uint32_t from, uint32_t to) {
    for (uint32_t t = from; t < to && t < j.gzs_items_cap; t++) j.gzs_items[t].member = ~0u;
}

// one thread per member: the gzip header, the chunks
__global__ __launch_bounds__(256) void k_gzsplan(DeviceJob j) {
    const uint32_t count = j.counters[16];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    j.gzs_mem[2 * i] = 0;
    j.gzs_mem[2 * i + 1] = 0;
    const uint32_t b = j.inf_list[i];
    const rpgpu_batch_result* R = &j.batches[b];
    if (((uint32_t)(uint16_t)R->attrs & 7u) != RPGPU_CODEC_GZIP) return;
    const uint64_t n = (uint64_t)(uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE);
    if (n < kGzsMin) return;
    const uint8_t* p = j.data + j.seg_off[R->segment] + R->file_pos + RPGPU_HEADER_SIZE;
    // RFC 1952 header: magic, CM 8, no reserved flags, no FHCRC
    if (p[0] != 0x1fu || p[1] != 0x8bu || p[2] != 8u || (p[3] & 0xe2u)) return;
    uint64_t h = 10;
    if (p[3] & 4u) h = 12 + ((uint64_t)p[10] | ((uint64_t)p[11] << 8));
    for (uint32_t f = 8; f <= 16; f <<= 1) {
        if (!(p[3] & f)) continue;
        while (h < n && p[h]) h++;
        if (h >= n) return;
        h++;
    }
    if (h + kGzsChunk > n) return;
    const uint64_t isize = rd32h(p + n - 4);
    uint64_t g = isize < 1032ull * n + 64 ? isize : 1032ull * n + 64;
    const uint64_t nd = n - h;
    uint32_t nk = (uint32_t)((nd + kGzsChunk - 1) / kGzsChunk);
    nk = nk < kGzsMaxK ? nk : kGzsMaxK;
    const uint64_t csz = (nd + nk - 1) / nk;
    const uint32_t base = atomicAdd(&j.counters[32], nk);
    if ((uint64_t)base + nk > j.gzs_items_cap) {
        gzs_null(j, base, base + nk);
        return;
    }
    for (uint32_t k = 0; k < nk; k++) {
        GzsItem& it = j.gzs_items[base + k];
        it.member = i;
        it.k = k;
        it.nk = nk;
        it.status = 0;
        it.begin = h + k * csz;
        it.end = h + (k + 1) * csz < n ? h + (k + 1) * csz : n;
        it.start = k == 0 ? 8 * h : ~0ull;
        it.stop = 0;
        it.out = 0;
        it.len = 0;
        it.guess = g;
        it.cap = 0;
    }
    j.gzs_mem[2 * i] = base;
    j.gzs_mem[2 * i + 1] = nk;
}

// the first dynamic-block header of each chunk k >= 1
constexpr uint32_t kGzsFindLds = 64 * 128 + kGzsWin;
__global__ __launch_bounds__(64) void k_gzsfind(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t l = lane();
    inf_lds_u8* tb = (inf_lds_u8*)lds + 128 * l;
    gzs_lds_u32* w = (gzs_lds_u32*)(lds + 64 * 128);
    const uint32_t nit = min(j.counters[32], j.gzs_items_cap);
    for (;;) {
        const uint32_t t = wave_fetch_add(&j.counters[33], 1u);
        if (t >= nit) break;
        GzsItem* it = &j.gzs_items[t];
        if (uni32(it->member) == ~0u || uni32(it->k) == 0) continue;
        const uint32_t b = uni32(j.inf_list[uni32(it->member)]);
        const InfIn in = inf_batch(j, &j.batches[b]);
        const uint64_t nbits = in.n * 8, pend = 8 * uni64(it->end);
        // the chunk's bytes (and 2 KiB past them) into LDS
        const uint64_t wa = (uni64(it->begin) + in.mis) & ~3ull;
        for (uint32_t d = l; d < kGzsWin / 4; d += 64) w[d] = inf_ld(in, wa + 4ull * d);
        // 64 bit positions per lane, 4096 per step: the fixed header bits
        // (BFINAL 0, BTYPE 2, HLIT <= 29, HDIST <= 29) of all 64 at once from
        // the lane's 160 stream bits (word shifts), the code-length code's
        // Kraft sum per survivor (~9 % of positions), then the full header
        // check (gzs_check) lane-parallel on the Kraft survivors in position
        // order.  (One position per lane per step spent ~100 instructions a
        // position: 26 ms of C6's member pass.)
        const uint64_t q_lo = 8 * uni64(it->begin);
        const uint64_t q_hi = pend < (nbits >= 128 ? nbits - 127 : 0) ? pend : (nbits >= 128 ? nbits - 127 : 0);
        const uint64_t pb0 = (q_lo + 8ull * in.mis) & ~63ull;  // physical bit, 64-aligned
        uint64_t found = ~0ull;
        for (uint64_t pb = pb0; found == ~0ull; pb += 4096) {
            const uint64_t plane = pb + 64ull * l;     // this lane's first physical bit
            const uint64_t ql = plane - 8ull * in.mis;  // ... as a stream bit position
            if (uni64(pb - 8ull * in.mis) >= q_hi) break;
            // valid positions ql + i: q_lo <= . < q_hi
            uint64_t vm = 0;
            if (ql + 64 > q_lo && ql < q_hi) {
                const uint32_t i0 = q_lo > ql ? (uint32_t)(q_lo - ql) : 0u;
                const uint32_t i1 = q_hi - ql < 64 ? (uint32_t)(q_hi - ql) : 64u;
                vm = (i1 >= 64 ? ~0ull : ((1ull << i1) - 1)) & ~((1ull << i0) - 1);
            }
            const uint64_t a = plane >> 3;
            const uint32_t d0 = gzs_dw(in, a, w, wa), d1 = gzs_dw(in, a + 4, w, wa), d2 = gzs_dw(in, a + 8, w, wa),
                           d3 = gzs_dw(in, a + 12, w, wa), d4 = gzs_dw(in, a + 16, w, wa);
            const uint64_t lo = (uint64_t)d1 << 32 | d0, hi = (uint64_t)d3 << 32 | d2;
#define GZS_SH(k) ((lo >> (k)) | (hi << (64 - (k))))
            uint64_t m = vm & ~lo & ~GZS_SH(1) & GZS_SH(2);
            m &= ~(GZS_SH(4) & GZS_SH(5) & GZS_SH(6) & GZS_SH(7));
            m &= ~(GZS_SH(9) & GZS_SH(10) & GZS_SH(11) & GZS_SH(12));
#undef GZS_SH
            // the code-length code of each survivor: HCLEN at i + 13, 19 x 3 bits after
            uint64_t km = 0;
            for (uint64_t mm = m; mm; mm &= mm - 1) {
                const uint32_t i = (uint32_t)__builtin_ctzll(mm), o = i + 13;
                const uint32_t k = o >= 64 ? o - 64 : 0u;
                const uint64_t v = o < 64 ? (lo >> o) | (hi << (64 - o))
                                          : (hi >> k) | (k ? (uint64_t)d4 << (64 - k) : 0ull);
                const uint32_t ncode = (uint32_t)(v & 15u) + 4;
                const uint64_t x = v >> 4;
                uint32_t kr = 0;
#pragma unroll
                for (uint32_t q = 0; q < 19; q++) {
                    const uint32_t L = (uint32_t)(x >> (3 * q)) & 7u;
                    if (q < ncode && L) kr += 128u >> L;
                }
                if (kr == 128u) km |= 1ull << i;
            }
            // the full check, each lane on its survivors in order; the answer
            // is the lowest position that passes once every lower survivor
            // (lower lanes' included) has failed
            uint64_t best = ~0ull;
            for (;;) {
                const uint64_t mine = km ? ql + (uint64_t)__builtin_ctzll(km) : ~0ull;
                const bool go = mine < best;
                if (!__ballot(go)) break;
                bool ok = false;
                if (go) {
                    ok = gzs_check(in, mine, tb, nbits, w, wa);
                    km &= km - 1;
                }
                uint64_t cand = ok ? mine : ~0ull;
#pragma unroll
                for (int sh = 32; sh > 0; sh >>= 1) {
                    const uint64_t o2 = __shfl_xor(cand, sh, 64);
                    cand = o2 < cand ? o2 : cand;
                }
                best = cand < best ? cand : best;
            }
            found = uni64(best);
        }
        if (l == 0) it->start = found;
    }
}

// each chunk from its block start to the next chunk's
__global__ __launch_bounds__(64) void k_gzsdecode(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    gzs_lds_u16* ring = (gzs_lds_u16*)lds;
    InfTabs* T = (InfTabs*)(lds + 2 * kGzsRing);
    const InfSymTabs ST = inf_sym_tabs();
    const uint32_t nit = min(j.counters[32], j.gzs_items_cap);
    unsigned long long* used = (unsigned long long*)(j.counters + 36);
    for (;;) {
        const uint32_t t = wave_fetch_add(&j.counters[34], 1u);
        if (t >= nit) break;
        GzsItem* it = &j.gzs_items[t];
        if (uni32(it->member) == ~0u) continue;
        const uint64_t start = uni64(it->start);
        if (start == ~0ull) continue;
        const uint32_t k = uni32(it->k), nk = uni32(it->nk);
        uint64_t stop = ~0ull;
        for (uint32_t u = t + 1; u < t + (nk - k); u++) {
            const uint64_t s2 = uni64(j.gzs_items[u].start);
            if (s2 != ~0ull) {
                stop = s2;
                break;
            }
        }
        const uint32_t b = uni32(j.inf_list[uni32(it->member)]);
        InfIn in = inf_batch(j, &j.batches[b]);
        // the region: twice the member's output per deflate byte over the
        // span, plus 16 K symbols, capped by the whole member's guess
        const uint64_t h = uni64(j.gzs_items[t - k].begin), g = uni64(it->guess);
        const uint64_t span = ((stop == ~0ull ? in.n * 8 : stop) - start) / 8 + 1;
        const uint64_t ratio = (g + (in.n - h) - 1) / (in.n - h);
        uint64_t want = 2 * ratio * span + 16384;
        want = want < g + 2048 ? want : g + 2048;
        // a fixed share of the pool per chunk: one payload-controlled ISIZE
        // cannot give each of a member's chunks the whole member's guess
        want = want < j.gzs_pool_syms / 32 ? want : j.gzs_pool_syms / 32;
        want = (want + 1023) & ~1023ull;
        want = want < 0xFFFFFC00ull ? want : 0xFFFFFC00ull;
        const uint64_t off = uni64(atomicAdd(used, lane() == 0 ? (unsigned long long)want : 0ull));
        int st = -3;
        uint64_t bp = start, total = 0;
        if (off + want <= j.gzs_pool_syms) {
            // positions -8192 .. -1: their placeholders
            for (uint32_t q = lane(); q < kGzsRing; q += 64) ring[q] = (uint16_t)(256u + 32768u - kGzsRing + q);
            GzsOut o;
            o.ring = ring;
            o.dst = j.gzs_pool + off;
            o.rs = __builtin_amdgcn_make_buffer_rsrc(o.dst, 0, (int)(2 * want < 0x7FFFFFFFull ? 2 * want : 0x7FFFFFFFull), kBufFlagsZs);
            o.flushed = 0;
            o.cap = want;
            o.over = false;
            st = gzs_run(in, T, o, ST, bp, stop, k != 0, total);
        }
        if (lane() == 0) {
            it->out = off;
            it->cap = (uint32_t)want;
            it->stop = bp;
            it->len = total;
            it->status = st;
        }
    }
}

// per member (256 threads): the chain, the bytes, the check, the plan
__global__ __launch_bounds__(256) void k_gzsresolve(DeviceJob j) {
    __shared__ uint32_t tab[256], raw[256], xp[256];
    __shared__ uint32_t chain[kGzsMaxK];
    __shared__ uint64_t coff[kGzsMaxK];
    __shared__ uint32_t s_i, s_n, s_verdict, s_bad;
    __shared__ uint64_t s_total, s_soff, s_end;
    const uint32_t tid = threadIdx.x;
    {
        uint32_t c = tid;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        tab[tid] = c;
    }
    const uint32_t count = j.counters[16];
    for (;;) {
        __syncthreads();
        if (tid == 0) s_i = atomicAdd(&j.counters[35], 1u);
        __syncthreads();
        const uint32_t i = s_i;
        if (i >= count) break;
        const uint32_t nk = j.gzs_mem[2 * i + 1];
        if (nk == 0) continue;
        const uint32_t b = j.inf_list[i];
        rpgpu_batch_result* R = &j.batches[b];
        const uint64_t S = j.seg_off[R->segment] + R->file_pos + RPGPU_HEADER_SIZE;
        const uint64_t n = (uint64_t)(uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE);
        const uint8_t* src = j.data + S;
        if (tid == 0) {
            // verdict: 0 decoded to the end (s_end: the final block's end, ~0
            // the input ran out), 1 a stream error (-1), 3 not closed: serial
            const GzsItem* I = j.gzs_items + j.gzs_mem[2 * i];
            uint32_t c = 0, nc = 0, v = 3;
            uint64_t tot = 0, end = ~0ull;
            for (;;) {
                const GzsItem& it = I[c];
                if (it.status == 1 || it.status == 2 || it.status == 3) {
                    chain[nc] = c;
                    coff[nc] = tot;
                    nc++;
                    tot += it.len;
                    if (it.status == 2) { v = 0; end = it.stop; break; }
                    if (it.status == 3) { v = 0; break; }
                    uint32_t u = c + 1;
                    while (u < nk && I[u].start == ~0ull) u++;
                    if (u >= nk || I[u].start != it.stop) break;  // (cannot happen: the decode stopped there)
                    c = u;
                    continue;
                }
                if (it.status == -1) v = 1;
                break;
            }
            uint64_t soff = 0;
            if (v == 0) {
                const uint64_t cap = (tot + 15) & ~15ull;
                soff = atomicAdd((unsigned long long*)j.inf_scratch_used, (unsigned long long)cap);
                if (soff + cap > j.inf_scratch_bytes) v = 3;
            }
            s_n = nc;
            s_total = tot;
            s_end = end;
            s_soff = soff;
            s_verdict = v;
            s_bad = 0;
        }
        __syncthreads();
        const uint32_t v0 = s_verdict;
        if (v0 == 3) continue;
        uint32_t rc = v0 == 1 ? 1u : 0u;  // 0 accept, 1 reject (-1), 2 reject (-2: the check)
        const uint64_t total = s_total;
        if (v0 == 0) {
            uint8_t* dst = j.inf_scratch + s_soff;
            const GzsItem* I = j.gzs_items + j.gzs_mem[2 * i];
            for (uint32_t w = 0; w < s_n; w++) {
                const GzsItem& it = I[chain[w]];
                const uint16_t* sy = j.gzs_pool + it.out;
                const uint64_t len = it.len, off = coff[w];
                bool bad = false;
                for (uint64_t e = 8ull * tid; e < len; e += 8ull * 256) {
                    const uint4 q = *(const uint4*)(sy + e);
                    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (uint32_t k = 0; k < 8; k++) {
                        if (e + k >= len) break;
                        const uint32_t s = (wd[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                        uint8_t y = (uint8_t)s;
                        if (s >= 256) {
                            const int64_t g = (int64_t)off + (int64_t)(s - 256) - (int64_t)kInfRing;
                            if (g < 0) bad = true;
                            else y = dst[g];
                        }
                        dst[off + e + k] = y;
                    }
                }
                if (bad) s_bad = 1;
                __syncthreads();
            }
            if (s_bad) {
                rc = 1;
            } else if (s_end != ~0ull) {
                // CHECK, LENGTH: inflate_member's rules on the trailer
                const uint64_t bp = (s_end + 7) & ~7ull, nbits = n * 8;
                if (nbits - bp >= 32) {
                    const uint64_t seg = ((total + 255) / 256 + 15) & ~15ull;
                    const uint64_t a = seg * tid, z = a + seg < total ? a + seg : total;
                    uint32_t c = 0;
                    for (uint64_t x = a; x < z; x++) c = tab[(c ^ dst[x]) & 0xFFu] ^ (c >> 8);
                    raw[tid] = c;
                    uint32_t pw = 1u << 31;
                    const uint64_t ln = z > a ? z - a : 0;
                    for (uint32_t k = 0; (ln >> k) != 0; k++)
                        if ((ln >> k) & 1) pw = ieee_mulmod(kX2nIeee[(3 + k) & 31], pw);
                    xp[tid] = z > a ? pw : 0u;
                    __syncthreads();
                    if (tid == 0) {
                        uint32_t crc = 0xFFFFFFFFu;
                        for (uint32_t t = 0; t < 256; t++)
                            if (xp[t]) crc = ieee_mulmod(xp[t], crc) ^ raw[t];
                        const uint8_t* tr = src + (bp >> 3);
                        if (rd32h(tr) != ~crc) s_bad = 2;
                        else if (nbits - bp >= 64 && rd32h(tr + 4) != (uint32_t)total) s_bad = 2;
                    }
                    __syncthreads();
                    if (s_bad) rc = 2;
                }
            }
        }
        if (tid == 0) {
            const uint64_t cap = rc == 1 ? 0 : (total + 15) & ~15ull;
            const int32_t rcount = R->record_count;
            j.dcap[b] = cap;
            j.slots[b] = ((j.flags & RPGPU_JOB_PARSE) && rcount > 0 && (uint64_t)rcount <= cap) ? (uint64_t)rcount : 0;
            j.inf_state[i] = rc != 0 ? 1u : 0u;
            j.inf_off[i] = rc == 1 ? 0 : s_soff;
            j.inf_total[i] = rc == 1 ? 0 : total;
            j.gzs_mem[2 * i + 1] = nk | (1u << 31);
        }
    }
}

hipError_t launch_gzsplan(const DeviceJob& j, hipStream_t s) {
    const uint32_t pg = (uint32_t)((j.batch_capacity + 255) / 256);
    hipLaunchKernelGGL(k_gzsplan, dim3(pg ? pg : 1), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_gzsplit(const DeviceJob& j, hipStream_t s, uint32_t grid, int part) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_gzsdecode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGzsLds);
        (void)hipFuncSetAttribute((const void*)k_gzsfind, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGzsFindLds);
        attr = true;
    }
    if (part != 2) hipLaunchKernelGGL(k_gzsfind, dim3(grid * 5), dim3(64), kGzsFindLds, s, j);
    if (part != 1) {
        hipLaunchKernelGGL(k_gzsdecode, dim3(grid * RPGPU_GZS_WGS), dim3(64), kGzsLds, s, j);
        hipLaunchKernelGGL(k_gzsresolve, dim3(grid * 2), dim3(256), 0, s, j);
    }
    return hipGetLastError();
}

hipError_t launch_inflate_plan(const DeviceJob& j, hipStream_t s, uint32_t grid, int pass) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_members_first, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMemLds);
        attr = true;
    }
    hipLaunchKernelGGL(k_members_first, dim3(grid), dim3(64), kMemLds, s, j, pass);
    return hipGetLastError();
}

hipError_t launch_zplan(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_zplan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMemLds);
        attr = true;
    }
    hipLaunchKernelGGL(k_zplan, dim3(grid), dim3(64), kMemLds, s, j);
    return hipGetLastError();
}

hipError_t launch_zparse(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_zlits, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kZlitsLds);
        (void)hipFuncSetAttribute((const void*)k_zparse, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMemLds);
        attr = true;
    }
    hipLaunchKernelGGL(k_zlits, dim3(grid * 2), dim3(64), kZlitsLds, s, j);
    hipLaunchKernelGGL(k_zparse, dim3(grid), dim3(64), kMemLds, s, j);
    return hipGetLastError();
}

hipError_t launch_zfallback(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_zfallback, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMemLds);
        attr = true;
    }
    hipLaunchKernelGGL(k_zfallback, dim3(grid), dim3(64), kMemLds, s, j);
    return hipGetLastError();
}

hipError_t launch_zexact(const DeviceJob& j, hipStream_t s, int pass) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_zexact, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kZsTabBytes);
        attr = true;
    }
    hipLaunchKernelGGL(k_zexact, dim3(1), dim3(64), kZsTabBytes, s, j, pass);
    return hipGetLastError();
}

hipError_t launch_inflate(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_members, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMemLds);
        attr = true;
    }
    hipLaunchKernelGGL(k_inflate_copy, dim3(grid), dim3(64 * 4), 0, s, j);
    hipLaunchKernelGGL(k_members, dim3(grid), dim3(64), kMemLds, s, j);
    return hipGetLastError();
}

}  // namespace rp
