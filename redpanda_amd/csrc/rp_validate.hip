// rp_validate.hip — k_validate: the batch CRC32C (model/record_utils.cc:68-91
// as checked by storage/log_replayer.cc:48-79), reset_size_checksum_metadata
// over decoded payloads (storage/parser_utils.cc:114-120) and the record walk
// into the offset index (model/record.h:616-627, model/record_utils.cc:94-181).
//
// One wave per batch, 16 waves per CU (4 per SIMD, so LDS and memory latency
// of one wave hide behind the others), persistent grid of one workgroup per
// CU.  A payload is processed in 16 KiB windows of 16 rows of 1 KiB; lane l
// loads bytes [1024 i + 16 l, +16) of each row i (one fully coalesced
// dwordx4 per row) and runs 4 braided CRC chains over them: braid (l, k) is
// dword k of the lane's 16 bytes in every row, so one step covers the word
// plus the 1020 bytes of the other 255 braids (tables T1023..T1020,
// replicated 32x in LDS: every lookup bank-conflict-free).  Row 15 folds the
// lane's four braids back into one state with plain word steps, and the 64
// lane states are merged with GF(2) shift tables over a shuffle tree (shift
// by 16 << m bytes, m = 0..5).
//
// The record walk: a uniform chain over the record length varints read
// through the scalar cache, then one record per lane read from L2 (the wave
// has just streamed these bytes) through 32-byte per-lane caches; the other
// 15 waves of the CU cover the latency.  Integer/byte work only: HBM-bound,
// no MFMA.
#include "rp_device.h"

namespace rp {

// Diagnostic build (-DRPGPU_STAMPS, librpgpu_stamps.so): per-phase s_memtime
// cycle totals summed over all waves, printed by k_print_stamps.  Never
// benchmarked.
#ifdef RPGPU_STAMPS
__device__ unsigned long long g_stamps[8];
__shared__ unsigned long long s_stamps[kVWaves][8];  // per-wave, flushed once at the end
#define STAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(i, d) do { if (lane() == 0) s_stamps[threadIdx.x >> 6][i] += (unsigned long long)(d); } while (0)
#else
#define STAMP(v)
#define STAMP_ADD(i, d)
#endif

DEV uint32_t L32(const uint8_t* lds, uint32_t a) { return *(const uint32_t*)(lds + a); }

// The lane id from a volatile asm: values derived from it cannot be hoisted
// out of the batch loop (loop-invariant per-lane pointers and masks would
// otherwise stay live for the whole kernel and push it into spills; they
// cost two VALU to recompute)
DEV uint32_t lane_v() {
    uint32_t r;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
    return r;
}

// constant address space: wave-uniform loads through it become s_load (the
// scalar cache), off the vector-memory queue the window stream keeps busy
typedef const __attribute__((address_space(4))) uint32_t cu32;

// LDS address keys of the four braid tables for this lane's copy:
// {slot * 128 + 4 c, -, row-set, -}; v_perm inserts the entry byte.
struct Keys {
    uint32_t k15, k14, k13, k12;
};
constexpr uint32_t kSel0 = 0x0C020400u;  // {key.b0, x.b0, key.b2, 0}
constexpr uint32_t kSel1 = 0x0C020500u;  // x byte 1
constexpr uint32_t kSel2 = 0x0C020600u;  // x byte 2
constexpr uint32_t kSel3 = 0x0C020700u;  // x byte 3

DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// One braid step from x = s ^ w: s' = T1023[x0] ^ T1022[x1] ^ T1021[x2] ^
// T1020[x3], the CRC of the word followed by the 1020 bytes of the other
// braids.  The state is kept as the pair (p, q) with s' = p ^ q, so the next
// step's x is one 3-input XOR (v_bitop3) with the next word.
DEV void braid_step(const uint8_t* lds, const Keys& K, uint32_t x, uint32_t& p, uint32_t& q) {
    const uint32_t a = L32(lds, __builtin_amdgcn_perm(x, K.k15, kSel0));
    const uint32_t b = L32(lds, __builtin_amdgcn_perm(x, K.k14, kSel1));
    const uint32_t c = L32(lds, __builtin_amdgcn_perm(x, K.k13, kSel2));
    const uint32_t d = L32(lds, __builtin_amdgcn_perm(x, K.k12, kSel3));
    p = xor3(a, b, c);
    q = d;
}

// slice-by-4 word step (T3..T0, single copy) from x = s ^ w, xored with e
DEV uint32_t word_step_x(const uint8_t* lds, uint32_t x, uint32_t e) {
    return xor3(xor3(L32(lds, kLdsSlice4Off + ((x & 0xFFu) << 2)), L32(lds, kLdsSlice4Off + 1024u + ((x >> 6) & 0x3FCu)),
                     L32(lds, kLdsSlice4Off + 2048u + ((x >> 14) & 0x3FCu))),
                L32(lds, kLdsSlice4Off + 3072u + ((x >> 22) & 0x3FCu)), e);
}

DEV uint32_t word_step(const uint8_t* lds, uint32_t s, uint32_t w) { return word_step_x(lds, s ^ w, 0u); }

DEV uint32_t byte_step(const uint8_t* lds, uint32_t s, uint32_t b) {
    return L32(lds, kLdsSlice4Off + 3072u + (((s ^ b) & 0xFFu) << 2)) ^ (s >> 8);
}

// advance a raw CRC state over 16 << k zero bytes, xored with e
DEV uint32_t shift_k(const uint8_t* lds, uint32_t s, uint32_t k, uint32_t e) {
    const uint32_t base = kLdsShiftOff + k * 4096u;
    return xor3(xor3(L32(lds, base + ((s & 0xFFu) << 2)), L32(lds, base + 1024u + ((s >> 6) & 0x3FCu)),
                     L32(lds, base + 2048u + ((s >> 14) & 0x3FCu))),
                L32(lds, base + 3072u + ((s >> 22) & 0x3FCu)), e);
}

// select a dword by index from values (never from addresses: a select of
// pointers would pin the register arrays in scratch)
DEV uint32_t pick4(uint4 v, uint32_t k) {
    const uint32_t x = v.x, y = v.y, z = v.z, w = v.w;
    const uint32_t lo = (k & 1u) ? y : x, hi = (k & 1u) ? w : z;
    return (k & 2u) ? hi : lo;
}

// One 16-byte row of the payload stream, loaded non-temporal: every byte is
// read once per launch, and with the default policy the window stream
// displaced lines other waves were still waiting on (measured on C1:
// k_validate 3.20 -> 2.96 ms; RPGPU_NT_WINDOW=0 restores the default policy
// for A/B).
#ifndef RPGPU_NT_WINDOW
#define RPGPU_NT_WINDOW 1
#endif
DEV uint4 ld_stream(const uint8_t* p) {
    if (RPGPU_NT_WINDOW) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_nontemporal_load((const v4u*)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *(const uint4*)p;
}

// A lane's share of the current window: dword k of row i in d[i] (rows
// 0..15, 16 bytes at 1024 i + 16 l).
struct Win {
    uint4 r[16];
};

// Bytes [S, E) of src (offsets from a 16-byte aligned base).  E16 = E rounded
// down to 16.  When E16 > S, windows are anchored at E16: window r covers
// [E16 - 16K (R - r), +16K) (window 0 may start before S) and the < 16-byte
// tail [E16, E) is folded in after them; otherwise the whole payload lies in
// the 16-byte row at E16 and is all tail.
struct Stream {
    const uint8_t* src;
    uint64_t S, E, E16, R;
};

DEV Stream make_stream(const uint8_t* src, uint64_t S, uint64_t E) {
    Stream st;
    st.src = src;
    st.S = S;
    st.E = E;
    st.E16 = E & ~15ull;
    st.R = st.E16 > S ? (st.E16 - S + kWinBytes - 1) / kWinBytes : 0;
    return st;
}

DEV int64_t win_base(const Stream& st, uint64_t r) {
    return (int64_t)st.E16 - (int64_t)kWinBytes * (int64_t)(st.R - r);
}

// window r, coalesced: row i of every lane is one 1 KiB wave load (rows
// wholly outside [S, E16) are zero)
DEV void load_window(const Stream& st, uint64_t r, Win& w) {
    const int64_t a = win_base(st, r) + 16 * (int64_t)lane_v();
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int64_t q = a + 1024 * i;
        uint4 t = make_uint4(0u, 0u, 0u, 0u);
        if (q + 16 > (int64_t)st.S && q < (int64_t)st.E16) t = ld_stream(st.src + q);
        w.r[i] = t;
    }
}

// rows [I0, I1) of window 0 only (the software pipeline issues a batch's
// window in two parts)
template <int I0, int I1>
DEV void load_rows(const Stream& st, Win& w) {
    const int64_t a = win_base(st, 0) + 16 * (int64_t)lane_v();
#pragma unroll
    for (int i = I0; i < I1; i++) {
        const int64_t q = a + 1024 * i;
        uint4 t = make_uint4(0u, 0u, 0u, 0u);
        if (q + 16 > (int64_t)st.S && q < (int64_t)st.E16) t = ld_stream(st.src + q);
        w.r[i] = t;
    }
}

// the 16-byte row at E16 holding the tail (uniform)
DEV uint4 load_tail(const Stream& st) {
    uint4 t = make_uint4(0u, 0u, 0u, 0u);
    if (st.E > st.E16) t = *(const uint4*)(st.src + st.E16);
    return t;
}

// lane l ^ X's value within 32-lane halves (ds_swizzle bit mode: and 0x1F,
// xor X; an immediate pattern, so no address VGPR stays live)
template <uint32_t X>
DEV uint32_t swz_xor(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (int)(0x1Fu | (X << 10)));
}

// CRC of one window from registers: the state at W0 + 16K.  Words before
// window offset o4 (4-aligned) are not part of the stream (read as zero);
// the state Tinj is injected at o4.
template <typename Mid>
DEV uint32_t crc_window(const uint8_t* lds, const Keys& K, const Win& d, uint32_t o4, uint32_t Tinj, bool do_mid,
                        Mid&& mid) {
    const uint32_t l = lane_v();
    const uint32_t i4 = o4 >> 10, l4 = (o4 >> 4) & 63u, k4 = (o4 >> 2) & 3u;
    const uint32_t lo = 16u * l;  // this lane's offset within a row
    uint32_t p[4] = {0u, 0u, 0u, 0u}, q[4] = {0u, 0u, 0u, 0u};  // braid k's state is p[k] ^ q[k]
    uint32_t s0 = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        uint32_t w[4] = {d.r[i].x, d.r[i].y, d.r[i].z, d.r[i].w};
        if ((uint32_t)i <= i4) {
            // the row holding o4 (and any before it): mask words before o4,
            // inject at o4 (uniform branch; rows after it take neither).  The
            // lane's row offsets lo + 4k against the uniform row threshold:
            // no per-row constants stay live across the batch loop
            const int32_t t = (int32_t)o4 - 1024 * i;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int32_t off = (int32_t)(lo + 4u * (uint32_t)k);
                w[k] = off >= t ? w[k] : 0u;
                p[k] ^= (off == t) ? Tinj : 0u;
            }
        }
        if (i == 8 && do_mid) mid();  // rows 0..7 are free: room for the caller's loads
        if (i < 15) {
#pragma unroll
            for (int k = 0; k < 4; k++) braid_step(lds, K, xor3(p[k], q[k], w[k]), p[k], q[k]);
        } else {
            // row 15: fold the braids (braid k sits at word k) with word steps
            uint32_t c = word_step_x(lds, xor3(p[0], q[0], w[0]), p[1] ^ q[1]);
            c = word_step_x(lds, c ^ w[1], p[2] ^ q[2]);
            c = word_step_x(lds, c ^ w[2], p[3] ^ q[3]);
            s0 = word_step_x(lds, c ^ w[3], 0u);
        }
    }
    // lane l's state sits 16 (63 - l) bytes before the window end:
    // shift-and-xor tree into lane 0.  At level m only lanes that are
    // multiples of 2^(m+1) matter, and for them l ^ 2^m = l + 2^m, so the
    // exchange is an xor swizzle (immediate pattern, no address VGPR) and the
    // last level a readlane of lane 32.
    static_assert(kShiftLevels == 6, "shift tree is written out for 64 lanes");
    uint32_t sv = s0;
    sv = shift_k(lds, sv, 0, swz_xor<1>(sv));
    sv = shift_k(lds, sv, 1, swz_xor<2>(sv));
    sv = shift_k(lds, sv, 2, swz_xor<4>(sv));
    sv = shift_k(lds, sv, 3, swz_xor<8>(sv));
    sv = shift_k(lds, sv, 4, swz_xor<16>(sv));
    return shift_k(lds, uni32(sv), 5, rl(sv, 32));
}

// fold the tail bytes [max(S, E16), E) held in gt into the state (uniform)
DEV uint32_t crc_tail(const uint8_t* lds, const Stream& st, const uint4& gt, uint32_t Tst) {
    if (st.E <= st.E16) return Tst;
    uint32_t x = (uint32_t)((st.S > st.E16 ? st.S : st.E16) - st.E16);
    const uint32_t nt = (uint32_t)(st.E - st.E16);
    const uint4 t = make_uint4(uni32(gt.x), uni32(gt.y), uni32(gt.z), uni32(gt.w));
    for (; (x & 3u) && x < nt; x++) Tst = byte_step(lds, Tst, (pick4(t, x >> 2) >> (8 * (x & 3u))) & 0xFFu);
    for (; x + 4 <= nt; x += 4) Tst = word_step(lds, Tst, pick4(t, x >> 2));
    for (; x < nt; x++) Tst = byte_step(lds, Tst, (pick4(t, x >> 2) >> (8 * (x & 3u))) & 0xFFu);
    return uni32(Tst);
}

// CRC state after [S, E) from the state Tst at S.  d holds window 0 on entry
// (issued by the caller); gt the tail row.  The < 4 bytes up to the first
// 4-aligned position are folded in first (scalar load), so the window only
// injects at a word boundary.  mid() runs once, half-way through the last
// window (or at the end when there is none).
template <typename Mid>
DEV uint32_t crc_stream(const uint8_t* lds, const Keys& K, const Stream& st, Win& d, const uint4& gt, uint32_t Tst,
                        Mid&& mid) {
    bool mid_done = false;
    if (st.R) {
        const uint64_t S4 = (st.S + 3) & ~3ull;
        if (S4 != st.S) {
            const uint32_t w = *(cu32*)(st.src + (st.S & ~3ull));
            for (uint64_t x = st.S; x < S4; x++) Tst = byte_step(lds, Tst, (w >> (8 * (uint32_t)(x & 3))) & 0xFFu);
            Tst = uni32(Tst);
        }
        if (st.R == 1) {
            // one window (the common case): mid() half-way through it
            const uint32_t o4 = (uint32_t)((int64_t)S4 - win_base(st, 0));
            // S4 can sit exactly at the end of window 0 (S within 3 bytes of
            // it): that window holds no stream bytes and the state passes on
            if (o4 < kWinBytes) {
                Tst = crc_window(lds, K, d, o4, Tst, true, mid);
                mid_done = true;
            }
        } else {
            // window 0 from the caller, then a fresh window per iteration (a
            // window carried around the loop would be copied and spilled)
            const uint32_t o4 = (uint32_t)((int64_t)S4 - win_base(st, 0));
            if (o4 < kWinBytes) Tst = crc_window(lds, K, d, o4, Tst, false, [] {});
            for (uint64_t r = 1; r < st.R; r++) {
                Win w;
                load_window(st, r, w);
                Tst = crc_window(lds, K, w, 0u, Tst, false, [] {});
            }
        }
    }
    if (!mid_done) mid();
    return crc_tail(lds, st, gt, Tst);
}

DEV uint32_t crc_stream(const uint8_t* lds, const Keys& K, const Stream& st, Win& d, const uint4& gt, uint32_t Tst) {
    return crc_stream(lds, K, st, d, gt, Tst, [] {});
}

// ---------------------------------------------------------------------------
// Record walk
// ---------------------------------------------------------------------------

// vint::deserialize (utils/vint.h:82-98) over at most `avail` bytes: LEB128
// stopping after 10 bytes, or at the end of input with the partial value.
// One- and two-byte varints (almost every length/delta) take a short path.
DEV int64_t varint12(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t avail, uint32_t& br) {
    uint64_t res;
    if (avail >= 2 && (r0 & 0x8080u) != 0x8080u) {
        const uint32_t b0 = r0 & 0xFFu;
        if (!(b0 & 0x80u)) { br = 1; res = b0; }
        else { br = 2; res = (b0 & 0x7Fu) | (((r0 >> 8) & 0x7Fu) << 7); }
    } else {
        const uint64_t lo = (uint64_t)r0 | ((uint64_t)r1 << 32);
        res = 0;
        uint32_t cnt = 0;
        const uint32_t lim = avail < 10 ? avail : 10u;
        for (uint32_t i = 0; i < lim; i++) {
            const uint64_t byte = (i < 8 ? (lo >> (8 * i)) : (r2 >> (8 * (i - 8)))) & 0xFF;
            cnt++;
            res |= (byte & 127) << (7 * i);
            if (!(byte & 128)) break;
        }
        br = cnt;
    }
    return (int64_t)((res >> 1) ^ (~(res & 1) + 1));
}

// Per-lane 48-byte register regions of the payload: three aligned 16-byte
// rows in grid coordinates (g = payload offset + mis, mis = p0 & 15, so every
// row is one aligned dwordx4).  Rows starting at or past the payload end read
// as zero; a row may run up to 15 bytes past it (buffers are readable to a
// 16-byte boundary past their end).
struct Region {
    uint32_t base;  // grid offset of r0
    uint4 r0, r1, r2;
};

DEV void load_region(const uint8_t* p0, uint32_t mis, uint32_t n, uint32_t base, Region& R) {
    const uint8_t* row = p0 - mis + base;
    const uint32_t lim = n + mis;
    R.base = base;
    R.r0 = R.r1 = R.r2 = make_uint4(0u, 0u, 0u, 0u);
    if (base < lim) R.r0 = *(const uint4*)row;
    if (base + 16u < lim) R.r1 = *(const uint4*)(row + 16);
    if (base + 32u < lim) R.r2 = *(const uint4*)(row + 32);
}

// dword k (0..11) of a region, selected by value (per-lane k)
DEV uint32_t pick12(const Region& R, uint32_t k) {
    const uint32_t a = pick4(R.r0, k), b = pick4(R.r1, k), c = pick4(R.r2, k);
    return k < 4u ? a : (k < 8u ? b : c);
}

// The record parser's byte source: the current region A, the record's tail
// region T (handed over up front), else a fresh region at the read position
// (one dependent load).
struct Reader {
    const uint8_t* p0;  // payload start (wave-uniform)
    uint32_t mis;       // p0 & 15
    uint32_t n;
    uint32_t pos;
    Region A, T;

    // region offset of pos, switching regions so 12 bytes from it are held
    DEV uint32_t locate() {
        const uint32_t g = pos + mis;
        if (g - A.base > 32u) {
            if (g - T.base <= 32u) A = T;
            else load_region(p0, mis, n, g & ~15u, A);
        }
        return g - A.base;
    }

    // iobuf_parser_base::read_varlong (bytes/iobuf_parser.h:48-52)
    DEV int64_t varlong() {
        const uint32_t o = locate(), k = o >> 2, sh = o & 3u, avail = n - pos;
        const uint32_t w0 = pick12(A, k), w1 = pick12(A, k + 1u);
        uint32_t r0 = __builtin_amdgcn_alignbyte(w1, w0, sh), r1 = 0u, r2 = 0u, br;
        if (avail >= 2 && (r0 & 0x8080u) == 0x8080u) {
            const uint32_t w2 = pick12(A, k + 2u), w3 = pick12(A, k + 3u);
            r1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
            r2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
        }
        const int64_t x = varint12(r0, r1, r2, avail, br);
        pos += br;
        return x;
    }
    DEV uint32_t byte() {
        const uint32_t o = locate();
        return (pick12(A, o >> 2) >> (8u * (o & 3u))) & 0xFFu;
    }
};

// iobuf_copy (bytes/iobuf.cc:133-157): -1 when (int)len < 0 (bad_alloc);
// a length past the end copies what is there, silently
template <class Src>
DEV int copy_bytes(Src& c, int64_t len) {
    const int32_t bl = (int32_t)(uint32_t)(uint64_t)len;
    if (bl < 0) return -1;
    const uint32_t left = c.n - c.pos;
    c.pos += ((uint32_t)bl < left) ? (uint32_t)bl : left;
    return 0;
}

struct Rec {
    uint32_t err;   // rpgpu_parse_err
    uint32_t end;
    int64_t ts;
    int32_t length, off, klen, vlen, hcount;
    uint32_t key_pos, val_pos, hdr_pos;
    int32_t attr;
};

// parse_one_record_copy_from_buffer (model/record_utils.cc:170-177) over
// parse_record_meta_from_buffer / do_parse_one_record_from_buffer /
// parse_record_headers (:94-160) from the source's position.  Src provides
// pos, n, varlong() and byte() (Reader: register regions).
// lane's LDS slab).
template <class Src>
DEV Rec parse_fields(Src& c) {
    Rec r;
    r.err = 0;
    r.key_pos = r.val_pos = r.hdr_pos = 0;
    r.ts = 0; r.length = r.off = r.klen = r.vlen = r.hcount = 0; r.attr = 0;
    const uint32_t n = c.n;
    const int64_t rsz = c.varlong();
    // consume_type<int8_t>: the only read that throws on short input
    if (c.pos >= n) { r.err = RPGPU_PARSE_ERR_ATTR_EOF; r.end = c.pos; return r; }
    r.attr = (int8_t)c.byte();
    c.pos++;
    r.ts = c.varlong();
    const int64_t off = c.varlong();
    const int64_t kl = c.varlong();
    r.key_pos = c.pos;
    if (kl > 0 && copy_bytes(c, kl)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    const int64_t vl = c.varlong();
    r.val_pos = c.pos;
    if (vl > 0 && copy_bytes(c, vl)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    const int64_t hc = c.varlong();
    r.hdr_pos = c.pos;
    // headers.reserve(count) throws for count < 0 or beyond the limit
    if (hc < 0 || hc > RPGPU_MAX_HEADER_RESERVE) { r.err = RPGPU_PARSE_ERR_HEADER_RESERVE; r.end = c.pos; return r; }
    for (int32_t h = 0; h < (int32_t)hc; h++) {
        if (c.pos >= n) break;
        const int64_t hk = c.varlong();
        if (hk > 0 && copy_bytes(c, hk)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
        const int64_t hv = c.varlong();
        if (hv > 0 && copy_bytes(c, hv)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    }
    r.length = (int32_t)rsz;
    r.off = (int32_t)off;
    r.klen = (int32_t)kl;
    r.vlen = (int32_t)vl;
    r.hcount = (int32_t)hc;
    r.end = c.pos;
    return r;
}

// from the record start, with the head and tail regions already loaded
// (record_regions)
DEV Rec parse_record(const uint8_t* p0, uint32_t mis, uint32_t n, uint32_t start, const Region& H, const Region& T) {
    Reader c;
    c.p0 = p0;
    c.mis = mis;
    c.n = n;
    c.pos = start;
    c.A = H;
    c.T = T;
    return parse_fields(c);
}

// Head and tail regions of a lane's record, issued together: three 16-byte
// rows at the start and three ending at (or just past) the chain's guess of
// its end, where the headers sit.  A typical record then costs one memory
// latency, whatever its length.
DEV void record_regions(const uint8_t* p0, uint32_t mis, uint32_t n, bool act, uint32_t start, uint32_t end,
                        Region& H, Region& T) {
    H.base = T.base = 0xFFFFFFF0u;
    H.r0 = H.r1 = H.r2 = T.r0 = T.r1 = T.r2 = make_uint4(0u, 0u, 0u, 0u);
    if (act) {
        const uint32_t hb = (start + mis) & ~15u;
        const uint32_t e16 = (end + mis + 15u) & ~15u;
        const uint32_t tb = (end != 0xFFFFFFFFu && e16 >= hb + 48u) ? e16 - 48u : hb;
        load_region(p0, mis, n, hb, H);
        load_region(p0, mis, n, tb, T);
    }
}

struct WalkResult {
    uint32_t parsed;
    uint32_t err;
    uint32_t trailing;
};

// 12 bytes at payload offset q (wave-uniform) through the scalar cache: the
// constant address space makes these s_loads, off the vector-memory queue
// the window stream keeps full.  The payload is read-only for the whole
// kernel; callers bound every use by the bytes available.
DEV void s12(const uint8_t* p0, uint32_t q, uint32_t& r0, uint32_t& r1, uint32_t& r2) {
    const uintptr_t a = (uintptr_t)(p0 + q);
    cu32* c = (cu32*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = c[0], w1 = c[1], w2 = c[2], w3 = c[3];
    r0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    r1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    r2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
}

// Byte source of the chain: 12 bytes at payload offset p (wave-uniform)
// through the scalar cache.  (A source reading a one-window payload from the
// window registers with v_movrels + v_readlane measured 2.3x slower per
// record than these loads.)
struct MemSrc {
    const uint8_t* p0;
    DEV void read(uint32_t p, uint32_t, uint32_t& r0, uint32_t& r1, uint32_t& r2) const { s12(p0, p, r0, r1, r2); }
};
// Speculative record starts and ends for records [done, done + want): a
// uniform chain over the length varints from `start`.  Lane m gets the start
// of record done + m and the position after it (the next start); returns how
// many lanes got a start.
template <typename Src>
DEV uint32_t chain_starts(const Src& src, uint32_t n, uint32_t start, uint32_t want, uint32_t& my_start,
                          uint32_t& my_end) {
    const uint32_t l = lane_v();
    my_start = my_end = 0xFFFFFFFFu;
    uint32_t p = start;
    uint32_t m = 0;
    for (; m < want; m++) {
        if (l == m) my_start = p;
        if (p >= n) { m++; break; }
        const uint32_t avail = n - p;
        uint32_t r0, r1, r2, br;
        src.read(p, avail, r0, r1, r2);
        const int64_t len = varint12(r0, r1, r2, avail, br);
        if (len < 0 || (uint64_t)len > n) { m++; break; }
        p = uni32(p + br + (uint32_t)len);
        if (l == m) my_end = p;
    }
    return m;
}

// The same starts and ends from k_dchain's precomputed chain of the payload
// (pre[k] = the position after record k, 0xFFFFFFFF where chain_starts
// stops): one coalesced load per 64 records instead of 64 dependent ones.
// s0 = the start of record `done` (0, or pre[done - 1]).
DEV uint32_t pre_starts(const uint32_t* pre, uint32_t s0, uint32_t done, uint32_t want, uint32_t& my_start,
                        uint32_t& my_end) {
    const uint32_t l = lane_v();
    const uint32_t e = l < want ? pre[done + l] : 0u;
    // lane l - 1's end is lane l's start (DPP wave_shr:1; lane 0 takes s0)
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x138, 0xF, 0xF, false);
    const uint64_t stops = __ballot(l < want && e == 0xFFFFFFFFu);
    const uint32_t m = stops ? (uint32_t)__builtin_ctzll(stops) + 1u : want;
    my_start = my_end = 0xFFFFFFFFu;
    if (l < m) {
        my_start = l == 0 ? s0 : prev;
        my_end = e;
    }
    return m;
}

// Lanes [0, m) parse one record each from their speculative starts; the
// prefix whose starts are confirmed by the previous record's exact end is
// committed to the index.  Returns false when a record failed (wr filled).
DEV bool parse_group(const uint8_t* p0, uint32_t mis, uint32_t n, uint32_t m, uint32_t my_start, const Region& H,
                     const Region& T, uint32_t batch_ord,
                     rpgpu_record_index* out, uint64_t out_cap, uint32_t& done, uint32_t& start, WalkResult& wr) {
    const uint32_t l = lane_v();
    Rec r;
    const bool act = l < m;
    if (act) r = parse_record(p0, mis, n, my_start, H, T);
    else { r.err = 0; r.end = 0xFFFFFFFFu; }
    // lane l - 1's values (DPP wave_shr:1; lane 0 ignores them)
    const uint32_t prev_end = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r.end, 0x138, 0xF, 0xF, false);
    const uint32_t prev_err = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r.err, 0x138, 0xF, 0xF, false);
    const bool match = (l == 0) || (prev_err == 0 && prev_end == my_start);
    const uint64_t bad = __ballot(act && !match);
    const uint32_t exact = bad ? (uint32_t)__builtin_ctzll(bad) : m;  // lanes [0, exact) are exact
    const uint64_t errs = __ballot(act && l < exact && r.err != 0);
    const uint32_t nok = errs ? (uint32_t)__builtin_ctzll(errs) : exact;  // records parsed OK
    if (l < nok && done + l < out_cap) {
        rpgpu_record_index e;
        e.batch = batch_ord;
        e.rec_pos = my_start;
        e.ts_delta = r.ts;
        e.length = r.length;
        e.offset_delta = r.off;
        e.key_len = r.klen;
        e.key_pos = r.key_pos;
        e.val_len = r.vlen;
        e.val_pos = r.val_pos;
        e.hdr_count = r.hcount;
        e.hdr_pos = r.hdr_pos;
        e.end_pos = r.end;
        e.attrs = (int8_t)r.attr;
        e.pad[0] = e.pad[1] = e.pad[2] = 0;
        e.reserved[0] = e.reserved[1] = 0;
        out[done + l] = e;
    }
    if (errs) {
        wr.parsed = done + nok;
        wr.err = rl(r.err, (int)nok);
        return false;
    }
    start = rl(r.end, (int)(exact - 1));
    done += exact;
    return true;
}

// record_batch::for_each_record (model/record.h:616-627) with speculative
// lane-parallel records: chain_starts guesses 64 record starts (and ends) at
// a time, record_regions loads each lane's head and tail rows, parse_group
// parses and commits the confirmed prefix.  The first group may be prepared
// by the caller around the CRC (Group: chain before it, regions issued
// half-way through it).
struct Group {
    bool first;
    uint32_t m, my_start, my_end;
    Region H, T;
};

DEV void group_init(Group& g) {
    g.first = false;
    g.m = 0;
    g.my_start = g.my_end = 0xFFFFFFFFu;
}

DEV WalkResult walk_records(const uint8_t* p0, uint32_t n, int32_t rc, uint32_t batch_ord, rpgpu_record_index* out,
                            uint64_t out_cap, Group& g, const uint32_t* pre = nullptr) {
    WalkResult wr;
    wr.parsed = 0;
    wr.err = 0;
    wr.trailing = 0;
    const uint32_t mis = (uint32_t)((uintptr_t)p0 & 15);
    const uint32_t total = (uint32_t)(rc > 0 ? rc : 0);
    uint32_t start = 0, done = 0;
    if (total == 0) {
        wr.trailing = n;
        return wr;
    }
    const MemSrc mem{p0};
    if (!g.first) {
        STAMP(w0);
        const uint32_t want = total < 64u ? total : 64u;
        g.m = pre ? pre_starts(pre, 0u, 0u, want, g.my_start, g.my_end) : chain_starts(mem, n, 0u, want, g.my_start, g.my_end);
        record_regions(p0, mis, n, lane_v() < g.m, g.my_start, g.my_end, g.H, g.T);
        STAMP(w1);
        STAMP_ADD(6, w1 - w0);
    }
    for (;;) {
        if (!parse_group(p0, mis, n, g.m, g.my_start, g.H, g.T, batch_ord, out, out_cap, done, start, wr)) return wr;
        if (done >= total) break;
        const uint32_t want = (total - done) < 64u ? (total - done) : 64u;
        // the precomputed chain holds while the parsed records confirm it
        // (they do unless a record's parse ends elsewhere than its length
        // says, which fails the walk first); otherwise chain from `start`
        if (pre && uni32(pre[done - 1]) != start) pre = nullptr;
        g.m = pre ? pre_starts(pre, start, done, want, g.my_start, g.my_end)
                  : chain_starts(mem, n, start, want, g.my_start, g.my_end);
        record_regions(p0, mis, n, lane_v() < g.m, g.my_start, g.my_end, g.H, g.T);
    }
    wr.parsed = done;
    wr.trailing = n - start;
    return wr;
}

// internal_header_only_crc (model/record_utils.cc:34-55) of the header that
// reset_size_checksum_metadata produces: codec bits cleared, size_bytes =
// 61 + decoded, crc = the decoded crc (storage/parser_utils.cc:53-56, 114-120)
DEV uint32_t decoded_header_crc(const Tables* T, const uint8_t* hdr, uint32_t new_size, uint32_t new_crc,
                                bool wire) {
    const uint32_t l = lane_v();
    uint32_t b = (l < RPGPU_HEADER_SIZE) ? (uint32_t)hdr[l] : 0u;
    if (wire) {
        // the adapted (disk) header: byte l from wire byte src(l), as in
        // wave_header_wire; type raft_data
        int src = 0;
        if (l >= 8 && l < 16) src = 15 - (int)l;
        else if (l >= 17 && l < 21) src = 37 - (int)l;
        else if (l >= 21 && l < RPGPU_HEADER_SIZE) src = 21 + be_index(l);
        b = (uint32_t)__shfl((int)b, src, 64);
        if (l == 16) b = 1u;
    }
    if (l >= 4 && l < 8) b = (new_size >> (8 * (l - 4))) & 0xFFu;
    if (l >= 17 && l < 21) b = (new_crc >> (8 * (l - 17))) & 0xFFu;
    if (l == 21) b &= ~7u;
    uint32_t x = (l >= 4 && l < RPGPU_HEADER_SIZE) ? T->hdr[60 - l][b] : 0u;
    // xor over the wave with immediate-pattern swizzles (no address VGPRs)
    x ^= swz_xor<1>(x);
    x ^= swz_xor<2>(x);
    x ^= swz_xor<4>(x);
    x ^= swz_xor<8>(x);
    x ^= swz_xor<16>(x);
    return ~(T->c57 ^ rl(x, 0) ^ rl(x, 32));
}

// first batch of segment s failing complete && crc_ok (log_replayer
// checkpoint, storage/log_replayer.cc:62-79); resolved by k_finalize_segments
DEV void note_bad(const DeviceJob& j, uint32_t seg, uint64_t b) {
    if (lane_v() == 0) {
        const uint64_t first = j.chunk_count[j.chunk_base[seg]];
        atomicMin(&j.seg_first_bad[seg], (uint32_t)(b - first));
    }
}

// Stored payloads with at most kLaneWalkMax records are walked one lane per
// batch by k_walk; k_validate walks the rest (and decoded payloads) with the
// wave-parallel walk.
#ifndef RPGPU_LANE_WALK_MAX
#define RPGPU_LANE_WALK_MAX 256
#endif
constexpr int32_t kLaneWalkMax = RPGPU_LANE_WALK_MAX;
DEV bool lane_walked(uint32_t flags, uint32_t codec, int32_t rc) {
    return (flags & RPGPU_F_COMPLETE) && codec == 0 && rc <= kLaneWalkMax;
}

// Per-batch descriptor, loaded one iteration ahead as ONE VGPR: lane i < 32
// holds dword i of the batch result, lanes 32..37 the index-slot and
// decode-arena words; the fields are read out with v_readlane when the batch
// is reached.  index_base carries the absolute payload start from k_emit
// (scratch, overwritten here), reserved1 the raw BE40 prefix CRC contribution.
constexpr int kDwSize = offsetof(rpgpu_batch_result, size_bytes) / 4;
constexpr int kDwCount = offsetof(rpgpu_batch_result, record_count) / 4;
constexpr int kDwCrc = offsetof(rpgpu_batch_result, crc) / 4;
constexpr int kDwFlags = offsetof(rpgpu_batch_result, flags) / 4;
constexpr int kDwSeg = offsetof(rpgpu_batch_result, segment) / 4;
constexpr int kDwBase = offsetof(rpgpu_batch_result, index_base) / 4;
constexpr int kDwDlen = offsetof(rpgpu_batch_result, decoded_len) / 4;
constexpr int kDwAttrs = offsetof(rpgpu_batch_result, attrs) / 4;
constexpr int kDwPraw = offsetof(rpgpu_batch_result, reserved1) / 4;
constexpr int kDwRes0 = offsetof(rpgpu_batch_result, reserved0) / 4;  // reserved0 in the high half
constexpr int kDwCcomp = offsetof(rpgpu_batch_result, crc_computed) / 4;
static_assert(offsetof(rpgpu_batch_result, reserved0) % 4 == 2, "reserved0: the high half of its dword");
static_assert(sizeof(rpgpu_batch_result) == 128 && offsetof(rpgpu_batch_result, attrs) % 4 == 0, "desc layout");

DEV uint32_t load_desc_raw(const DeviceJob& j, uint64_t b) {
    const uint32_t l = lane_v();
    const uint32_t* p = l < 32u ? (const uint32_t*)&j.batches[b] + l
                      : l < 34u ? (const uint32_t*)&j.slots[b] + (l - 32u)
                      : l < 36u ? (const uint32_t*)&j.slots[b + 1] + (l - 34u)
                                : (const uint32_t*)&j.dcap[b] + (l & 1u);
    return l < 38u ? *p : 0u;
}

struct Desc {
    uint32_t flags, crc, praw, codec, seg, dlen;
    uint64_t S, n, ib, islots, doff;
    int32_t rc;
    uint32_t scc;    // the stored crc was composed by k_crc_compose (reserved0 bit 1): ccomp holds it
    uint32_t ccomp;
};

DEV Desc desc_of(uint32_t raw) {
    Desc d;
    d.flags = rl(raw, kDwFlags);
    d.crc = rl(raw, kDwCrc);
    d.praw = rl(raw, kDwPraw);
    d.S = (uint64_t)rl(raw, kDwBase) | ((uint64_t)rl(raw, kDwBase + 1) << 32);
    d.n = rl(raw, kDwSize) - RPGPU_HEADER_SIZE;
    d.rc = (int32_t)rl(raw, kDwCount);
    d.codec = rl(raw, kDwAttrs) & 7u;
    d.seg = rl(raw, kDwSeg);
    d.dlen = rl(raw, kDwDlen);
    d.ib = (uint64_t)rl(raw, 32) | ((uint64_t)rl(raw, 33) << 32);
    d.islots = ((uint64_t)rl(raw, 34) | ((uint64_t)rl(raw, 35) << 32)) - d.ib;
    d.doff = (uint64_t)rl(raw, 36) | ((uint64_t)rl(raw, 37) << 32);
    d.scc = (rl(raw, kDwRes0) >> 16) & 2u;
    d.ccomp = rl(raw, kDwCcomp);
    return d;
}

// the stored payload of a batch as a stream (empty when there is none)
DEV Stream stored_stream(const DeviceJob& j, const Desc& d, bool valid) {
    return (valid && (d.flags & RPGPU_F_COMPLETE) && !d.scc) ? make_stream(j.data, d.S, d.S + d.n)
                                                               : make_stream(j.data, 0, 0);
}

// the record walk of one payload into the batch's index slots
DEV WalkResult walk_batch(const DeviceJob& j, const Desc& ds, const uint8_t* p0, uint32_t n, uint64_t b, bool& idx_ok,
                          Group& g0, const uint32_t* pre = nullptr) {
    idx_ok = ds.ib + ds.islots <= j.record_capacity;
    rpgpu_record_index* out = idx_ok ? j.records + ds.ib : nullptr;
    const uint64_t cap = idx_ok ? ds.islots : 0;
    return walk_records(p0, n, ds.rc, (uint32_t)b, out, cap, g0, pre);
}

// a decoded payload whose record chain k_dchain precomputes (k_validate_decoded
// takes it from there iff this holds for both): its walk runs, its
// record_count index slots exist and hold the chain, and its records are
// long enough that each chain step is a line of its own (>= 256 B on
// average; shorter records share lines, which the wave's scalar chain reads
// at cache latency: C5's 100-byte records ran 3.6 -> 4.0 ms lane-chained)
// and few enough for one lane's serial chain
constexpr uint32_t kDchainMinRecBytes = 256, kDchainMaxRecs = 1024;
DEV bool dchain_ok(const DeviceJob& j, uint32_t flags, int32_t rc, uint64_t ib, uint64_t islots, uint32_t dlen) {
    // (disk layout only: k_dchain runs beside k_validate, which sets the
    // CRC_OK bit the wire layout's walk depends on)
    return j.dchain && (flags & RPGPU_F_CODEC_OK) && (j.flags & RPGPU_JOB_PARSE) &&
           j.layout == RPGPU_LAYOUT_DISK && rc > 0 && (uint64_t)rc <= islots &&
           ib + islots <= j.record_capacity && (uint32_t)rc <= kDchainMaxRecs &&
           dlen >= kDchainMinRecBytes * (uint32_t)rc;
}

// LDS image of the CRC tables (every workgroup of the validate kernels).
// braid tables: word i -> row-set rs = i >> 14, entry e = (i >> 6) & 255,
// slot = (i >> 5) & 1, copy = i & 31; (rs, slot) = (0,0) T1023, (0,1)
// T1022, (1,0) T1021, (1,1) T1020
DEV void init_lds_tables(uint8_t* lds, const Tables* T) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 32768u; i += blockDim.x)
        ((uint32_t*)(lds + kLdsBraidOff))[i] = T->braid[((i >> 14) << 1) | ((i >> 5) & 1u)][(i >> 6) & 255u];
    // slice tables: T3, T2, T1, T0
    for (uint32_t i = tid; i < 1024u; i += blockDim.x) ((uint32_t*)(lds + kLdsSlice4Off))[i] = T->hdr[3 - (i >> 8)][i & 255u];
    // shift tables: 16 << m bytes, m = 0..5
    for (uint32_t i = tid; i < kShiftLevels * 1024u; i += blockDim.x)
        ((uint32_t*)(lds + kLdsShiftOff))[i] = ((const uint32_t*)T->shift)[i];
    __syncthreads();
}

// this lane's copy of the four braid tables
DEV Keys make_keys() {
    const uint32_t bank = (lane_v() & 31u) * 4u;
    Keys K;
    K.k15 = (0u << 16) | (0u + bank);
    K.k14 = (0u << 16) | (128u + bank);
    K.k13 = (1u << 16) | (0u + bank);
    K.k12 = (1u << 16) | (128u + bank);
    return K;
}

// Walk result -> verdict bits (model/record.h:616-627 sync, :680-697 async)
DEV uint32_t walk_flags(const DeviceJob& j, const WalkResult& w, bool idx_ok, uint32_t& perr) {
    uint32_t f = RPGPU_F_PARSED;
    perr = w.err;
    if (perr == 0) {
        f |= RPGPU_F_PARSE_ASYNC_OK;
        if (w.trailing == 0) f |= RPGPU_F_PARSE_OK;
        else perr = RPGPU_PARSE_ERR_TRAILING;
    }
    if (f & RPGPU_F_PARSE_OK) {
        if (idx_ok) f |= RPGPU_F_INDEX_WRITTEN;
        else { perr = RPGPU_PARSE_ERR_INDEX_CAPACITY; if (lane_v() == 0) atomicOr(&j.counters[1], 2u); }
    }
    return f;
}

// Rows of a batch's window that may be issued one iteration ahead, before
// the previous batch's walk (whose chain reads through the scalar cache, so
// it never waits on them).  Measured on the C1 workload: 0, 4, 8 and 10 rows
// within 1% of each other (the walk, not the window latency, is exposed), so
// only the descriptor is prefetched.
constexpr int kPreRows = 0;

// ---------------------------------------------------------------------------
// Lane record walk (k_walk)
// ---------------------------------------------------------------------------
template <class J>
DEV void note_bad_lane(const J& j, uint32_t seg, uint64_t b) {
    const uint64_t first = j.chunk_count[j.chunk_base[seg]];
    atomicMin(&j.seg_first_bad[seg], (uint32_t)(b - first));
}

// One lane's walk of one stored payload.  The bytes a lane parses sit in
// LDS rather than registers (held in registers, every field read was a
// 12-way select: ~1,200 VALU per record), in regions of 6 rows of 16 bytes
// at a 16-byte aligned grid offset.  Record k's step needs ONE region, C_k =
// the 96 bytes around its guessed end: the 48 bytes before it hold record
// k's headers, the 48 after it record k + 1's length .. key length, key and
// value length (16-byte keys), so the next step parses its head from C_k.
//
// The regions of a wave's 64 lanes are fetched together, cooperatively: the
// 384 rows are spread over 6 global_load_lds wave-instructions so that each
// instruction reads ~10 regions' contiguous rows (~17 cache lines) instead
// of one row from each of 64 regions (64 lines).  The lane-per-region
// gather was bound by the texture addresser (TA ~86% busy, ~126 cycles per
// instruction).  Row r of lane w's region lands at slot + 96 w + 16 r.  Two
// slots per wave alternate by step parity: H (C_{k-1}, the record's head)
// and C_k (loaded this step).
// 6 rows: 48 bytes before the guessed end (record k's headers) and 48 after
// it (record k + 1's length .. value length).  5-row regions (48 / 32: 10 KiB
// of LDS per wave, four workgroups per CU instead of three) measured slower
// on C1 (walk 1.34 -> 1.49 ms): the walk is not short of walks in flight.
#ifndef RPGPU_WALK_ROWS
#define RPGPU_WALK_ROWS 6
#endif
constexpr uint32_t kRegionRows = RPGPU_WALK_ROWS;
constexpr uint32_t kRegionBytes = 16u * kRegionRows;
constexpr uint32_t kRegionBefore = 48u;  // bytes of C_k before the 16-aligned guessed end
static_assert(kRegionBytes > kRegionBefore && 64u * kRegionBytes >= 4096u, "region / staging geometry");
constexpr uint32_t kRegionReach = kRegionBytes - 16u;  // a read needs 16 bytes from its offset
constexpr uint32_t kSlotBytes = 64u * kRegionBytes;
constexpr uint32_t kWalkLdsWave = 2u * kSlotBytes;

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;
#ifndef RPGPU_WALK_AUX
#define RPGPU_WALK_AUX 2  // region fetch non-temporal (measured: walk 1.36 -> 1.30 ms); 0 = default policy
#endif

DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Region layout in a slot.  Cooperative fetch (default): lane w's region is
// contiguous at slot + 96 w.  Per-lane fetch (RPGPU_WALK_COOP_LOAD=0, kept
// for A/B): each lane issues its own six global_load_lds, which land
// lane-linear, so row r of lane w sits at slot + 1024 r + 16 w.  Measured on
// C1: walk 1.36 ms cooperative, 1.45 ms per-lane.
#ifndef RPGPU_WALK_COOP_LOAD
#define RPGPU_WALK_COOP_LOAD 1
#endif
constexpr bool kCoopLoad = RPGPU_WALK_COOP_LOAD != 0;
DEV uint32_t region_off(uint32_t o) { return kCoopLoad ? o : (o >> 4) * 1024u + (o & 12u); }
DEV uint32_t region_lane(uint32_t l) { return kCoopLoad ? kRegionBytes * l : 16u * l; }

// rows of the region at grid offset base that start inside the payload
// (the others are never parsed and are not loaded)
DEV uint32_t region_rows(uint32_t n, uint32_t mis, uint32_t base) {
    const uint32_t lim = n + mis;
    if (base >= lim) return 0u;
    const uint32_t r = (lim - base + 15u) >> 4;
    return r < kRegionRows ? r : kRegionRows;
}

// Wave-cooperative fetch (all 64 lanes active): lane w wants `rows` rows from
// global address g (16-byte aligned) into its region of the slot at the
// wave-uniform LDS address `slot`.
DEV void coop_load(uint8_t* slot, const uint8_t* g, uint32_t rows) {
    const uint32_t l = lane_v();
    const uint64_t ga = (uint64_t)(uintptr_t)g;
    const int lo = (int)(uint32_t)ga, hi = (int)(uint32_t)(ga >> 32), nr = (int)rows;
#pragma unroll
    for (uint32_t m = 0; m < kRegionRows; m++) {
        const uint32_t q = 64u * m + l, w = q / kRegionRows, r = q - w * kRegionRows;
        const int src = (int)(w * 4u);
        const uint32_t wlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, lo);
        const uint32_t whi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, hi);
        const uint32_t wnr = (uint32_t)__builtin_amdgcn_ds_bpermute(src, nr);
        if (r < wnr) {
            const uint8_t* row = (const uint8_t*)(uintptr_t)(((uint64_t)whi << 32) | wlo) + 16u * r;
            __builtin_amdgcn_global_load_lds((gbl_void*)row, (lds_void*)(slot + 1024u * m), 16, 0, RPGPU_WALK_AUX);
        }
    }
}

// Wave-cooperative index store (all 64 lanes active): lane w's 64-byte entry
// e goes to dst (null: nothing to write).  The entries are staged in LDS
// (`stage`, 4 KiB, wave-uniform) and written 16 per wave-instruction, each
// as 4 lanes x 16 contiguous bytes, instead of one 16-byte piece of each of
// 64 scattered entries per instruction (the index stores were a third of
// the walk's time).
#ifndef RPGPU_NT_INDEX
#define RPGPU_NT_INDEX 0  // index entries stored non-temporal (A/B knob)
#endif
DEV void coop_store(uint8_t* stage, const rpgpu_record_index& e, rpgpu_record_index* dst) {
    static_assert(sizeof(rpgpu_record_index) == 64, "index entry is 4 x 16 bytes");
    const uint32_t l = lane_v();
    const uint4* src = (const uint4*)&e;
    uint4* mine = (uint4*)(stage + 64u * l);
    if (dst) {
        mine[0] = src[0];
        mine[1] = src[1];
        mine[2] = src[2];
        mine[3] = src[3];
    }
    const uint64_t da = (uint64_t)(uintptr_t)dst;
    const int lo = (int)(uint32_t)da, hi = (int)(uint32_t)(da >> 32);
#pragma unroll
    for (uint32_t m = 0; m < 4u; m++) {
        const uint32_t w = 16u * m + (l >> 2), qtr = l & 3u;
        const int src_lane = (int)(w * 4u);
        const uint32_t wlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane, lo);
        const uint32_t whi = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane, hi);
        if (wlo | whi) {
            const uint4 v = *(const uint4*)(stage + 64u * w + 16u * qtr);
            uint4* d = (uint4*)((uint8_t*)(uintptr_t)(((uint64_t)whi << 32) | wlo) + 16u * qtr);
            if (RPGPU_NT_INDEX) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                v4u x;
                x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
                __builtin_nontemporal_store(x, (v4u*)d);
            } else *d = v;
        }
    }
}

// one lane's own region load (rare: a record the guess did not cover), with
// plain loads and ds_writes into its region of a slot
DEV void lane_region_load(const uint8_t* p0, uint32_t mis, uint32_t n, uint32_t base, uint8_t* region) {
    const uint8_t* row = p0 - mis + base;
    const uint32_t rows = region_rows(n, mis, base);
#pragma unroll
    for (uint32_t r = 0; r < kRegionRows; r++)
        if (r < rows) *(uint4*)(region + region_off(16u * r)) = *(const uint4*)(row + 16u * r);
}

// dword at 4-aligned offset o (< kRegionBytes) of a lane's region
DEV uint32_t region_dw(const uint8_t* region, uint32_t o) {
    return *(const uint32_t*)(region + region_off(o));
}

// The record parser's byte source over LDS regions: the current region A,
// the tail region T (C_k), else a fresh region at the read position (one
// dependent load, into H's region: the read position has left H, and C_k
// must survive as the next step's H).
struct LdsReader {
    const uint8_t* p0;  // payload start
    uint32_t mis;       // p0 & 15
    uint32_t n;
    uint32_t pos;
    const uint8_t* a;   // region being read (LDS)
    const uint8_t* t;
    uint8_t* h;
    uint32_t a_base, t_base;

    DEV uint32_t locate() {
        const uint32_t g = pos + mis;
        if (g - a_base > kRegionReach) {
            if (g - t_base <= kRegionReach) {
                a_base = t_base;
                a = t;
            } else {
                a_base = g & ~15u;
                a = h;
                lane_region_load(p0, mis, n, a_base, h);
            }
        }
        return g - a_base;
    }
    // iobuf_parser_base::read_varlong (bytes/iobuf_parser.h:48-52)
    DEV int64_t varlong() {
        const uint32_t o = locate(), k = o & ~3u, sh = o & 3u, avail = n - pos;
        const uint32_t w0 = region_dw(a, k), w1 = region_dw(a, k + 4u);
        uint32_t r0 = __builtin_amdgcn_alignbyte(w1, w0, sh), r1 = 0u, r2 = 0u, br;
        if (avail >= 2 && (r0 & 0x8080u) == 0x8080u) {
            const uint32_t w2 = region_dw(a, k + 8u), w3 = region_dw(a, k + 12u);
            r1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
            r2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
        }
        const int64_t x = varint12(r0, r1, r2, avail, br);
        pos += br;
        return x;
    }
    DEV uint32_t byte() {
        const uint32_t o = locate();
        return (region_dw(a, o & ~3u) >> (8u * (o & 3u))) & 0xFFu;
    }
};

struct LaneWalk {
    const uint8_t* p0;
    rpgpu_record_index* out;  // the batch's index slots (null when they overflow)
    uint32_t mis, n, total, done, start, cap, ord;
    uint32_t h_base;  // grid offset of the region holding `start`
};

DEV void lane_walk_begin(LaneWalk& w, const uint8_t* p0, uint32_t n, int32_t rc, uint32_t batch_ord,
                         rpgpu_record_index* out, uint32_t cap) {
    w.p0 = p0;
    w.out = out;
    w.mis = (uint32_t)((uintptr_t)p0 & 15);
    w.n = n;
    w.total = (uint32_t)(rc > 0 ? rc : 0);
    w.done = 0;
    w.start = 0;
    w.cap = cap;
    w.ord = batch_ord;
    w.h_base = w.mis & ~15u;
}

// the guessed end of the record at w.start from its length varint (H holds
// 16 bytes from it), and C_k's grid offset: 48 bytes each side of it
DEV uint32_t lane_c_base(const LaneWalk& w, const uint8_t* H) {
    const uint32_t n = w.n, mis = w.mis, start = w.start;
    uint32_t guess = 0xFFFFFFFFu;
    if (start < n) {
        const uint32_t o = start + mis - w.h_base, k = o & ~3u, sh = o & 3u;
        const uint32_t w0 = region_dw(H, k), w1 = region_dw(H, k + 4u), w2 = region_dw(H, k + 8u),
                       w3 = region_dw(H, k + 12u);
        uint32_t br;
        const int64_t len = varint12(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                     __builtin_amdgcn_alignbyte(w3, w2, sh), n - start, br);
        if (len >= 0 && (uint64_t)len <= n) guess = start + br + (uint32_t)len;
    }
    const uint32_t e16 = (guess + mis + 15u) & ~15u;
    return (guess != 0xFFFFFFFFu && e16 >= w.h_base + kRegionBefore) ? e16 - kRegionBefore : w.h_base;
}

// One record of a lane walk (w.total > 0), H and C_k in LDS: parse the record
// at w.start, hand its index entry out (e, dst: null when there is none to
// write) and move on.  Returns true when the batch is finished (wr filled);
// otherwise `fresh` says whether the next record's head is outside C_k and
// must be loaded before its step.
DEV bool lane_record_step(LaneWalk& w, WalkResult& wr, uint8_t* H, const uint8_t* Ck, uint32_t cb, bool& fresh,
                          rpgpu_record_index& e, rpgpu_record_index*& dst) {
    const uint32_t n = w.n, mis = w.mis, start = w.start;
    LdsReader c;
    c.p0 = w.p0;
    c.mis = mis;
    c.n = n;
    c.pos = start;
    c.a = H;
    c.t = Ck;
    c.h = H;
    c.a_base = w.h_base;
    c.t_base = cb;
    const Rec r = parse_fields(c);
    if (r.err) {
        wr.parsed = w.done;
        wr.err = r.err;
        wr.trailing = 0;
        return true;
    }
    // the index entry is written by the wave's cooperative store (coop_store)
    if (w.done < w.cap) {
        e.batch = w.ord;
        e.rec_pos = start;
        e.ts_delta = r.ts;
        e.length = r.length;
        e.offset_delta = r.off;
        e.key_len = r.klen;
        e.key_pos = r.key_pos;
        e.val_len = r.vlen;
        e.val_pos = r.val_pos;
        e.hdr_count = r.hcount;
        e.hdr_pos = r.hdr_pos;
        e.end_pos = r.end;
        e.attrs = (int8_t)r.attr;
        e.pad[0] = e.pad[1] = e.pad[2] = 0;
        e.reserved[0] = e.reserved[1] = 0;
        dst = w.out + w.done;
    }
    w.done++;
    w.start = r.end;
    if (w.done >= w.total) {
        wr.parsed = w.done;
        wr.err = 0;
        wr.trailing = n - w.start;
        return true;
    }
    // the next record's head: in C_k when the guess held
    const uint32_t g = w.start + mis;
    fresh = g - cb > kRegionReach;
    w.h_base = fresh ? (g & ~15u) : cb;
    return false;
}

// What a lane walk touches of the job
struct WalkCtx {
    const uint8_t* data;
    const uint64_t* seg_off;
    rpgpu_batch_result* batches;
    const uint64_t* slots;
    rpgpu_record_index* records;
    uint64_t record_capacity;
    uint32_t* counters;
    const uint64_t* chunk_count;  // note_bad (wire only)
    const uint64_t* chunk_base;
    uint32_t* seg_first_bad;
};

DEV WalkCtx walk_ctx(const DeviceJob& j) {
    return WalkCtx{j.data, j.seg_off, j.batches, j.slots, j.records, j.record_capacity, j.counters,
                   j.chunk_count, j.chunk_base, j.seg_first_bad};
}

// A lane-walked batch's descriptor, read by the walking lane itself: the
// payload, its record count and index slots.  Returns false when the batch
// is not lane-walked (incomplete, compressed or > kLaneWalkMax records).
DEV bool lane_walk_setup(const WalkCtx& j, uint64_t b, LaneWalk& w, bool& idx_ok) {
    const rpgpu_batch_result* R = &j.batches[b];
    const int32_t rc = R->record_count;
    if (!lane_walked(R->flags, (uint32_t)R->attrs & 7u, rc)) return false;
    const uint64_t S = j.seg_off[R->segment] + R->file_pos + RPGPU_HEADER_SIZE;
    const uint32_t n = (uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE);
    const uint64_t ib = j.slots[b], islots = j.slots[b + 1] - ib;
    idx_ok = ib + islots <= j.record_capacity;
    lane_walk_begin(w, j.data + S, n, rc, (uint32_t)b, idx_ok ? j.records + ib : nullptr,
                    idx_ok ? (uint32_t)islots : 0u);
    return true;
}

// A lane walk's verdict bits into the batch result (model/record.h:616-627
// sync, :680-697 async).  flags is OR-ed: the CRC wave may be writing its
// own bits into the same word at the same time.
DEV void lane_walk_finish(const WalkCtx& j, uint64_t b, const WalkResult& w, bool idx_ok, bool wire) {
    rpgpu_batch_result* R = &j.batches[b];
    uint32_t f = RPGPU_F_PARSED, perr = w.err;
    if (perr == 0) {
        f |= RPGPU_F_PARSE_ASYNC_OK;
        if (w.trailing == 0) f |= RPGPU_F_PARSE_OK;
        else perr = RPGPU_PARSE_ERR_TRAILING;
    }
    if (f & RPGPU_F_PARSE_OK) {
        if (idx_ok) f |= RPGPU_F_INDEX_WRITTEN;
        else { perr = RPGPU_PARSE_ERR_INDEX_CAPACITY; atomicOr(&j.counters[1], 2u); }
    }
    // wire: a failed sync record parse is the first batch do_load_slice
    // rejects (kafka/protocol/batch_reader.cc:129-151)
    if (wire && !(f & RPGPU_F_PARSE_OK)) note_bad_lane(j, R->segment, b);
    atomicOr(&R->flags, f);
    R->records_parsed = w.parsed;
    R->parse_err = (uint8_t)perr;
}

__global__ __launch_bounds__(1024) void k_validate(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const Tables* T = j.tables;
    const uint32_t tid = threadIdx.x;
    init_lds_tables(lds, T);
    const uint32_t l = lane_v();
    const Keys K = make_keys();
    const uint32_t c40 = uni32(T->c40);

    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    const uint64_t nw = (uint64_t)gridDim.x * kVWaves;
#ifdef RPGPU_STAMPS
    if (l == 0)
        for (int i = 0; i < 8; i++) s_stamps[tid >> 6][i] = 0;
#endif
    STAMP(tk0);
    uint64_t b = (uint64_t)blockIdx.x * kVWaves + (tid >> 6);
    if (b < nb) {
        uint32_t raw = load_desc_raw(j, b);
        Desc dn = desc_of(raw);
        Stream sn = stored_stream(j, dn, true);
        Win v;
        load_rows<0, kPreRows>(sn, v);
        for (; b < nb; b += nw) {
            const Desc d = dn;
            const Stream st = sn;
            const uint64_t bn = b + nw;
            const bool more = bn < nb;
            raw = load_desc_raw(j, more ? bn : b);
            load_rows<kPreRows, 16>(st, v);  // the rest of this batch's window
            const uint4 gt = load_tail(st);
            // the next batch's descriptor and first rows (into the rows the
            // CRC has consumed)
            auto prefetch = [&]() __attribute__((always_inline)) {
                dn = desc_of(raw);
                sn = stored_stream(j, dn, more);
                load_rows<0, kPreRows>(sn, v);
            };
            rpgpu_batch_result* R = &j.batches[b];
            STAMP(ta);
            if (!(d.flags & RPGPU_F_COMPLETE)) {
                if (l == 0) { R->index_base = d.ib; R->decoded_off = d.doff; R->reserved1 = 0; }
                note_bad(j, d.seg, b);
                prefetch();
                continue;
            }
            uint32_t f = d.flags;
            uint32_t parsed = 0, perr = 0;
            // uncompressed: the first record chain runs now, while the
            // window's lines are arriving in L2 (its scalar loads hit or merge
            // with them; after the CRC they would be evicted again)
            const bool wire = j.layout == RPGPU_LAYOUT_WIRE;
            const bool walk = d.codec == 0 && (j.flags & RPGPU_JOB_PARSE) && !lane_walked(f, d.codec, d.rc);
            Group g0;
            group_init(g0);
            g0.first = walk && d.rc > 0;
            const uint8_t* p0 = j.data + d.S;
            const uint32_t n = (uint32_t)d.n;
            if (g0.first) {
                const uint32_t total = (uint32_t)d.rc;
                g0.m = chain_starts(MemSrc{p0}, n, 0u, total < 64u ? total : 64u, g0.my_start, g0.my_end);
            }
            STAMP(tb);
            STAMP_ADD(6, tb - ta);
            // stored payload: batch crc.  CRC state after the BE40 prefix with
            // init ~0 = c40 ^ the prefix's raw contribution (from k_emit).
            // Half-way through, the first group's head and tail rows are
            // issued into the registers the CRC has freed.
            // a large stored payload (disk layout) has its CRC computed in
            // kSplitParts chunks on other waves (k_crc_split) and merged by
            // GF(2) shifts (k_crc_combine), which then sets the verdict
            // (a payload whose crc k_crc_compose assembled from the raw-block
            // CRCs of k_raw_copy and its other bytes: taken as it is)
            const bool split = !wire && !d.scc && d.n >= j.split_min;
            uint32_t crc = 0;
            if (d.scc) crc = d.ccomp;
            else if (!split) crc = ~crc_stream(lds, K, st, v, gt, d.praw ^ c40);
            record_regions(p0, (uint32_t)((uintptr_t)p0 & 15), n, g0.first && lane_v() < g0.m, g0.my_start, g0.my_end,
                           g0.H, g0.T);
            STAMP(tb2);
            STAMP_ADD(0, tb2 - tb);
            // on the wire valid_crc is only computed for v2 batches, and
            // adapt() parses records only after both checks passed
            // (kafka/protocol/kafka_batch_adapter.cc:157-181)
            if (split) {
                if (l == 0) j.split_list[atomicAdd(&j.counters[3], 1u)] = (uint32_t)b;
            } else if (crc == d.crc && (!wire || (f & RPGPU_F_WIRE_V2))) {
                f |= RPGPU_F_CRC_OK;
            } else if (!wire) {
                note_bad(j, d.seg, b);
            }
            prefetch();
            if (walk && (!wire || (f & RPGPU_F_CRC_OK))) {
                bool idx_ok;
                const WalkResult w = walk_batch(j, d, p0, n, b, idx_ok, g0);
                f |= walk_flags(j, w, idx_ok, perr);
                parsed = w.parsed;
            }
            // wire: the first batch batch_reader::do_load_slice rejects
            // (kafka/protocol/batch_reader.cc:129-151): not v2 / bad crc, codec
            // bits 5-7 (compressed() throws), or a failed sync record parse
            if (wire && (!(f & RPGPU_F_CRC_OK) || (f & RPGPU_F_CODEC_INVALID) ||
                         ((f & RPGPU_F_PARSED) && !(f & RPGPU_F_PARSE_OK))))
                note_bad(j, d.seg, b);
            STAMP(tc);
            STAMP_ADD(1, tc - tb2);
            if (l == 0) {
                R->crc_computed = crc;
                R->flags = f;
                R->index_base = d.ib;
                R->decoded_off = d.doff;
                R->records_parsed = parsed;
                R->parse_err = (uint8_t)perr;
                // a decoded payload is finished by k_validate_decoded, which
                // still needs the prefix contribution (so does k_crc_combine)
                if (!(d.codec != 0 && (f & RPGPU_F_CODEC_OK)) && !split) R->reserved1 = 0;
            }
            STAMP(td);
            STAMP_ADD(5, td - tc);
            STAMP_ADD(3, 1);
        }
    }
    STAMP(tk1);
    STAMP_ADD(4, tk1 - tk0);
#ifdef RPGPU_STAMPS
    if (l == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&g_stamps[i], s_stamps[tid >> 6][i]);
#endif
}

#ifdef RPGPU_STAMPS
__global__ void k_print_stamps() {
    const double n = (double)g_stamps[3];
    printf("RPGPU_STAMPS batches=%.0f cycles/batch/wave: desc=%.0f crc(+loads)=%.0f walk=%.0f (chain %.0f) stores=%.0f "
           "total=%.0f\n",
           n, g_stamps[2] / n, g_stamps[0] / n, g_stamps[1] / n, g_stamps[6] / n, g_stamps[5] / n, g_stamps[4] / n);
    for (int i = 0; i < 8; i++) g_stamps[i] = 0;
}
#endif

// ---------------------------------------------------------------------------
// Large stored payloads (north_star: "large batches are split into chunks
// whose partial CRCs are merged with GF(2) crc-combine shifts").  A payload
// of kSplitMin bytes or more would hold one k_validate wave for up to
// 64 KiB-row windows in series while the other waves idle at the end of a
// skewed job; instead k_validate lists it and k_crc_split spreads its
// kSplitParts chunks over all waves (claimed one at a time).  Each chunk's
// linear CRC L_k (zero initial state) is merged in k_crc_combine:
//   state = x^(8 n) * S0  ^  sum_k x^(8 (n - end_k)) * L_k   (mod P)
// with S0 the state after the BE40 prefix, the products in GF(2)[x] mod the
// reflected CRC32C polynomial (zlib's multmodp / x2nmodp scheme).
// ---------------------------------------------------------------------------
DEV uint64_t split_cut(uint64_t n, uint32_t k) { return k >= kSplitParts ? n : (n * k / kSplitParts) & ~15ull; }

__global__ __launch_bounds__(1024) void k_crc_split(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t count = j.counters[3];
    if (count == 0) return;
    init_lds_tables(lds, j.tables);
    const Keys K = make_keys();
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[15], 1u);
        if (i >= count * kSplitParts) break;
        const uint32_t item = i / kSplitParts, part = i % kSplitParts;
        const uint64_t b = uni32(j.split_list[item]);
        const Desc d = desc_of(load_desc_raw(j, b));
        // k_validate replaced index_base (the payload start) by the index
        // slot: the payload follows the 61-byte header at file_pos
        const uint64_t S = uni64(j.batches[b].file_pos) + uni64(j.seg_off[d.seg]) + RPGPU_HEADER_SIZE;
        const Stream st = make_stream(j.data, S + split_cut(d.n, part), S + split_cut(d.n, part + 1));
        Win v;
        load_window(st, 0, v);
        const uint4 gt = load_tail(st);
        const uint32_t L = crc_stream(lds, K, st, v, gt, 0u);
        if (lane_v() == 0) j.split_part[i] = L;
    }
}

// one wave per listed payload: lanes 0..15 shift the chunk CRCs, lane 16 the
// prefix state, an xor over the wave merges them; then the verdict
__global__ __launch_bounds__(256) void k_crc_combine(DeviceJob j) {
    const uint32_t item = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= j.counters[3]) return;
    const uint32_t l = lane_v();
    const uint64_t b = uni32(j.split_list[item]);
    const Desc d = desc_of(load_desc_raw(j, b));
    uint32_t t = 0;
    if (l < kSplitParts) t = crc_shift(j.split_part[item * kSplitParts + l], d.n - split_cut(d.n, l + 1));
    else if (l == kSplitParts) t = crc_shift(d.praw ^ j.tables->c40, d.n);
    t = wave_xor(t);
    const uint32_t crc = ~t;
    if (crc != d.crc) note_bad(j, d.seg, b);
    if (l == 0) {
        rpgpu_batch_result* R = &j.batches[b];
        R->crc_computed = crc;
        if (crc == d.crc) R->flags = d.flags | RPGPU_F_CRC_OK;
        if (!(d.codec != 0 && (d.flags & RPGPU_F_CODEC_OK))) R->reserved1 = 0;
    }
}

// k_crc_compose (round 6): the stored crc of an LZ4F payload decoded block by
// block, assembled without reading its stored (raw) blocks again.  k_raw_copy
// copied every independent raw block without a block checksum to the arena
// and took its linear CRC on the way (BlockItem.crc; the decoded bytes are the
// stored ones); the payload's other bytes (frame header, size words,
// compressed blocks, checksums, end mark, anything after it) are CRC'd here
// from the stored payload, and the pieces merged in order by GF(2) shifts:
//   state = x^(8 len) * state  ^  L(block)     per raw block,
// from the BE40 prefix state S0, exactly the state k_validate's stream
// reaches.  C2: 12 of its 12.9 GB of stored payload are raw blocks that
// k_validate read a second time.  One wave per decode item; k_validate takes
// the result (Desc.scc) instead of streaming the payload.
constexpr uint64_t kComposeMin = 64u << 10;
// sum over the wave of block sizes (each <= 4 MiB, so 64 of them fit 32 bits)
DEV uint32_t wave_sum_u32(uint32_t v) {
    for (int o = 32; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return uni32(v);
}
__global__ __launch_bounds__(1024) void k_crc_compose(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t count = j.counters[2];
    // worth it only when raw blocks are most of the job's stored bytes (C2:
    // 12 of 12.9 GB); otherwise k_validate streams every payload as before
    // (C5, a few raw blocks among snappy and compressed LZ4: the kernel's
    // pass over the decode list cost more than it saved)
    const uint64_t raw_bytes = *(const volatile uint64_t*)(j.counters + 24);
    if (count == 0 || j.counters[40] == 0 || 2 * raw_bytes < j.data_len) return;
    init_lds_tables(lds, j.tables);
    const Keys K = make_keys();
    const uint32_t l = lane_v(), c40 = uni32(j.tables->c40);
    auto gap = [&](uint64_t a, uint64_t e, uint32_t state) __attribute__((always_inline)) {
        if (e - a <= 64) {
            // a short gap (size words, checksums, the frame header): lane k
            // holds byte k, folded in with uniform word / byte steps (a
            // window here cost a load round trip and 16 rows of braids)
            const uint32_t nb = (uint32_t)(e - a);
            const uint32_t by = l < nb ? (uint32_t)j.data[a + l] : 0u;
            uint32_t k = 0;
            for (; k + 4 <= nb; k += 4)
                state = uni32(word_step(lds, state, rl(by, (int)k) | (rl(by, (int)k + 1) << 8) |
                                                        (rl(by, (int)k + 2) << 16) | (rl(by, (int)k + 3) << 24)));
            for (; k < nb; k++) state = uni32(byte_step(lds, state, rl(by, (int)k)));
            return state;
        }
        const Stream st = make_stream(j.data, a, e);
        Win v;
        load_window(st, 0, v);
        const uint4 gt = load_tail(st);
        return crc_stream(lds, K, st, v, gt, state);
    };
    for (;;) {
        const uint32_t item = wave_fetch_add(&j.counters[12], 1u);
        if (item >= count) break;
        if (uni32(j.plans[item].mode) != 1u) continue;
        const uint32_t first = uni32(j.plans[item].first), nb = uni32(j.plans[item].nb);
        // composed only where raw blocks are most of a large payload: a
        // payload of mostly compressed blocks streams faster through
        // k_validate than its gaps do here one window latency each (C5:
        // validate 3.67 -> 3.98 ms with every payload holding a raw block
        // composed)
        uint64_t rawb = 0;
        for (uint32_t k0 = 0; k0 < nb; k0 += 64) {
            const uint32_t k = k0 + l;
            const bool r = k < nb && j.blocks[first + k].fast == kLzfRaw;
            rawb += wave_sum_u32(r ? j.blocks[first + k].csize : 0u);
        }
        const uint64_t b = uni32(j.decode_list[item]);
        const Desc d = desc_of(load_desc_raw(j, b));
        if (!(d.flags & RPGPU_F_COMPLETE) || d.n < kComposeMin || 4 * rawb < 3 * d.n) continue;
        uint32_t state = d.praw ^ c40;
        uint64_t pos = d.S;  // (index_base still holds the payload start: k_validate runs after)
        for (uint32_t k = 0; k < nb; k++) {
            if (uni32(j.blocks[first + k].fast) != kLzfRaw) continue;
            const uint64_t a = uni64(j.blocks[first + k].src);
            const uint32_t len = uni32(j.blocks[first + k].csize);
            if (a > pos) state = gap(pos, a, state);
            state = crc_shift(state, len) ^ uni32(j.blocks[first + k].crc);
            pos = a + len;
        }
        if (d.S + d.n > pos) state = gap(pos, d.S + d.n, state);
        if (l == 0) {
            rpgpu_batch_result* R = &j.batches[b];
            R->crc_computed = ~state;
            R->reserved0 = (uint16_t)(R->reserved0 | 2u);
        }
    }
}

// k_dchain (round 6): the record chain of every decoded payload, one LANE per
// payload, so that all of a job's chains are in flight at once.  (The chain
// is one dependent load per record: k_validate_decoded's wave-uniform
// chain_starts paid ~520 of them per C2 batch, for one batch after another
// on each wave, 3.3 ms for C2's 16 M records.)  pre[k] = the position after
// record k's length varint and body, exactly chain_starts' arithmetic, and
// 0xFFFFFFFF where it stops (a start at or past the end, a bad length);
// written at the payload's index slots of the record pool (j.dchain), read
// back 64 at a time by walk_records (pre_starts).
#ifndef RPGPU_DCHAIN_PRIO
#define RPGPU_DCHAIN_PRIO 2
#endif
__global__ __launch_bounds__(256) void k_dchain(DeviceJob j) {
    // above k_content_xxh's waves on a shared SIMD: an XXH32 chain keeps the
    // SIMD's VALU busy back to back (its quarter-rate multiply per stripe), and
    // a chain lane waiting behind it held k_dchain's end with it (0.9 -> 1.9 ms)
    __builtin_amdgcn_s_setprio(RPGPU_DCHAIN_PRIO);
    const uint32_t nlz = j.counters[2], ngz = j.counters[16], count = nlz + ngz + j.counters[19];
    const uint8_t* const aend = j.decoded + j.decoded_capacity;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x) {
        const uint64_t b = i < nlz ? j.decode_list[i] : i < nlz + ngz ? j.inf_list[i - nlz] : j.host_list[i - nlz - ngz];
        const rpgpu_batch_result& R = j.batches[b];
        const uint32_t flags = R.flags;
        const int32_t rc = R.record_count;
        const uint64_t ib = j.slots[b], islots = j.slots[b + 1] - ib;
        if (!dchain_ok(j, flags, rc, ib, islots, R.decoded_len)) continue;
        const uint8_t* p0 = j.decoded + j.dcap[b];
        const uint32_t n = R.decoded_len;
        uint32_t* pre = j.dchain + ib;
        uint32_t p = 0;
        for (int32_t k = 0; k < rc; k++) {
            if (p >= n) {
                pre[k] = 0xFFFFFFFFu;
                break;
            }
            // 12 bytes at p: four aligned dwords (byte loads at the arena's end)
            const uint8_t* q = p0 + p;
            const uint32_t* a = (const uint32_t*)((uintptr_t)q & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)((uintptr_t)q & 3);
            uint32_t w0, w1, w2, w3;
            if ((const uint8_t*)(a + 4) <= aend) {
                w0 = a[0]; w1 = a[1]; w2 = a[2]; w3 = a[3];
            } else {
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                for (uint32_t t = 0; t < 16; t++)
                    if ((const uint8_t*)a + t < aend) w[t >> 2] |= (uint32_t)((const uint8_t*)a)[t] << (8 * (t & 3));
                w0 = w[0]; w1 = w[1]; w2 = w[2]; w3 = w[3];
            }
            uint32_t br;
            const int64_t len = varint12(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                         __builtin_amdgcn_alignbyte(w3, w2, sh), n - p, br);
            if (len < 0 || (uint64_t)len > n) {
                pre[k] = 0xFFFFFFFFu;
                break;
            }
            p = p + br + (uint32_t)len;
            pre[k] = p;
        }
    }
}

// reset_size_checksum_metadata (storage/parser_utils.cc:114-120) and the
// record walk over every payload k_decode uncompressed: one wave per
// worklist item, after k_validate has written the stored-payload verdict.
// The new crc covers the BE40 prefix with the codec bits of attrs cleared
// (BE40 byte 1) followed by the decoded bytes.
__global__ __launch_bounds__(1024) void k_validate_decoded(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    // the LZ4 / snappy decode list, then the gzip members
    const uint32_t nlz = j.counters[2], ngz = j.counters[16], count = nlz + ngz + j.counters[19];
    if (count == 0) return;
    const Tables* T = j.tables;
    init_lds_tables(lds, T);
    const uint32_t l = lane_v();
    const Keys K = make_keys();
    const uint32_t c40 = uni32(T->c40);
    // items claimed one at a time (counters[13]): payloads run 200 B .. 1 MiB,
    // and a static stride left waves holding several of the largest
    for (;;) {
        const uint32_t i = wave_fetch_add(&j.counters[13], 1u);
        if (i >= count) break;
        const uint64_t b = uni32(i < nlz ? j.decode_list[i] : i < nlz + ngz ? j.inf_list[i - nlz] : j.host_list[i - nlz - ngz]);
        rpgpu_batch_result* R = &j.batches[b];
        Desc d = desc_of(load_desc_raw(j, b));
        if (!(d.flags & RPGPU_F_CODEC_OK)) continue;
        // k_validate replaced index_base (the payload start) by the index
        // slot; the header sits at file_pos in its segment
        const uint64_t hdr = uni64(R->file_pos) + uni64(j.seg_off[d.seg]);
        const uint64_t dl = d.dlen;
        // block-parallel frames: k_decode_finish merged the streaming CRCs
        // of k_lz_exec's flushes (reserved0 = 1); frames decoded whole (the
        // sequential list) are read back here
        uint32_t dcrc;
        if (uni32((uint32_t)R->reserved0) & 1u) {
            dcrc = uni32(R->decoded_crc);
        } else {
            const Stream ds = make_stream(j.decoded, d.doff, d.doff + dl);
            Win dv;
            load_window(ds, 0, dv);
            const uint4 dgt = load_tail(ds);
            dcrc = ~crc_stream(lds, K, ds, dv, dgt, d.praw ^ T->hdr[38][d.codec] ^ c40);
        }
        const uint32_t dhcrc = decoded_header_crc(T, j.data + hdr, (uint32_t)(RPGPU_HEADER_SIZE + dl), dcrc,
                                                  j.layout == RPGPU_LAYOUT_WIRE);
        uint32_t f = d.flags, perr = 0, parsed = 0;
        if ((j.flags & RPGPU_JOB_PARSE) && (j.layout != RPGPU_LAYOUT_WIRE || (d.flags & RPGPU_F_CRC_OK))) {
            bool idx_ok;
            Group g0;
            group_init(g0);
            const uint32_t* pre = dchain_ok(j, d.flags, d.rc, d.ib, d.islots, d.dlen) ? j.dchain + d.ib : nullptr;
            const WalkResult w = walk_batch(j, d, j.decoded + d.doff, (uint32_t)dl, b, idx_ok, g0, pre);
            f |= walk_flags(j, w, idx_ok, perr);
            parsed = w.parsed;
        }
        if (l == 0) {
            R->flags = f;
            R->records_parsed = parsed;
            R->parse_err = (uint8_t)perr;
            R->decoded_crc = dcrc;
            R->decoded_header_crc = dhcrc;
            R->reserved0 = 0;
            R->reserved1 = 0;
        }
    }
}

// k_walk: the record walk of stored (uncompressed) payloads with at most
// kLaneWalkMax records, one LANE per batch, after k_validate has written the
// CRC verdicts.  record_batch::for_each_record (model/record.h:616-627) is
// sequential by nature: record k + 1 starts where record k's parse ended
// (parse_fields: model/record_utils.cc:94-181).  Every lane of a wave takes
// one step per turn of a wave-uniform loop (the cooperative region fetch
// needs all 64 lanes):
//   idle  -> take the lane's next batch (grid-stride); its first region is
//            fetched this turn (state head)
//   head  -> its region arrived: walk from the next turn
//   walk  -> fetch C_k, parse record k, commit it
// Batches with more records are walked by the wave-parallel walk inside
// k_validate.
__global__ __launch_bounds__(256) void k_walk(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    enum : uint32_t { kIdle = 0, kHead = 1, kWalk = 2, kFin = 3 };
    uint8_t* wave = lds + (threadIdx.x >> 6) * kWalkLdsWave;
    const uint32_t l = lane_v();
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    const bool wire = j.layout == RPGPU_LAYOUT_WIRE;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const WalkCtx c = walk_ctx(j);
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t st = kIdle;
    bool first = true, idx_ok = false;
    LaneWalk w;
    for (uint32_t step = 0;; step++) {
        uint8_t* hslot = wave + (step & 1u) * kSlotBytes;   // H of this turn
        uint8_t* cslot = wave + (~step & 1u) * kSlotBytes;  // fetched this turn
        if (st == kIdle) {
            if (!first) b += stride;
            first = false;
            if (b >= nb) st = kFin;
            else if (!(wire && !(j.batches[b].flags & RPGPU_F_CRC_OK)) && lane_walk_setup(c, b, w, idx_ok)) {
                if (w.total == 0) {
                    WalkResult wr;
                    wr.parsed = 0; wr.err = 0; wr.trailing = w.n;
                    lane_walk_finish(c, b, wr, idx_ok, wire);
                } else st = kHead;
            }
        }
        uint32_t want = 0, rows = 0;
        if (st == kWalk) want = lane_c_base(w, hslot + region_lane(l));
        else if (st == kHead) want = w.h_base;
        if (st == kWalk || st == kHead) rows = region_rows(w.n, w.mis, want);
        if (__ballot(st != kFin) == 0) break;
        if (kCoopLoad) coop_load(cslot, w.p0 - w.mis + want, rows);
        else {
            const uint8_t* g = w.p0 - w.mis + want;
#pragma unroll
            for (uint32_t r = 0; r < kRegionRows; r++)
                if (r < rows)
                    __builtin_amdgcn_global_load_lds((gbl_void*)(g + 16u * r), (lds_void*)(cslot + 1024u * r), 16, 0, 0);
        }
        wait_vm();
        rpgpu_record_index e;
        rpgpu_record_index* dst = nullptr;
        if (st == kWalk) {
            WalkResult wr;
            bool fresh = false;
            if (lane_record_step(w, wr, hslot + region_lane(l), cslot + region_lane(l), want, fresh, e, dst)) {
                lane_walk_finish(c, b, wr, idx_ok, wire);
                st = kIdle;
            } else if (fresh) st = kHead;
        } else if (st == kHead) st = kWalk;
        // H is spent: its slot stages the entries
        coop_store(hslot, e, dst);
    }
}

// ---------------------------------------------------------------------------
// Write side: stamp the headers of batches about to be
// written, one wave per batch (claimed one at a time):
//   * RPGPU_STAMP_OFFSETS — disk_log_appender::operator() (storage/
//     disk_log_appender.cc:72-74, :113-119): base_offset = the appender's
//     next offset, which then moves to last_offset + 1 (the caller's
//     exclusive scan of last_offset_delta + 1 gives every batch its value);
//   * RPGPU_STAMP_CRC — reset_size_checksum_metadata (storage/parser_utils.cc:
//     114-120): size_bytes = 61 + payload, crc = crc_record_batch (BE40 prefix
//     then the payload, the same braided window CRC as k_validate);
//   * header_crc = internal_header_only_crc (model/record_utils.cc:34-55)
//     over the final header, always.
// ---------------------------------------------------------------------------
// BE40 prefix byte k (model/record_utils.cc:68-80) = disk header byte be_src(k)
DEV uint32_t be40_src(uint32_t k) {
    // fields: attrs 2 @21, lod 4 @23, first_ts 8 @27, max_ts 8 @35, pid 8 @43,
    // epoch 2 @51, base_seq 4 @53, record_count 4 @57 (each byte-reversed)
    return k < 2 ? 22 - k : k < 6 ? 26 - (k - 2) : k < 14 ? 34 - (k - 6) : k < 22 ? 42 - (k - 14) : k < 30 ? 50 - (k - 22)
         : k < 32 ? 52 - (k - 30) : k < 36 ? 56 - (k - 32) : 60 - (k - 36);
}

__global__ __launch_bounds__(1024) void k_stamp(uint8_t* data, const uint64_t* __restrict__ pos,
                                                const uint32_t* __restrict__ plen,
                                                const uint64_t* __restrict__ offs, int64_t next, uint32_t n,
                                                uint32_t flags, const Tables* T, uint32_t* cursor) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    init_lds_tables(lds, T);
    const uint32_t l = lane_v();
    const Keys K = make_keys();
    const uint32_t c40 = uni32(T->c40);
    for (;;) {
        const uint32_t i = wave_fetch_add(cursor, 1u);
        if (i >= n) break;
        const uint64_t p = uni64(pos[i]);
        const uint32_t L = uni32(plen[i]);
        uint8_t* h = data + p;
        uint32_t b = l < RPGPU_HEADER_SIZE ? (uint32_t)h[l] : 0u;
        if (flags & RPGPU_STAMP_OFFSETS) {
            const uint64_t bo = (uint64_t)next + uni64(offs[i]);
            if (l >= 8 && l < 16) b = (uint32_t)(bo >> (8 * (l - 8))) & 0xFFu;
        }
        if (flags & RPGPU_STAMP_CRC) {
            const uint32_t size = RPGPU_HEADER_SIZE + L;
            if (l >= 4 && l < 8) b = (size >> (8 * (l - 4))) & 0xFFu;
            // raw CRC contribution of the BE40 prefix: lane k < 40 holds its byte
            const uint32_t pb = (uint32_t)__shfl((int)b, (int)be40_src(l < 40 ? l : 0), 64);
            uint32_t x = l < 40 ? T->hdr[39 - l][pb] : 0u;
            x ^= swz_xor<1>(x);
            x ^= swz_xor<2>(x);
            x ^= swz_xor<4>(x);
            x ^= swz_xor<8>(x);
            x ^= swz_xor<16>(x);
            const uint32_t praw = rl(x, 0) ^ rl(x, 32);
            const Stream st = make_stream(data, p + RPGPU_HEADER_SIZE, p + RPGPU_HEADER_SIZE + L);
            Win w;
            load_window(st, 0, w);
            const uint4 gt = load_tail(st);
            const uint32_t crc = ~crc_stream(lds, K, st, w, gt, praw ^ c40);
            if (l >= 17 && l < 21) b = (crc >> (8 * (l - 17))) & 0xFFu;
        }
        // header_crc over bytes 4..60 of the stamped header
        uint32_t x = (l >= 4 && l < RPGPU_HEADER_SIZE) ? T->hdr[60 - l][b] : 0u;
        x ^= swz_xor<1>(x);
        x ^= swz_xor<2>(x);
        x ^= swz_xor<4>(x);
        x ^= swz_xor<8>(x);
        x ^= swz_xor<16>(x);
        const uint32_t hc = ~(T->c57 ^ rl(x, 0) ^ rl(x, 32));
        if (l < 4) b = (hc >> (8 * l)) & 0xFFu;
        if (l < 21) h[l] = (uint8_t)b;
    }
}

// per batch last_offset_delta + 1 (the appender's offset step), scanned by the caller
__global__ __launch_bounds__(256) void k_stamp_steps(const uint8_t* data, const uint64_t* __restrict__ pos, uint32_t n,
                                                     uint64_t* steps) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* h = data + pos[i] + 23;
    const int32_t lod = (int32_t)((uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24));
    steps[i] = (uint64_t)((int64_t)lod + 1);
}

hipError_t launch_stamp_steps(const uint8_t* data, const uint64_t* pos, uint32_t n, uint64_t* steps, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_stamp_steps, dim3((n + 255) / 256), dim3(256), 0, s, data, pos, n, steps);
    return hipGetLastError();
}

hipError_t launch_stamp(uint8_t* data, const uint64_t* pos, const uint32_t* plen, const uint64_t* offs, int64_t next,
                        uint32_t n, uint32_t flags, const Tables* T, uint32_t* cursor, uint32_t grid, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_stamp, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsValidateBytes);
        attr = true;
    }
    hipLaunchKernelGGL(k_stamp, dim3(grid), dim3(64 * kVWaves), kLdsValidateBytes, s, data, pos, plen, offs, next, n,
                       flags, T, cursor);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// kafka::writer_serialize_batch (kafka/protocol/response_writer.h:241-276):
// disk-layout batches -> a Kafka v2 record set, one wave per batch.  The
// wire header is the disk header re-encoded big-endian: base_offset,
// batch_length = size_bytes - 61 + 61 - 8 - 4, partition leader epoch 0,
// magic 2, crc, attrs, last_offset_delta, first/max timestamp, producer id,
// epoch, base_sequence, record_count; the payload follows unchanged.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_to_wire(const uint8_t* __restrict__ disk, uint8_t* __restrict__ wire,
                                                 const uint64_t* __restrict__ src, const uint64_t* __restrict__ dst,
                                                 uint32_t n) {
    const uint32_t l = lane_v();
    for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
        const uint8_t* h = disk + uni64(src[i]);
        uint8_t* o = wire + uni64(dst[i]);
        uint32_t b = l < RPGPU_HEADER_SIZE ? (uint32_t)h[l] : 0u;
        const int32_t size = (int32_t)(rl(b, 4) | (rl(b, 5) << 8) | (rl(b, 6) << 16) | (rl(b, 7) << 24));
        const uint32_t blen = (uint32_t)(size - 12);
        // wire byte l <- disk byte src(l), reversed within each field
        int from = -1;
        uint32_t w = 0;
        if (l < 8) from = 15 - (int)l;                        // base_offset (disk 8..15)
        else if (l < 12) w = (blen >> (8 * (11 - l))) & 0xFFu;  // batch_length
        else if (l < 16) w = 0;                               // partition leader epoch
        else if (l == 16) w = 2;                              // magic
        else if (l < 21) from = 20 - ((int)l - 17);           // crc (disk 17..20)
        else if (l < RPGPU_HEADER_SIZE) from = (int)be40_src(l - 21);  // attrs .. record_count (the BE40 prefix)
        const uint32_t v = (uint32_t)__shfl((int)b, from < 0 ? 0 : from, 64);
        if (from >= 0) w = v;
        if (l < RPGPU_HEADER_SIZE) o[l] = (uint8_t)w;
        const uint32_t pl = (uint32_t)size - RPGPU_HEADER_SIZE;
        const uint8_t* ps = h + RPGPU_HEADER_SIZE;
        uint8_t* pd = o + RPGPU_HEADER_SIZE;
        for (uint32_t c = 0; c < pl; c += 1024) {
            const uint32_t k = c + 16 * l;
            if (k + 16 <= pl) {
                uint4 t;
                __builtin_memcpy(&t, ps + k, 16);
                __builtin_memcpy(pd + k, &t, 16);
            } else if (k < pl) {
                for (uint32_t e = k; e < pl; e++) pd[e] = ps[e];
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_wire_sizes(const rpgpu_batch_result* __restrict__ batches,
                                                    const uint64_t* __restrict__ seg_off, uint64_t first, uint32_t n,
                                                    uint64_t* src, uint64_t* sizes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rpgpu_batch_result& r = batches[first + i];
    src[i] = seg_off[r.segment] + r.file_pos;
    sizes[i] = (uint64_t)(uint32_t)r.size_bytes;
}

hipError_t launch_to_wire(const uint8_t* disk, uint8_t* wire, const rpgpu_batch_result* batches, const uint64_t* seg_off,
                          uint64_t first, uint32_t n, uint64_t* src, uint64_t* dst, void* scan_tmp, size_t scan_bytes,
                          uint32_t grid, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_wire_sizes, dim3((n + 255) / 256), dim3(256), 0, s, batches, seg_off, first, n, src, dst);
    hipError_t e = scan_exclusive_u64(dst, n, scan_tmp, scan_bytes, s);  // dst[n] = total
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_to_wire, dim3(grid), dim3(256), 0, s, disk, wire, src, dst, n);
    return hipGetLastError();
}

hipError_t launch_walk(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    if (j.flags & RPGPU_JOB_PARSE)
        hipLaunchKernelGGL(k_walk, dim3(grid), dim3(256), 4 * kWalkLdsWave, s, j);  // 48 KiB: 3 per CU
    return hipGetLastError();
}

hipError_t launch_crc_compose(const DeviceJob& j, hipStream_t s, uint32_t grid, uint32_t waves) {
    (void)hipFuncSetAttribute((const void*)k_crc_compose, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsValidateBytes);
    if (j.crc_compose && (j.flags & RPGPU_JOB_DECODE) && j.decoded && j.raw_list && j.layout == RPGPU_LAYOUT_DISK)
        hipLaunchKernelGGL(k_crc_compose, dim3(grid), dim3(64 * waves), kLdsValidateBytes, s, j);
    return hipGetLastError();
}

hipError_t launch_validate(const DeviceJob& j, hipStream_t s, uint32_t grid, bool compose) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_validate, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsValidateBytes);
        (void)hipFuncSetAttribute((const void*)k_validate_decoded, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kLdsValidateBytes);
        (void)hipFuncSetAttribute((const void*)k_crc_split, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kLdsValidateBytes);
        (void)hipFuncSetAttribute((const void*)k_crc_compose, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kLdsValidateBytes);
        attr = true;
    }
    if (compose && j.crc_compose && (j.flags & RPGPU_JOB_DECODE) && j.decoded && j.raw_list && j.layout == RPGPU_LAYOUT_DISK)
        hipLaunchKernelGGL(k_crc_compose, dim3(grid), dim3(64 * kVWaves), kLdsValidateBytes, s, j);
    hipLaunchKernelGGL(k_validate, dim3(grid), dim3(64 * kVWaves), kLdsValidateBytes, s, j);
#ifdef RPGPU_STAMPS
    hipLaunchKernelGGL(k_print_stamps, dim3(1), dim3(1), 0, s);
#endif
    if (j.layout != RPGPU_LAYOUT_WIRE && j.data_len >= j.split_min) {
        hipLaunchKernelGGL(k_crc_split, dim3(grid), dim3(64 * kVWaves), kLdsValidateBytes, s, j);
        hipLaunchKernelGGL(k_crc_combine, dim3((j.split_capacity + 3) / 4), dim3(256), 0, s, j);
    }
    return hipGetLastError();
}

// k_dchain: lanes with no payload exit at once; a grid of 2 workgroups per CU
// covers C2's 31 K payloads in one pass
bool dchain_wanted(const DeviceJob& j) {
    return (j.flags & RPGPU_JOB_DECODE) && (j.flags & RPGPU_JOB_PARSE) && j.decoded && j.dchain &&
           j.layout == RPGPU_LAYOUT_DISK;
}
hipError_t launch_dchain(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    if (dchain_wanted(j)) hipLaunchKernelGGL(k_dchain, dim3(grid * 2), dim3(256), 0, s, j);  // 8 waves per CU beside k_validate's 16
    return hipGetLastError();
}

hipError_t launch_validate_decoded(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    if ((j.flags & RPGPU_JOB_DECODE) && j.decoded)
        hipLaunchKernelGGL(k_validate_decoded, dim3(grid), dim3(64 * kVWaves), kLdsValidateBytes, s, j);
    return hipGetLastError();
}

}  // namespace rp
