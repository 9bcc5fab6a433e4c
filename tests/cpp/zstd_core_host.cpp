// Host instantiation of the device zstd decoder's logic (rp_zstd_core.h),
// TEST INFRASTRUCTURE ONLY: tests/test_zstd_core.py fuzzes it against
// libzstd through the reference's loop (the oracle) so that the acceptance
// rules the device kernels run are pinned on the CPU, where thousands of
// mutated frames take seconds.  The product never loads this library.
#include <stdint.h>
#include <string.h>

#include <vector>

#define ZS_FN static inline
#include "../../redpanda_amd/csrc/rp_zstd_core.h"

namespace {

uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
const uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
               P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
uint64_t round1(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
uint64_t merge(uint64_t acc, uint64_t v) { return (acc ^ round1(0, v)) * P1 + P4; }
uint64_t xxh64(const uint8_t* p, size_t n) {
    const uint8_t* e = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        while (p + 32 <= e) {
            v1 = round1(v1, rd64(p)); v2 = round1(v2, rd64(p + 8)); v3 = round1(v3, rd64(p + 16)); v4 = round1(v4, rd64(p + 24));
            p += 32;
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = merge(h, v1); h = merge(h, v2); h = merge(h, v3); h = merge(h, v4);
    } else {
        h = P5;
    }
    h += n;
    while (p + 8 <= e) { h ^= round1(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
    if (p + 4 <= e) { h ^= (uint64_t)rd32(p) * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
    while (p < e) { h ^= (*p) * P5; h = rotl(h, 11) * P1; p++; }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

struct HostEnv {
    const uint8_t* src;
    uint64_t n;
    std::vector<uint8_t> out;
    size_t fstart = 0;
    uint32_t b(uint64_t i) const { return i < n ? src[i] : 0u; }
    uint64_t le(uint64_t i, uint32_t k) const {
        uint64_t v = 0;
        for (uint32_t j = 0; j < k; j++) v |= (uint64_t)b(i + j) << (8 * j);
        return v;
    }
    uint64_t lb(rp::zs::Bits&, uint64_t i) const { return le(i, 8); }
    uint32_t U(uint32_t x) const { return x; }
    rp::zs::SeqSym sym(const rp::zs::SeqSym& s) const { return s; }
    void raw(uint64_t pos, uint64_t k) { out.insert(out.end(), src + pos, src + pos + k); }
    void fill(uint32_t v, uint64_t k) { out.insert(out.end(), (size_t)k, (uint8_t)v); }
    void lit(uint32_t v) { out.push_back((uint8_t)v); }
    void match(uint64_t off, uint64_t ml) {
        for (uint64_t i = 0; i < ml; i++) out.push_back(out[out.size() - off]);
    }
    void frame_begin() { fstart = out.size(); }
    int check(uint32_t v) { return (uint32_t)xxh64(out.data() + fstart, out.size() - fstart) == v ? 1 : 0; }
};

// Eager literals (rp::zs::EagerLits, as the device's lane parser decodes
// them): every Huffman literal of a block decoded before its sequences, taken
// from a per-block buffer in consumption order
struct EagerHostEnv : HostEnv {
    std::vector<uint8_t> blk;
    size_t took = 0;
    // eager sequences (rp::zs::EagerSeqs, as k_zlits decodes them ahead):
    // the block's whole sequence stream decoded at once, then applied
    rp::zs::Tabs* T = nullptr;
    std::vector<rp::zs::RawSeq> seqs;
    size_t next = 0;
    bool ok = false;
    bool seqs_take(uint64_t sp, uint64_t n, uint32_t nseq, uint32_t llog, uint32_t olog, uint32_t mlog) {
        rp::zs::Bits d;
        if (!rp::zs::bits_init(*this, d, sp, n)) return false;  // block() rejects in place
        rp::zs::SeqState q;
        rp::zs::seq_begin(*this, d, q, llog, olog, mlog);
        seqs.resize(nseq);
        for (uint32_t k = 0; k < nseq; k++) rp::zs::seq_decode(*this, T, d, q, seqs[k]);
        ok = rp::zs::bits_reload(*this, d) >= rp::zs::kCompleted;
        next = 0;
        return true;
    }
    void seq_next(rp::zs::RawSeq& r) { r = seqs[next++]; }
    // the block() loop over the taken sequences (the device applies 64 at a
    // time across lanes; here the plain restatement, pinning the hook)
    bool seqs_apply(rp::zs::Frame& F, rp::zs::Lits& L, uint64_t& r0, uint64_t& r1, uint64_t& r2, uint64_t& bo,
                    uint64_t capb, uint32_t nseq) {
        for (uint32_t k = 0; k < nseq; k++) {
            const rp::zs::RawSeq& s = seqs[k];
            uint64_t off;
            if (s.kind == 0) { off = s.v; r2 = r1; r1 = r0; r0 = off; }
            else if (s.kind == 1) { if (s.ll != 0) off = r0; else { off = r1; r1 = r0; r0 = off; } }
            else {
                uint64_t t = s.v == 3 ? r0 - 1 : (s.v == 1 ? r1 : r2);
                t += !t;
                if (s.v != 1) r2 = r1;
                r1 = r0;
                r0 = off = t;
            }
            const uint64_t ll = s.ll, ml = s.ml;
            if (ll + ml > capb - bo) return false;
            if (ll > (uint64_t)(L.size - L.used)) return false;
            take(ll);
            L.used += (uint32_t)ll;
            bo += ll;
            F.fo += ll;
            if (off > F.fo - F.seg0 + F.prevlen) return false;
            if (off > F.fo - F.seg0 && F.prevlen - (off - (F.fo - F.seg0)) < F.fo - F.seg0 + rp::zs::kRingDirty)
                return false;
            match(off, ml);
            bo += ml;
            F.fo += ml;
        }
        return true;
    }
    bool seqs_ok() const { return ok; }
    void take(uint64_t k) {
        out.insert(out.end(), blk.begin() + took, blk.begin() + took + k);
        took += k;
    }
    void raw_ahead(uint64_t pos, uint64_t k) {
        blk.assign(src + pos, src + pos + k);
        took = 0;
    }
    void fill_ahead(uint32_t v, uint64_t k) {
        blk.assign((size_t)k, (uint8_t)v);
        took = 0;
    }
    void huf_all(rp::zs::Tabs* T, rp::zs::Lits& L, uint32_t hlog) {
        blk.assign(L.size, 0);
        took = 0;
        for (uint32_t k = 0; k < L.ns; k++) {
            for (uint32_t i = 0; i < L.cnt[k]; i++)
                blk[(size_t)k * L.seg + i] =
                    (uint8_t)rp::zs::huf_one(*this, T, L.s[k], L.pend[k], L.cnt[k] - i, L.x2, hlog);
            L.dec[k] = L.cnt[k];
        }
    }
};

// The DCtx's output buffer emulated byte for byte (rp::zs::ExactRing): what
// libzstd's ZSTD_execSequence (x86-64, SSE2 COPY16) writes, overcopies
// included, so that a match reaching into the previous ring segment where
// the current one has written reads libzstd's bytes.  WILDCOPY_PAIRS selects
// the x86 ZSTD_wildcopy loop shape (one COPY16, then two per iteration).
#ifndef WILDCOPY_PAIRS
#define WILDCOPY_PAIRS 1
#endif
struct ExactHostEnv : EagerHostEnv {
    std::vector<uint8_t> buf;  // the DCtx's outBuff (or the caller's output room: single pass)
    uint64_t op = 0, oend = 0;
    std::vector<uint8_t> pad;  // bytes a wildcopy reads past the block's literals
    uint8_t L(size_t i) const { return i < blk.size() ? blk[i] : pad[i - blk.size()]; }
    void ring_begin(uint64_t size) {
        oend = size;
        if (buf.size() < size + 256) buf.resize(size + 256, 0);
        op = 0;
        prevlen = 0;
    }
    void ring_wrap() {
        prevlen = op;
        op = 0;
    }
    void lit_pad(int mode, uint64_t pos, uint32_t rle) {
        pad.assign(64, 0);
        if (mode == 1)
            for (int i = 0; i < 64; i++) pad[i] = (pos + i < n) ? src[pos + i] : 0;
        else if (mode == 2)
            for (int i = 0; i < 64; i++) pad[i] = (uint8_t)rle;
    }
    void emit(uint64_t a, uint64_t k) { out.insert(out.end(), buf.begin() + a, buf.begin() + a + k); }
    // exact writes (raw / RLE blocks, the last literals): memcpy / memset
    void raw(uint64_t pos, uint64_t k) {
        memcpy(&buf[op], src + pos, k);
        emit(op, k);
        op += k;
    }
    void fill(uint32_t v, uint64_t k) {
        memset(&buf[op], (int)v, k);
        emit(op, k);
        op += k;
    }
    void take(uint64_t k) {
        for (uint64_t i = 0; i < k; i++) buf[op + i] = L(took + i);
        emit(op, k);
        op += k;
        took += k;
    }
    // COPY16 / COPY8: the whole source loaded, then stored
    void copy_n(uint64_t d, uint64_t s, int k) {
        uint8_t t[16];
        for (int i = 0; i < k; i++) t[i] = buf[s + i];
        for (int i = 0; i < k; i++) buf[d + i] = t[i];
    }
    // ZSTD_wildcopy from the output buffer (src_before_dst: overlap allowed)
    void wild_buf(uint64_t d, uint64_t s, int64_t length, bool overlap) {
        const uint64_t e = d + (uint64_t)length;
        if (overlap && d - s < 16) {
            do { copy_n(d, s, 8); d += 8; s += 8; } while (d < e);
            return;
        }
#if WILDCOPY_PAIRS
        copy_n(d, s, 16);
        if (16 >= length) return;
        d += 16; s += 16;
        do { copy_n(d, s, 16); d += 16; s += 16; copy_n(d, s, 16); d += 16; s += 16; } while (d < e);
#else
        do { copy_n(d, s, 16); d += 16; s += 16; } while (d < e);
#endif
    }
    // ZSTD_wildcopy from the literal buffer (no overlap)
    void wild_lit(uint64_t d, size_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
#if WILDCOPY_PAIRS
        for (int i = 0; i < 16; i++) buf[d + i] = L(s + i);
        if (16 >= length) return;
        d += 16; s += 16;
        do {
            for (int i = 0; i < 32; i++) buf[d + i] = L(s + i);
            d += 32; s += 32;
        } while (d < e);
#else
        do { for (int i = 0; i < 16; i++) buf[d + i] = L(s + i); d += 16; s += 16; } while (d < e);
#endif
    }
    // ZSTD_overlapCopy8
    void overlap8(uint64_t& d, uint64_t& s, uint64_t offset) {
        if (offset < 8) {
            static const uint32_t dec32[] = {0, 1, 2, 1, 4, 4, 4, 4};
            static const int dec64[] = {8, 8, 8, 7, 8, 9, 10, 11};
            const int sub2 = dec64[offset];
            buf[d] = buf[s]; buf[d + 1] = buf[s + 1]; buf[d + 2] = buf[s + 2]; buf[d + 3] = buf[s + 3];
            s += dec32[offset];
            copy_n(d + 4, s, 4);
            s -= sub2;
        } else {
            copy_n(d, s, 8);
        }
        s += 8;
        d += 8;
    }
    void memmove_buf(uint64_t d, uint64_t s, uint64_t k) {
        std::vector<uint8_t> t(buf.begin() + s, buf.begin() + s + k);
        memcpy(&buf[d], t.data(), k);
    }
    // ZSTD_safecopy (near the buffer end)
    void safecopy_buf(uint64_t d, uint64_t oend_w, uint64_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
        if (length < 8) { while (d < e) buf[d++] = buf[s++]; return; }
        overlap8(d, s, d - s);
        if (e <= oend_w) { wild_buf(d, s, length, true); return; }
        if (d <= oend_w) { wild_buf(d, s, (int64_t)(oend_w - d), true); s += oend_w - d; d = oend_w; }
        while (d < e) buf[d++] = buf[s++];
    }
    void safecopy_lit(uint64_t d, uint64_t oend_w, size_t s, int64_t length) {
        const uint64_t e = d + (uint64_t)length;
        if (length < 8) { while (d < e) buf[d++] = L(s++); return; }
        if (e <= oend_w) { wild_lit(d, s, length); return; }
        if (d <= oend_w) { wild_lit(d, s, (int64_t)(oend_w - d)); s += oend_w - d; d = oend_w; }
        while (d < e) buf[d++] = L(s++);
    }
    // ZSTD_execSequence / ZSTD_execSequenceEnd; prefixStart = 0, the
    // previous segment (extDict) = [0, prevlen) of the same buffer
    uint64_t prevlen = 0;
    void exec_seq(uint64_t ll, uint64_t off, uint64_t ml) {
        const uint64_t o0 = op, oLitEnd = op + ll, oMatchEnd = oLitEnd + ml, oend_w = oend - 32;
        const bool end_path = oMatchEnd > oend_w;
        if (end_path) safecopy_lit(op, oend_w, took, (int64_t)ll);
        else {
            for (int i = 0; i < 16; i++) buf[op + i] = L(took + i);
            if (ll > 16) wild_lit(op + 16, took + 16, (int64_t)ll - 16);
        }
        took += ll;
        uint64_t d = oLitEnd, m = oLitEnd - off, rem = ml;
        if (off > oLitEnd) {  // extDict: the previous segment's place in the buffer
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
        if (end_path) safecopy_buf(d, oend_w, m, (int64_t)rem);
        else if (off >= 16) wild_buf(d, m, (int64_t)rem, false);
        else {
            overlap8(d, m, off);
            if (rem > 8) wild_buf(d, m, (int64_t)rem - 8, true);
        }
        op = oMatchEnd;
        emit(o0, ll + ml);
    }
};

}  // namespace

template <>
struct rp::zs::EagerLits<ExactHostEnv> {
    static constexpr bool value = true;
};
template <>
struct rp::zs::ExactRing<ExactHostEnv> {
    static constexpr bool value = true;
};

extern "C" int zs_host_decode_exact(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* total) {
    static rp::zs::Tabs T;
    ExactHostEnv e;
    e.src = src;
    e.n = n;
    e.T = &T;
    uint64_t t = 0;
    bool unsure = false;
    const int rc = n == 0 ? -1 : rp::zs::payload(e, &T, n, t, unsure);
    *total = rc == 0 ? t : 0;
    if (rc == 0 && t > e.out.size()) return -9;
    if (rc == 0) memcpy(dst, e.out.data(), t < cap ? t : cap);
    return rc;
}

template <>
struct rp::zs::EagerLits<EagerHostEnv> {
    static constexpr bool value = true;
};
template <>
struct rp::zs::EagerSeqs<EagerHostEnv> {
    static constexpr bool value = true;
};

extern "C" int zs_host_decode_eager(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* total) {
    static rp::zs::Tabs T;
    EagerHostEnv e;
    e.src = src;
    e.n = n;
    e.T = &T;
    uint64_t t = 0;
    bool unsure = false;
    const int rc = n == 0 ? -1 : rp::zs::payload(e, &T, n, t, unsure);
    *total = rc == 0 ? t : 0;
    if (rc == 0 && t > e.out.size()) return -9;
    if (rc == 0) memcpy(dst, e.out.data(), t < cap ? t : cap);
    return rc;
}

extern "C" int zs_host_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* total) {
    static rp::zs::Tabs T;
    HostEnv e;
    e.src = src;
    e.n = n;
    uint64_t t = 0;
    bool unsure = false;
    const int rc = n == 0 ? -1 : rp::zs::payload(e, &T, n, t, unsure);
    *total = rc == 0 ? t : 0;
    if (rc == 0 && t > e.out.size()) return -9;  // bookkeeping mismatch
    if (rc == 0) memcpy(dst, e.out.data(), t < cap ? t : cap);
    return rc;
}

extern "C" uint64_t zs_host_xxh64(const uint8_t* p, uint64_t n) { return xxh64(p, n); }
