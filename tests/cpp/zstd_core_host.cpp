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

}  // namespace

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
