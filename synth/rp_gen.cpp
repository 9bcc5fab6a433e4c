// rp_gen.cpp — synthetic segment generator (synth/rpgen.h; test and bench
// data, never linked into the engine).
//
// Mirrors the reference's test batch recipe (storage/tests/utils/
// random_batch.cc:50-154: records with ts/offset deltas = index, two headers
// of <=10-byte key/value, alnum payloads from random/generators.h:60-70 whose
// charset excludes its last character) but seeded with mt19937_64 so every
// run reproduces.  Batches are written in the on-disk layout
// (storage/segment_appender_utils.cc:28-54) with crc / header_crc computed as
// model/record_utils.cc:34-91 does.  Compressed batches go through the
// reference's own codec libraries (liblz4 LZ4F with blockIndependent +
// contentSize like lz4_frame_compressor.cc:69-113; snappy-java framing like
// snappy_java_compressor.cc:57-74; raw snappy like snappy_standard_compressor;
// gzip like gzip_compressor.cc deflateInit2(15 + 16); zstd with the content
// size like stream_zstd.cc), loaded with dlopen.
#include <dlfcn.h>
#include <nmmintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include <lz4frame.h>
#include <snappy-c.h>
#include <zlib.h>
#include <zstd.h>

#include "rpgen.h"

constexpr uint32_t kHeaderSize = 61;  // model::packed_record_batch_header_size (model/record.h:473-487)

namespace {

// --- codec libraries (the reference's: liblz4, libsnappy, zlib, libzstd) ----
bool lz4f_frame(const std::vector<uint8_t>& in, std::vector<uint8_t>& out, bool linked, bool cc, bool bc) {
    LZ4F_preferences_t p;
    std::memset(&p, 0, sizeof p);
    p.compressionLevel = 1;
    p.frameInfo.blockMode = linked ? LZ4F_blockLinked : LZ4F_blockIndependent;
    p.frameInfo.contentSize = in.size();
    p.frameInfo.blockSizeID = LZ4F_max64KB;  // 64 KiB blocks, as Kafka producers use
    p.frameInfo.contentChecksumFlag = cc ? LZ4F_contentChecksumEnabled : LZ4F_noContentChecksum;
    p.frameInfo.blockChecksumFlag = bc ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
    const size_t bound = LZ4F_compressFrameBound(in.size(), &p);
    out.resize(bound);
    const size_t n = LZ4F_compressFrame(out.data(), bound, in.data(), in.size(), &p);
    if (LZ4F_isError(n)) return false;
    out.resize(n);
    return true;
}

bool snappy_block(const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
    size_t cl = snappy_max_compressed_length(n);
    out.resize(cl);
    if (snappy_compress((const char*)in, n, (char*)out.data(), &cl) != SNAPPY_OK) return false;
    out.resize(cl);
    return true;
}

// gzip_compressor::compress (compression/internal/gzip_compressor.cc): deflateInit2
// (Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY)
bool gzip_member(const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    out.resize(deflateBound(&zs, in.size()) + 64);
    zs.next_in = const_cast<uint8_t*>(in.data());
    zs.avail_in = (uInt)in.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    const int r = deflate(&zs, Z_FINISH);
    out.resize(zs.total_out);
    deflateEnd(&zs);
    return r == Z_STREAM_END;
}

// stream_zstd::do_compress (compression/stream_zstd.cc): content size always set
bool zstd_frame(const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
    out.resize(ZSTD_compressBound(in.size()));
    const size_t n = ZSTD_compress(out.data(), out.size(), in.data(), in.size(), 3);
    if (ZSTD_isError(n)) return false;
    out.resize(n);
    return true;
}

// --- encoding helpers ---------------------------------------------------------
void put_vint(std::vector<uint8_t>& o, int64_t x) {
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    while (v >= 0x80) { o.push_back((uint8_t)(v | 0x80)); v >>= 7; }
    o.push_back((uint8_t)v);
}
size_t vint_size(int64_t x) {
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; n++; }
    return n;
}
void wr_le(uint8_t* p, uint64_t v, int n) { for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i)); }
void wr_be(uint8_t* p, uint64_t v, int n) { for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * (n - 1 - i))); }

// 61 alnum characters: random/generators.h uses chars.size() - 2 as the max
// index, so its last character ('9') is never produced.
const char kChars[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";

struct Rng {
    std::mt19937_64 g;
    uint64_t buf = 0;
    int left = 0;
    explicit Rng(uint64_t seed) : g(seed) {}
    uint64_t next() { return g(); }
    uint32_t below(uint32_t n) { return (uint32_t)(g() % n); }
    char alnum() {
        for (;;) {
            if (left == 0) { buf = g(); left = 10; }
            uint32_t v = buf & 63;
            buf >>= 6;
            left--;
            if (v < 61) return kChars[v];
        }
    }
    void fill_alnum(uint8_t* p, size_t n) { for (size_t i = 0; i < n; i++) p[i] = (uint8_t)alnum(); }
};

struct RecSpec {
    int32_t klen, vlen;
    int32_t hk[2], hv[2];
};

size_t rec_body_size(int idx, const RecSpec& r, int nh) {
    size_t s = 1 + vint_size(idx) + vint_size(idx) + vint_size(r.klen) + (size_t)r.klen + vint_size(r.vlen) + (size_t)r.vlen +
               vint_size(nh);
    for (int h = 0; h < nh; h++) s += vint_size(r.hk[h]) + (size_t)r.hk[h] + vint_size(r.hv[h]) + (size_t)r.hv[h];
    return s;
}
size_t rec_total(int idx, const RecSpec& r, int nh) {
    size_t b = rec_body_size(idx, r, nh);
    return vint_size((int64_t)b) + b;
}

// payload kinds for compressible batches (random, alnum text, repetitive json)
enum Kind { K_ALNUM = 0, K_RANDOM = 1, K_JSON = 2 };

void fill_kind(Rng& rng, uint8_t* p, size_t n, int kind, uint64_t& json_ctr) {
    if (kind == K_RANDOM) {
        for (size_t i = 0; i < n; i += 8) {
            uint64_t v = rng.next();
            for (size_t k = 0; k < 8 && i + k < n; k++) p[i + k] = (uint8_t)(v >> (8 * k));
        }
    } else if (kind == K_JSON) {
        static const char* keys[] = {"\"user\":", "\"event\":\"click\",", "\"ts\":", "\"page\":\"/home\",", "\"ok\":true,"};
        size_t i = 0;
        while (i < n) {
            char tmp[64];
            int k = snprintf(tmp, sizeof tmp, "{%s%llu,%s%s%llu}", keys[json_ctr % 5], (unsigned long long)(json_ctr % 97),
                             keys[(json_ctr + 1) % 5], keys[2], (unsigned long long)(1600000000000ull + json_ctr));
            json_ctr++;
            for (int q = 0; q < k && i < n; q++) p[i++] = (uint8_t)tmp[q];
        }
    } else {
        rng.fill_alnum(p, n);
    }
}

// Encode records into `out` so that the encoded size is exactly `target`
// (when target >= the minimal record size).  Returns the record count.
int encode_records(Rng& rng, std::vector<uint8_t>& out, size_t target, const rpgen_spec* sp, int kind, uint64_t& jc) {
    const int nh = (int)sp->headers_per_record;
    const int32_t vbase = sp->value_bytes ? (int32_t)sp->value_bytes : 1024;
    const int32_t kbase = sp->key_bytes ? (int32_t)sp->key_bytes : 16;
    int idx = 0;
    size_t used = 0;
    std::vector<RecSpec> specs;
    for (;;) {
        RecSpec r;
        r.klen = kbase;
        r.vlen = vbase / 2 + (int32_t)rng.below((uint32_t)vbase + 1);
        for (int h = 0; h < 2; h++) { r.hk[h] = 1 + (int32_t)rng.below(10); r.hv[h] = 1 + (int32_t)rng.below(10); }
        const size_t full = rec_total(idx, r, nh);
        const size_t left = target - used;
        // if another full record plus a minimal one would not fit, size this
        // one as the last record and pad its value to hit the target exactly
        RecSpec minr = r;
        minr.vlen = 0;
        if (left < full + rec_total(idx + 1, minr, nh) + 64) {
            // last record: search key/header-value padding and the value
            // length for an exact fit (varint widths make some totals
            // unreachable with the value alone)
            bool found = false;
            RecSpec last = r;
            for (int dk = 0; dk < 4 && !found; dk++) {
                for (int dh = 0; dh < 10 && !found; dh++) {
                    RecSpec t = r;
                    t.klen = r.klen + dk;
                    if (nh > 0) t.hv[0] = r.hv[0] + dh;
                    t.vlen = 0;
                    const size_t base = rec_total(idx, t, nh);
                    if (base > left) continue;
                    int32_t v = (int32_t)(left - base);
                    while (v > 0 && rec_total(idx, RecSpec{t.klen, v, {t.hk[0], t.hk[1]}, {t.hv[0], t.hv[1]}}, nh) > left) v--;
                    t.vlen = v;
                    if (rec_total(idx, t, nh) == left) { last = t; found = true; }
                }
            }
            if (!found) break;
            specs.push_back(last);
            used += left;
            idx++;
            break;
        }
        specs.push_back(r);
        used += full;
        idx++;
    }
    out.clear();
    out.reserve(target);
    for (int i = 0; i < (int)specs.size(); i++) {
        const RecSpec& r = specs[i];
        put_vint(out, (int64_t)rec_body_size(i, r, nh));
        out.push_back(0);  // attributes
        put_vint(out, i);  // timestamp delta
        put_vint(out, i);  // offset delta
        put_vint(out, r.klen);
        size_t o = out.size();
        out.resize(o + (size_t)r.klen);
        rng.fill_alnum(out.data() + o, (size_t)r.klen);
        put_vint(out, r.vlen);
        o = out.size();
        out.resize(o + (size_t)r.vlen);
        fill_kind(rng, out.data() + o, (size_t)r.vlen, kind, jc);
        put_vint(out, nh);
        for (int h = 0; h < nh; h++) {
            put_vint(out, r.hk[h]);
            o = out.size();
            out.resize(o + (size_t)r.hk[h]);
            rng.fill_alnum(out.data() + o, (size_t)r.hk[h]);
            put_vint(out, r.hv[h]);
            o = out.size();
            out.resize(o + (size_t)r.hv[h]);
            rng.fill_alnum(out.data() + o, (size_t)r.hv[h]);
        }
    }
    return (int)specs.size();
}

// slot -> payload bytes under the batch's codec attribute
bool compress_payload(int slot, const std::vector<uint8_t>& in, std::vector<uint8_t>& out, bool linked, bool cc,
                      bool bc) {
    switch (slot) {
    case RPGEN_LZ4:
        return lz4f_frame(in, out, linked, cc, bc);
    case RPGEN_SNAPPY_JAVA: {
        static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        out.assign(magic, magic + 8);
        uint8_t v[8];
        wr_le(v, 1, 4);  // version, min_version: native little endian (snappy_java_compressor.cc:86-88)
        wr_le(v + 4, 1, 4);
        out.insert(out.end(), v, v + 8);
        const size_t chunk = 32 << 10;
        std::vector<uint8_t> tmp;
        for (size_t i = 0; i < in.size() || i == 0; i += chunk) {
            const size_t len = std::min(chunk, in.size() - i);
            if (!snappy_block(in.data() + i, len, tmp)) return false;
            uint8_t be[4];
            wr_be(be, (uint32_t)tmp.size(), 4);
            out.insert(out.end(), be, be + 4);
            out.insert(out.end(), tmp.begin(), tmp.end());
            if (in.empty()) break;
        }
        return true;
    }
    case RPGEN_SNAPPY_RAW:
        return snappy_block(in.data(), in.size(), out);
    case RPGEN_GZIP:
        return gzip_member(in, out);
    case RPGEN_ZSTD:
        return zstd_frame(in, out);
    }
    return false;
}

int slot_codec(int slot) { return slot == RPGEN_SNAPPY_RAW ? RPGEN_SNAPPY_JAVA : slot; }

}  // namespace

extern "C" __attribute__((target("sse4.2"))) uint32_t rpgen_crc32c(uint32_t crc, const uint8_t* p, uint64_t n) {
    uint64_t l = crc ^ 0xFFFFFFFFu;
    while (n && ((uintptr_t)p & 7)) { l = _mm_crc32_u8((uint32_t)l, *p++); n--; }
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        l = _mm_crc32_u64(l, v);
        p += 8;
        n -= 8;
    }
    uint32_t s = (uint32_t)l;
    while (n) { s = _mm_crc32_u8(s, *p++); n--; }
    return s ^ 0xFFFFFFFFu;
}

extern "C" int64_t rpgen_segment(const rpgen_spec* sp, uint32_t segment_index, uint8_t* out) {
    if (!sp || !out) return -1;
    Rng rng(sp->seed * 0x9E3779B97F4A7C15ull + (uint64_t)segment_index * 0xD1B54A32D192ED03ull + 1);
    const uint64_t len = sp->segment_bytes;
    std::memset(out, 0, len);
    uint64_t pos = 0;
    int64_t nb = 0;
    int64_t offset = sp->base_offset + (int64_t)segment_index * 100000000ll;
    int64_t ts = 1600000000000ll + (int64_t)segment_index * 1000000ll;
    uint64_t jc = 0;
    std::vector<uint8_t> recs, comp;
    const uint32_t minb = sp->min_batch_bytes ? sp->min_batch_bytes : 200;
    const uint32_t maxb = sp->max_batch_bytes ? sp->max_batch_bytes : (1u << 20);
    uint64_t wsum = 0;
    for (int s = 0; s < RPGEN_SLOTS; s++) wsum += sp->codec_weights[s];
    const bool mixed = wsum > sp->codec_weights[RPGEN_NONE];
    for (;;) {
        uint32_t target = sp->batch_bytes;
        if (!target) {
            // log-uniform (or uniform) in [min, max]
            const double u = (double)(rng.next() >> 11) / 9007199254740992.0;
            target = sp->size_uniform ? (uint32_t)(minb + u * (double)(maxb - minb))
                                      : (uint32_t)(minb * std::exp(u * std::log((double)maxb / (double)minb)));
            if (target < minb) target = minb;
        }
        if (target < kHeaderSize + 16) target = kHeaderSize + 16;
        int slot = RPGEN_NONE;
        if (mixed) {
            uint64_t r = rng.next() % wsum;
            for (slot = 0; slot < RPGEN_SLOTS - 1 && r >= sp->codec_weights[slot]; slot++) r -= sp->codec_weights[slot];
        }
        const int kind = slot ? (int)rng.below(3) : K_ALNUM;
        bool linked = false, cc = false, bc = false;
        if (slot == RPGEN_LZ4) {
            linked = rng.below(1000000) < sp->lz4_linked_ppm;
            cc = rng.below(1000000) < sp->lz4_content_checksum_ppm;
            bc = rng.below(1000000) < sp->lz4_block_checksum_ppm;
        }
        // uncompressed: size_bytes == target exactly; compressed: the
        // decoded payload is target - 61 bytes
        const uint64_t room = len - pos;
        if (room < (uint64_t)kHeaderSize + 32) break;
        const size_t body = target - kHeaderSize;
        if (!slot && body + kHeaderSize > room && !sp->truncate_tail) break;
        const int nrec = encode_records(rng, recs, body, sp, kind, jc);
        if (nrec <= 0) break;
        const std::vector<uint8_t>* payload = &recs;
        if (slot) {
            if (!compress_payload(slot, recs, comp, linked, cc, bc)) slot = RPGEN_NONE;
            else payload = &comp;
        }
        const int codec = slot_codec(slot);
        const uint64_t size = kHeaderSize + payload->size();
        if (size > room && !sp->truncate_tail) break;
        // a batch that does not fit is built in scratch and cut at the end
        std::vector<uint8_t> scratch;
        uint8_t* h = out + pos;
        if (size > room) {
            scratch.resize(size);
            h = scratch.data();
        }
        // header fields (header_crc and crc filled below)
        wr_le(h + 4, (uint32_t)size, 4);
        wr_le(h + 8, (uint64_t)offset, 8);
        h[16] = 1;  // raft_data
        wr_le(h + 21, (uint16_t)codec, 2);
        wr_le(h + 23, (uint32_t)(nrec - 1), 4);
        wr_le(h + 27, (uint64_t)ts, 8);
        wr_le(h + 35, (uint64_t)(ts + nrec - 1), 8);
        wr_le(h + 43, (uint64_t)-1ll, 8);
        wr_le(h + 51, (uint16_t)0xFFFF, 2);
        wr_le(h + 53, (uint32_t)0xFFFFFFFFu, 4);
        wr_le(h + 57, (uint32_t)nrec, 4);
        std::memcpy(h + kHeaderSize, payload->data(), payload->size());
        // crc: BE(attrs..record_count) ++ payload (model/record_utils.cc:68-91)
        uint8_t be[40];
        wr_be(be + 0, (uint16_t)codec, 2);
        wr_be(be + 2, (uint32_t)(nrec - 1), 4);
        wr_be(be + 6, (uint64_t)ts, 8);
        wr_be(be + 14, (uint64_t)(ts + nrec - 1), 8);
        wr_be(be + 22, (uint64_t)-1ll, 8);
        wr_be(be + 30, (uint16_t)0xFFFF, 2);
        wr_be(be + 32, (uint32_t)0xFFFFFFFFu, 4);
        wr_be(be + 36, (uint32_t)nrec, 4);
        uint32_t crc = rpgen_crc32c(0, be, 40);
        crc = rpgen_crc32c(crc, h + kHeaderSize, payload->size());
        wr_le(h + 17, crc, 4);
        wr_le(h + 0, rpgen_crc32c(0, h + 4, 57), 4);
        if (size > room) {
            std::memcpy(out + pos, h, room);  // truncated tail: header valid, payload cut
            break;
        }
        // fault injection (config 5 corruption injector)
        const uint32_t roll = (uint32_t)(rng.next() % 1000000u);
        if (roll < sp->corrupt_ppm_payload && payload->size() > 0) {
            const uint64_t bit = rng.next() % (payload->size() * 8);
            h[kHeaderSize + bit / 8] ^= (uint8_t)(1u << (bit % 8));
        } else if (roll < sp->corrupt_ppm_payload + sp->corrupt_ppm_header) {
            const uint64_t bit = rng.next() % (61 * 8);
            h[bit / 8] ^= (uint8_t)(1u << (bit % 8));
        } else if (roll < sp->corrupt_ppm_payload + sp->corrupt_ppm_header + sp->corrupt_ppm_zero) {
            std::memset(h, 0, kHeaderSize);
        }
        pos += size;
        offset += nrec;
        ts += nrec;
        nb++;
    }
    return nb;
}
