// rp_gen.cpp — synthetic segment generator behind rpgpu_gen_segment.
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
// snappy_java_compressor.cc:57-74), loaded with dlopen.
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "rpgpu.h"

namespace {

// --- codec libraries ---------------------------------------------------------
struct LZ4FPrefs {  // LZ4F_preferences_t (lz4 1.9.x ABI)
    struct {
        unsigned blockSizeID, blockMode, contentChecksumFlag, frameType;
        unsigned long long contentSize;
        unsigned dictID, blockChecksumFlag;
    } frameInfo;
    int compressionLevel;
    unsigned autoFlush, favorDecSpeed, reserved[3];
};
typedef size_t (*lz4f_bound_t)(size_t, const LZ4FPrefs*);
typedef size_t (*lz4f_compress_t)(void*, size_t, const void*, size_t, const LZ4FPrefs*);
typedef unsigned (*lz4f_iserr_t)(size_t);
typedef int (*snappy_compress_t)(const char*, size_t, char*, size_t*);
typedef size_t (*snappy_bound_t)(size_t);

struct Codecs {
    lz4f_bound_t lz4f_bound = nullptr;
    lz4f_compress_t lz4f_compress = nullptr;
    lz4f_iserr_t lz4f_iserr = nullptr;
    snappy_compress_t snappy_compress = nullptr;
    snappy_bound_t snappy_bound = nullptr;
};

const Codecs& codecs() {
    static Codecs c;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* lz4_names[] = {"liblz4.so.1", "/opt/conda/lib/liblz4.so.1", "/lib/x86_64-linux-gnu/liblz4.so.1"};
        for (const char* n : lz4_names) {
            void* h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (!h) continue;
            c.lz4f_bound = (lz4f_bound_t)dlsym(h, "LZ4F_compressFrameBound");
            c.lz4f_compress = (lz4f_compress_t)dlsym(h, "LZ4F_compressFrame");
            c.lz4f_iserr = (lz4f_iserr_t)dlsym(h, "LZ4F_isError");
            if (c.lz4f_bound && c.lz4f_compress && c.lz4f_iserr) break;
        }
        const char* sn_names[] = {"libsnappy.so.1", "/opt/conda/lib/libsnappy.so.1"};
        for (const char* n : sn_names) {
            void* h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (!h) continue;
            c.snappy_compress = (snappy_compress_t)dlsym(h, "snappy_compress");
            c.snappy_bound = (snappy_bound_t)dlsym(h, "snappy_max_compressed_length");
            if (c.snappy_compress && c.snappy_bound) break;
        }
    });
    return c;
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
int encode_records(Rng& rng, std::vector<uint8_t>& out, size_t target, const rpgpu_gen_spec* sp, int kind, uint64_t& jc) {
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

bool compress_payload(int codec, const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
    const Codecs& c = codecs();
    if (codec == RPGPU_CODEC_LZ4) {
        if (!c.lz4f_compress) return false;
        LZ4FPrefs p;
        std::memset(&p, 0, sizeof p);
        p.compressionLevel = 1;
        p.frameInfo.blockMode = 1;  // LZ4F_blockIndependent
        p.frameInfo.contentSize = in.size();
        p.frameInfo.blockSizeID = 4;  // 64 KiB blocks, as Kafka producers use
        const size_t bound = c.lz4f_bound(in.size(), &p);
        out.resize(bound);
        const size_t n = c.lz4f_compress(out.data(), bound, in.data(), in.size(), &p);
        if (c.lz4f_iserr(n)) return false;
        out.resize(n);
        return true;
    }
    if (codec == RPGPU_CODEC_SNAPPY) {
        if (!c.snappy_compress) return false;
        static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        out.assign(magic, magic + 8);
        uint8_t v[8];
        wr_le(v, 1, 4);
        wr_le(v + 4, 1, 4);
        out.insert(out.end(), v, v + 8);
        const size_t chunk = 32 << 10;
        std::vector<char> tmp(c.snappy_bound(chunk));
        for (size_t i = 0; i < in.size() || i == 0; i += chunk) {
            const size_t len = std::min(chunk, in.size() - i);
            size_t cl = tmp.size();
            if (c.snappy_compress((const char*)in.data() + i, len, tmp.data(), &cl) != 0) return false;
            uint8_t be[4];
            wr_be(be, (uint32_t)cl, 4);
            out.insert(out.end(), be, be + 4);
            out.insert(out.end(), tmp.data(), tmp.data() + cl);
            if (in.empty()) break;
        }
        return true;
    }
    return false;
}

}  // namespace

extern "C" int64_t rpgpu_gen_segment(const rpgpu_gen_spec* sp, uint32_t segment_index, uint8_t* out) {
    if (!sp || !out) return RPGPU_E_INVALID;
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
    for (;;) {
        uint32_t target = sp->batch_bytes;
        if (!target) {
            // log-uniform in [min, max]
            const double u = (double)(rng.next() >> 11) / 9007199254740992.0;
            target = (uint32_t)(minb * std::exp(u * std::log((double)maxb / (double)minb)));
            if (target < minb) target = minb;
        }
        if (target < RPGPU_HEADER_SIZE + 16) target = RPGPU_HEADER_SIZE + 16;
        // codec choice
        int codec = 0;
        if (sp->codec_mix & ~1u) {
            uint32_t allowed[8];
            int na = 0;
            for (int c = 0; c < 5; c++)
                if (sp->codec_mix & (1u << c)) allowed[na++] = (uint32_t)c;
            codec = na ? (int)allowed[rng.below((uint32_t)na)] : 0;
            if (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD) codec = 0;
        }
        const int kind = codec ? (int)rng.below(3) : K_ALNUM;
        // uncompressed: size_bytes == target exactly; compressed: the
        // decoded payload is target - 61 bytes
        const uint64_t room = len - pos;
        if (room < (uint64_t)RPGPU_HEADER_SIZE + 32) break;
        size_t body = target - RPGPU_HEADER_SIZE;
        if (!codec && body + RPGPU_HEADER_SIZE > room) break;
        const int nrec = encode_records(rng, recs, body, sp, kind, jc);
        if (nrec <= 0) break;
        const std::vector<uint8_t>* payload = &recs;
        if (codec) {
            if (!compress_payload(codec, recs, comp)) { codec = 0; }
            else payload = &comp;
        }
        const uint64_t size = RPGPU_HEADER_SIZE + payload->size();
        if (size > room) break;
        uint8_t* h = out + pos;
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
        std::memcpy(h + RPGPU_HEADER_SIZE, payload->data(), payload->size());
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
        uint32_t crc = rpgpu_crc32c_extend(0, be, 40);
        crc = rpgpu_crc32c_extend(crc, h + RPGPU_HEADER_SIZE, payload->size());
        wr_le(h + 17, crc, 4);
        wr_le(h + 0, rpgpu_crc32c_extend(0, h + 4, 57), 4);
        // fault injection (config 5 corruption injector)
        const uint32_t roll = (uint32_t)(rng.next() % 1000000u);
        if (roll < sp->corrupt_ppm_payload && payload->size() > 0) {
            const uint64_t bit = rng.next() % (payload->size() * 8);
            h[RPGPU_HEADER_SIZE + bit / 8] ^= (uint8_t)(1u << (bit % 8));
        } else if (roll < sp->corrupt_ppm_payload + sp->corrupt_ppm_header) {
            const uint64_t bit = rng.next() % (61 * 8);
            h[bit / 8] ^= (uint8_t)(1u << (bit % 8));
        } else if (roll < sp->corrupt_ppm_payload + sp->corrupt_ppm_header + sp->corrupt_ppm_zero) {
            std::memset(h, 0, RPGPU_HEADER_SIZE);
        }
        pos += size;
        offset += nrec;
        ts += nrec;
        nb++;
    }
    return nb;
}
