/*
 * rpgpu_redpanda.h — the reference's hot-path surfaces, re-declared in C++17
 * over the C-ABI in rpgpu.h, so a caller of Redpanda's batch path swaps the
 * include and keeps its code:
 *
 *   crc::crc32c                           hashing/crc32c.h:19-40
 *   model::record_batch_attributes        model/record.h:255-351
 *   model::record_batch_header            model/record.h:354-417
 *   model::internal_header_only_crc,
 *   model::crc_record_batch_header,
 *   model::crc_record_batch               model/record_utils.h:23-35 (.cc:34-91)
 *   storage::parser_errc                  storage/parser_errc.h:18-25
 *   storage::batch_consumer               storage/parser.h:32-87
 *   storage::continuous_batch_parser      storage/parser.h:94-136 (parser.cc:96-254)
 *   storage::log_replayer                 storage/log_replayer.h/.cc:27-114
 *   compression::compressor::uncompress   compression/compression.h:21-24
 *   kafka::batch_reader,
 *   kafka::kafka_batch_adapter            kafka/protocol/batch_reader.h, batch_reader.cc:50-156,
 *                                         kafka/protocol/kafka_batch_adapter.h:60-76 (.cc:126-188)
 *
 * Differences forced by leaving Seastar: futures become synchronous calls,
 * ss::input_stream becomes a byte span of a whole segment, iobuf a
 * contiguous byte buffer.  The parser validates the whole segment on the GPU
 * through rpgpu_validate_host (pinned, double-buffered host -> device
 * staging in the context), then replays the per-batch verdicts into the consumer
 * in chain order, so accept / skip / stop decisions and byte accounting
 * follow continuous_batch_parser::consume exactly.  No exception crosses the
 * C-ABI; these wrappers rethrow where the reference throws.
 */
#ifndef RPGPU_REDPANDA_H_
#define RPGPU_REDPANDA_H_

#include <cstddef>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <memory>
#include <algorithm>
#include <optional>
#include <ostream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "rpgpu.h"

namespace rpgpu {

// Contiguous byte buffer standing in for iobuf (bytes/iobuf.h).
class iobuf {
public:
    iobuf() = default;
    iobuf(const uint8_t* p, size_t n) : _b(p, p + n) {}
    explicit iobuf(std::vector<uint8_t> b) : _b(std::move(b)) {}
    size_t size_bytes() const { return _b.size(); }
    bool empty() const { return _b.empty(); }
    const uint8_t* data() const { return _b.data(); }
    uint8_t* data() { return _b.data(); }
    const std::vector<uint8_t>& bytes() const { return _b; }

private:
    std::vector<uint8_t> _b;
};

// One rpgpu context (HIP stream + device scratch) on one device; one per
// host thread / shard, as the reference's shard-per-core ownership requires.
class engine {
public:
    explicit engine(int device = 0) {
        const int rc = rpgpu_create(device, &_ctx);
        if (rc != RPGPU_OK) throw std::runtime_error(std::string("rpgpu_create: ") + rpgpu_strerror(rc));
    }
    engine(const engine&) = delete;
    engine& operator=(const engine&) = delete;
    ~engine() {
        if (_ctx) rpgpu_destroy(_ctx);
    }
    rpgpu_ctx* ctx() const { return _ctx; }
    void check(int rc, const char* what) const {
        if (rc != RPGPU_OK)
            throw std::runtime_error(std::string(what) + ": " + rpgpu_strerror(rc) + " (" + rpgpu_last_error(_ctx) + ")");
    }

    // The engine used by the surfaces below when none is passed explicitly.
    static engine& local() {
        thread_local engine e(0);
        return e;
    }

private:
    rpgpu_ctx* _ctx = nullptr;
};

// RAII device buffer
class dev_buffer {
public:
    dev_buffer(engine& e, size_t bytes) : _e(e) { _e.check(rpgpu_dev_alloc(_e.ctx(), bytes, &_p), "rpgpu_dev_alloc"); }
    dev_buffer(const dev_buffer&) = delete;
    dev_buffer& operator=(const dev_buffer&) = delete;
    ~dev_buffer() {
        if (_p) rpgpu_dev_free(_e.ctx(), _p);
    }
    void* get() const { return _p; }

private:
    engine& _e;
    void* _p = nullptr;
};

// XXH64 (seed 0 in the reference's incremental_xxhash64, hashing/xx.h:36-71);
// the checksum of the on-disk segment index (storage/index_state.cc:27-48).
inline uint64_t xxh64(const uint8_t* p, size_t n, uint64_t seed = 0) {
    constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                       P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
    auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
    auto rd64 = [](const uint8_t* q) { uint64_t v; std::memcpy(&v, q, 8); return v; };
    auto rd32 = [](const uint8_t* q) { uint32_t v; std::memcpy(&v, q, 4); return v; };
    auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
    auto merge = [&](uint64_t acc, uint64_t v) { return (acc ^ round(0, v)) * P1 + P4; };
    const uint8_t* const end = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; p + 32 <= end; p += 32) {
            v1 = round(v1, rd64(p));
            v2 = round(v2, rd64(p + 8));
            v3 = round(v3, rd64(p + 16));
            v4 = round(v4, rd64(p + 24));
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = merge(merge(merge(merge(h, v1), v2), v3), v4);
    } else {
        h = seed + P5;
    }
    h += (uint64_t)n;
    for (; p + 8 <= end; p += 8) h = rotl(h ^ round(0, rd64(p)), 27) * P1 + P4;
    if (p + 4 <= end) {
        h = rotl(h ^ ((uint64_t)rd32(p) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; p++) h = rotl(h ^ ((uint64_t)*p * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

}  // namespace rpgpu

// ---------------------------------------------------------------------------
// crc::crc32c — hashing/crc32c.h:19-40 (google crc32c::Extend semantics)
// ---------------------------------------------------------------------------
namespace crc {
class crc32c {
public:
    template <typename T, typename = std::enable_if_t<std::is_integral_v<T>, T>>
    void extend(T num) noexcept {
        extend(reinterpret_cast<const uint8_t*>(&num), sizeof(T));
    }
    void extend(const uint8_t* data, size_t size) { _crc = rpgpu_crc32c_extend(_crc, data, size); }
    void extend(const char* data, size_t size) { extend(reinterpret_cast<const uint8_t*>(data), size); }
    uint32_t value() const { return _crc; }

private:
    uint32_t _crc = 0;
};
}  // namespace crc

// ---------------------------------------------------------------------------
// model — record batch types and CRC helpers
// ---------------------------------------------------------------------------
namespace model {

// model/compression.h:35-48
enum class compression : uint8_t { none = 0, gzip = 1, snappy = 2, lz4 = 3, zstd = 4 };

// model/record.h:255-351
class record_batch_attributes final {
public:
    static constexpr uint16_t compression_mask = 0x7;
    static constexpr uint16_t timestamp_type_mask = 0x8;
    static constexpr uint16_t transactional_mask = 0x10;
    static constexpr uint16_t control_mask = 0x20;
    using type = int16_t;

    record_batch_attributes() noexcept = default;
    explicit record_batch_attributes(type v) noexcept : _a((uint16_t)v) {}
    type value() const { return (type)_a; }
    bool is_control() const { return _a & control_mask; }
    bool is_transactional() const { return _a & transactional_mask; }
    bool is_valid_compression() const { return (_a & compression_mask) <= 4; }
    // throws for codec values 5..7, as the reference does
    model::compression compression() const {
        const uint16_t v = _a & compression_mask;
        if (v > 4) throw std::runtime_error("Unknown compression value: " + std::to_string(v));
        return (model::compression)v;
    }
    void remove_compression() { _a &= (uint16_t)~compression_mask; }
    record_batch_attributes& operator|=(model::compression c) {
        _a |= (uint16_t)((uint16_t)c & compression_mask);
        return *this;
    }
    bool operator==(const record_batch_attributes& o) const { return _a == o._a; }
    bool operator!=(const record_batch_attributes& o) const { return _a != o._a; }

private:
    uint16_t _a = 0;
};

// model/record.h:473-487 (the comment there says 57; the fields sum to 61)
constexpr size_t packed_record_batch_header_size = RPGPU_HEADER_SIZE;

// model/record.h:354-417 (context fields dropped: not serialized)
struct record_batch_header {
    uint32_t header_crc{0};
    int32_t size_bytes{0};
    int64_t base_offset{0};
    int8_t type{0};
    int32_t crc{0};
    record_batch_attributes attrs;
    int32_t last_offset_delta{0};
    int64_t first_timestamp{0};
    int64_t max_timestamp{0};
    int64_t producer_id{0};
    int16_t producer_epoch{0};
    int32_t base_sequence{0};
    int32_t record_count{0};

    int64_t last_offset() const { return base_offset + last_offset_delta; }
    bool operator==(const record_batch_header& o) const {
        return size_bytes == o.size_bytes && base_offset == o.base_offset && crc == o.crc && attrs == o.attrs &&
               last_offset_delta == o.last_offset_delta && first_timestamp == o.first_timestamp &&
               max_timestamp == o.max_timestamp && record_count == o.record_count;
    }
    bool operator!=(const record_batch_header& o) const { return !(*this == o); }

    // from an engine verdict (the fields storage::header_from_iobuf decodes)
    static record_batch_header from(const rpgpu_batch_result& r) {
        record_batch_header h;
        h.header_crc = r.header_crc;
        h.size_bytes = r.size_bytes;
        h.base_offset = r.base_offset;
        h.type = r.type;
        h.crc = (int32_t)r.crc;
        h.attrs = record_batch_attributes(r.attrs);
        h.last_offset_delta = r.last_offset_delta;
        h.first_timestamp = r.first_timestamp;
        h.max_timestamp = r.max_timestamp;
        h.producer_id = r.producer_id;
        h.producer_epoch = r.producer_epoch;
        h.base_sequence = r.base_sequence;
        h.record_count = r.record_count;
        return h;
    }
};

namespace detail {
template <typename T>
inline void put_be(uint8_t*& p, T v) {
    using U = std::make_unsigned_t<T>;
    U u = (U)v;
    for (int i = (int)sizeof(T) - 1; i >= 0; i--) *p++ = (uint8_t)(u >> (8 * i));
}
}  // namespace detail

// model/record_utils.cc:34-55: fields hashed in native (little-endian) order
inline uint32_t internal_header_only_crc(const record_batch_header& h) {
    crc::crc32c c;
    c.extend(h.size_bytes);
    c.extend(h.base_offset);
    c.extend(h.type);
    c.extend(h.crc);
    c.extend(h.attrs.value());
    c.extend(h.last_offset_delta);
    c.extend(h.first_timestamp);
    c.extend(h.max_timestamp);
    c.extend(h.producer_id);
    c.extend(h.producer_epoch);
    c.extend(h.base_sequence);
    c.extend(h.record_count);
    return c.value();
}

// model/record_utils.cc:68-80: the Kafka crc prefix, big-endian
inline void crc_record_batch_header(crc::crc32c& c, const record_batch_header& h) {
    uint8_t b[RPGPU_CRC_PREFIX_SIZE];
    uint8_t* p = b;
    detail::put_be(p, h.attrs.value());
    detail::put_be(p, h.last_offset_delta);
    detail::put_be(p, h.first_timestamp);
    detail::put_be(p, h.max_timestamp);
    detail::put_be(p, h.producer_id);
    detail::put_be(p, h.producer_epoch);
    detail::put_be(p, h.base_sequence);
    detail::put_be(p, h.record_count);
    c.extend(b, sizeof b);
}

// model/record_utils.cc:82-91
inline int32_t crc_record_batch(const record_batch_header& h, const rpgpu::iobuf& records) {
    crc::crc32c c;
    crc_record_batch_header(c, h);
    c.extend(records.data(), records.size_bytes());
    return (int32_t)c.value();
}

}  // namespace model

// ---------------------------------------------------------------------------
// compression::compressor::uncompress — compression/compression.h:21-24
// (lz4 and snappy decoded on the GPU, gzip and zstd by the reference's loops
// over zlib / libzstd on the host; throws std::runtime_error where the
// reference throws, std::logic_error only when zlib / libzstd is absent)
// ---------------------------------------------------------------------------
namespace compression {
using type = model::compression;
struct compressor {
    static rpgpu::iobuf uncompress(const rpgpu::iobuf& in, type t, rpgpu::engine& e = rpgpu::engine::local()) {
        // the frame's planned size (LZ4F block sizes / content size, snappy
        // length varints), as the batch pipeline reserves it; gzip / zstd
        // (no plan) start at 4x and grow on RPGPU_E_OVERFLOW to the size the
        // decoder reports
        const uint64_t plan = rpgpu_uncompress_bound((int)t, in.data(), in.size_bytes());
        size_t cap = plan ? (size_t)plan : in.size_bytes() * 4 + 64, got = 0;
        for (;;) {
            std::vector<uint8_t> out(cap);
            const int rc = rpgpu_uncompress(e.ctx(), (int)t, in.data(), in.size_bytes(), out.data(), cap, &got);
            if (rc == RPGPU_OK) {
                out.resize(got);
                return rpgpu::iobuf(std::move(out));
            }
            if (rc == RPGPU_E_OVERFLOW) {
                cap = got > cap ? got : cap * 2;
                continue;
            }
            if (rc == RPGPU_E_UNSUPPORTED) throw std::logic_error(rpgpu_last_error(e.ctx()));
            throw std::runtime_error(rpgpu_last_error(e.ctx()));
        }
    }
    // compression/compression.cc:17-33 (lz4: lz4_frame_compressor.cc:72-113,
    // snappy: snappy_java_compressor.cc:58-75) on the device, byte for byte
    // what liblz4 / libsnappy give through those wrappers.  `frag`: the
    // size of the input iobuf's fragments (snappy-java writes one chunk per
    // fragment; 0 = one contiguous fragment).  gzip / zstd run on the host,
    // the reference's loops over zlib / libzstd.
    static rpgpu::iobuf compress(const rpgpu::iobuf& in, type t, rpgpu::engine& e = rpgpu::engine::local(),
                                 size_t frag = 0) {
        if (t == type::none) throw std::runtime_error("compressor: nothing to compress for 'none'");
        const int codec = (int)t;
        size_t cap = rpgpu_compress_bound(codec, in.size_bytes(), frag), got = 0;
        std::vector<uint8_t> out(cap ? cap : 1);
        const void* src = in.data();
        const size_t n = in.size_bytes();
        void* dst = out.data();
        int st = 0;
        e.check(rpgpu_compress_batch(e.ctx(), 1, &codec, &src, &n, &frag, &dst, &cap, &got, &st),
                "rpgpu_compress_batch");
        if (st != RPGPU_OK) throw std::runtime_error("rpgpu_compress_batch: status " + std::to_string(st));
        out.resize(got);
        return rpgpu::iobuf(std::move(out));
    }
};
}  // namespace compression

// ---------------------------------------------------------------------------
// storage — parser surfaces
// ---------------------------------------------------------------------------
namespace storage {

namespace internal {
// storage/parser_utils.cc:114-120 (host: one header at a time)
inline void reset_size_checksum_metadata(model::record_batch_header& hdr, const rpgpu::iobuf& records) {
    hdr.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + records.size_bytes());
    hdr.crc = model::crc_record_batch(hdr, records);
    hdr.header_crc = model::internal_header_only_crc(hdr);
}

// storage/parser_utils.cc:96-111: the payload compressed with c, the
// compression bits set in attrs, then size, crc and header_crc reset
inline std::pair<model::record_batch_header, rpgpu::iobuf>
compress_batch(model::compression c, model::record_batch_header h, const rpgpu::iobuf& records,
               rpgpu::engine& e = rpgpu::engine::local()) {
    if (c == model::compression::none) throw std::invalid_argument("Asked to compress a batch with type `none`");
    rpgpu::iobuf payload = compression::compressor::compress(records, c, e);
    h.attrs |= c;  // compression bit must be set first
    reset_size_checksum_metadata(h, payload);
    return {h, std::move(payload)};
}
}  // namespace internal

// The write side in bulk (rpgpu_stamp): a buffer of on-disk batches about to
// be appended gets, on the device and in batch order, what
// disk_log_appender::operator() (storage/disk_log_appender.cc:72-74,
// :113-119) and reset_size_checksum_metadata give each one: base offsets
// from `next_offset` (returns the appender's next offset after the last
// batch), size_bytes and crc, then header_crc.  `buf` holds the batches
// back to back; each payload runs to the next header (or the end).
inline int64_t stamp_batches(uint8_t* buf, size_t len, const std::vector<size_t>& positions, int64_t next_offset,
                             uint32_t flags = RPGPU_STAMP_OFFSETS | RPGPU_STAMP_CRC,
                             rpgpu::engine& e = rpgpu::engine::local()) {
    const size_t n = positions.size();
    if (n == 0) return next_offset;
    std::vector<uint64_t> pos(n);
    std::vector<uint32_t> plen(n);
    int64_t next = next_offset;
    for (size_t i = 0; i < n; i++) {
        const size_t end = i + 1 < n ? positions[i + 1] : len;
        if (positions[i] + RPGPU_HEADER_SIZE > end) throw std::invalid_argument("stamp_batches: short batch");
        pos[i] = positions[i];
        plen[i] = (uint32_t)(end - positions[i] - RPGPU_HEADER_SIZE);
        int32_t lod;
        std::memcpy(&lod, buf + positions[i] + 23, 4);
        next = (int64_t)((uint64_t)next + (uint64_t)(int64_t)lod + 1u);
    }
    // through the context's grow-only pinned + device staging: one H2D, the
    // kernels, one D2H
    e.check(rpgpu_stamp_host(e.ctx(), buf, len, pos.data(), plen.data(), (uint32_t)n, next_offset, flags),
            "rpgpu_stamp_host");
    return (flags & RPGPU_STAMP_OFFSETS) ? next : next_offset;
}

// storage/parser_errc.h:18-25
enum class parser_errc : int {
    none = RPGPU_ERRC_NONE,
    end_of_stream = RPGPU_ERRC_END_OF_STREAM,
    header_only_crc_missmatch = RPGPU_ERRC_HEADER_ONLY_CRC_MISSMATCH,
    input_stream_not_enough_bytes = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES,
    fallocated_file_read_zero_bytes_for_header = RPGPU_ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER,
    not_enough_bytes_in_parser_for_one_record = RPGPU_ERRC_NOT_ENOUGH_BYTES_IN_PARSER_FOR_ONE_RECORD,
};

// outcome::result<size_t, parser_errc>
struct parse_result {
    size_t value{0};
    std::optional<parser_errc> error;
    explicit operator bool() const { return !error.has_value(); }
};

// storage/parser.h:32-87
class batch_consumer {
public:
    using stop_parser = bool;  // ss::bool_class<stop_parser_tag>
    enum class consume_result : int8_t { accept_batch, stop_parser, skip_batch };

    batch_consumer() noexcept = default;
    virtual ~batch_consumer() noexcept = default;
    virtual consume_result accept_batch_start(const model::record_batch_header&) const = 0;
    virtual void consume_batch_start(model::record_batch_header, size_t physical_base_offset, size_t size_on_disk) = 0;
    virtual void skip_batch_start(model::record_batch_header, size_t physical_base_offset, size_t size_on_disk) = 0;
    virtual void consume_records(rpgpu::iobuf&&) = 0;
    virtual stop_parser consume_batch_end() = 0;
    virtual void print(std::ostream&) const = 0;
};

inline std::ostream& operator<<(std::ostream& os, const batch_consumer& c) {
    c.print(os);
    return os;
}

namespace detail {
// One disk-layout segment validated on the GPU (chain discovery, header_crc,
// batch crc): the per-batch verdicts in chain order and the segment summary.
struct segment_scan {
    std::vector<rpgpu_batch_result> batches;
    rpgpu_segment_summary summary{};
    // filled when an index rebuild was requested (rpgpu_segment_index)
    rpgpu_index_state index{};
    std::vector<uint32_t> rel_offset, rel_time;
    std::vector<uint64_t> position;
};

struct index_request {
    int64_t base_offset;  // the segment's base offset (segment_index / index_state.base_offset)
    uint64_t step;        // segment_index::_step
};

inline segment_scan scan_segment(rpgpu::engine& e, const uint8_t* seg, size_t len,
                                 uint32_t layout = RPGPU_LAYOUT_DISK, uint32_t flags = RPGPU_JOB_CRC,
                                 const index_request* want_index = nullptr) {
    // rpgpu_validate_host: the context's pinned, double-buffered staging
    // (256 MiB groups copied while the previous group validates), no
    // per-call device allocation.  The result arrays are sized for the
    // worst case (a batch per 61 bytes) but left uninitialised, so only the
    // entries the job writes are touched.
    segment_scan out;
    const size_t cap = len / RPGPU_HEADER_SIZE + 2;
    std::unique_ptr<rpgpu_batch_result[]> b(new rpgpu_batch_result[cap]);
    std::unique_ptr<uint32_t[]> ro, rt;
    std::unique_ptr<uint64_t[]> ps;
    const uint8_t* segs[1] = {seg};
    const uint64_t sizes[1] = {(uint64_t)len};
    rpgpu_job_totals t{};
    rpgpu_host_job j{};
    j.segments = segs;
    j.seg_sizes = sizes;
    j.n_segments = 1;
    j.layout = layout;
    j.flags = flags;
    j.batches = b.get();
    j.batch_capacity = cap;
    j.summaries = &out.summary;
    j.totals = &t;
    if (want_index) {
        ro.reset(new uint32_t[cap]);
        rt.reset(new uint32_t[cap]);
        ps.reset(new uint64_t[cap]);
        out.index = rpgpu_index_state{};
        out.index.base_offset = want_index->base_offset;
        j.index_step = want_index->step;
        j.index_states = &out.index;
        j.rel_offset = ro.get();
        j.rel_time = rt.get();
        j.position = ps.get();
    }
    e.check(rpgpu_validate_host(e.ctx(), &j), "rpgpu_validate_host");
    const size_t nb = (size_t)std::min<uint64_t>(t.n_batches, cap);
    out.batches.assign(b.get(), b.get() + nb);
    if (want_index) {
        const size_t a = (size_t)out.index.first_entry, n = (size_t)out.index.n_entries;
        out.rel_offset.assign(ro.get() + a, ro.get() + a + n);
        out.rel_time.assign(rt.get() + a, rt.get() + a + n);
        out.position.assign(ps.get() + a, ps.get() + a + n);
    }
    return out;
}
}  // namespace detail

// ss::input_stream<char> as the parser reads it: successive reads from
// file position 0, 0 bytes at the end of the stream.
class input_stream {
public:
    virtual ~input_stream() = default;
    // up to n bytes into dst; 0 = end of stream
    virtual size_t read(uint8_t* dst, size_t n) = 0;
};

// a file read from position 0 (log_replayer::recover opens the segment with
// make_file_input_stream at 0, storage/log_replayer.cc:95-114)
class file_input_stream final : public input_stream {
public:
    explicit file_input_stream(const char* path) : _f(std::fopen(path, "rb")) {
        if (!_f) throw std::runtime_error(std::string("file_input_stream: cannot open ") + path);
    }
    ~file_input_stream() override {
        if (_f) std::fclose(_f);
    }
    size_t read(uint8_t* dst, size_t n) override { return std::fread(dst, 1, n, _f); }

private:
    std::FILE* _f;
};

// bytes already in host memory, read in pieces of at most `piece`
class memory_input_stream final : public input_stream {
public:
    memory_input_stream(const uint8_t* p, size_t n, size_t piece = SIZE_MAX) : _p(p), _n(n), _piece(piece) {}
    size_t read(uint8_t* dst, size_t n) override {
        const size_t k = std::min(std::min(n, _piece), _n - _at);
        std::memcpy(dst, _p + _at, k);
        _at += k;
        return k;
    }

private:
    const uint8_t* _p;
    size_t _n, _piece, _at = 0;
};

// storage/parser.h:94-136.  Two inputs: a whole segment in host memory (a
// file's bytes from position 0, as log_replayer reads it), or an
// input_stream read ahead in windows (default 64 MiB).  A window is
// validated on the GPU in one job; the chain's stop inside it is final
// unless the window merely ended there (a short header or payload at its
// end while the stream has more): then the bytes from that batch on are
// kept, the window refilled and validated again from there, so the events
// are exactly those of one job over the whole stream.  A batch larger than
// the window doubles it.
class continuous_batch_parser {
public:
    static constexpr size_t default_readahead = 64u << 20;

    continuous_batch_parser(std::unique_ptr<batch_consumer> consumer, const uint8_t* segment, size_t len,
                            rpgpu::engine& e = rpgpu::engine::local()) noexcept
      : _consumer(std::move(consumer)), _seg(segment), _win_len(len), _in_eof(true), _e(e) {}
    continuous_batch_parser(std::unique_ptr<batch_consumer> consumer, std::unique_ptr<input_stream> in,
                            size_t readahead = default_readahead, rpgpu::engine& e = rpgpu::engine::local())
      : _consumer(std::move(consumer)), _in(std::move(in)), _readahead(std::max<size_t>(readahead, 64)), _e(e) {}
    continuous_batch_parser(const continuous_batch_parser&) = delete;
    continuous_batch_parser& operator=(const continuous_batch_parser&) = delete;

    // continuous_batch_parser::consume (storage/parser.cc:218-254) over the
    // GPU's verdicts.  The segment (or the stream's first window) is
    // validated on the first call; later calls resume where the previous one
    // stopped.
    parse_result consume() {
        if (_err != parser_errc::none) return {0, _err};
        for (;;) {
            const step s = consume_one();
            if (_eof) break;
            if (s.err != parser_errc::none) {
                _err = s.err;
                break;
            }
            if (s.stop) break;
        }
        if (_bytes_consumed) return {_bytes_consumed, std::nullopt};  // partial reads
        if (_err == parser_errc::none || _err == parser_errc::end_of_stream ||
            _err == parser_errc::fallocated_file_read_zero_bytes_for_header)
            return {_bytes_consumed, std::nullopt};
        return {0, _err};
    }

    void close() {}

private:
    struct step {
        parser_errc err = parser_errc::none;
        bool stop = false;
    };

    // The verdict of the chain's next batch (nullptr: the chain ended, see
    // _term): from the current window's scan, refilled as the stream goes.
    const rpgpu_batch_result* next_batch() {
        for (;;) {
            if (_scan && _i < _scan->batches.size()) return &_scan->batches[_i];
            if (_scan && _final) return nullptr;
            scan_window();
        }
    }

    // Validate the window from the chain's position (the first batch not yet
    // delivered); read more of the stream first when there is one.
    void scan_window() {
        if (_in) {
            const size_t keep = _scan ? _keep_from : 0;
            if (keep) {
                std::memmove(_buf.data(), _buf.data() + keep, _win_len - keep);
                _win_len -= keep;
                _win_base += keep;
            }
            if (_buf.size() < _readahead) _buf.resize(_readahead);
            if (_scan && keep == 0 && _win_len == _buf.size()) _buf.resize(_buf.size() * 2);  // a batch > the window
            while (_win_len < _buf.size() && !_in_eof) {
                const size_t k = _in->read(_buf.data() + _win_len, _buf.size() - _win_len);
                if (k == 0) _in_eof = true;
                _win_len += k;
            }
            _seg = _buf.data();
        }
        _scan = detail::scan_segment(_e, _seg, _win_len);
        _i = 0;
        const rpgpu_segment_summary& s = _scan->summary;
        // the window ended, not the stream: the chain resumes at the stop
        _final = !(s.terminal_eof && !_in_eof);
        if (!_final) {
            _keep_from = (size_t)s.terminal_pos;
            // an incomplete last batch (its payload runs past the window) is
            // read again with the next window
            while (!_scan->batches.empty() && !(_scan->batches.back().flags & RPGPU_F_COMPLETE))
                _scan->batches.pop_back();
        }
    }

    // consume_one (storage/parser.cc:178-190) = consume_header + consume_records
    step consume_one() {
        for (;;) {
            if (!_pending) {
                // read_header_impl (storage/parser.cc:139-176): the chain's
                // next header, or the verdict that ended the chain.  A read
                // past the end of the data is an empty read: end_of_stream.
                if (!next_batch()) {
                    if (_eof) return {parser_errc::end_of_stream, false};
                    if (_scan->summary.terminal_eof) _eof = true;
                    return {(parser_errc)_scan->summary.terminal_errc, false};
                }
                _pending = true;
            }
            const rpgpu_batch_result& r = *next_batch();
            const model::record_batch_header h = model::record_batch_header::from(r);
            const bool complete = (r.flags & RPGPU_F_COMPLETE) != 0;
            const size_t size = (size_t)(int64_t)h.size_bytes;
            switch (_consumer->accept_batch_start(h)) {
            case batch_consumer::consume_result::stop_parser:
                return {parser_errc::none, true};  // the header stays pending
            case batch_consumer::consume_result::skip_batch:
                _consumer->skip_batch_start(h, _physical_base_offset, size);
                _physical_base_offset += size;
                // verify_read_iobuf: a short read sets eof and returns before
                // add_bytes_and_reset, so the header stays pending
                if (!complete) {
                    _eof = true;
                    return {parser_errc::input_stream_not_enough_bytes, false};
                }
                add_bytes_and_reset(size);
                continue;
            case batch_consumer::consume_result::accept_batch:
                break;
            }
            _consumer->consume_batch_start(h, _physical_base_offset, size);
            _physical_base_offset += size;
            // consume_records: add_bytes_and_reset runs whether or not the
            // payload could be read
            step out;
            if (!complete) {
                _eof = true;
                out.err = parser_errc::input_stream_not_enough_bytes;
            } else {
                const uint8_t* payload = _seg + r.file_pos + RPGPU_HEADER_SIZE;  // window-relative
                _consumer->consume_records(
                  rpgpu::iobuf(payload, (uint32_t)(r.size_bytes - (int32_t)RPGPU_HEADER_SIZE)));
                out.stop = _consumer->consume_batch_end();
            }
            add_bytes_and_reset(size);
            return out;
        }
    }

    void add_bytes_and_reset(size_t size) {
        _bytes_consumed += size;
        _pending = false;
        _i++;
    }

    std::unique_ptr<batch_consumer> _consumer;
    const uint8_t* _seg = nullptr;  // the window's bytes (the whole segment without a stream)
    std::unique_ptr<input_stream> _in;
    std::vector<uint8_t> _buf;      // the stream's window
    size_t _win_len = 0;            // valid bytes at _seg
    size_t _win_base = 0;           // stream position of _seg[0]
    size_t _readahead = 0;
    size_t _keep_from = 0;          // window position the chain resumes at (not final)
    bool _in_eof = false;           // the stream returned 0 bytes
    bool _final = false;            // the window scan's terminal verdict ends the chain
    rpgpu::engine& _e;
    std::optional<detail::segment_scan> _scan;
    size_t _i = 0;         // window chain ordinal of the next (or pending) header
    bool _pending = false; // _header is set
    bool _eof = false;     // _input.eof()
    parser_errc _err = parser_errc::none;
    size_t _bytes_consumed{0};
    size_t _physical_base_offset{0};
};

// storage/index_state.h:37-75: the sparse offset/time -> file position index
// of one segment, as recovery rebuilds it.
struct index_state {
    int64_t base_offset{0};
    int64_t max_offset{0};
    int64_t base_timestamp{0};
    int64_t max_timestamp{0};
    std::vector<uint32_t> relative_offset_index;
    std::vector<uint32_t> relative_time_index;
    std::vector<uint64_t> position_index;
    uint32_t bitflags{0};
    bool empty() const { return relative_offset_index.empty(); }

    static constexpr int8_t ondisk_version = 3;  // index_state.h:38

    // index_state::checksum_state (storage/index_state.cc:27-48): xxhash64 of
    // bitflags, base/max offset, base/max timestamp, the entry count and the
    // three arrays, each as its native little-endian bytes
    uint64_t checksum_state() const {
        std::vector<uint8_t> b;
        put_fields(b);
        return rpgpu::xxh64(b.data(), b.size());
    }

    // index_state::checksum_and_serialize (storage/index_state.cc:189-236): the
    // .base_index file body
    std::vector<uint8_t> checksum_and_serialize() const {
        std::vector<uint8_t> body;
        put_fields(body);
        const uint64_t checksum = rpgpu::xxh64(body.data(), body.size());
        const uint32_t size = (uint32_t)(8 + body.size());  // checksum + the hashed fields
        std::vector<uint8_t> out;
        out.reserve(1 + 4 + size);
        put(out, ondisk_version);
        put(out, size);
        put(out, checksum);
        out.insert(out.end(), body.begin(), body.end());
        return out;
    }

    // index_state::hydrate_from_buffer (storage/index_state.cc:104-186): nullopt
    // on an unknown version, a size mismatch or a bad checksum (the reference
    // then rebuilds the index from the log); a read past the buffer throws
    // std::out_of_range, as the reference's iobuf_parser does
    // (bytes/details/io_iterator_consumer.h:64-84)
    static std::optional<index_state> hydrate_from_buffer(const uint8_t* p, size_t n) {
        size_t at = 0;
        auto take = [&](auto& v) {
            if (n - at < sizeof(v)) throw std::out_of_range("index_state: short read");
            std::memcpy(&v, p + at, sizeof(v));
            at += sizeof(v);
        };
        int8_t version;
        uint32_t size, vsize;
        uint64_t checksum;
        index_state r;
        take(version);
        if (version != ondisk_version) return std::nullopt;
        take(size);
        if (n - at != size) return std::nullopt;
        take(checksum);
        take(r.bitflags);
        take(r.base_offset);
        take(r.max_offset);
        take(r.base_timestamp);
        take(r.max_timestamp);
        take(vsize);
        if ((n - at) / 16 < vsize) throw std::out_of_range("index_state: short read");
        r.relative_offset_index.resize(vsize);
        r.relative_time_index.resize(vsize);
        r.position_index.resize(vsize);
        for (auto& v : r.relative_offset_index) take(v);
        for (auto& v : r.relative_time_index) take(v);
        for (auto& v : r.position_index) take(v);
        if (r.checksum_state() != checksum) return std::nullopt;
        return r;
    }

private:
    template <class T>
    static void put(std::vector<uint8_t>& b, T v) {
        const auto* q = reinterpret_cast<const uint8_t*>(&v);
        b.insert(b.end(), q, q + sizeof(T));
    }
    void put_fields(std::vector<uint8_t>& b) const {
        put(b, bitflags);
        put(b, base_offset);
        put(b, max_offset);
        put(b, base_timestamp);
        put(b, max_timestamp);
        put(b, (uint32_t)relative_offset_index.size());
        for (uint32_t v : relative_offset_index) put(b, v);
        for (uint32_t v : relative_time_index) put(b, v);
        for (uint64_t v : position_index) put(b, v);
    }
};

// storage/segment_index.h:30-100 (the lookups over a rebuilt index_state)
class segment_index {
public:
    static constexpr size_t default_data_buffer_step = RPGPU_INDEX_DEFAULT_STEP;  // segment_index.h:49
    struct entry {
        int64_t offset;
        int64_t timestamp;
        size_t filepos;
    };
    explicit segment_index(index_state st) : _state(std::move(st)) {}
    const index_state& state() const { return _state; }

    // segment_index::find_nearest(model::offset) (storage/segment_index.cc:89-107):
    // the last entry whose offset is <= o
    std::optional<entry> find_nearest(int64_t o) const {
        if (o < _state.base_offset || _state.empty()) return std::nullopt;
        const uint32_t i = (uint32_t)(o - _state.base_offset);
        const auto& ro = _state.relative_offset_index;
        auto it = std::upper_bound(ro.begin(), ro.end(), i);
        if (it == ro.begin()) return std::nullopt;
        return translate(size_t(std::distance(ro.begin(), it)) - 1);
    }
    // segment_index::find_nearest(model::timestamp) (storage/segment_index.cc:74-87):
    // the first entry whose relative time is >= t
    std::optional<entry> find_nearest_timestamp(int64_t t) const {
        if (t < _state.base_timestamp || _state.empty()) return std::nullopt;
        const uint32_t i = (uint32_t)(t - _state.base_timestamp);
        const auto& rt = _state.relative_time_index;
        auto it = std::lower_bound(rt.begin(), rt.end(), i);
        if (it == rt.end()) return std::nullopt;
        return translate(size_t(std::distance(rt.begin(), it)));
    }

private:
    entry translate(size_t k) const {
        return entry{_state.base_offset + (int64_t)_state.relative_offset_index[k],
                     _state.base_timestamp + (int64_t)_state.relative_time_index[k], (size_t)_state.position_index[k]};
    }
    index_state _state;
};

// storage/log_replayer.h:159-165 + log_replayer.cc:95-114: recover a segment
// from file position 0; the checkpoint is the last batch whose crc matched
// before the first one that did not.  Computed on the GPU in one submit.
class log_replayer {
public:
    struct checkpoint {
        std::optional<int64_t> last_offset;
        std::optional<size_t> truncate_file_pos;
    };

    static checkpoint recover(const uint8_t* segment, size_t len, rpgpu::engine& e = rpgpu::engine::local()) {
        const detail::segment_scan sc = detail::scan_segment(e, segment, len);
        checkpoint c;
        if (sc.summary.has_checkpoint) {
            c.last_offset = sc.summary.ckpt_last_offset;
            c.truncate_file_pos = (size_t)sc.summary.ckpt_truncate_pos;
        }
        return c;
    }

    // Recovery that also rebuilds the segment's sparse index the way
    // checksumming_consumer does (log_replayer.cc:62-74 -> segment_index::maybe_track).
    // Where the reference vasserts (a batch below the index base offset) this
    // throws std::runtime_error.
    static checkpoint recover(const uint8_t* segment, size_t len, int64_t base_offset, index_state& idx,
                              size_t step = segment_index::default_data_buffer_step,
                              rpgpu::engine& e = rpgpu::engine::local()) {
        const detail::index_request rq{base_offset, step};
        detail::segment_scan sc = detail::scan_segment(e, segment, len, RPGPU_LAYOUT_DISK, RPGPU_JOB_CRC, &rq);
        if (sc.index.assert_batch == -2) throw std::runtime_error("log_replayer: batch capacity overflow");
        if (sc.index.assert_batch >= 0) throw std::runtime_error("index_state::maybe_index: offset below base_offset");
        idx.base_offset = sc.index.base_offset;
        idx.max_offset = sc.index.max_offset;
        idx.base_timestamp = sc.index.base_timestamp;
        idx.max_timestamp = sc.index.max_timestamp;
        idx.relative_offset_index = std::move(sc.rel_offset);
        idx.relative_time_index = std::move(sc.rel_time);
        idx.position_index = std::move(sc.position);
        checkpoint c;
        if (sc.summary.has_checkpoint) {
            c.last_offset = sc.summary.ckpt_last_offset;
            c.truncate_file_pos = (size_t)sc.summary.ckpt_truncate_pos;
        }
        return c;
    }
};

}  // namespace storage

// ---------------------------------------------------------------------------
// kafka — the produce path's record-set reader over the wire layout
// ---------------------------------------------------------------------------
namespace kafka {

// kafka/protocol/errors.h (the one code this path raises)
enum class error_code : int16_t { none = 0, corrupt_message = 2 };

// kafka/protocol/exceptions.h
struct exception : std::runtime_error {
    exception(error_code e, const std::string& msg) : std::runtime_error(msg), error(e) {}
    error_code error;
};

// kafka/protocol/kafka_batch_adapter.h:60-76: the verdict of adapt() on one
// wire batch.  `batch` holds the adapted header (size_bytes = batch_length
// + 12, type raft_data) when the batch was accepted; `records` its payload.
struct kafka_batch_adapter {
    bool v2_format{false};
    bool valid_crc{false};
    std::optional<model::record_batch_header> batch;
    rpgpu::iobuf records;
};

// kafka/protocol/batch_reader.h: a Kafka v2 record set as a produce request
// carries it.  The whole set is validated on the GPU in one rpgpu_submit
// (layout RPGPU_LAYOUT_WIRE: CRC, record parse), then consumed batch by
// batch with the reference's verdicts and exceptions.
class batch_reader {
public:
    batch_reader(const uint8_t* record_set, size_t len, rpgpu::engine& e = rpgpu::engine::local())
      : _buf(record_set), _len(len),
        _scan(storage::detail::scan_segment(e, record_set, len, RPGPU_LAYOUT_WIRE, RPGPU_JOB_CRC | RPGPU_JOB_PARSE)) {}

    bool empty() const { return _pos >= _len; }
    size_t size_bytes() const { return _len - _pos; }

    // batch_reader::last_offset (batch_reader.cc:92-103): last_offset of the
    // final batch, structurally; a short header throws corrupt_message and a
    // batch running past the end (or shorter than its own header) makes the
    // parser's skip throw std::out_of_range
    int64_t last_offset() const {
        int64_t last = 0;
        for (size_t i = _i; i < _scan.batches.size(); i++) {
            const rpgpu_batch_result& r = _scan.batches[i];
            if (!(r.flags & RPGPU_F_COMPLETE)) throw std::out_of_range("batch_reader: batch past the end");
            last = (int64_t)((uint64_t)r.base_offset + (uint64_t)(int64_t)r.last_offset_delta);
        }
        check_terminal();
        return last;
    }

    // batch_reader::consume_batch (batch_reader.cc:112-121) + adapt()
    // (kafka_batch_adapter.cc:126-188)
    kafka_batch_adapter consume_batch() {
        if (_i >= _scan.batches.size()) {
            check_terminal();
            throw exception(error_code::corrupt_message, "Invalid kafka header parsing: no batch left");
        }
        const rpgpu_batch_result& r = _scan.batches[_i];
        if (!(r.flags & RPGPU_F_COMPLETE)) throw std::out_of_range("batch_reader: batch past the end");
        kafka_batch_adapter kba;
        kba.v2_format = (r.flags & RPGPU_F_WIRE_V2) != 0;
        kba.valid_crc = kba.v2_format && (r.flags & RPGPU_F_CRC_OK);
        _i++;
        _pos = (size_t)r.file_pos + (size_t)(int64_t)r.size_bytes;
        if (!kba.valid_crc) return kba;
        // record_batch::compressed() -> attributes::compression() throws for
        // codec values 5..7, out of adapt()
        if (r.flags & RPGPU_F_CODEC_INVALID)
            throw std::runtime_error("Unknown compression value: " + std::to_string(r.attrs & 7));
        if (!(r.flags & RPGPU_F_COMPRESSED) && !(r.flags & RPGPU_F_PARSE_OK)) return kba;  // for_each_record threw
        kba.batch = model::record_batch_header::from(r);
        kba.records = rpgpu::iobuf(_buf + r.file_pos + RPGPU_HEADER_SIZE,
                                   (size_t)((int64_t)r.size_bytes - (int64_t)RPGPU_HEADER_SIZE));
        return kba;
    }

private:
    void check_terminal() const {
        const rpgpu_segment_summary& sm = _scan.summary;
        if (sm.terminal_errc == RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES) {
            // fewer than 61 bytes left: read_record_batch_info throws; a
            // batch_length too small for the header makes the skip throw
            if (sm.terminal_eof) throw exception(error_code::corrupt_message, "Invalid kafka header parsing");
            throw std::out_of_range("batch_reader: batch shorter than its header");
        }
    }

    const uint8_t* _buf;
    size_t _len;
    storage::detail::segment_scan _scan;
    size_t _i = 0;
    size_t _pos = 0;
};

}  // namespace kafka

#endif  // RPGPU_REDPANDA_H_
