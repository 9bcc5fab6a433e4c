// Driver for the C++ drop-in surfaces in include/rpgpu_redpanda.h, used by
// tests/test_cpp_surfaces.py.  Each mode prints one event per line; the
// Python side compares the events with a restatement of the reference's
// loops over the same bytes.
//
//   surfaces_test cpu <segment>                 host walk: model:: crc helpers
//   surfaces_test parse <segment> M R S E       continuous_batch_parser replay
//   surfaces_test parse_stream <segment> M R S E W   ... over a file stream, W-byte windows
//   surfaces_test recover <segment>             log_replayer checkpoint
//   surfaces_test recover_bench <reps> <seg>... log_replayer::recover timing (host path)
//   surfaces_test index <segment> <base> <q>... log_replayer recovery + segment_index rebuild,
//                                               find_nearest(offset) for each q
//   surfaces_test uncompress (<codec> <in> <out>)+  compressor::uncompress
//   surfaces_test wire <record_set>             kafka::batch_reader
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <sstream>

#include "rpgpu_redpanda.h"

static std::vector<uint8_t> slurp(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(2); }
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

template <typename T>
static T le(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof v);
    return v;
}

// storage::header_from_iobuf (storage/parser.cc:36-76): the disk header is
// little-endian, in declaration order
static model::record_batch_header header_at(const uint8_t* p) {
    model::record_batch_header h;
    h.header_crc = le<uint32_t>(p + 0);
    h.size_bytes = le<int32_t>(p + 4);
    h.base_offset = le<int64_t>(p + 8);
    h.type = (int8_t)p[16];
    h.crc = le<int32_t>(p + 17);
    h.attrs = model::record_batch_attributes(le<int16_t>(p + 21));
    h.last_offset_delta = le<int32_t>(p + 23);
    h.first_timestamp = le<int64_t>(p + 27);
    h.max_timestamp = le<int64_t>(p + 35);
    h.producer_id = le<int64_t>(p + 43);
    h.producer_epoch = le<int16_t>(p + 51);
    h.base_sequence = le<int32_t>(p + 53);
    h.record_count = le<int32_t>(p + 57);
    return h;
}

// the disk header back (header_at's inverse)
template <class T>
static void put_le(uint8_t* p, T v) { std::memcpy(p, &v, sizeof v); }
static void header_to(const model::record_batch_header& h, uint8_t* p) {
    put_le(p + 0, h.header_crc);
    put_le(p + 4, h.size_bytes);
    put_le(p + 8, h.base_offset);
    p[16] = (uint8_t)h.type;
    put_le(p + 17, h.crc);
    put_le(p + 21, h.attrs.value());
    put_le(p + 23, h.last_offset_delta);
    put_le(p + 27, h.first_timestamp);
    put_le(p + 35, h.max_timestamp);
    put_le(p + 43, h.producer_id);
    put_le(p + 51, h.producer_epoch);
    put_le(p + 53, h.base_sequence);
    put_le(p + 57, h.record_count);
}

static int self_checks() {
    // crc::crc32c: the standard check value, and extend() composes
    const char* s = "123456789";
    crc::crc32c a;
    a.extend(s, 9);
    crc::crc32c b;
    b.extend(s, 4);
    b.extend(s + 4, 5);
    if (a.value() != 0xE3069283u || b.value() != a.value()) return 1;
    crc::crc32c c;
    c.extend((int32_t)0x01020304);
    const uint8_t le4[4] = {4, 3, 2, 1};
    if (c.value() != rpgpu_crc32c_extend(0, le4, 4)) return 2;
    // attributes: codec bits, control / transactional bits, invalid codecs throw
    model::record_batch_attributes at(0x33);
    if (at.compression() != model::compression::lz4 || !at.is_control() || !at.is_transactional()) return 3;
    bool threw = false;
    try {
        (void)model::record_batch_attributes(0x6).compression();
    } catch (const std::runtime_error&) {
        threw = true;
    }
    if (!threw) return 4;
    model::record_batch_attributes at2(0x12);
    at2.remove_compression();
    at2 |= model::compression::snappy;
    if (at2.value() != 0x12) return 5;
    return 0;
}

static int mode_cpu(const std::vector<uint8_t>& seg) {
    const int sc = self_checks();
    std::printf("SELF %d\n", sc);
    // a log_replayer-style host walk (storage/log_replayer.cc:62-79) using
    // only the model:: surfaces
    size_t pos = 0;
    while (seg.size() - pos >= model::packed_record_batch_header_size) {
        const model::record_batch_header h = header_at(seg.data() + pos);
        if (h.header_crc == 0) break;
        const bool hok = model::internal_header_only_crc(h) == h.header_crc;
        if (!hok) break;
        const size_t size = (size_t)(int64_t)h.size_bytes;
        if (size < model::packed_record_batch_header_size || seg.size() - pos < size) break;
        rpgpu::iobuf rec(seg.data() + pos + model::packed_record_batch_header_size,
                         size - model::packed_record_batch_header_size);
        const bool cok = model::crc_record_batch(h, rec) == h.crc;
        std::printf("B %zu %d %lld %d %d %d\n", pos, h.size_bytes, (long long)h.base_offset, (int)hok, (int)cok,
                    (int)h.attrs.value());
        pos += size;
    }
    return sc;
}

// Consumer with scripted decisions by chain ordinal k: skip when k % M == R,
// stop_parser once at k == S, consume_batch_end() returns stop at k == E.
class scripted_consumer final : public storage::batch_consumer {
public:
    scripted_consumer(int m, int r, int s, int e) : _m(m), _r(r), _s(s), _e(e) {}
    consume_result accept_batch_start(const model::record_batch_header& h) const override {
        std::printf("ASK %d %lld\n", _k, (long long)h.base_offset);
        if (_k == _s && !_stopped) {
            _stopped = true;
            return consume_result::stop_parser;
        }
        if (_m > 0 && _k % _m == _r) return consume_result::skip_batch;
        return consume_result::accept_batch;
    }
    void consume_batch_start(model::record_batch_header h, size_t phys, size_t size) override {
        std::printf("START %d %lld %zu %zu %d\n", _k, (long long)h.base_offset, phys, size, h.record_count);
    }
    void skip_batch_start(model::record_batch_header h, size_t phys, size_t size) override {
        std::printf("SKIP %d %lld %zu %zu\n", _k, (long long)h.base_offset, phys, size);
        _k++;
    }
    void consume_records(rpgpu::iobuf&& b) override {
        crc::crc32c c;
        c.extend(b.data(), b.size_bytes());
        std::printf("RECORDS %d %zu %u\n", _k, b.size_bytes(), c.value());
    }
    stop_parser consume_batch_end() override {
        const bool stop = _k == _e;
        std::printf("END %d %d\n", _k, (int)stop);
        _k++;
        return stop;
    }
    void print(std::ostream& os) const override { os << "scripted_consumer{" << _k << "}"; }

private:
    int _m, _r, _s, _e;
    int _k = 0;
    mutable bool _stopped = false;
};

static void print_result(const storage::parse_result& r) {
    if (r) std::printf("RESULT ok %zu\n", r.value);
    else std::printf("RESULT err %d\n", (int)*r.error);
}

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: surfaces_test <mode> ...\n"); return 2; }
    const std::string mode = argv[1];
    try {
        if (mode == "cpu") return mode_cpu(slurp(argv[2]));
        if (mode == "parse" && argc == 7) {
            const std::vector<uint8_t> seg = slurp(argv[2]);
            storage::continuous_batch_parser p(
              std::make_unique<scripted_consumer>(std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                                                  std::atoi(argv[6])),
              seg.data(), seg.size());
            // a stop ends one consume(); the caller resumes, as the
            // reference's readers do after a stop_parser
            for (int call = 0; call < 3; call++) {
                print_result(p.consume());
            }
            p.close();
            return 0;
        }
        if (mode == "parse_stream" && argc == 8) {
            // the same replay over a file input stream read ahead in windows
            // of argv[7] bytes
            storage::continuous_batch_parser p(
              std::make_unique<scripted_consumer>(std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                                                  std::atoi(argv[6])),
              std::make_unique<storage::file_input_stream>(argv[2]), (size_t)std::atoll(argv[7]));
            for (int call = 0; call < 3; call++) {
                print_result(p.consume());
            }
            p.close();
            return 0;
        }
        if (mode == "recover") {
            const std::vector<uint8_t> seg = slurp(argv[2]);
            const storage::log_replayer::checkpoint c = storage::log_replayer::recover(seg.data(), seg.size());
            if (c.last_offset) std::printf("CKPT 1 %lld %zu\n", (long long)*c.last_offset, *c.truncate_file_pos);
            else std::printf("CKPT 0\n");
            return 0;
        }
        if (mode == "recover_bench" && argc >= 4) {
            // log_replayer::recover over host segments (the pinned,
            // double-buffered host path): wall time per pass after a warm-up
            std::vector<std::vector<uint8_t>> segs;
            for (int a = 3; a < argc; a++) segs.push_back(slurp(argv[a]));
            const int reps = std::atoi(argv[2]);
            size_t bytes = 0;
            for (auto& sg : segs) bytes += sg.size();
            for (auto& sg : segs) (void)storage::log_replayer::recover(sg.data(), sg.size());  // warm-up
            const auto t0 = std::chrono::steady_clock::now();
            long long ck = 0;
            for (int r = 0; r < reps; r++)
                for (auto& sg : segs) {
                    const storage::log_replayer::checkpoint c = storage::log_replayer::recover(sg.data(), sg.size());
                    ck += c.last_offset ? *c.last_offset : -1;
                }
            const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::printf("RECOVER_BENCH bytes=%zu reps=%d seconds=%.4f GBps=%.2f ckpt_sum=%lld\n", bytes, reps, sec,
                        (double)bytes * reps / sec / 1e9, ck);
            return 0;
        }
        if (mode == "xxh64") {  // host only: the .base_index checksum primitive
            const std::vector<uint8_t> b = slurp(argv[2]);
            std::printf("%llu\n", (unsigned long long)rpgpu::xxh64(b.data(), b.size()));
            return 0;
        }
        if (mode == "index") {
            const std::vector<uint8_t> seg = slurp(argv[2]);
            storage::index_state st;
            try {
                const storage::log_replayer::checkpoint c =
                  storage::log_replayer::recover(seg.data(), seg.size(), std::atoll(argv[3]), st);
                if (c.last_offset) std::printf("CKPT 1 %lld %zu\n", (long long)*c.last_offset, *c.truncate_file_pos);
                else std::printf("CKPT 0\n");
            } catch (const std::runtime_error& e) {
                std::printf("VASSERT\n");
                return 0;
            }
            std::printf("STATE %lld %lld %lld %lld %zu\n", (long long)st.base_offset, (long long)st.max_offset,
                        (long long)st.base_timestamp, (long long)st.max_timestamp, st.relative_offset_index.size());
            for (size_t k = 0; k < st.relative_offset_index.size(); k++)
                std::printf("E %u %u %llu\n", st.relative_offset_index[k], st.relative_time_index[k],
                            (unsigned long long)st.position_index[k]);
            {
                // .base_index round trip (index_state::checksum_and_serialize / hydrate_from_buffer)
                std::vector<uint8_t> ser = st.checksum_and_serialize();
                std::printf("SER ");
                for (uint8_t c : ser) std::printf("%02x", c);
                std::printf("\n");
                const auto back = storage::index_state::hydrate_from_buffer(ser.data(), ser.size());
                const bool same = back && back->relative_offset_index == st.relative_offset_index &&
                                  back->relative_time_index == st.relative_time_index &&
                                  back->position_index == st.position_index && back->max_offset == st.max_offset &&
                                  back->max_timestamp == st.max_timestamp;
                ser[ser.size() / 2] ^= 0x40;  // a flipped bit: checksum mismatch -> rebuild
                bool rejected;  // nullopt, or a short read (the flip may land in a length field)
                try {
                    rejected = !storage::index_state::hydrate_from_buffer(ser.data(), ser.size());
                } catch (const std::out_of_range&) {
                    rejected = true;
                }
                std::printf("HYDRATE %d %d\n", same ? 1 : 0, rejected ? 1 : 0);
                // short reads throw (the reference's iobuf_parser): an empty
                // buffer, and a vsize past the bytes present
                auto outcome = [](const std::vector<uint8_t>& b) {
                    try {
                        return storage::index_state::hydrate_from_buffer(b.data(), b.size()) ? "value" : "nullopt";
                    } catch (const std::out_of_range&) {
                        return "out_of_range";
                    }
                };
                std::vector<uint8_t> shortv = st.checksum_and_serialize();
                const size_t vs_at = 1 + 4 + 8 + 4 + 8 * 4;  // version, size, checksum, bitflags, 4 x i64
                uint32_t vsz;
                std::memcpy(&vsz, shortv.data() + vs_at, 4);
                vsz += 1000;
                std::memcpy(shortv.data() + vs_at, &vsz, 4);
                std::printf("HYDRATE_SHORT %s %s\n", outcome(std::vector<uint8_t>()), outcome(shortv));
            }
            const storage::segment_index idx(std::move(st));
            for (int a = 4; a < argc; a++) {
                const auto e = idx.find_nearest(std::atoll(argv[a]));
                if (e) std::printf("NEAR %lld %zu\n", (long long)e->offset, e->filepos);
                else std::printf("NEAR none\n");
            }
            return 0;
        }
        if (mode == "wire") {
            const std::vector<uint8_t> rs = slurp(argv[2]);
            {
                kafka::batch_reader r(rs.data(), rs.size());
                try {
                    std::printf("L %lld\n", (long long)r.last_offset());
                } catch (const kafka::exception&) {
                    std::printf("L corrupt\n");
                } catch (const std::out_of_range&) {
                    std::printf("L out_of_range\n");
                }
            }
            kafka::batch_reader r(rs.data(), rs.size());
            while (!r.empty()) {
                try {
                    const kafka::kafka_batch_adapter kba = r.consume_batch();
                    if (kba.batch) {
                        crc::crc32c c;
                        c.extend(kba.records.data(), kba.records.size_bytes());
                        std::printf("B %d %d 1 %lld %d %zu %u\n", (int)kba.v2_format, (int)kba.valid_crc,
                                    (long long)kba.batch->base_offset, kba.batch->size_bytes, kba.records.size_bytes(),
                                    c.value());
                    } else {
                        std::printf("B %d %d 0\n", (int)kba.v2_format, (int)(kba.v2_format && kba.valid_crc));
                    }
                } catch (const kafka::exception&) {
                    std::printf("X corrupt\n");
                    break;
                } catch (const std::out_of_range&) {
                    std::printf("X out_of_range\n");
                    break;
                } catch (const std::runtime_error&) {
                    std::printf("X runtime_error\n");
                    break;
                }
            }
            return 0;
        }
        if (mode == "stamp" && argc == 7) {
            // stamp <in> <positions.txt> <out> <next_offset> <flags>: storage::stamp_batches
            std::vector<uint8_t> buf = slurp(argv[2]);
            std::vector<size_t> pos;
            {
                std::ifstream f(argv[3]);
                size_t v;
                while (f >> v) pos.push_back(v);
            }
            const int64_t next = storage::stamp_batches(buf.data(), buf.size(), pos, std::atoll(argv[5]),
                                                        (uint32_t)std::atoi(argv[6]));
            std::ofstream f(argv[4], std::ios::binary);
            f.write((const char*)buf.data(), (std::streamsize)buf.size());
            std::printf("S %lld\n", (long long)next);
            return 0;
        }
        if (mode == "compress_batch" && argc == 5) {
            // compress_batch <codec> <batch.bin> <out.bin>: one disk-layout
            // batch (61-byte header + payload) through
            // storage::internal::compress_batch, written back in disk layout
            const std::vector<uint8_t> in = slurp(argv[3]);
            model::record_batch_header h = header_at(in.data());
            const rpgpu::iobuf records(in.data() + RPGPU_HEADER_SIZE, in.size() - RPGPU_HEADER_SIZE);
            auto r = storage::internal::compress_batch((model::compression)std::atoi(argv[2]), h, records);
            uint8_t hd[RPGPU_HEADER_SIZE];
            header_to(r.first, hd);
            std::ofstream f(argv[4], std::ios::binary);
            f.write((const char*)hd, RPGPU_HEADER_SIZE);
            f.write((const char*)r.second.data(), (std::streamsize)r.second.size_bytes());
            std::printf("C %d %zu\n", r.first.size_bytes, r.second.size_bytes());
            return 0;
        }
        if (mode == "uncompress" && argc >= 5 && (argc - 2) % 3 == 0) {
            // one or more (codec, in, out) triples: one line each
            for (int a = 2; a + 2 < argc; a += 3) {
                const std::vector<uint8_t> in = slurp(argv[a + 1]);
                try {
                    const rpgpu::iobuf out = compression::compressor::uncompress(
                      rpgpu::iobuf(in.data(), in.size()), (compression::type)std::atoi(argv[a]));
                    std::ofstream f(argv[a + 2], std::ios::binary);
                    f.write((const char*)out.data(), (std::streamsize)out.size_bytes());
                    std::printf("U ok %zu\n", out.size_bytes());
                } catch (const std::logic_error& e) {
                    std::printf("U logic_error\n");
                } catch (const std::runtime_error& e) {
                    std::printf("U runtime_error\n");
                }
            }
            return 0;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 3;
    }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
