/*
 * rp_oracle.h — CPU restatement of the reference's record-batch hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (redpanda_amd/, librpgpu.so) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to /root/reference/src/v) or, for third-party arithmetic absent from the
 * reference tree, the library and version whose published algorithm it
 * restates (google crc32c @47b40d22, lz4 1.9.3, snappy 1.1.8 — SURVEY.md §8(c)).
 *
 * Pinning: CRC32C by RFC 3720 vectors; header/CRC/record fields by fixtures
 * generated from the reference's own Python reader (tools/metadata_viewer);
 * LZ4F and snappy by differential tests against liblz4 1.9.3 / libsnappy
 * 1.1.8 (oracle/_ref), see tests/golden/README.md.
 */
#ifndef RP_ORACLE_H_
#define RP_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#include "../include/rpgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* --- hashing/crc32c.h:19-40 -> google crc32c::Extend (table, bytewise) */
uint32_t rpo_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
/* same function, SSE4.2 crc32q with 3 interleaved streams (the shape of
 * google crc32c's x86 path) — used as the timed CPU baseline */
uint32_t rpo_crc32c_extend_hw(uint32_t crc, const uint8_t* p, size_t n);
/* raw GF(2) helpers used by tests: crc of A||B from crc(A), crc(B), |B| */
uint32_t rpo_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* --- XXH32 (lz4 1.9.3 xxhash.c), used by LZ4F checksums */
uint32_t rpo_xxh32(const uint8_t* p, size_t n, uint32_t seed);

/* --- utils/vint.h:82-98 (vint::deserialize) and :37-39 (decode_zigzag) */
int64_t rpo_vint_deserialize(const uint8_t* p, size_t avail, size_t* bytes_read);
/* utils/vint.h:45-67 (vint::serialize); returns bytes written (<=10) */
size_t rpo_vint_serialize(int64_t v, uint8_t* out);

/* --- model::record_batch_header (model/record.h:354-417) */
typedef struct rpo_header {
    uint32_t header_crc;
    int32_t size_bytes;
    int64_t base_offset;
    int8_t type;
    int32_t crc;
    int16_t attrs;
    int32_t last_offset_delta;
    int64_t first_timestamp;
    int64_t max_timestamp;
    int64_t producer_id;
    int16_t producer_epoch;
    int32_t base_sequence;
    int32_t record_count;
} rpo_header;

/* storage/parser.cc:36-76 (header_from_iobuf, little endian) */
void rpo_header_from_disk(const uint8_t* p, rpo_header* h);
/* kafka/protocol/kafka_batch_adapter.cc:32-91 (read_header, big endian);
 * returns the magic byte */
int rpo_header_from_wire(const uint8_t* p, rpo_header* h);
/* storage/segment_appender_utils.cc:28-54 (disk_header_to_iobuf) */
void rpo_header_to_disk(const rpo_header* h, uint8_t* out61);
/* model/record_utils.cc:34-55 */
uint32_t rpo_internal_header_only_crc(const rpo_header* h);
/* model/record_utils.cc:68-91 (crc_record_batch_header + crc_extend_iobuf) */
uint32_t rpo_crc_record_batch(const rpo_header* h, const uint8_t* payload, size_t n);

/* --- record walk: model/record.h:616-627 / :680-697 over
 *     model/record_utils.cc:94-181.  Returns records fully parsed; sets
 *     *parse_err (rpgpu_parse_err of the async walk) and *trailing (bytes
 *     left after record_count records when no error).  Writes at most
 *     index_cap entries. */
uint32_t rpo_walk_records(const uint8_t* payload, size_t n, int32_t record_count,
                          uint32_t batch_ordinal, rpgpu_record_index* index,
                          uint64_t index_cap, uint8_t* parse_err, uint64_t* trailing);

/* --- compression::compressor::uncompress (compression/compression.cc:34-55)
 *     for lz4 (lz4_frame_compressor.cc:115-213) and snappy
 *     (snappy_java_compressor.cc:76-129, snappy_standard_compressor.cc:43-78).
 *     Return 0 ok, -1 where the reference throws, -2 if cap too small. */
int rpo_lz4f_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
int rpo_snappy_raw_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
int rpo_snappy_java_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
int rpo_uncompress(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
/* gzip_compressor::uncompress (compression/internal/gzip_compressor.cc:
 * 161-230) over zlib 1.2.11 inflate (inflateInit2(15 + 32): gzip or zlib
 * wrapper): a restatement of zlib's inflate state machine.  *out_len = the
 * bytes the stream yields (the reference's sizing pass: everything decoded
 * before the end of the first member, an error, or the end of the input);
 * at most cap of them are written.  0 ok, -1 where the reference throws
 * (Z_DATA_ERROR / Z_NEED_DICT), -2 when cap is too small. */
int rpo_gzip_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
/* LZ4 block (lz4 1.9.3 LZ4_decompress_safe_usingDict): history = bytes
 * immediately before dst that matches may reference (0 for independent). */
int rpo_lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap,
                         size_t history);
/* decode-arena reservation for one compressed payload (engine plan rule,
 * shared with the GPU planner; see DESIGN.md "decode arena") */
uint64_t rpo_decode_capacity(int codec, const uint8_t* src, size_t n);
/* the same for a gzip member (the engine's sizing pass) and a host-decoded
 * zstd payload */
uint64_t rpo_gzip_plan(const uint8_t* src, size_t n);
uint64_t rpo_zstd_plan(const uint8_t* src, size_t n);
/* stream_zstd::do_uncompress (compression/stream_zstd.cc:152-178) over
 * libzstd (dlopen'd); -3 when libzstd is absent */
int rpo_zstd_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* --- segment pipeline: continuous_batch_parser::consume
 *     (storage/parser.cc:96-254) driving checksumming_consumer
 *     (storage/log_replayer.cc:27-91) plus decompress_batch
 *     (storage/parser_utils.cc:43-60) and the record walk. */
typedef struct rpo_job_state {
    uint64_t batch_base;      /* job-wide ordinal of the next batch */
    uint64_t index_base;      /* next free record-index slot */
    uint64_t decoded_base;    /* next free decoded-arena byte */
    uint32_t overflow;
} rpo_job_state;

/* Processes one disk-layout segment; appends to batches/index/arena.
 * Returns batches emitted (>=0) or <0 on batch-capacity overflow. */
int64_t rpo_scan_segment(const uint8_t* seg, uint64_t len, uint32_t segment, uint32_t job_flags,
                         rpgpu_batch_result* batches, uint64_t batch_cap,
                         rpgpu_record_index* index, uint64_t index_cap,
                         uint8_t* decoded, uint64_t decoded_cap,
                         rpgpu_segment_summary* summary, rpo_job_state* st);

/* Whole job over concatenated segments (the rpgpu_job contract, host memory). */
int rpo_run_job(const uint8_t* data, const uint64_t* seg_offsets, uint32_t n_segments,
                uint32_t job_flags, rpgpu_batch_result* batches, uint64_t batch_cap,
                rpgpu_record_index* index, uint64_t index_cap, uint8_t* decoded,
                uint64_t decoded_cap, rpgpu_segment_summary* summaries,
                rpgpu_job_totals* totals, uint64_t* valid_bitmap);

/* kafka::writer_serialize_batch (kafka/protocol/response_writer.h:241-276)
 * over batches [first, first + n) of a job's results; out NULL sizes */
uint64_t rpo_serialize_wire(const uint8_t* data, const uint64_t* seg_offsets, const rpgpu_batch_result* batches,
                            uint64_t first, uint64_t n, uint8_t* out);

/* validity rule behind rpgpu_job.d_valid_bitmap */
int rpo_batch_valid(const rpgpu_batch_result* b, uint32_t job_flags);
int rpo_batch_valid_layout(const rpgpu_batch_result* b, uint32_t job_flags, uint32_t layout);
int64_t rpo_scan_segment_layout(const uint8_t* seg, uint64_t len, uint32_t segment, uint32_t job_flags,
                                uint32_t layout, rpgpu_batch_result* batches, uint64_t batch_cap,
                                rpgpu_record_index* index, uint64_t index_cap,
                                uint8_t* decoded, uint64_t decoded_cap,
                                rpgpu_segment_summary* sm, rpo_job_state* st);
int rpo_run_job_layout(const uint8_t* data, const uint64_t* seg_offsets, uint32_t n_segments,
                       uint32_t job_flags, uint32_t layout, rpgpu_batch_result* batches, uint64_t batch_cap,
                       rpgpu_record_index* index, uint64_t index_cap, uint8_t* decoded,
                       uint64_t decoded_cap, rpgpu_segment_summary* summaries,
                       rpgpu_job_totals* totals, uint64_t* valid_bitmap);

/* CPU baseline: validate (crc + header crc + record walk) a segment set with
 * `threads` workers, one segment-slice per worker (Seastar shard-per-core);
 * returns batches validated, wall time in *seconds. */
int64_t rpo_baseline_validate(const uint8_t* data, const uint64_t* seg_offsets,
                              uint32_t n_segments, int threads, int use_hw_crc,
                              double* seconds, uint64_t* bytes);


/* --- segment index rebuild: checksumming_consumer::consume_batch_end
 *     (storage/log_replayer.cc:62-74) -> segment_index::maybe_track
 *     (storage/segment_index.cc:58-72) -> index_state::maybe_index
 *     (storage/index_state.cc:48-95), replayed over each segment's crc-good
 *     prefix of a completed job.  Same contract as rpgpu_segment_index. */
int rpo_segment_index(const rpgpu_batch_result* batches, uint64_t batch_cap,
                      const rpgpu_segment_summary* summaries, uint32_t n_segments, uint64_t step,
                      rpgpu_index_state* states, uint32_t* rel_offset, uint32_t* rel_time,
                      uint64_t* position);

/* Write side: header stamping in batch order (flags: 1 offsets, 2 size+crc;
 * header_crc always), see rp_oracle.c */
void rpo_stamp_batches(uint8_t* data, const uint64_t* pos, const uint32_t* plen, uint32_t n, int64_t next_offset,
                       uint32_t flags);

/* Write side: compression::compressor::compress (lz4 frame, snappy-java
 * with `frag`-byte iobuf fragments, 0 = one fragment), see rp_oracle.c */
int rpo_lz4_compress_block(const uint8_t* s, int n, uint8_t* dst, int cap);
size_t rpo_lz4f_compress_bound(size_t n);
size_t rpo_lz4f_compress(const uint8_t* s, size_t n, uint8_t* dst);
size_t rpo_snappy_compress_block(const uint8_t* s, uint32_t n, uint8_t* op);
size_t rpo_snappy_raw_compress(const uint8_t* s, size_t n, uint8_t* dst);
size_t rpo_snappy_java_compress_bound(size_t n, size_t frag);
size_t rpo_snappy_java_compress(const uint8_t* s, size_t n, size_t frag, uint8_t* dst);

#ifdef __cplusplus
}
#endif

#endif /* RP_ORACLE_H_ */
