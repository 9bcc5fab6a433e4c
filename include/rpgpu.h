/*
 * rpgpu.h — C-ABI boundary of the MI355X record-batch validation/decode engine.
 *
 * This is the drop-in boundary for Redpanda's batch hot path.
 * Every entry point below replaces one reference interface; the reference
 * file:line it stands in for is cited next to it (paths relative to
 * /root/reference/src/v).  Plain pointers and sizes only — no HIP, torch or
 * C++ types cross this boundary, and no exception ever does: every call
 * returns an int status (0 = ok, <0 = rpgpu_status).
 *
 * Layouts of the per-batch result, the per-record index and the segment
 * summary are part of the contract: the CPU oracle (oracle/) emits the same
 * structs, so parity is a memcmp.
 */
#ifndef RPGPU_H_
#define RPGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Constants                                                                 */
/* ------------------------------------------------------------------------ */

/* model::packed_record_batch_header_size (model/record.h:473-487): the
 * comment there says 57 but the fields sum to 61. */
#define RPGPU_HEADER_SIZE 61u
/* kafka::internal::kafka_header_size (kafka/protocol/kafka_batch_adapter.h:25-37) */
#define RPGPU_KAFKA_HEADER_SIZE 61u
/* bytes of the Kafka CRC prefix rebuilt big-endian from the header
 * (model/record_utils.cc:68-80: attrs..record_count) */
#define RPGPU_CRC_PREFIX_SIZE 40u

/* model::compression (model/compression.h:35-48) */
enum rpgpu_codec {
    RPGPU_CODEC_NONE = 0,
    RPGPU_CODEC_GZIP = 1,
    RPGPU_CODEC_SNAPPY = 2, /* snappy-java framing, falls back to raw snappy */
    RPGPU_CODEC_LZ4 = 3,    /* LZ4 frame */
    RPGPU_CODEC_ZSTD = 4,
};

/* storage::parser_errc (storage/parser_errc.h:18-25), same numbering. */
enum rpgpu_parser_errc {
    RPGPU_ERRC_NONE = 0,
    RPGPU_ERRC_END_OF_STREAM = 1,
    RPGPU_ERRC_HEADER_ONLY_CRC_MISSMATCH = 2,
    RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES = 3,
    RPGPU_ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER = 4,
    RPGPU_ERRC_NOT_ENOUGH_BYTES_IN_PARSER_FOR_ONE_RECORD = 5,
};

/* Library status codes (return values). */
enum rpgpu_status {
    RPGPU_OK = 0,
    RPGPU_E_INVALID = -1,      /* bad argument */
    RPGPU_E_NO_DEVICE = -2,    /* no HIP device / HIP call failed */
    RPGPU_E_NOMEM = -3,        /* device or host allocation failed */
    RPGPU_E_OVERFLOW = -4,     /* caller-provided output capacity too small */
    RPGPU_E_CODEC = -5,        /* uncompress failed (maps to std::runtime_error) */
    RPGPU_E_UNSUPPORTED = -6,  /* codec not decoded by this engine (gzip/zstd) */
    RPGPU_E_HIP = -7,          /* kernel launch / runtime error */
};
/* rpgpu_poll: the job is still running (a positive, non-error status). */
#define RPGPU_PENDING 1

/* ------------------------------------------------------------------------ */
/* Per-batch verdict flags (rpgpu_batch_result.flags).  Each bit is pinned    */
/* to one reference function ("composite verdict").         */
/* ------------------------------------------------------------------------ */
#define RPGPU_F_HEADER_OK (1u << 0)      /* read_header_impl accepted: header_crc != 0 and == internal_header_only_crc (storage/parser.cc:139-176) */
#define RPGPU_F_COMPLETE (1u << 1)       /* size_bytes-61 payload bytes present (storage/parser.cc:206-216) */
#define RPGPU_F_CRC_OK (1u << 2)         /* (uint32)hdr.crc == crc32c(BE hdr40 ++ stored payload) (storage/log_replayer.cc:62-79, model/record_utils.cc:68-91) */
#define RPGPU_F_COMPRESSED (1u << 3)     /* attrs codec != none */
#define RPGPU_F_CODEC_INVALID (1u << 4)  /* codec value 5..7: record_batch_attributes::compression() throws (model/record.h:283-300) */
#define RPGPU_F_CODEC_UNSUPPORTED (1u << 5) /* zstd in a job without RPGPU_JOB_DECODE (kept from the host-only zstd path) */
#define RPGPU_F_CODEC_OK (1u << 6)       /* compressor::uncompress succeeded (compression/compression.cc:34-55) */
#define RPGPU_F_PARSED (1u << 7)         /* a record walk was run over the (decoded) payload */
#define RPGPU_F_PARSE_ASYNC_OK (1u << 8) /* model::for_each_record completed without throwing (model/record.h:680-697) */
#define RPGPU_F_PARSE_OK (1u << 9)       /* record_batch::for_each_record: no throw AND no trailing bytes (model/record.h:616-627) */
#define RPGPU_F_INDEX_WRITTEN (1u << 10) /* record index entries [index_base, index_base+records_parsed) are valid */
#define RPGPU_F_WIRE_V2 (1u << 11)       /* wire layout: magic == 2 (kafka/protocol/kafka_batch_adapter.cc:39-43) */
#define RPGPU_F_DECODE_OVERFLOW (1u << 12) /* decoded bytes did not fit the reserved arena slot */

/* rpgpu_batch_result.parse_err: why the record walk stopped (0 = no error). */
enum rpgpu_parse_err {
    RPGPU_PARSE_ERR_NONE = 0,
    RPGPU_PARSE_ERR_ATTR_EOF = 1,        /* consume_type<int8_t> out_of_range (bytes/details/io_iterator_consumer.h:64-84) */
    RPGPU_PARSE_ERR_COPY_NEGATIVE = 2,   /* iobuf_copy with (int)len < 0 -> bad_alloc (bytes/iobuf.cc:133-157) */
    RPGPU_PARSE_ERR_HEADER_RESERVE = 3,  /* headers.reserve(count) throws (model/record_utils.cc:99) */
    RPGPU_PARSE_ERR_TRAILING = 4,        /* sync for_each_record: bytes left after record_count records */
    RPGPU_PARSE_ERR_INDEX_CAPACITY = 5,  /* more records than the reserved index slots (record_count > payload) */
};

/* Reference-environment limit for headers.reserve(header_count): libstdc++
 * throws length_error above max_size() and Seastar throws bad_alloc when the
 * shard cannot allocate count*sizeof(record_header) (=64 B).  The latter is
 * environment dependent; this engine pins it at 2 GiB of reservation. */
#define RPGPU_MAX_HEADER_RESERVE (1ll << 25)

/* ------------------------------------------------------------------------ */
/* Output layouts                                                            */
/* ------------------------------------------------------------------------ */

/* One entry per batch reached by the continuous_batch_parser chain whose
 * header passed read_header_impl (storage/parser.cc:139-176), in chain order.
 * 128 bytes. */
typedef struct rpgpu_batch_result {
    uint64_t file_pos;            /* physical offset of the header in its segment */
    int64_t base_offset;          /* record_batch_header fields as decoded by   */
    int64_t first_timestamp;      /* storage::header_from_iobuf                 */
    int64_t max_timestamp;        /* (storage/parser.cc:36-76)                  */
    int64_t producer_id;
    int32_t size_bytes;           /* stored size (header + payload) */
    int32_t record_count;
    int32_t last_offset_delta;
    int32_t base_sequence;
    uint32_t header_crc;          /* stored header_crc */
    uint32_t crc;                 /* stored crc (as uint32) */
    uint32_t crc_computed;        /* crc32c(BE hdr40 ++ stored payload) */
    uint32_t header_crc_computed; /* internal_header_only_crc(header) */
    uint32_t flags;               /* RPGPU_F_* */
    uint32_t segment;             /* segment index within the job */
    uint64_t index_base;          /* first record-index slot of this batch */
    uint64_t decoded_off;         /* offset of the decoded payload in the decoded arena (compressed batches) */
    uint32_t records_parsed;      /* records fully parsed before stop */
    uint32_t decoded_len;         /* decoded payload bytes (== stored payload len when not compressed) */
    uint32_t decoded_crc;         /* reset_size_checksum_metadata: new crc over decoded payload (storage/parser_utils.cc:114-120) */
    uint32_t decoded_header_crc;  /* reset_size_checksum_metadata: new header_crc */
    int16_t attrs;
    int16_t producer_epoch;
    int8_t type;
    uint8_t parse_err;            /* rpgpu_parse_err */
    uint16_t reserved0;
    uint64_t reserved1;
} rpgpu_batch_result;

/* One entry per parsed record (model/record_utils.cc:94-181).  Positions are
 * byte offsets inside the batch's (decoded) payload.  64 bytes. */
typedef struct rpgpu_record_index {
    uint32_t batch;               /* job-wide batch ordinal */
    uint32_t rec_pos;             /* offset of the record's length varint */
    int64_t ts_delta;             /* timestamp_delta */
    int32_t length;               /* record::size_bytes (length varint, int32) */
    int32_t offset_delta;         /* static_cast<int32_t>(offset delta varint) */
    int32_t key_len;              /* key_length as stored by model::record (int32) */
    uint32_t key_pos;             /* first key byte */
    int32_t val_len;
    uint32_t val_pos;
    int32_t hdr_count;            /* number of record headers */
    uint32_t hdr_pos;             /* first byte after the header-count varint */
    uint32_t end_pos;             /* first byte after this record */
    int8_t attrs;                 /* record attributes byte */
    uint8_t pad[3];
    uint32_t reserved[2];
} rpgpu_record_index;

/* Per segment: where and why the parser chain stopped, and the
 * log_replayer checkpoint (storage/log_replayer.cc:62-79, log_replayer.h:159-165). */
typedef struct rpgpu_segment_summary {
    uint64_t first_batch;         /* job-wide ordinal of the segment's first batch */
    uint64_t n_batches;           /* batches with a valid header on the chain */
    uint64_t terminal_pos;        /* file position where the chain stopped */
    uint64_t bytes_consumed;      /* continuous_batch_parser::_bytes_consumed */
    int32_t terminal_errc;        /* rpgpu_parser_errc that ended the chain */
    int32_t terminal_eof;         /* 1 if the stop came from a short read (input_stream::eof()) */
    int32_t has_checkpoint;       /* checkpoint fields valid */
    uint32_t first_bad;           /* chain ordinal of the first batch failing crc (== n_batches if none) */
    int64_t ckpt_last_offset;     /* checkpoint.last_offset */
    uint64_t ckpt_truncate_pos;   /* checkpoint.truncate_file_pos */
    uint64_t n_records;           /* index slots reserved for this segment */
    uint64_t reserved[2];
} rpgpu_segment_summary;

/* Whole-job totals, written by the device. */
typedef struct rpgpu_job_totals {
    uint64_t n_batches;
    uint64_t n_records;           /* index slots used */
    uint64_t decoded_bytes;       /* arena bytes reserved */
    uint64_t batch_capacity_needed;
    uint64_t record_capacity_needed;
    uint64_t decoded_capacity_needed;
    uint32_t overflow;            /* nonzero: an output capacity was too small */
    uint32_t n_rewalks;           /* discovery chunks whose speculative entry had to be re-walked */
    uint64_t reserved[2];
} rpgpu_job_totals;

/* ------------------------------------------------------------------------ */
/* Context / memory                                                          */
/* ------------------------------------------------------------------------ */

typedef struct rpgpu_ctx rpgpu_ctx;

/* Number of visible HIP devices (0 when none). */
int rpgpu_device_count(void);
/* One context per host thread or Seastar shard (ownership
 * row): it owns a HIP stream pair and device scratch.  Not thread-safe. */
int rpgpu_create(int device, rpgpu_ctx** out);
int rpgpu_destroy(rpgpu_ctx* ctx);
const char* rpgpu_strerror(int status);
const char* rpgpu_last_error(rpgpu_ctx* ctx);

int rpgpu_dev_alloc(rpgpu_ctx* ctx, size_t bytes, void** out);
int rpgpu_dev_free(rpgpu_ctx* ctx, void* p);
/* pinned host memory for the double-buffered H2D staging */
int rpgpu_host_alloc(rpgpu_ctx* ctx, size_t bytes, void** out);
int rpgpu_host_free(rpgpu_ctx* ctx, void* p);
int rpgpu_memcpy_h2d(rpgpu_ctx* ctx, void* dst, const void* src, size_t n, void* stream);
int rpgpu_memcpy_d2h(rpgpu_ctx* ctx, void* dst, const void* src, size_t n, void* stream);
int rpgpu_memset(rpgpu_ctx* ctx, void* dst, int value, size_t n, void* stream);
int rpgpu_sync(rpgpu_ctx* ctx, void* stream);

/* ------------------------------------------------------------------------ */
/* crc::crc32c (hashing/crc32c.h:19-40)                                      */
/* ------------------------------------------------------------------------ */

/* google crc32c::Extend(crc, p, n) semantics: Extend(0, p, n) is the standard
 * CRC32C (Castagnoli, reflected 0x82F63B78, init/xorout ~0).  Host-side
 * (SSE4.2) for the small per-call sizes crc::crc32c sees; bulk segment CRC
 * runs on the GPU through rpgpu_submit. Pure, thread-safe, no allocation. */
uint32_t rpgpu_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);

/* ------------------------------------------------------------------------ */
/* Segment engine (new; replaces the per-batch loops of                      */
/* storage::continuous_batch_parser::consume (storage/parser.cc:218-254),    */
/* log_replayer::recover_in_thread (storage/log_replayer.cc:95-114),         */
/* storage::internal::decompress_batch (storage/parser_utils.cc:43-60) and   */
/* kafka_batch_adapter::adapt (kafka/protocol/kafka_batch_adapter.cc:126)).  */
/* ------------------------------------------------------------------------ */

enum rpgpu_layout {
    RPGPU_LAYOUT_DISK = 0, /* Redpanda on-disk: 61-byte LE header (storage/segment_appender_utils.cc:28-54) */
    RPGPU_LAYOUT_WIRE = 1, /* Kafka v2 wire: BE header (kafka/protocol/kafka_batch_adapter.cc:32-91) */
};

#define RPGPU_JOB_CRC (1u << 0)     /* compute the payload crc (always on in recovery) */
#define RPGPU_JOB_PARSE (1u << 1)   /* walk records into the index */
#define RPGPU_JOB_DECODE (1u << 2)  /* uncompress lz4/snappy/gzip/zstd payloads into the arena (on the device) */
/* With RPGPU_JOB_DECODE: decode zstd batches on the host instead (SURVEY.md
 * §8(b)'s CPU fallback: stream_zstd::do_uncompress over libzstd,
 * compression/stream_zstd.cc:152-178), into the same arena, then CRC and walk
 * them on the device like every other decoded payload.  Same plan and
 * verdicts as the device decoder; the submit then synchronizes on its stream
 * once the chain is planned (the payloads' sizes and bytes cross to the host
 * and back), so rpgpu_submit_async returns after that point. */
#define RPGPU_JOB_HOST_CODECS (1u << 3)

/* All pointers are DEVICE pointers, caller-owned.  Segments are concatenated
 * in d_data; segment s spans [d_seg_offsets[s], d_seg_offsets[s+1]). */
typedef struct rpgpu_job {
    const uint8_t* d_data;
    const uint64_t* d_seg_offsets;   /* n_segments + 1 entries */
    const uint64_t* h_seg_offsets;   /* HOST copy of the same offsets (sizes the launch grids) */
    uint32_t n_segments;
    uint32_t layout;                 /* rpgpu_layout */
    uint32_t flags;                  /* RPGPU_JOB_* */
    uint32_t chunk_bytes;            /* discovery chunk size (0 = default 256 KiB) */
    rpgpu_batch_result* d_batches;   /* capacity batch_capacity */
    uint64_t batch_capacity;
    rpgpu_record_index* d_records;   /* capacity record_capacity (may be NULL if !PARSE) */
    uint64_t record_capacity;
    uint8_t* d_decoded;              /* decoded arena (may be NULL if !DECODE); bytes are defined only at
                                        [decoded_off, +decoded_len) of batches with RPGPU_F_CODEC_OK (the
                                        reference throws and keeps nothing for the others); 16-B aligned */
    uint64_t decoded_capacity;
    rpgpu_segment_summary* d_summaries; /* n_segments entries */
    rpgpu_job_totals* d_totals;      /* one entry */
    uint64_t* d_valid_bitmap;        /* optional: 1 bit per batch, set = crc_ok && header_ok (&& parse_ok if PARSE) */
    /* Optional chain seeds (the index-seeded mode of SURVEY.md §8(b)): known
     * batch header positions of each segment, ascending, e.g. the
     * position_index of its .base_index (storage/index_state.h:23-100,
     * index_state::hydrate_from_buffer, storage/index_state.cc:104-186).
     * Segment s's seeds are d_seeds[d_seed_offsets[s] .. d_seed_offsets[s+1]).
     * Discovery then enters each chunk by following the chain from the last
     * seed before it instead of scanning its bytes.  Seeds are verified like
     * any discovered header (a wrong or stale index only costs re-walks);
     * results are identical with or without them.  NULL = scan. */
    const uint64_t* d_seeds;
    const uint64_t* d_seed_offsets;  /* device, n_segments + 1 entries */
} rpgpu_job;

/* Enqueue the whole pipeline (discover -> resolve -> plan -> validate/decode)
 * on `stream` (hipStream_t, NULL = the context's stream).  Asynchronous:
 * results are valid after rpgpu_sync / an event on that stream.  Capacity
 * overflow is reported in d_totals (overflow != 0), never by writing out of
 * bounds. */
int rpgpu_submit(rpgpu_ctx* ctx, const rpgpu_job* job, void* stream);

/* Asynchronous completion for a reactor that must not block (SURVEY.md
 * §8(b) segment-engine row; storage::continuous_batch_parser::consume
 * returns a future, storage/parser.h:94-136): the same pipeline as
 * rpgpu_submit, plus a completion event on the launch stream.
 * rpgpu_poll is non-blocking: RPGPU_OK once every output is written,
 * RPGPU_PENDING while the job runs, < 0 on a device error.  rpgpu_wait
 * blocks until then.  rpgpu_release frees the handle (after completion or
 * not: the job itself is not cancelled). */
typedef struct rpgpu_pending rpgpu_pending;
int rpgpu_submit_async(rpgpu_ctx* ctx, const rpgpu_job* job, void* stream, rpgpu_pending** out);
int rpgpu_poll(rpgpu_pending* p);
int rpgpu_wait(rpgpu_pending* p);
int rpgpu_release(rpgpu_pending* p);

/* Output sizes a job needs, before it runs (the segment-engine row's "sized
 * by a query call").  Reads only d_data, d_seg_offsets, h_seg_offsets,
 * n_segments, layout, flags and chunk_bytes of `job`; the chain is
 * discovered and planned into context scratch.  Synchronous on `stream`. */
typedef struct rpgpu_capacity {
    uint64_t n_batches;          /* batch_capacity needed */
    uint64_t record_capacity;    /* record index slots needed (RPGPU_JOB_PARSE) */
    uint64_t decoded_capacity;   /* decoded arena bytes needed (RPGPU_JOB_DECODE; 0 otherwise) */
    uint64_t reserved;
} rpgpu_capacity;
int rpgpu_query_capacity(rpgpu_ctx* ctx, const rpgpu_job* job, void* stream, rpgpu_capacity* out);

/* Device time of the pipeline stages, measured with HIP events recorded on
 * the launch stream, averaged over every timed rpgpu_submit since the
 * previous call (milliseconds; the call resets the average).  Indices:
 * 0 = whole pipeline, 1 = discover, 2 = resolve+emit+plan, 3 = validate,
 * 4 = decode (0 when the job has no RPGPU_JOB_DECODE), 5 = lane record walk
 * of stored payloads (k_walk; 0 without RPGPU_JOB_PARSE). */
int rpgpu_last_timings(rpgpu_ctx* ctx, float* ms, int n);
/* Enable/disable per-kernel event timing (off by default). */
int rpgpu_set_timing(rpgpu_ctx* ctx, int enable);

/* ------------------------------------------------------------------------ */
/* storage::segment_index rebuild during recovery                            */
/* (checksumming_consumer::consume_batch_end -> segment_index::maybe_track,  */
/* storage/log_replayer.cc:62-74, storage/segment_index.cc:58-72 ->          */
/* index_state::maybe_index, storage/index_state.cc:48-95).                  */
/* ------------------------------------------------------------------------ */

/* segment_index::default_data_buffer_step (storage/segment_index.h:49) */
#define RPGPU_INDEX_DEFAULT_STEP 32768u

/* Per segment: the index_state header fields (storage/index_state.h:37-65)
 * after replaying maybe_track over the segment's crc-good batch prefix
 * [0, summary.first_bad).  64 bytes. */
typedef struct rpgpu_index_state {
    int64_t base_offset;          /* IN: the segment's base offset (index_state.base_offset, kept by reset()) */
    int64_t max_offset;           /* last tracked batch's last_offset */
    int64_t base_timestamp;       /* first tracked batch's first_timestamp */
    int64_t max_timestamp;        /* max over tracked batches of max(first_timestamp, max_timestamp) */
    uint64_t first_entry;         /* entries of this segment live at [first_entry, first_entry + n_entries)
                                     of the entry arrays (== summary.first_batch) */
    uint64_t n_entries;           /* relative_offset_index.size() */
    int64_t assert_batch;         /* -1, or the segment ordinal of the first tracked batch whose
                                     base_offset < base_offset: the reference vasserts (aborts) there,
                                     so tracking stops before it */
    uint64_t tracked;             /* batches replayed through maybe_track */
} rpgpu_index_state;

/* Device pointers.  d_batches/d_summaries are the outputs of a completed
 * disk-layout rpgpu_submit (same stream, or synchronised).  d_states has
 * n_segments entries with base_offset filled in by the caller.  The three
 * entry arrays (relative_offset_index, relative_time_index, position_index)
 * need batch_capacity slots each.  step = segment_index::_step. */
int rpgpu_segment_index(rpgpu_ctx* ctx, const rpgpu_batch_result* d_batches, uint64_t batch_capacity,
                        const rpgpu_segment_summary* d_summaries, uint32_t n_segments, uint64_t step,
                        rpgpu_index_state* d_states, uint32_t* d_rel_offset, uint32_t* d_rel_time,
                        uint64_t* d_position, void* stream);

/* ------------------------------------------------------------------------ */
/* Write side: header stamping of batches about to be written (SURVEY.md     */
/* §8(f) row 3)                                                              */
/* ------------------------------------------------------------------------ */
/* disk_log_appender::operator() (storage/disk_log_appender.cc:72-74): the
 * batch gets the appender's next offset as base_offset, the appender moves
 * on to last_offset + 1 (:113-119). */
#define RPGPU_STAMP_OFFSETS (1u << 0)
/* storage::internal::reset_size_checksum_metadata (storage/parser_utils.cc:
 * 114-120): size_bytes = 61 + payload bytes, crc = crc_record_batch. */
#define RPGPU_STAMP_CRC (1u << 1)

/* n disk-layout batches in the device buffer d_data (16-byte aligned, with 16
 * readable bytes past the last payload): batch i's 61-byte header at
 * d_pos[i], its payload (d_payload_len[i] bytes) right after it.  In place,
 * in batch order: RPGPU_STAMP_OFFSETS numbers them from next_offset,
 * RPGPU_STAMP_CRC resets size and crc, and header_crc
 * (model::internal_header_only_crc) is always recomputed last.  Batches must
 * not overlap.  Asynchronous on `stream`. */
int rpgpu_stamp(rpgpu_ctx* ctx, uint8_t* d_data, const uint64_t* d_pos, const uint32_t* d_payload_len, uint32_t n,
                int64_t next_offset, uint32_t flags, void* stream);

/* kafka::writer_serialize_batch (kafka/protocol/response_writer.h:241-276)
 * for batches [first, first + n) of a completed disk-layout job (its
 * d_batches, over the job's d_data / d_seg_offsets): each batch's Kafka v2
 * wire header (big endian; batch_length = size_bytes - 12, partition leader
 * epoch 0, magic 2, the stored crc) followed by its payload, back to back in
 * d_wire (capacity: the batches' size_bytes summed).  *d_total (a device
 * u64) receives the record set's length.  Asynchronous on `stream`. */
int rpgpu_serialize_wire(rpgpu_ctx* ctx, const uint8_t* d_data, const uint64_t* d_seg_offsets,
                         const rpgpu_batch_result* d_batches, uint64_t first, uint32_t n, uint8_t* d_wire,
                         uint64_t* d_total, void* stream);

/* ------------------------------------------------------------------------ */
/* compression::compressor::uncompress (compression/compression.h:21-24)     */
/* ------------------------------------------------------------------------ */

/* Decode one payload (host pointers).  LZ4 and snappy run on the device;
 * gzip and zstd run on the host, the reference's own loops over zlib /
 * libzstd (gzip_compressor.cc:161-230, stream_zstd.cc:152-178: the CPU
 * fallback of SURVEY.md §8(b)).  *out_len receives the decoded size;
 * returns RPGPU_E_CODEC where the reference throws std::runtime_error,
 * RPGPU_E_OVERFLOW if cap is too small (out_len then holds the size needed),
 * RPGPU_E_UNSUPPORTED when zlib / libzstd cannot be loaded.  ctx may be
 * NULL for gzip / zstd (no device work). */
int rpgpu_uncompress(rpgpu_ctx* ctx, int codec, const void* in, size_t n,
                     void* out, size_t cap, size_t* out_len);

/* n payloads in one device round trip (the per-batch call sites
 * storage/parser_utils.cc:51 and kafka/protocol/kafka_batch_adapter.cc:259,
 * batched).  Arrays of n entries; status[i] is what rpgpu_uncompress would
 * return for payload i.  Returns RPGPU_OK when every payload has a status. */
int rpgpu_uncompress_batch(rpgpu_ctx* ctx, uint32_t n, const int* codecs, const void* const* in,
                           const size_t* in_len, void* const* out, const size_t* cap, size_t* out_len,
                           int* status);

/* ------------------------------------------------------------------------ */
/* compression::compressor::compress (compression/compression.cc:17-33): the */
/* write side's storage::internal::compress_batch (storage/parser_utils.cc:   */
/* 97-111).  SURVEY.md §8(f) row 3.                                          */
/* ------------------------------------------------------------------------ */

/* Bytes compressor::compress can produce for n input bytes: the LZ4 frame
 * (lz4_frame_compressor.cc:72-113) or the snappy-java stream over frag-byte
 * iobuf fragments (snappy_java_compressor.cc:58-75; frag 0 = one fragment),
 * or a safe bound for the host gzip / zstd streams.  0 for RPGPU_CODEC_NONE. */
size_t rpgpu_compress_bound(int codec, size_t n, size_t frag);

/* n payloads compressed on the device in one round trip (host pointers), the
 * bytes liblz4 1.9.3 / libsnappy 1.1.8 produce through the reference's
 * wrappers, bit for bit: RPGPU_CODEC_LZ4 -> LZ4 frame {independent 64 KiB
 * blocks, content size, level 1}; RPGPU_CODEC_SNAPPY -> snappy-java with one
 * chunk per frag[i]-byte fragment (frag may be NULL: one fragment, a
 * contiguous iobuf).  status[i]: RPGPU_OK; RPGPU_E_OVERFLOW when cap[i] <
 * the output (out_len[i] then holds its size); RPGPU_E_CODEC for
 * RPGPU_CODEC_NONE (the reference throws "nothing to compress").  gzip and
 * zstd run on the host, the reference's loops over zlib / libzstd
 * (gzip_compressor.cc:126-161, stream_zstd.cc:84-104; RPGPU_E_UNSUPPORTED
 * when the library cannot be loaded). */
int rpgpu_compress_batch(rpgpu_ctx* ctx, uint32_t n, const int* codecs, const void* const* in, const size_t* in_len,
                         const size_t* frag, void* const* out, const size_t* cap, size_t* out_len, int* status);

/* ------------------------------------------------------------------------ */
/* Host segment path (log_replayer over files, storage/log_replayer.cc:       */
/* 95-114): pinned, double-buffered H2D of host-resident segments.  Segments */
/* are copied in staging groups on a copy stream while the previous group    */
/* validates, and each group's outputs come back while the next one runs.    */
/* Outputs are HOST pointers and hold exactly what ONE rpgpu_submit over all */
/* the segments returns: job-wide batch ordinals (record_index.batch),       */
/* index_base, decoded_off and summary.first_batch.                          */
/* ------------------------------------------------------------------------ */
typedef struct rpgpu_host_job {
    const uint8_t* const* segments;  /* host pointers (pinned or pageable) */
    const uint64_t* seg_sizes;
    uint32_t n_segments;
    uint32_t layout;
    uint32_t flags;
    uint32_t group_kib;              /* staging group size in KiB (0 = 256 MiB): segments are copied and
                                        validated in groups of at most this many bytes (a larger segment
                                        is a group of its own) */
    rpgpu_batch_result* batches;     /* host, capacity batch_capacity */
    uint64_t batch_capacity;
    rpgpu_segment_summary* summaries; /* host, n_segments */
    rpgpu_job_totals* totals;        /* host */
    /* optional (NULL / 0: not returned): the per-record index
     * (RPGPU_JOB_PARSE) and the decoded arena (RPGPU_JOB_DECODE); a capacity
     * that is too small sets totals.overflow bit 2 / 4, as on the device */
    rpgpu_record_index* records;
    uint64_t record_capacity;
    uint8_t* decoded;
    uint64_t decoded_capacity;
    /* optional segment index rebuild (rpgpu_segment_index over each group's
     * results, disk layout): index_step != 0 fills index_states[n_segments]
     * (base_offset is an IN field) and the three entry arrays (batch_capacity
     * entries each; segment s's entries at [first_entry, first_entry +
     * n_entries), first_entry == its summary.first_batch) */
    uint64_t index_step;
    rpgpu_index_state* index_states;
    uint32_t* rel_offset;
    uint32_t* rel_time;
    uint64_t* position;
} rpgpu_host_job;

int rpgpu_validate_host(rpgpu_ctx* ctx, const rpgpu_host_job* job);

/* Decoded-size plan of one lz4 / snappy payload from its frame structure
 * alone (the arena rule rpgpu_submit reserves per batch): an upper bound of
 * what compressor::uncompress returns for a payload it accepts; 0 for an
 * empty, unplannable or gzip / zstd payload (the caller then grows on
 * RPGPU_E_OVERFLOW).  Host only, no context. */
uint64_t rpgpu_uncompress_bound(int codec, const void* in, size_t n);

/* rpgpu_stamp over a HOST buffer, in place (storage::stamp_batches): staged
 * through the context's pinned and device scratch (grow-only), one H2D, the
 * kernels, one D2H.  Synchronous.  d_pos / d_payload_len as rpgpu_stamp,
 * but host arrays. */
int rpgpu_stamp_host(rpgpu_ctx* ctx, uint8_t* buf, size_t len, const uint64_t* pos, const uint32_t* payload_len,
                     uint32_t n, int64_t next_offset, uint32_t flags);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RPGPU_H_ */
