/*
 * rpgen.h — synthetic Redpanda segment generator (test and benchmark data).
 *
 * NOT part of the product: librpgen.so is loaded by tests/, bench.py and
 * __graft_entry__.smoke() to make seeded workloads of the BASELINE.json
 * configurations.  It follows the reference's test batch
 * recipe (storage/tests/utils/random_batch.cc:50-154) and compresses through
 * the reference's codec libraries (liblz4 / libsnappy / zlib / libzstd,
 * loaded with dlopen).  The engine (librpgpu.so) never links it.
 */
#ifndef RPGEN_H_
#define RPGEN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* codec slots of rpgen_spec.codec_weights */
enum rpgen_codec_slot {
    RPGEN_NONE = 0,
    RPGEN_GZIP = 1,        /* gzip member (zlib deflate, as gzip_compressor.cc writes) */
    RPGEN_SNAPPY_JAVA = 2, /* xerial snappy-java framing (snappy_java_compressor.cc:57-74) */
    RPGEN_LZ4 = 3,         /* LZ4 frame (lz4_frame_compressor.cc:69-113) */
    RPGEN_ZSTD = 4,        /* zstd frame */
    RPGEN_SNAPPY_RAW = 5,  /* raw snappy block under codec 2 (snappy_standard_compressor) */
    RPGEN_SLOTS = 6,
};

typedef struct rpgen_spec {
    uint64_t seed;
    uint64_t segment_bytes;          /* exact bytes per segment */
    uint32_t batch_bytes;            /* target size_bytes per batch (0 = variable, see min/max) */
    uint32_t min_batch_bytes;        /* variable mode: log-uniform in [min, max] (decoded size for codecs) */
    uint32_t max_batch_bytes;
    uint32_t value_bytes;            /* approximate record value size */
    uint32_t key_bytes;
    uint32_t headers_per_record;
    uint32_t codec_weights[RPGEN_SLOTS]; /* relative weights; all zero = uncompressed only */
    uint32_t lz4_linked_ppm;         /* LZ4 frames with linked blocks, per million LZ4 batches */
    uint32_t lz4_content_checksum_ppm;
    uint32_t lz4_block_checksum_ppm;
    uint32_t corrupt_ppm_payload;    /* payload bit flips per million batches */
    uint32_t corrupt_ppm_header;     /* header bit flips per million batches */
    uint32_t corrupt_ppm_zero;       /* zeroed headers per million batches */
    uint32_t truncate_tail;          /* 1: the batch that does not fit is written cut at the segment end */
    uint32_t size_uniform;           /* variable mode: 1 = uniform in [min, max] instead of log-uniform */
    int64_t base_offset;
} rpgen_spec;

/* Fill `out` (segment_bytes) with one segment; returns the number of batches
 * written whole, or <0.  Without truncate_tail the room that cannot hold
 * another batch is zero-filled (fallocated). */
int64_t rpgen_segment(const rpgen_spec* spec, uint32_t segment_index, uint8_t* out);

/* CRC32C (Castagnoli) extend, host SSE4.2. */
uint32_t rpgen_crc32c(uint32_t crc, const uint8_t* p, uint64_t n);

#ifdef __cplusplus
}
#endif

#endif /* RPGEN_H_ */
