// rp_internal.h — shared between the device kernels (rp_kernels.hip) and the
// host runtime (rp_runtime.hip).  Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rpgpu.h"

namespace rp {

constexpr uint64_t kNone = ~0ull;
constexpr uint32_t kCrcPoly = 0x82F63B78u;

// CRC chunking of the validate kernel: every lane owns two consecutive
// streams of kStream bytes; a wave round covers 64 * 2 * kStream bytes.
constexpr uint32_t kStream = 128;
constexpr uint32_t kLaneBytes = 2 * kStream;       // 256
constexpr uint32_t kRoundBytes = 64 * kLaneBytes;  // 16 KiB
constexpr uint32_t kCombineLevels = 7;             // shift by kStream * 2^l, l = 0..6

// LDS image of the validate kernel (bytes).
//  [0, 128 KiB): slice-by-4 CRC tables replicated 32x so lane L always hits
//                bank L%32 (2 tables per 256-byte row: see rp_kernels.hip)
//  [128 KiB, 156 KiB): combine tables, 7 levels x 4 byte-tables x 256
constexpr uint32_t kLdsSliceBytes = 128u << 10;
constexpr uint32_t kLdsCombineOff = kLdsSliceBytes;
constexpr uint32_t kLdsCombineBytes = kCombineLevels * 4 * 256 * 4;
constexpr uint32_t kLdsValidateBytes = kLdsCombineOff + kLdsCombineBytes;

// Constant tables, built on the host once per context.
struct Tables {
    uint32_t slice[4][256];          // T_k[b]: byte b followed by k zero bytes (raw CRC)
    uint32_t hdr[57][256];           // T_d for d = 0..56 (parallel header CRC)
    uint32_t comb[kCombineLevels][4][256]; // shift by kStream*2^l bytes, per state byte
    uint32_t c57;                    // state 0xFFFFFFFF advanced over 57 zero bytes
    uint32_t c40;                    // state 0xFFFFFFFF advanced over 40 zero bytes
    uint32_t pad[2];
};

// Discovery record per chunk (speculative walk), 32 bytes.
struct ChunkRec {
    uint64_t entry;   // first header position found in the chunk (kNone if none)
    uint64_t exit;    // first chain position >= chunk end, or terminal position
    uint32_t count;   // batches (with valid header) whose header starts in the chunk
    int32_t term;     // -1: ran through; else parser errc | (eof << 8)
    uint64_t tpos;    // terminal position when term >= 0
};

// Per-segment resolve output.
struct SegTerm {
    uint64_t pos;
    int32_t errc;
    int32_t eof;
};

struct DeviceJob {
    const uint8_t* data;
    uint64_t data_len;            // bytes of d_data (= h_seg_offsets[n_segments])
    const uint64_t* seg_off;      // n_segments + 1
    const uint64_t* chunk_base;   // n_segments + 1 : first global chunk index of each segment
    uint32_t n_segments;
    uint32_t flags;
    uint32_t chunk_bytes;
    uint32_t total_chunks;
    ChunkRec* chunks;
    uint64_t* chunk_count;        // total_chunks (+1) : resolved counts -> exclusive scan in place
    uint64_t* chunk_entry;        // total_chunks : resolved entry position
    SegTerm* seg_term;
    rpgpu_batch_result* batches;
    uint64_t batch_capacity;
    uint64_t* slots;              // batch_capacity (+1): planned index slots -> scan
    uint64_t* dcap;               // batch_capacity (+1): planned decode bytes -> scan
    rpgpu_record_index* records;
    uint64_t record_capacity;
    uint8_t* decoded;
    uint64_t decoded_capacity;
    rpgpu_segment_summary* summaries;
    rpgpu_job_totals* totals;
    uint64_t* bitmap;
    const Tables* tables;
    uint32_t* counters;           // [0]: rewalks, [1]: overflow bits
};

// kernel launchers (rp_kernels.hip)
hipError_t launch_chunk_base(const DeviceJob& j, hipStream_t s);
hipError_t launch_discover(const DeviceJob& j, hipStream_t s);
hipError_t launch_resolve(const DeviceJob& j, hipStream_t s);
hipError_t launch_emit(const DeviceJob& j, hipStream_t s);
hipError_t launch_validate(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_finalize(const DeviceJob& j, hipStream_t s);
hipError_t scan_exclusive_u64(uint64_t* data, uint64_t n, void* temp, size_t temp_bytes, hipStream_t s);
// n = min(*d_n, n_cap), read on the device
hipError_t scan_exclusive_u64_devn(uint64_t* data, const uint64_t* d_n, uint64_t n_cap, void* temp, hipStream_t s);
size_t scan_temp_bytes(uint64_t n);

}  // namespace rp
