// rp_internal.h — shared between the device kernels (rp_kernels.hip) and the
// host runtime (rp_runtime.hip).  Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rpgpu.h"

namespace rp {

constexpr uint64_t kNone = ~0ull;
constexpr uint32_t kCrcPoly = 0x82F63B78u;

// Shift tables: advance a raw CRC state over 16 << m zero bytes (m = 0..5):
// the cross-lane merge tree of the validate kernel.
constexpr uint32_t kShiftLevels = 6;
// Braid stride of the validate kernel: lane l's 16 bytes of window row i sit
// at 1024 i + 16 l, so a braid word is followed by 1020 bytes of other braids.
constexpr uint32_t kBraidSkip = 1020;

// Validate kernel (rp_validate.hip): one wave per batch, 16 waves per
// workgroup (4 per SIMD), one workgroup per CU.  A payload is processed in
// 16 KiB windows of 16 rows of 1 KiB: lane l holds bytes [1024 i + 16 l, +16)
// of every row i (one coalesced dwordx4 load per row).
constexpr uint32_t kVWaves = 16;
constexpr uint32_t kWinBytes = 16384;
// LDS image of the validate kernel (bytes):
//  [0, 128 KiB)    braid tables T1023..T1020 (byte followed by 1023..1020
//                  zero bytes),
//                  32 copies so lane L always hits bank L % 32: two 64 KiB
//                  row-sets, entry e row = 256 B, table A at [0,128) and
//                  table B at [128,256), copy c at 4c
//  [128, 132 KiB)  slice tables T3..T0 (single copy): word/byte steps
//  [132, 156 KiB)  shift tables: 6 levels, shift by 16 << m bytes
constexpr uint32_t kLdsBraidOff = 0;
constexpr uint32_t kLdsSlice4Off = 131072;
constexpr uint32_t kLdsShiftOff = kLdsSlice4Off + 4096;
constexpr uint32_t kLdsValidateBytes = kLdsShiftOff + kShiftLevels * 4096;
static_assert(kLdsValidateBytes <= 160u * 1024u, "validate LDS image exceeds 160 KiB");

// Constant tables, built on the host once per context.
struct Tables {
    uint32_t slice[4][256];          // T_k[b]: byte b followed by k zero bytes (raw CRC)
    uint32_t hdr[57][256];           // T_d for d = 0..56 (parallel header CRC)
    uint32_t braid[4][256];          // T_{1023-t}[b]: byte b followed by 1023 - t zero bytes
    uint32_t shift[kShiftLevels][4][256]; // state byte j (value b << 8j) over 16 << m zero bytes
    uint32_t c57;                    // state 0xFFFFFFFF advanced over 57 zero bytes
    uint32_t c40;                    // state 0xFFFFFFFF advanced over 40 zero bytes
    uint32_t pad[2];
    // streaming CRC of decoded output (k_lz_exec): lane l's 16-byte state
    // moved to its 1 KiB row end, x^(8 * 16 (63 - l)); and the inverse
    // shifts x^(-8 z) (z = 0..1023) that take a zero-padded last row back to
    // the true end
    uint32_t lane_rowend[64];
    uint32_t inv_shift[1024];
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

// One piece of a planned compressed payload: an LZ4F block, a snappy-java
// chunk, or a whole raw snappy stream.  Independent pieces decode into their
// planned arena position; the blocks of a linked LZ4F frame are decoded in
// order by one wave, which rewrites `dst` with the position each landed at.
struct BlockItem {
    uint64_t src;    // absolute offset of the block data in the job's data
    uint64_t dst;    // absolute offset in the decoded arena (planned; actual for linked blocks)
    uint32_t csize;  // block data bytes
    uint32_t kind;   // kBlk* bits
    int32_t out;     // decoded bytes, -1 on failure (written by k_lz_exec)
    uint32_t cap;    // bytes reserved at dst (LZ4: the block maximum = the decoder's output bound)
    uint32_t crc;    // linear CRC32C (zero state, no final xor) of the decoded bytes, from k_lz_exec's
                     // flush; a linked frame's whole output on its first block
    uint32_t fast;   // kLzf*: walked by k_lzf_walk (executed from its records by k_lz_exec)
};
// BlockItem.fast: 0 k_lz_walk walks it; kLzfListed the planner gave it to
// k_lzf_walk (frecs reserved: PieceState.first_slab); kLzfReady walked into
// frecs by k_lzf_walk + k_lzf_tail (k_lz_exec executes those records);
// kLzfReject rejected there (out = -1 written)
// kLzfRaw: an independent raw block k_raw_copy copies (out / crc written there)
constexpr uint32_t kLzfNone = 0, kLzfReady = 1, kLzfReject = 2, kLzfListed = 3, kLzfRaw = 4;
// kBlkWhole: a raw (non-xerial) snappy payload, snappy_standard_compressor
// semantics (length 0 is an empty result whatever follows)
constexpr uint32_t kBlkRaw = 1, kBlkChecksum = 2, kBlkSnappy = 4, kBlkLinked = 8, kBlkWhole = 16;

// One parsed sequence of an LZ4 block / snappy tag: literal bytes
// [lip, lip + ll) of the piece's stream, then ml bytes copied from `off`
// back (ml = 0: literal only).  Written by the parse phase of k_lz_exec,
// executed by its wave phase.
struct SeqRec {
    uint32_t lip, ll, ml, off;
};
// k_lz_walk stores each piece's records in slabs of kSlabRecs taken from
// one pool (bump counter); slab_next chains a piece's slabs
constexpr uint32_t kSlabRecs = 512;
constexpr uint32_t kRecsPerLane = 256;                // k_lz_exec's own walk (pool exhausted): records per pass
// k_lz_exec waves (one LDS ring each) per CU: one workgroup of that many
// waves per CU, as compiled into rp_codec.hip (its ring size decides it)
uint32_t lz_exec_wgs_per_cu();

// A piece's walk result (k_lz_walk -> k_lz_exec)
struct PieceState {
    int32_t ip, op, need, st;   // the walk's PState (st: 1 done, -1 rejected, 0 suspended: pool exhausted)
    uint32_t ulen, safe;
    uint32_t nrec;              // records stored
    uint32_t first_slab;        // 0xFFFFFFFF: none
};

// Per decode item: how its payload is being decoded
struct FramePlan {
    uint32_t mode;   // 0 decoded whole by one wave, 1 LZ4F blocks, 2 snappy-java chunks, 3 no arena room
    uint32_t first;  // first BlockItem
    uint32_t nb;     // number of BlockItems
    uint32_t ccs;    // LZ4F: content checksum present
    uint64_t content_size;  // LZ4F: content size (0 = absent)
    uint32_t ccs_val;       // LZ4F: stored content checksum
    uint32_t csf;           // LZ4F: content size present
    uint32_t xxh;           // k_content_xxh's verdict: 0 not taken, 1 match, 2 mismatch
    uint32_t pad;
};

// zstd members parsed into records (rp_inflate.hip zstd_fast_item): inf_state
// kZsFast, inf_off -> a ZsFastDesc in the scratch pool; k_zexec (rp_codec.hip)
// executes them into their arena slots
constexpr uint32_t kZsFast = 3;
constexpr uint32_t kZsFastHdr = 128;  // descriptor bytes before the literal buffer
struct ZsFastDesc {
    uint64_t nlit, nrec, lit_off, rec_off;  // literal bytes, records; offsets from the descriptor
    uint64_t lcap, rcap;                    // literal buffer / record array capacities (k_zplan's header walk)
    uint64_t items, nitems;                 // the member's Huffman literal blocks (ZsLitItem), offset from the descriptor
    uint64_t sitems, nsitems;               // its sequence sections (ZsSeqItem)
    uint64_t pad[6];
};
static_assert(sizeof(ZsFastDesc) == kZsFastHdr, "descriptor size");
// One block's sequence section, planned by k_zplan (its three FSE tables
// snapshot, the stream) and decoded ahead by k_zlits into 16-byte raw
// sequences (rp_zstd_core.h RawSeq: lengths and the offset code), which the
// lane parser then only applies
struct ZsSeqItem {
    uint64_t src, n;   // member payload (offset in d_data), bytes
    uint64_t seqs;     // scratch offset of its raw sequences
    uint64_t tab;      // scratch offset of the ll / of / ml table snapshot
    uint64_t sp, sn;   // stream start (member offset), bytes
    uint32_t nseq, llog, olog, mlog;
    uint32_t status;   // 0 not decoded, 1 decoded and the stream ended exactly, 2 decoded, it did not
    uint32_t pad;
};
constexpr uint64_t kZsSeqTab = 10240;  // ll[512] + of[256] + ml[512] SeqSyms
// One block's Huffman literal section, planned by k_zplan (table snapshot,
// stream bounds, where its literals go) and decoded ahead by k_zlits, one
// wave per block, while k_zparse later only takes the bytes
struct ZsLitItem {
    uint64_t src;      // member payload (offset in d_data)
    uint64_t n;        // member bytes
    uint64_t lits;     // scratch offset of the block's literals
    uint64_t tab;      // scratch offset of the Huffman table snapshot (1 << hlog entries)
    uint64_t s0[4];    // stream starts (member offsets)
    uint32_t sn[4];    // stream bytes
    uint32_t cnt[4];   // symbols per stream
    uint32_t lsz, seg, ns, hlog, x2;
    uint32_t status;   // 0 not decoded, 1 decoded and every stream ended exactly, 2 decoded, a stream did not
};
constexpr uint32_t kZsPlanned = 5;  // inf_state: k_zplan sized and planned the member for k_zparse
// inf_state: a zstd member whose decode reached into the overwritten part of
// the previous ring segment (zs::RingDirtyHook): k_zexact decodes it over the
// exact DCtx-buffer environment (first pass), and again into its arena slot
// when it outgrew the scratch slot (kZsExactAgain)
constexpr uint32_t kZsExact = 6, kZsExactAgain = 7;

// one chunk of a large gzip member decoded on its own wave (rp_inflate.hip,
// k_gzsplan / k_gzsfind / k_gzsdecode / k_gzsresolve)
struct GzsItem {
    uint32_t member;     // inf_list index (~0: unused)
    uint32_t k, nk;      // chunk ordinal, chunks of the member
    int32_t status;      // k_gzsdecode's verdict (0: not decoded)
    uint64_t begin, end; // deflate bytes searched for the chunk's first block header
    uint64_t start;      // bit offset of that block (~0: none found)
    uint64_t stop;       // bit offset the decode ended at
    uint64_t out;        // pool offset (symbols) of the decoded symbols
    uint64_t len;        // symbols decoded
    uint64_t guess;      // the member's output guess (sizes the region)
    uint32_t cap, pad;   // region symbols
};
#ifndef RPGPU_GZS_MIN  // (A/B variants: scripts/build_exp.py -DRPGPU_GZS_MIN=... / -DRPGPU_GZS_CHUNK=...)
#define RPGPU_GZS_MIN 16384
#endif
#ifndef RPGPU_GZS_CHUNK
#define RPGPU_GZS_CHUNK 16384
#endif
constexpr uint64_t kGzsMin = RPGPU_GZS_MIN;      // stored gzip payloads this large take the split decode
constexpr uint64_t kGzsChunk = RPGPU_GZS_CHUNK;  // deflate bytes per chunk
constexpr uint32_t kGzsMaxK = 256;     // chunks per member at most

// job counters (DeviceJob::counters), zeroed per submit
constexpr size_t kCounterBytes = 256;

struct DeviceJob {
    const uint8_t* data;
    uint64_t data_len;            // bytes of d_data (= h_seg_offsets[n_segments])
    const uint64_t* seg_off;      // n_segments + 1
    const uint64_t* chunk_base;   // n_segments + 1 : first global chunk index of each segment
    uint32_t n_segments;
    uint32_t flags;
    uint32_t layout;              // rpgpu_layout
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
    uint32_t* counters;           // [0] rewalks, [1] overflow bits, [2] decode items, [3] split batches,
                                  // [4] block items reserved, [5] sequential-frame claim cursor,
                                  // [6] sequential frames, [7] linked frames, [8] k_lz_exec claim cursor,
                                  // [9] slab pool cursor, [10] k_lz_walk lane_list cursor, [11] long pieces,
                                  // [12] (unused), [13] k_validate_decoded claim cursor,
                                  // [14] k_decode_finish claim cursor, [15] k_crc_split claim cursor,
                                  // [16] gzip / zstd members (inf_list), [17] k_members_first / [18] k_members claim cursors,
                                  // [19] host-decoded members (host_list), [20] k_members_first's second claim cursor,
                                  // [21] k_zexec claim cursor, [22] / [23] k_zparse claim cursors, [26] k_zfallback claim cursor,
                                  // [28] planned literal blocks (zs_items), [29] k_zlits / [30] k_zplan claim cursors,
                                  // [32] gzip split items (gzs_items), [33] / [34] / [35] k_gzsfind / k_gzsdecode /
                                  // k_gzsresolve claim cursors, [36..37] gzs_pool symbols used (u64),
                                  // [38] / [39] wlong_list count / cursor, [40] raw_list count, [41] lane_list count,
                                  // [42..43] frecs used (u64), [45] lzf_list count, [46] k_lzf_walk claim cursor,
                                  // [47] lzf_tail count; [12] k_crc_compose claim cursor, [24..25] bytes
                                  // k_raw_copy copied (u64), [44] k_decode_finish's checksummed-frame claim cursor,
                                  // [27] zstd members for k_zexact, [31] k_zexact's buffers (pool offset / 16 + 1),
                                  // [48] / [49] k_members_first's claim cursors of its pass 2
    uint32_t* decode_list;        // batch_capacity: ordinals of batches to uncompress
    uint32_t* seq_list;           // batch_capacity: decode items decoded whole by one lane
    uint32_t* link_list;          // batch_capacity: decode items whose linked LZ4F blocks one wave decodes in order
    uint32_t* long_list;          // block_capacity: pieces k_lz_exec runs alone ([11] count)
    uint32_t* wlong_list;         // block_capacity: the long pieces k_lz_walk may walk one wave each (not
                                  // k_lzf_walk's; [38] count, [39] cursor)
    uint32_t* split_list;         // split_capacity: stored payloads >= kSplitMin whose CRC runs in kSplitParts
                                  // chunks on separate waves ([3] count)
    uint32_t* split_part;         // split_capacity * kSplitParts: the chunks' linear CRCs
    uint32_t split_capacity;
    uint64_t split_min;           // payloads this large are split: max(kSplitMin, 2 x the job's bytes per k_validate wave)
    SeqRec* seqs;                 // k_lz_exec's own walks: kRecsPerLane per resident wave
    uint32_t exec_waves;          // k_lz_exec waves (lz_exec_wgs_per_cu() per workgroup; sizes `seqs`)
    PieceState* pstate;           // block_capacity: walk results
    SeqRec* pool;                 // record slabs
    uint32_t crc_compose;         // k_crc_compose assembles LZ4F stored crcs from k_raw_copy's block CRCs
    uint32_t* dchain;             // k_dchain's record-chain ends of decoded payloads, at their index slots (the
                                  // record pool, free again once decode is done); nullptr = k_validate_decoded chains
    uint32_t* slab_next;          // pool_slabs: next slab of the same piece
    uint32_t pool_slabs;
    uint2* frecs;                 // LZ4 sequence records of k_lzf_walk (executed by k_lz_exec), 8 B each
    uint64_t frec_cap;            // records frecs holds
    uint32_t* lzf_list;           // block_capacity: blocks k_lzf_walk takes (planner-listed, [45] count)
    uint32_t* lane_list;          // block_capacity: the blocks k_lz_walk's lane loop considers ([41] count, [10] cursor)
    uint32_t* raw_list;           // block_capacity: independent raw blocks k_raw_copy copies ([40] count)
    uint32_t* lzf_tail;           // block_capacity: blocks whose tails k_lzf_tail runs ([47] count)
    BlockItem* blocks;            // block work list ([4] items reserved, [5] claim cursor)
    uint32_t block_capacity;
    FramePlan* plans;             // one per decode item
    uint32_t* seg_first_bad;      // n_segments: first chain ordinal failing complete && crc_ok (atomicMin)
    const uint64_t* seeds;        // optional chain seeds (index-seeded discovery), per segment ascending
    const uint64_t* seed_off;     // n_segments + 1
    uint32_t* inf_list;           // batch_capacity: ordinals of gzip / zstd batches (k_members_first / k_members)
    uint32_t* inf_state;          // batch_capacity: 0 decoded into scratch, 1 rejected, 2 decode again (k_inflate),
                                  // kZsFast parsed into records (k_zexec), 4 left by k_zparse to k_zfallback
    uint64_t* inf_off;            // batch_capacity: scratch offset of each member's first-pass output
    uint64_t* inf_total;          // batch_capacity: decoded bytes of each member
    uint8_t* inf_scratch;         // first-pass output pool (context scratch)
    uint64_t inf_scratch_bytes;
    uint64_t* inf_scratch_used;   // bump allocator of the pool (zeroed per job)
    uint32_t zs_fast;             // zstd members may take the parse / execute split (kZsFast)
    uint32_t zs_split;            // k_zparse (side stream) owns the zstd members' first pass
    uint64_t* zs_items;           // zs_items_cap: scratch offsets of the planned literal blocks (k_zplan -> k_zlits)
    uint32_t zs_items_cap;
    uint32_t* host_list;          // batch_capacity: ordinals of host-decoded (zstd) batches (RPGPU_JOB_HOST_CODECS)
    uint32_t* gzs_mem;            // 2 x batch_capacity, per member: first item, chunks | 1 << 31 once resolved
                                  // (null: no split decode, k_members_first takes every gzip member)
    GzsItem* gzs_items;           // gzs_items_cap
    uint32_t gzs_items_cap;
    uint16_t* gzs_pool;           // decoded symbols of the chunks (bytes, or 256 + a window position)
    uint64_t gzs_pool_syms;
};

// one host-decoded batch (RPGPU_JOB_HOST_CODECS): its payload, the host's
// verdict and where its bytes sit in the staging buffers
struct HostItem {
    uint64_t src;        // payload offset in d_data
    uint64_t stage;      // offset in the payload / decoded staging
    uint64_t out_len;    // decoded bytes
    uint64_t cap;        // arena reservation (0 when rejected)
    uint32_t n;          // payload bytes
    uint32_t ord;        // batch ordinal
    int32_t record_count;
    int32_t status;      // 0 decoded, -1 the reference throws
};
hipError_t launch_host_desc(const DeviceJob& j, HostItem* items, uint32_t n, hipStream_t s);
hipError_t launch_host_gather(const DeviceJob& j, const HostItem* items, uint32_t n, uint8_t* stage, hipStream_t s);
hipError_t launch_host_patch(const DeviceJob& j, const HostItem* items, uint32_t n, hipStream_t s);
hipError_t launch_host_scatter(const DeviceJob& j, const HostItem* items, uint32_t n, const uint8_t* stage,
                               hipStream_t s);

// kernel launchers (rp_kernels.hip)
hipError_t launch_chunk_base(const DeviceJob& j, hipStream_t s);
hipError_t launch_discover(const DeviceJob& j, hipStream_t s);
hipError_t launch_resolve(const DeviceJob& j, hipStream_t s);
hipError_t launch_emit(const DeviceJob& j, hipStream_t s);
hipError_t launch_validate(const DeviceJob& j, hipStream_t s, uint32_t grid, bool compose = true);  // rp_validate.hip
hipError_t launch_crc_compose(const DeviceJob& j, hipStream_t s, uint32_t grid, uint32_t waves = 16);
bool dchain_wanted(const DeviceJob& j);                                         // rp_validate.hip
hipError_t launch_dchain(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_validate_decoded(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_walk(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_decode(const DeviceJob& j, hipStream_t s, uint32_t grid);    // rp_codec.hip
hipError_t launch_decode_blocks(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_lz_walk(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_lz_exec(const DeviceJob& j, hipStream_t s);
hipError_t launch_raw_copy(const DeviceJob& j, hipStream_t s, uint32_t cus);
hipError_t launch_lzf_walk(const DeviceJob& j, hipStream_t s, uint32_t cus);
hipError_t launch_decode_finish(const DeviceJob& j, hipStream_t s, uint32_t grid, bool defer = false);
hipError_t launch_content_xxh(const DeviceJob& j, hipStream_t s, uint32_t grid);  // k_decode_finish(defer)'s checksums
hipError_t launch_content_apply(const DeviceJob& j, hipStream_t s, uint32_t grid);  // their mismatches, after the join
// gzip members (rp_inflate.hip): first pass (into scratch) before the slot
// scans, then the copy into the arena and the second pass where needed
hipError_t launch_inflate_plan(const DeviceJob& j, hipStream_t s, uint32_t grid, int pass = 0);
hipError_t launch_inflate(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_zparse(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_zplan(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_gzsplan(const DeviceJob& j, hipStream_t s);
hipError_t launch_gzsplit(const DeviceJob& j, hipStream_t s, uint32_t grid, int part = 0);  // part 1: find, 2: decode + resolve, 0: all
hipError_t launch_zfallback(const DeviceJob& j, hipStream_t s, uint32_t grid);
hipError_t launch_zexact(const DeviceJob& j, hipStream_t s, int pass);  // rp_inflate.hip
hipError_t launch_zstamps(hipStream_t s, int print);  // RPGPU_ZSTAMPS builds: reset / print the decoder stamps
hipError_t launch_zexec(const DeviceJob& j, hipStream_t s);  // rp_codec.hip
// one payload, one wave (rpgpu_uncompress); res[0] = rc (0 / -1 / -2), res[1] = out_len
hipError_t launch_uncompress_one(int codec, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap,
                                 int64_t* res, hipStream_t s);
// rpgpu_uncompress_batch: one payload per lane
struct UncItem {
    uint64_t src, n;    // input bytes [src, src + n) of the staged inputs
    uint64_t dst, cap;  // output slot [dst, dst + cap) (cap includes 16 bytes of wild-copy room)
    int32_t codec, pad;
};
// compressor::compress (rp_compress.hip): 64 KiB blocks into scratch slots
// of kCompSlot bytes (>= snappy::MaxCompressedLength(65536)), then one frame
// per payload
constexpr uint32_t kCompSlot = 76800;
// large stored payloads (disk layout): CRC in kSplitParts chunks, one wave
// each, merged by GF(2) shifts (k_crc_split / k_crc_combine).  Only payloads
// above twice a wave's share of the job are split (DeviceJob::split_min): a
// job of many batches is balanced by k_validate's stride already, and
// splitting C2 / C5's batches at 256 KiB measured slower (validate 8.8 ->
// 9.9 ms), a separate pass where the stride overlapped them.
constexpr uint64_t kSplitMin = 256u << 10;
constexpr uint32_t kSplitParts = 16;
struct CompBlock {
    uint64_t src;                    // staged input offset (a fragment starts 16-byte aligned; 8 readable bytes past it)
    uint32_t n, codec;               // block bytes (<= 65536), RPGPU_CODEC_LZ4 / _SNAPPY
    uint32_t frag_len, frag_blocks;  // snappy: on a fragment's first block, the fragment's bytes and blocks
};
struct CompPayload {
    uint64_t n, out;                 // input bytes; output offset
    uint32_t first, nblocks, codec, pad;
};
hipError_t launch_compress(const uint8_t* in, const CompBlock* blocks, uint32_t nb, const CompPayload* pay, uint32_t np,
                           uint8_t* scratch, uint32_t* sizes, uint8_t* out, uint64_t* out_len, hipStream_t s);
hipError_t launch_uncompress_many(const UncItem* items, uint32_t count, const uint8_t* in, uint64_t in_total,
                                  uint8_t* out, int64_t* res, hipStream_t s);
hipError_t launch_finalize(const DeviceJob& j, hipStream_t s);
// rpgpu_serialize_wire (rp_validate.hip): batches [first, first + n) of a job's
// results; src/dst: n + 1 u64 each (dst ends as the exclusive scan, dst[n] = total)
hipError_t launch_to_wire(const uint8_t* disk, uint8_t* wire, const rpgpu_batch_result* batches, const uint64_t* seg_off,
                          uint64_t first, uint32_t n, uint64_t* src, uint64_t* dst, void* scan_tmp, size_t scan_bytes,
                          uint32_t grid, hipStream_t s);
// rpgpu_stamp (rp_validate.hip): base offset of batch i = next + offs[i]
// (RPGPU_STAMP_OFFSETS: offs = exclusive scan of the steps), cursor zeroed
hipError_t launch_stamp_steps(const uint8_t* data, const uint64_t* pos, uint32_t n, uint64_t* steps, hipStream_t s);
hipError_t launch_stamp(uint8_t* data, const uint64_t* pos, const uint32_t* plen, const uint64_t* offs, int64_t next,
                        uint32_t n, uint32_t flags, const Tables* T, uint32_t* cursor, uint32_t grid, hipStream_t s);
hipError_t scan_exclusive_u64(uint64_t* data, uint64_t n, void* temp, size_t temp_bytes, hipStream_t s);
// n = min(*d_n, n_cap), read on the device
hipError_t scan_exclusive_u64_devn(uint64_t* data, const uint64_t* d_n, uint64_t n_cap, void* temp, hipStream_t s);
size_t scan_temp_bytes(uint64_t n);

// rp_index.hip: segment index rebuild (rpgpu_segment_index), one wave per segment
hipError_t launch_segment_index(const rpgpu_batch_result* batches, uint64_t cap, const rpgpu_segment_summary* sums,
                                uint32_t n_segments, uint64_t step, rpgpu_index_state* states, uint32_t* rel_offset,
                                uint32_t* rel_time, uint64_t* position, hipStream_t s);
size_t segment_index_ws_bytes(uint32_t n_segments, uint64_t cap);
hipError_t launch_segment_index_pieces(const rpgpu_batch_result* batches, uint64_t cap,
                                       const rpgpu_segment_summary* sums, uint32_t n_segments, uint64_t step,
                                       rpgpu_index_state* states, uint32_t* rel_offset, uint32_t* rel_time,
                                       uint64_t* position, void* ws, hipStream_t s);

}  // namespace rp
