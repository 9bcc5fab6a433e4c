// rp_device.h — device helpers shared by the kernel translation units
// (rp_kernels.hip, rp_validate.hip, rp_codec.hip).  Wave64 idioms only.
#pragma once

#include "rp_internal.h"

namespace rp {

#define DEV __device__ __forceinline__

DEV uint32_t lane() { return __lane_id(); }

DEV uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
    return v;
}
DEV uint32_t wave_or(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}
DEV uint32_t rl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
// readfirstlane/readlane return int: go through uint32_t so the low half is
// never sign-extended into the high half (positions >= 2 GiB).
DEV uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
DEV uint64_t uni64(uint64_t v) {
    return (uint64_t)uni32((uint32_t)v) | ((uint64_t)uni32((uint32_t)(v >> 32)) << 32);
}
// the dword holding rpgpu_batch_result.reserved0 (its high half), for the
// atomic bit updates of kernels that run side by side (k_crc_compose,
// k_content_xxh)
static_assert(offsetof(rpgpu_batch_result, reserved0) % 4 == 2, "reserved0 is the high half of a dword");
DEV uint32_t* reserved0_word(rpgpu_batch_result* R) {
    return (uint32_t*)((uint8_t*)R + offsetof(rpgpu_batch_result, reserved0) - 2);
}

// byte k (0..60) of a header whose bytes are spread one per lane
DEV uint32_t hb(uint32_t b, int k) { return rl(b, k); }
DEV uint32_t h32(uint32_t b, int k) { return hb(b, k) | (hb(b, k + 1) << 8) | (hb(b, k + 2) << 16) | (hb(b, k + 3) << 24); }
DEV uint64_t h64(uint32_t b, int k) { return (uint64_t)h32(b, k) | ((uint64_t)h32(b, k + 4) << 32); }
DEV uint32_t h16(uint32_t b, int k) { return hb(b, k) | (hb(b, k + 1) << 8); }

// ---------------------------------------------------------------------------
// Wave-cooperative header read: read_header_impl (storage/parser.cc:139-176).
// Lane l holds header byte l; internal_header_only_crc (model/record_utils.cc:
// 34-55) is computed in parallel: byte l at distance 60-l from the end
// contributes T_{60-l}[b] (raw CRC), the ~0 init contributes c57.
// ---------------------------------------------------------------------------
struct Hdr {
    int32_t status;   // -1 ok, else parser errc
    int32_t eof;
    uint32_t hcrc, computed;
    int32_t size;
    uint64_t need;    // (uint32_t)(size - 61)
    uint32_t b;       // this lane's header byte
};

DEV Hdr wave_header(const uint8_t* __restrict__ seg, uint64_t len, uint64_t p, const Tables* __restrict__ T) {
    Hdr h;
    h.eof = 0;
    h.b = 0;
    h.hcrc = h.computed = 0;
    h.size = 0;
    h.need = 0;
    const uint64_t rem = len - p;
    if (rem == 0) { h.status = RPGPU_ERRC_END_OF_STREAM; h.eof = 1; return h; }
    if (rem < RPGPU_HEADER_SIZE) { h.status = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES; h.eof = 1; return h; }
    const uint32_t l = lane();
    uint32_t b = (l < RPGPU_HEADER_SIZE) ? (uint32_t)seg[p + l] : 0u;
    uint32_t contrib = (l >= 4 && l < RPGPU_HEADER_SIZE) ? T->hdr[60 - l][b] : 0u;
    uint32_t raw = wave_xor(contrib);
    h.b = b;
    h.computed = ~(T->c57 ^ raw);
    h.hcrc = h32(b, 0);
    h.size = (int32_t)h32(b, 4);
    h.need = (uint32_t)((uint32_t)h.size - RPGPU_HEADER_SIZE);
    if (h.hcrc == 0) { h.status = RPGPU_ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER; return h; }
    if (h.hcrc != h.computed) { h.status = RPGPU_ERRC_HEADER_ONLY_CRC_MISSMATCH; return h; }
    h.status = -1;
    return h;
}

// 4 bytes at an arbitrary byte address, from the aligned dwords around it.
// The second dword is only touched when the bytes straddle it, so the read
// never goes past the last byte asked for.
DEV uint32_t ldu32(const uint8_t* p) {
    uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t hi = 0;
    if (sh) hi = q[1];
    return __builtin_amdgcn_alignbyte(hi, q[0], sh);
}

// BE40 prefix position of disk header byte l (21..60): fields are reversed
// byte-wise (model/record_utils.cc:68-80).
DEV int be_index(uint32_t l) {
    // field starts on disk and lengths: attrs 21/2, lod 23/4, first_ts 27/8,
    // max_ts 35/8, pid 43/8, epoch 51/2, base_seq 53/4, record_count 57/4
    int fs, fl;
    if (l < 23) { fs = 21; fl = 2; }
    else if (l < 27) { fs = 23; fl = 4; }
    else if (l < 35) { fs = 27; fl = 8; }
    else if (l < 43) { fs = 35; fl = 8; }
    else if (l < 51) { fs = 43; fl = 8; }
    else if (l < 53) { fs = 51; fl = 2; }
    else if (l < 57) { fs = 53; fl = 4; }
    else { fs = 57; fl = 4; }
    return (fs - 21) + (fl - 1 - ((int)l - fs));
}

// big-endian fields of a header spread one byte per lane
DEV uint32_t hbe16(uint32_t b, int k) { return (hb(b, k) << 8) | hb(b, k + 1); }
DEV uint32_t hbe32(uint32_t b, int k) { return (hbe16(b, k) << 16) | hbe16(b, k + 2); }
DEV uint64_t hbe64(uint32_t b, int k) { return ((uint64_t)hbe32(b, k) << 32) | hbe32(b, k + 4); }

// ---------------------------------------------------------------------------
// Wave-cooperative Kafka v2 wire header: batch_reader::read_record_batch_info
// (kafka/protocol/batch_reader.cc:50-88) + kafka_batch_adapter::read_header
// (kafka/protocol/kafka_batch_adapter.cc:32-91).  Lane l holds wire byte l.
// The chain is structural: size = batch_length + 12; a size below 61 cannot
// hold the header adapt() reads (it throws).  There is no header_crc on the
// wire: `computed` is internal_header_only_crc of the adapted header (the
// value the batch carries on disk), from disk byte l = wire byte src(l).
// ---------------------------------------------------------------------------
DEV Hdr wave_header_wire(const uint8_t* __restrict__ seg, uint64_t len, uint64_t p, const Tables* __restrict__ T) {
    Hdr h;
    h.eof = 0;
    h.b = 0;
    h.hcrc = h.computed = 0;
    h.size = 0;
    h.need = 0;
    const uint64_t rem = len - p;
    if (rem == 0) { h.status = RPGPU_ERRC_END_OF_STREAM; h.eof = 1; return h; }
    if (rem < RPGPU_HEADER_SIZE) { h.status = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES; h.eof = 1; return h; }
    const uint32_t l = lane();
    const uint32_t b = (l < RPGPU_HEADER_SIZE) ? (uint32_t)seg[p + l] : 0u;
    h.b = b;
    const uint32_t bl = hbe32(b, 8);
    if ((int64_t)(int32_t)bl + 12 < (int64_t)RPGPU_HEADER_SIZE) { h.status = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES; return h; }
    h.size = (int32_t)(bl + 12u);
    h.need = (uint32_t)((uint32_t)h.size - RPGPU_HEADER_SIZE);
    // adapted (disk, little-endian) byte l: size_bytes 4..7, base_offset
    // 8..15 (wire 7..0), type 16 (raft_data), then every field byte-reversed
    // in place (the BE40 prefix is wire[21..61))
    int src = 0;
    if (l >= 8 && l < 16) src = 15 - (int)l;
    else if (l >= 17 && l < 21) src = 37 - (int)l;
    else if (l >= 21 && l < RPGPU_HEADER_SIZE) src = 21 + be_index(l);
    const uint32_t moved = (uint32_t)__shfl((int)b, src, 64);
    uint32_t d = moved;
    if (l >= 4 && l < 8) d = ((uint32_t)h.size >> (8 * (l - 4))) & 0xFFu;
    if (l == 16) d = 1u;
    const uint32_t contrib = (l >= 4 && l < RPGPU_HEADER_SIZE) ? T->hdr[60 - l][d] : 0u;
    h.computed = ~(T->c57 ^ wave_xor(contrib));
    h.status = -1;
    return h;
}

DEV Hdr wave_header_of(uint32_t layout, const uint8_t* __restrict__ seg, uint64_t len, uint64_t p,
                       const Tables* __restrict__ T) {
    return layout == RPGPU_LAYOUT_WIRE ? wave_header_wire(seg, len, p, T) : wave_header(seg, len, p, T);
}

// ---------------------------------------------------------------------------
// Lane-private header read: the same verdicts as wave_header_of, one header
// per LANE, so 64 chains advance per wave instruction.  The 61 bytes arrive
// in four 16-byte loads (the last at +45, so nothing past byte 60 is read);
// header_crc is the xor of 57 independent lookups T_{60-k}[byte k] in the LDS
// image of Tables::hdr (`th`, 57 x 256 words), so its latency is one LDS
// round, not 57.
// ---------------------------------------------------------------------------
struct LHdr {
    int32_t status;  // -1 ok, else parser errc
    int32_t eof;
    uint32_t hcrc, computed;
    int32_t size;
    uint64_t need;   // (uint32_t)(size - 61)
    uint32_t w[16];  // header bytes 0..63 (61..63 zero)
};

DEV uint4 ld16u(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // one global_load_dwordx4 (unaligned access is native)
    return v;
}

// header bytes [0, 61) of seg + p into w[0..15]
DEV void lane_header_bytes(const uint8_t* __restrict__ h, uint32_t (&w)[16]) {
    const uint4 a = ld16u(h), b = ld16u(h + 16), c = ld16u(h + 32), d = ld16u(h + 45);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w;
    // d holds bytes 45..60: byte 48 + i = d byte 3 + i
    w[12] = __builtin_amdgcn_alignbyte(d.y, d.x, 3);
    w[13] = __builtin_amdgcn_alignbyte(d.z, d.y, 3);
    w[14] = __builtin_amdgcn_alignbyte(d.w, d.z, 3);
    w[15] = d.w >> 24;
}

DEV uint32_t lb(const uint32_t (&w)[16], int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }
DEV uint32_t l32(const uint32_t (&w)[16], int k) {
    return (k & 3) ? __builtin_amdgcn_alignbyte(w[(k >> 2) + 1], w[k >> 2], k & 3) : w[k >> 2];
}
DEV uint64_t l64(const uint32_t (&w)[16], int k) { return (uint64_t)l32(w, k) | ((uint64_t)l32(w, k + 4) << 32); }
DEV uint32_t l16(const uint32_t (&w)[16], int k) { return l32(w, k) & 0xFFFFu; }
DEV uint32_t lbe32(const uint32_t (&w)[16], int k) { return __builtin_bswap32(l32(w, k)); }
DEV uint64_t lbe64(const uint32_t (&w)[16], int k) { return ((uint64_t)lbe32(w, k) << 32) | lbe32(w, k + 4); }
DEV uint32_t lbe16(const uint32_t (&w)[16], int k) { return (lb(w, k) << 8) | lb(w, k + 1); }

// wire byte the adapted (disk) header byte l comes from (wave_header_wire)
constexpr int wire_src(int l) {
    return (l >= 8 && l < 16) ? 15 - l
         : (l >= 17 && l < 21) ? 37 - l
         : (l >= 21 && l < 61) ? 21 + ((l < 23 ? 0 : l < 27 ? 2 : l < 35 ? 6 : l < 43 ? 14 : l < 51 ? 22 : l < 53 ? 30
                                        : l < 57 ? 32 : 36) +
                                       ((l < 23 ? 2 : l < 27 ? 4 : l < 35 ? 8 : l < 43 ? 8 : l < 51 ? 8 : l < 53 ? 2
                                        : 4) - 1 - (l - (l < 23 ? 21 : l < 27 ? 23 : l < 35 ? 27 : l < 43 ? 35
                                                         : l < 51 ? 43 : l < 53 ? 51 : l < 57 ? 53 : 57))))
         : 0;
}

DEV LHdr lane_header(uint32_t layout, const uint8_t* __restrict__ seg, uint64_t len, uint64_t p,
                     const uint32_t* __restrict__ th, uint32_t c57) {
    LHdr h;
    h.eof = 0;
    h.hcrc = h.computed = 0;
    h.size = 0;
    h.need = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) h.w[i] = 0;
    const uint64_t rem = len - p;
    if (rem == 0) { h.status = RPGPU_ERRC_END_OF_STREAM; h.eof = 1; return h; }
    if (rem < RPGPU_HEADER_SIZE) { h.status = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES; h.eof = 1; return h; }
    lane_header_bytes(seg + p, h.w);
    uint32_t raw = 0;
    if (layout == RPGPU_LAYOUT_WIRE) {
        const uint32_t bl = lbe32(h.w, 8);
        if ((int64_t)(int32_t)bl + 12 < (int64_t)RPGPU_HEADER_SIZE) {
            h.status = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES;
            return h;
        }
        h.size = (int32_t)(bl + 12u);
        h.need = (uint32_t)((uint32_t)h.size - RPGPU_HEADER_SIZE);
#pragma unroll
        for (int k = 4; k < 61; k++) {
            const uint32_t d = (k < 8) ? (((uint32_t)h.size >> (8 * (k - 4))) & 0xFFu) : (k == 16) ? 1u : lb(h.w, wire_src(k));
            raw ^= th[(60 - k) * 256 + d];
        }
        h.computed = ~(c57 ^ raw);
        h.status = -1;
        return h;
    }
#pragma unroll
    for (int k = 4; k < 61; k++) raw ^= th[(60 - k) * 256 + lb(h.w, k)];
    h.computed = ~(c57 ^ raw);
    h.hcrc = h.w[0];
    h.size = (int32_t)h.w[1];
    h.need = (uint32_t)((uint32_t)h.size - RPGPU_HEADER_SIZE);
    if (h.hcrc == 0) { h.status = RPGPU_ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER; return h; }
    if (h.hcrc != h.computed) { h.status = RPGPU_ERRC_HEADER_ONLY_CRC_MISSMATCH; return h; }
    h.status = -1;
    return h;
}

// raw CRC contribution of the BE40 prefix of the batch crc (model/record_utils.cc:
// 68-80): disk byte k (21..60) lands at BE position be(k); on the wire the
// prefix is bytes [21, 61) as they stand
DEV uint32_t lane_prefix_raw(uint32_t layout, const uint32_t (&w)[16], const uint32_t* __restrict__ th) {
    uint32_t x = 0;
    if (layout == RPGPU_LAYOUT_WIRE) {
#pragma unroll
        for (int k = 21; k < 61; k++) x ^= th[(39 - (k - 21)) * 256 + lb(w, k)];
    } else {
#pragma unroll
        for (int k = 21; k < 61; k++) x ^= th[(39 - (wire_src(k) - 21)) * 256 + lb(w, k)];
    }
    return x;
}

// the LDS image of Tables::hdr for lane_header (57 KiB)
constexpr uint32_t kLdsHdrBytes = 57u * 256u * 4u;
DEV void init_lds_hdr(uint32_t* th, const Tables* T) {
    for (uint32_t i = threadIdx.x; i < 57u * 256u; i += blockDim.x) th[i] = (&T->hdr[0][0])[i];
    __syncthreads();
}

#define HD __host__ __device__ inline

HD uint32_t rd32h(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

// ---------------------------------------------------------------------------
// Decode-arena plan rule (engine rule, restated by the oracle as
// rpo_decode_capacity): bytes reserved for one compressed payload, from its
// frame structure alone, before any decode.  Shared by k_emit and the
// rpgpu_uncompress host path.
// ---------------------------------------------------------------------------
HD uint32_t xxh32_small(const uint8_t* p, uint32_t n) {
    // XXH32 for n < 16 (the LZ4F header checksum input is <= 14 bytes)
    const uint32_t P1 = 0x9E3779B1u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u, P2 = 0x85EBCA77u;
    uint32_t h = P5 + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) {
        uint32_t v = (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
        h += v * P3;
        h = ((h << 17) | (h >> 15)) * P4;
    }
    for (; i < n; i++) { h += p[i] * P5; h = ((h << 11) | (h >> 21)) * P1; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}


HD int snappy_varint32_dev(const uint8_t* s, uint64_t n, uint32_t* v) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        uint32_t b = s[i];
        if (i < 4) {
            r |= (b & 127) << (7 * i);
            if (b < 128) { *v = r; return (int)i + 1; }
        } else {
            r |= (b & 127) << 28;
            if (b < 16) { *v = r; return 5; }
            return -1;
        }
    }
    return -1;
}

// Same rule as the oracle's rpo_decode_capacity (engine plan rule): the
// frame's planned bytes rounded up to 16, so every slot of the decoded
// arena starts 16-byte aligned (whole-chunk stores)
HD uint64_t decode_capacity_raw(int codec, const uint8_t* s, uint64_t n);
HD uint64_t decode_capacity_dev(int codec, const uint8_t* s, uint64_t n) {
    return (decode_capacity_raw(codec, s, n) + 15) & ~15ull;
}
HD uint64_t decode_capacity_raw(int codec, const uint8_t* s, uint64_t n) {
    if (n == 0) return 0;
    if (codec == RPGPU_CODEC_LZ4) {
        if (n < 7) return 0;
        uint32_t magic = rd32h(s);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u || magic != 0x184D2204u) return 0;
        uint32_t flg = s[4];
        uint64_t hs = 7 + (((flg >> 3) & 1) ? 8 : 0) + ((flg & 1) ? 4 : 0);
        if (n < hs) return 0;
        if ((flg >> 1) & 1) return 0;
        if (((flg >> 6) & 3) != 1) return 0;
        uint32_t bd = s[5];
        if ((bd >> 7) & 1) return 0;
        uint32_t bsid = (bd >> 4) & 7;
        if (bsid < 4 || (bd & 15)) return 0;
        if (((xxh32_small(s + 4, (uint32_t)(hs - 5)) >> 8) & 0xFF) != s[hs - 1]) return 0;
        const uint64_t bmax = bsid == 4 ? (64u << 10) : bsid == 5 ? (256u << 10) : bsid == 6 ? (1u << 20) : (4u << 20);
        const uint32_t bcs = (flg >> 4) & 1;
        uint64_t cap = 0, pos = hs;
        while (n - pos >= 4) {
            uint32_t bh = rd32h(s + pos);
            if (bh == 0) break;
            uint64_t bsz = bh & 0x7FFFFFFFu;
            if (bsz > bmax) break;
            cap += (bh & 0x80000000u) ? bsz : bmax;
            pos += 4;
            uint64_t adv = bsz + (bcs ? 4 : 0);
            if (n - pos < adv) break;
            pos += adv;
        }
        return cap;
    }
    if (codec == RPGPU_CODEC_SNAPPY) {
        const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        bool java = n >= 16;
        for (int i = 0; i < 8 && java; i++) java = s[i] == magic[i];
        uint32_t ulen;
        if (!java) {
            if (snappy_varint32_dev(s, n, &ulen) < 0) return 0;
            return ((uint64_t)ulen <= 22ull * n + 64) ? ulen : 0;
        }
        uint64_t cap = 0, pos = 16;
        while (n - pos >= 4) {
            int32_t clen = (int32_t)(((uint32_t)s[pos] << 24) | ((uint32_t)s[pos + 1] << 16) |
                                     ((uint32_t)s[pos + 2] << 8) | s[pos + 3]);
            if (clen <= 0 || n - pos - 4 < (uint64_t)clen) break;
            if (snappy_varint32_dev(s + pos + 4, (uint64_t)clen, &ulen) < 0) break;
            if ((uint64_t)ulen > 22ull * (uint64_t)clen + 64) break;
            cap += ulen;
            pos += 4 + (uint64_t)clen;
        }
        return cap;
    }
    return 0;
}


// ---------------------------------------------------------------------------
// GF(2) arithmetic modulo the reflected CRC32C polynomial (zlib's multmodp /
// x2nmodp scheme; bit 31 is x^0): merging partial CRCs (k_crc_combine) and
// the pieces of a decoded payload (k_decode_finish).  x has order 2^31 - 1
// modulo this polynomial, so x^(2^k) repeats with period 31.
// ---------------------------------------------------------------------------
static __constant__ uint32_t kX2n[31] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0x82F63B78u, 0x6EA2D55Cu, 0x18B8EA18u,
    0x510AC59Au, 0xB82BE955u, 0xB8FDB1E7u, 0x88E56F72u, 0x74C360A4u, 0xE4172B16u, 0x0D65762Au, 0x35D73A62u,
    0x28461564u, 0xBF455269u, 0xE2EA32DCu, 0xFE7740E6u, 0xF946610Bu, 0x3C204F8Fu, 0x538586E3u, 0x59726915u,
    0x734D5309u, 0xBC1AC763u, 0x7D0722CCu, 0xD289CABEu, 0xE94CA9BCu, 0x05B74F3Fu, 0xA51E1F42u};

// a * b mod P (a != 0)
DEV uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}
// the raw state s advanced over n zero bytes: x^(8 n) * s mod P
DEV uint32_t crc_shift(uint32_t s, uint64_t n) {
    uint32_t p = 1u << 31;  // x^0
    for (uint32_t k = 3; n; n >>= 1, k = (k == 30u) ? 0u : k + 1u)
        if (n & 1) p = multmodp(kX2n[k], p);
    return multmodp(p, s);
}

// Wave-uniform atomic fetch-add of `v` (lane 0's contribution; the other
// lanes add 0).  Every lane executes the atomic: written as
// `if (lane() == 0) x = atomicAdd(..)` followed by readfirstlane, the
// compiler's divergence analysis took the claimed value for a per-lane one
// and built a claim loop with a per-lane exit whose lanes never all left
// (the round-2 wave decoder did not terminate).
DEV uint32_t wave_fetch_add(uint32_t* p, uint32_t v) {
    return uni32(atomicAdd(p, lane() == 0 ? v : 0u));
}

}  // namespace rp
