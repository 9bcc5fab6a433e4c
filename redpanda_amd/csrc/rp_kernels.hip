// rp_kernels.hip — CDNA4 (gfx950) kernels of the record-batch engine.
//
// Pipeline per job (all on one stream, see rp_runtime.hip):
//   k_discover   speculative chain walk per chunk      (storage/parser.cc:139-254)
//   k_resolve    verify/repair speculation per segment (same chain semantics)
//   scan         chunk batch counts -> batch ordinals
//   k_emit       walk again, write headers + plan      (storage/parser.cc:36-76)
//   scan x2      index slots / decode-arena bytes
//   k_validate   CRC32C + record walk per batch        (model/record_utils.cc:68-181)
//   k_finalize   checkpoint, bitmap, totals            (storage/log_replayer.cc:62-79)
//
// Integer/byte work only: HBM-bound, no MFMA.  The CRC runs from LDS tables
// replicated 32x so every lane reads its own bank (conflict-free ds_read_b32).
#include "rp_internal.h"

namespace rp {

#define DEV __device__ __forceinline__

// Bounds-checked build (-DRPGPU_CHECKED, librpgpu_checked.so): every data
// access of k_validate is checked against the allocation and reported with
// printf instead of faulting.  Fault localisation only; never benchmarked.
#ifdef RPGPU_CHECKED
#include <cstdio>
#define RP_CHECK(flag, cond, fmt, ...)                                               \
    do {                                                                            \
        if (!(cond)) {                                                              \
            if (__lane_id() == 0) printf("RPGPU_CHECK %d " fmt "\n", __LINE__, __VA_ARGS__); \
            flag = true;                                                            \
        }                                                                           \
    } while (0)
#endif

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

// ---------------------------------------------------------------------------
// Discovery
// ---------------------------------------------------------------------------
DEV uint32_t find_segment(const uint64_t* __restrict__ chunk_base, uint32_t nseg, uint64_t g) {
    uint32_t lo = 0, hi = nseg;  // largest s with chunk_base[s] <= g
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (chunk_base[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

// Cheap plausibility test of a candidate header at q (speculation only: a
// wrong guess is caught by k_resolve, so this never decides a verdict).
DEV bool prefilter(const uint8_t* __restrict__ seg, uint64_t len, uint64_t q) {
    if (len - q < RPGPU_HEADER_SIZE) return false;
    uint32_t hcrc = ldu32(seg + q);
    int32_t size = (int32_t)ldu32(seg + q + 4);
    if (hcrc == 0 || size < (int32_t)RPGPU_HEADER_SIZE) return false;
    if ((uint64_t)size > len - q) return false;
    uint32_t t = ldu32(seg + q + 16);
    int8_t type = (int8_t)(t & 0xFF);
    if (type < 1 || type > 32) return false;
    uint32_t attrs = (ldu32(seg + q + 21) & 0xFFFF);
    if ((attrs & 7) > 4) return false;
    int32_t rc = (int32_t)ldu32(seg + q + 57);
    if (rc < 0 || rc > size) return false;
    return true;
}

struct WalkOut {
    uint64_t exit;
    uint64_t tpos;
    uint32_t count;
    int32_t term;
};

// Follow the chain from p while headers start before ce.
DEV WalkOut wave_walk(const uint8_t* __restrict__ seg, uint64_t len, uint64_t p, uint64_t ce, const Tables* __restrict__ T) {
    WalkOut w;
    w.count = 0;
    w.term = -1;
    w.tpos = 0;
    while (p < ce) {
        Hdr h = wave_header(seg, len, p, T);
        if (h.status >= 0) { w.term = h.status | (h.eof << 8); w.tpos = p; break; }
        if (len - p - RPGPU_HEADER_SIZE < h.need) {
            w.count++;
            w.term = RPGPU_ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES | (1 << 8);
            w.tpos = p;
            break;
        }
        w.count++;
        p += RPGPU_HEADER_SIZE + h.need;
    }
    w.exit = p;
    return w;
}

__global__ __launch_bounds__(256) void k_discover(DeviceJob j) {
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= j.total_chunks) return;
    const uint32_t s = find_segment(j.chunk_base, j.n_segments, g);
    const uint64_t w = g - j.chunk_base[s];
    const uint64_t off = j.seg_off[s], len = j.seg_off[s + 1] - off;
    const uint8_t* seg = j.data + off;
    const uint64_t cs = w * j.chunk_bytes;
    const uint64_t ce = (cs + j.chunk_bytes < len) ? cs + j.chunk_bytes : len;
    uint64_t entry = kNone;
    if (w == 0) {
        entry = 0;
    } else {
        for (uint64_t q0 = cs; q0 < ce && entry == kNone; q0 += 64) {
            const uint64_t q = q0 + lane();
            bool cand = (q < ce) && prefilter(seg, len, q);
            uint64_t mask = __ballot(cand);
            while (mask) {
                const uint32_t bit = __builtin_ctzll(mask);
                mask &= mask - 1;
                const uint64_t qc = q0 + bit;
                Hdr h = wave_header(seg, len, qc, j.tables);
                if (h.status < 0 && len - qc - RPGPU_HEADER_SIZE >= h.need) { entry = qc; break; }
            }
        }
    }
    WalkOut o;
    if (entry == kNone) {
        o.exit = kNone; o.count = 0; o.term = -1; o.tpos = 0;
    } else {
        o = wave_walk(seg, len, entry, ce, j.tables);
    }
    if (lane() == 0) {
        ChunkRec r;
        r.entry = entry;
        r.exit = o.exit;
        r.count = o.count;
        r.term = o.term;
        r.tpos = o.tpos;
        j.chunks[g] = r;
    }
}

// ---------------------------------------------------------------------------
// Resolve: one 256-thread workgroup per segment.  Chunk w's speculation is
// right iff its entry equals the true chain position entering it (the exit of
// the nearest earlier chunk that holds a header start).  Mismatches are
// re-walked from the true position by wave 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_resolve(DeviceJob j) {
    const uint32_t s = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const uint64_t c0 = j.chunk_base[s];
    const uint64_t W = j.chunk_base[s + 1] - c0;
    const uint64_t off = j.seg_off[s], len = j.seg_off[s + 1] - off;
    const uint8_t* seg = j.data + off;
    const uint64_t CS = j.chunk_bytes;

    __shared__ uint64_t s_exit[256];
    __shared__ int32_t s_term[256];
    __shared__ int32_t s_scan[256];
    __shared__ uint32_t s_first, s_tfirst;
    __shared__ uint64_t s_T, s_pred;
    __shared__ int32_t s_ended;
    __shared__ SegTerm s_st;

    if (tid == 0) { s_T = 0; s_ended = 0; s_st.pos = len; s_st.errc = RPGPU_ERRC_END_OF_STREAM; s_st.eof = 1; }
    __syncthreads();
    uint64_t w0 = 0;
    while (w0 < W && !s_ended) {
        const uint64_t w = w0 + tid;
        const bool valid = w < W;
        ChunkRec r;
        r.entry = kNone; r.exit = kNone; r.count = 0; r.term = -1; r.tpos = 0;
        if (valid) r = j.chunks[c0 + w];
        const bool has = valid && r.entry != kNone;
        s_exit[tid] = r.exit;
        s_term[tid] = r.term;
        s_scan[tid] = has ? (int32_t)tid : -1;
        if (tid == 0) { s_first = 256; s_tfirst = 256; }
        __syncthreads();
        // inclusive max-scan of the last chunk index holding a header start
        for (int o = 1; o < 256; o <<= 1) {
            int32_t v = s_scan[tid];
            int32_t u = (tid >= (uint32_t)o) ? s_scan[tid - o] : -1;
            __syncthreads();
            s_scan[tid] = v > u ? v : u;
            __syncthreads();
        }
        const int32_t prev = (tid > 0) ? s_scan[tid - 1] : -1;
        const uint64_t pred = (prev >= 0) ? s_exit[prev] : s_T;
        const int32_t pterm = (prev >= 0) ? s_term[prev] : -1;
        const uint64_t cs = w * CS;
        const uint64_t ce = (cs + CS < len) ? cs + CS : len;
        bool bad = false;
        if (valid) {
            if (pterm >= 0) bad = true;                      // chain already ended
            else if (!has) bad = !(pred >= ce);              // the chain must jump over it
            else bad = (pred != r.entry);
        }
        if (bad) atomicMin(&s_first, tid);
        __syncthreads();
        const uint32_t first = s_first;
        if (valid && tid < first) {
            j.chunk_count[c0 + w] = has ? r.count : 0;
            j.chunk_entry[c0 + w] = has ? r.entry : kNone;
            if (has && r.term >= 0) atomicMin(&s_tfirst, tid);
        }
        __syncthreads();
        if (s_tfirst < 256) {
            // the chain ends inside a verified chunk
            if (tid == 0) {
                const ChunkRec t = j.chunks[c0 + w0 + s_tfirst];
                s_st.pos = t.tpos;
                s_st.errc = t.term & 0xFF;
                s_st.eof = (t.term >> 8) & 1;
                s_ended = 1;
            }
            __syncthreads();
            w0 = w0 + s_tfirst + 1;
            break;
        }
        if (first >= 256 || w0 + first >= W) {
            // whole block verified: carry the exit of its last header chunk
            if (tid == 0) {
                int32_t last = s_scan[255];
                if (last >= 0) s_T = s_exit[last];
            }
            __syncthreads();
            w0 += 256;
            continue;
        }
        // speculation failed at chunk wf: re-walk it from the true position
        const uint64_t wf = w0 + first;
        if (tid == first) s_pred = pred;
        __syncthreads();
        const uint64_t P = s_pred;
        if (tid < 64) {
            const uint64_t cs2 = wf * CS;
            const uint64_t ce2 = (cs2 + CS < len) ? cs2 + CS : len;
            WalkOut o;
            uint64_t entry = kNone;
            if (P >= ce2) {
                o.exit = P; o.count = 0; o.term = -1; o.tpos = 0;
            } else {
                entry = P;
                o = wave_walk(seg, len, P, ce2, j.tables);
            }
            if (tid == 0) {
                ChunkRec nr;
                nr.entry = entry; nr.exit = o.exit; nr.count = o.count; nr.term = o.term; nr.tpos = o.tpos;
                j.chunks[c0 + wf] = nr;
                j.chunk_count[c0 + wf] = o.count;
                j.chunk_entry[c0 + wf] = entry;
                atomicAdd(&j.counters[0], 1u);
                if (o.term >= 0) {
                    s_st.pos = o.tpos; s_st.errc = o.term & 0xFF; s_st.eof = (o.term >> 8) & 1;
                    s_ended = 1;
                }
                s_T = o.exit;
            }
        }
        __syncthreads();
        w0 = wf + 1;
    }
    // chunks past the end of the chain hold no batches
    for (uint64_t w = w0 + tid; w < W; w += 256) {
        if (s_ended) {
            j.chunk_count[c0 + w] = 0;
            j.chunk_entry[c0 + w] = kNone;
        }
    }
    if (tid == 0) {
        if (!s_ended) { s_st.pos = s_T; s_st.errc = RPGPU_ERRC_END_OF_STREAM; s_st.eof = 1; }
        j.seg_term[s] = s_st;
    }
}

// ---------------------------------------------------------------------------
// Emit: walk each chunk again from its resolved entry; write the decoded
// header (storage/parser.cc:36-76) and plan index slots / decode bytes.
// ---------------------------------------------------------------------------
DEV uint32_t xxh32_small(const uint8_t* p, uint32_t n) {
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

DEV uint32_t rd32b(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

DEV int snappy_varint32_dev(const uint8_t* s, uint64_t n, uint32_t* v) {
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

// Same rule as the oracle's rpo_decode_capacity (engine plan rule).
DEV uint64_t decode_capacity_dev(int codec, const uint8_t* s, uint64_t n) {
    if (n == 0) return 0;
    if (codec == RPGPU_CODEC_LZ4) {
        if (n < 7) return 0;
        uint32_t magic = rd32b(s);
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
            uint32_t bh = rd32b(s + pos);
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
        static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
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

__global__ __launch_bounds__(256) void k_emit(DeviceJob j) {
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= j.total_chunks) return;
    const uint64_t base_ord = j.chunk_count[g];
    const uint64_t cnt = j.chunk_count[g + 1] - base_ord;
    if (cnt == 0) return;
    const uint32_t s = find_segment(j.chunk_base, j.n_segments, g);
    const uint64_t off = j.seg_off[s], len = j.seg_off[s + 1] - off;
    const uint8_t* seg = j.data + off;
    const Tables* T = j.tables;
    const uint32_t l = lane();
    uint64_t p = j.chunk_entry[g];
    for (uint64_t i = 0; i < cnt; i++) {
#ifdef RPGPU_CHECKED
        {
            bool bad = false;
            RP_CHECK(bad, p < len, "emit g=%llu i=%llu cnt=%llu p=%llu len=%llu entry=%llu", (unsigned long long)g,
                     (unsigned long long)i, (unsigned long long)cnt, (unsigned long long)p, (unsigned long long)len,
                     (unsigned long long)j.chunk_entry[g]);
            if (bad) break;
        }
#endif
        Hdr h = wave_header(seg, len, p, T);  // known valid (resolved chain)
        const uint64_t ord = base_ord + i;
        const bool complete = (len - p - RPGPU_HEADER_SIZE) >= h.need;
        // prefix state of the batch crc: CRC over the BE40 prefix, init ~0
        uint32_t pc = (l >= 21 && l < RPGPU_HEADER_SIZE) ? T->hdr[39 - be_index(l)][h.b] : 0u;
        uint32_t praw = wave_xor(pc);
        const uint32_t attrs = h16(h.b, 21);
        const int32_t rc = (int32_t)h32(h.b, 57);
        const uint32_t codec = attrs & 7;
        uint64_t slots = 0, cap = 0;
        const bool decodable = (codec == RPGPU_CODEC_LZ4 || codec == RPGPU_CODEC_SNAPPY) && (j.flags & RPGPU_JOB_DECODE);
        if (complete) {
            if (codec == 0) {
                if ((j.flags & RPGPU_JOB_PARSE) && rc > 0 && (uint64_t)rc <= h.need) slots = (uint64_t)rc;
            } else if (decodable) {
                cap = uni64(decode_capacity_dev((int)codec, seg + p + RPGPU_HEADER_SIZE, h.need));
                if ((j.flags & RPGPU_JOB_PARSE) && rc > 0 && (uint64_t)rc <= cap) slots = (uint64_t)rc;
            }
        }
        if (l == 0 && ord < j.batch_capacity) {
            rpgpu_batch_result r;
            r.file_pos = p;
            r.base_offset = (int64_t)h64(h.b, 8);
            r.first_timestamp = (int64_t)h64(h.b, 27);
            r.max_timestamp = (int64_t)h64(h.b, 35);
            r.producer_id = (int64_t)h64(h.b, 43);
            r.size_bytes = h.size;
            r.record_count = rc;
            r.last_offset_delta = (int32_t)h32(h.b, 23);
            r.base_sequence = (int32_t)h32(h.b, 53);
            r.header_crc = h.hcrc;
            r.crc = h32(h.b, 17);
            r.crc_computed = 0;
            r.header_crc_computed = h.computed;
            uint32_t f = RPGPU_F_HEADER_OK;
            if (complete) f |= RPGPU_F_COMPLETE;
            if (codec) f |= RPGPU_F_COMPRESSED;
            if (codec >= 5) f |= RPGPU_F_CODEC_INVALID;
            if (complete && (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD)) f |= RPGPU_F_CODEC_UNSUPPORTED;
            r.flags = f;
            r.segment = s;
            r.index_base = 0;
            r.decoded_off = 0;
            r.records_parsed = 0;
            r.decoded_len = (complete && codec == 0) ? (uint32_t)h.need : 0;
            r.decoded_crc = 0;
            r.decoded_header_crc = 0;
            r.attrs = (int16_t)attrs;
            r.producer_epoch = (int16_t)h16(h.b, 51);
            r.type = (int8_t)hb(h.b, 16);
            r.parse_err = 0;
            r.reserved0 = 0;
            // scratch for k_validate: raw CRC contribution of the BE prefix
            r.reserved1 = praw;
            j.batches[ord] = r;
            j.slots[ord] = slots;
            j.dcap[ord] = cap;
        }
        if (!complete) break;
        p += RPGPU_HEADER_SIZE + h.need;
    }
}

// ---------------------------------------------------------------------------
// Exclusive scan of u64 (3 passes, tile = 4096).  The element count is read
// from device memory so the batch count never round-trips to the host.
// ---------------------------------------------------------------------------
constexpr uint32_t kScanTile = 4096;

__global__ __launch_bounds__(256) void k_scan_tiles(uint64_t* data, const uint64_t* d_n, uint64_t n_host, uint64_t* tile_sums) {
    const uint64_t n = d_n ? (*d_n < n_host ? *d_n : n_host) : n_host;
    const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
    if (t0 >= n) return;
    __shared__ uint64_t s[256];
    uint64_t v[16];
    uint64_t sum = 0;
    const uint64_t b = t0 + threadIdx.x * 16;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        v[i] = (b + i < n) ? data[b + i] : 0;
        sum += v[i];
    }
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        uint64_t x = (threadIdx.x >= (uint32_t)o) ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += x;
        __syncthreads();
    }
    uint64_t run = s[threadIdx.x] - sum;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        if (b + i < n) data[b + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 255) tile_sums[blockIdx.x] = s[255];
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t* tile_sums, const uint64_t* d_n, uint64_t n_host, uint64_t* total_out) {
    const uint64_t n = d_n ? (*d_n < n_host ? *d_n : n_host) : n_host;
    const uint64_t nt = (n + kScanTile - 1) / kScanTile;
    __shared__ uint64_t s[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t t0 = 0; t0 < nt; t0 += 1024) {
        const uint64_t t = t0 + threadIdx.x;
        uint64_t v = t < nt ? tile_sums[t] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            uint64_t x = (threadIdx.x >= (uint32_t)o) ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += x;
            __syncthreads();
        }
        if (t < nt) tile_sums[t] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) total_out[0] = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint64_t* data, const uint64_t* d_n, uint64_t n_host, const uint64_t* tile_sums) {
    const uint64_t n = d_n ? (*d_n < n_host ? *d_n : n_host) : n_host;
    const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
    if (t0 >= n) return;
    const uint64_t add = tile_sums[blockIdx.x];
    for (uint64_t i = t0 + threadIdx.x; i < t0 + kScanTile && i < n; i += 256) data[i] += add;
}

// ---------------------------------------------------------------------------
// Validate: CRC32C over BE40 prefix ++ payload, record walk.
// ---------------------------------------------------------------------------

// LDS address of T_k[e] in the replicated image:
//   row-set rs (64 KiB) holds two tables, A at bytes [0,128) of each 256-byte
//   row and B at [128,256); copy c of entry e sits at e*256 + slot*128 + 4c,
//   i.e. bank c: lane L reads copy L%32 and never conflicts.
// v_perm_b32 assembles {key.b0, x.b_j, key.b2, 0} = address in one op.
constexpr uint32_t kSel0 = 0x0C020400u;  // x byte 0
constexpr uint32_t kSel1 = 0x0C020500u;  // x byte 1
constexpr uint32_t kSel2 = 0x0C020600u;  // x byte 2
constexpr uint32_t kSel3 = 0x0C020700u;  // x byte 3

struct Keys {
    uint32_t k3, k2, k1, k0;  // keys of T3, T2, T1, T0
};

DEV uint32_t lds32(const uint8_t* lds, uint32_t addr) { return *(const uint32_t*)(lds + addr); }

DEV uint32_t step4(const uint8_t* lds, const Keys& K, uint32_t s, uint32_t w) {
    const uint32_t x = s ^ w;
    const uint32_t a = lds32(lds, __builtin_amdgcn_perm(x, K.k3, kSel0));
    const uint32_t b = lds32(lds, __builtin_amdgcn_perm(x, K.k2, kSel1));
    const uint32_t c = lds32(lds, __builtin_amdgcn_perm(x, K.k1, kSel2));
    const uint32_t d = lds32(lds, __builtin_amdgcn_perm(x, K.k0, kSel3));
    return (a ^ b) ^ (c ^ d);
}

DEV uint32_t step1(const uint8_t* lds, const Keys& K, uint32_t s, uint32_t byte) {
    return lds32(lds, __builtin_amdgcn_perm(s ^ byte, K.k0, kSel0)) ^ (s >> 8);
}

// shift a raw CRC state forward over kStream*2^lvl zero bytes
DEV uint32_t shift_lvl(const uint8_t* lds, uint32_t s, uint32_t lvl) {
    const uint32_t* t = (const uint32_t*)(lds + kLdsCombineOff) + lvl * 1024;
    return t[s & 0xFF] ^ t[256 + ((s >> 8) & 0xFF)] ^ t[512 + ((s >> 16) & 0xFF)] ^ t[768 + (s >> 24)];
}


// 16 bytes at an arbitrary address, zero past `lim` (exclusive, absolute).
DEV void load16u(const uint8_t* p, const uint8_t* lim, uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uintptr_t L = (uintptr_t)lim;
    uint32_t d0 = ((uintptr_t)(q + 0) < L) ? q[0] : 0;
    uint32_t d1 = ((uintptr_t)(q + 1) < L) ? q[1] : 0;
    uint32_t d2 = ((uintptr_t)(q + 2) < L) ? q[2] : 0;
    uint32_t d3 = ((uintptr_t)(q + 3) < L) ? q[3] : 0;
    uint32_t d4 = ((uintptr_t)(q + 4) < L) ? q[4] : 0;
    r0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    r2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    r3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
}

// vint::deserialize (utils/vint.h:82-98) over at most `avail` bytes.
DEV int64_t varint16(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint64_t avail, uint32_t& br) {
    const uint64_t lo = (uint64_t)r0 | ((uint64_t)r1 << 32);
    const uint64_t hi = (uint64_t)r2 | ((uint64_t)r3 << 32);
    uint64_t res = 0;
    uint32_t n = 0;
    const uint32_t lim = avail < 10 ? (uint32_t)avail : 10u;
    for (uint32_t i = 0; i < lim; i++) {
        const uint64_t byte = (i < 8 ? (lo >> (8 * i)) : (hi >> (8 * (i - 8)))) & 0xFF;
        n++;
        res |= (byte & 127) << (7 * i);
        if (!(byte & 128)) break;
    }
    br = n;
    return (int64_t)((res >> 1) ^ (~(res & 1) + 1));
}

struct Reader {
    const uint8_t* base;  // payload start
    const uint8_t* lim;   // payload end (absolute)
    uint64_t n;
    uint64_t pos;
};

DEV int64_t rd_varlong(Reader& c) {
    uint32_t r0, r1, r2, r3, br;
    load16u(c.base + c.pos, c.lim, r0, r1, r2, r3);
    int64_t v = varint16(r0, r1, r2, r3, c.n - c.pos, br);
    c.pos += br;
    return v;
}

// iobuf_copy (bytes/iobuf.cc:133-157): -1 when (int)len < 0 (bad_alloc)
DEV int copy_bytes(Reader& c, int64_t len) {
    const int32_t bl = (int32_t)(uint32_t)(uint64_t)len;
    if (bl < 0) return -1;
    const uint64_t left = c.n - c.pos;
    c.pos += ((uint64_t)bl < left) ? (uint64_t)bl : left;
    return 0;
}

struct Rec {
    uint32_t err;   // rpgpu_parse_err
    uint64_t end;
    int64_t ts;
    int32_t length, off, klen, vlen, hcount;
    uint32_t key_pos, val_pos, hdr_pos;
    int32_t attr;
};

// parse_one_record_copy_from_buffer (model/record_utils.cc:170-177)
DEV Rec parse_record(const uint8_t* base, const uint8_t* lim, uint64_t n, uint64_t start) {
    Rec r;
    Reader c{base, lim, n, start};
    r.err = 0;
    r.key_pos = r.val_pos = r.hdr_pos = 0;
    r.ts = 0; r.length = r.off = r.klen = r.vlen = r.hcount = 0; r.attr = 0;
    const int64_t rsz = rd_varlong(c);
    if (c.pos >= n) { r.err = RPGPU_PARSE_ERR_ATTR_EOF; r.end = c.pos; return r; }
    r.attr = (int8_t)base[c.pos];
    c.pos++;
    r.ts = rd_varlong(c);
    const int64_t off = rd_varlong(c);
    const int64_t kl = rd_varlong(c);
    r.key_pos = (uint32_t)c.pos;
    if (kl > 0 && copy_bytes(c, kl)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    const int64_t vl = rd_varlong(c);
    r.val_pos = (uint32_t)c.pos;
    if (vl > 0 && copy_bytes(c, vl)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    const int64_t hc = rd_varlong(c);
    r.hdr_pos = (uint32_t)c.pos;
    if (hc < 0 || hc > RPGPU_MAX_HEADER_RESERVE) { r.err = RPGPU_PARSE_ERR_HEADER_RESERVE; r.end = c.pos; return r; }
    for (int64_t h = 0; h < hc; h++) {
        if (c.pos >= n) break;
        const int64_t hk = rd_varlong(c);
        if (hk > 0 && copy_bytes(c, hk)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
        const int64_t hv = rd_varlong(c);
        if (hv > 0 && copy_bytes(c, hv)) { r.err = RPGPU_PARSE_ERR_COPY_NEGATIVE; r.end = c.pos; return r; }
    }
    r.length = (int32_t)rsz;
    r.off = (int32_t)off;
    r.klen = (int32_t)kl;
    r.vlen = (int32_t)vl;
    r.hcount = (int32_t)hc;
    r.end = c.pos;
    return r;
}

struct WalkResult {
    uint32_t parsed;
    uint32_t err;
    uint64_t trailing;
};

// record_batch::for_each_record (model/record.h:616-627) with speculative
// lane-parallel records: a scalar chain over the length varints guesses where
// records start, lanes parse one record each, and only the prefix whose
// starts are confirmed by the previous record's exact end is committed.
DEV WalkResult walk_records(const uint8_t* base, uint64_t n, int32_t rc, uint32_t batch_ord,
                            rpgpu_record_index* out, uint64_t out_cap) {
    WalkResult wr;
    wr.parsed = 0;
    wr.err = 0;
    wr.trailing = 0;
    const uint32_t l = lane();
    const uint8_t* lim = base + n;
    uint64_t start = 0;
    uint32_t done = 0;
    while (done < (uint32_t)(rc > 0 ? rc : 0)) {
        const uint32_t want = ((uint32_t)rc - done) < 64u ? ((uint32_t)rc - done) : 64u;
        // speculative starts (uniform chain on the length varint)
        uint64_t my_start = kNone;
        uint64_t p = start;
        uint32_t m = 0;
        for (; m < want; m++) {
            if (l == m) my_start = p;
            if (p >= n) { m++; break; }
            uint32_t r0, r1, r2, r3, br;
            load16u(base + p, lim, r0, r1, r2, r3);
            r0 = uni32(r0); r1 = uni32(r1); r2 = uni32(r2); r3 = uni32(r3);
            const int64_t len = varint16(r0, r1, r2, r3, n - p, br);
            if (len < 0 || (uint64_t)len > n) { m++; break; }
            p = p + br + (uint64_t)len;
        }
        // each lane parses its record exactly
        Rec r;
        const bool act = l < m;
        if (act) r = parse_record(base, lim, n, my_start);
        else { r.err = 0; r.end = kNone; }
        const uint64_t prev_end = __shfl_up(r.end, 1, 64);
        const uint32_t prev_err = __shfl_up(r.err, 1, 64);
        const bool match = (l == 0) || (prev_err == 0 && prev_end == my_start);
        const uint64_t bad = __ballot(act && !match);
        const uint32_t exact = bad ? (uint32_t)__builtin_ctzll(bad) : m;  // lanes [0, exact) are exact
        const uint64_t errs = __ballot(act && l < exact && r.err != 0);
        const uint32_t nok = errs ? (uint32_t)__builtin_ctzll(errs) : exact;  // records parsed OK
        if (l < nok && done + l < out_cap) {
#ifdef RPGPU_CHECKED
            if (my_start >= n) printf("RPGPU_CHECK walk start %llu n %llu\n", (unsigned long long)my_start, (unsigned long long)n);
#endif
            rpgpu_record_index e;
            e.batch = batch_ord;
            e.rec_pos = (uint32_t)my_start;
            e.ts_delta = r.ts;
            e.length = r.length;
            e.offset_delta = r.off;
            e.key_len = r.klen;
            e.key_pos = r.key_pos;
            e.val_len = r.vlen;
            e.val_pos = r.val_pos;
            e.hdr_count = r.hcount;
            e.hdr_pos = r.hdr_pos;
            e.end_pos = (uint32_t)r.end;
            e.attrs = (int8_t)r.attr;
            e.pad[0] = e.pad[1] = e.pad[2] = 0;
            e.reserved[0] = e.reserved[1] = 0;
            out[done + l] = e;
        }
        if (errs) {
            wr.parsed = done + nok;
            wr.err = uni32(__shfl(r.err, nok, 64));
            return wr;
        }
        start = uni64(__shfl(r.end, exact - 1, 64));
        done += exact;
    }
    wr.parsed = done;
    wr.trailing = n - start;
    return wr;
}

__global__ __launch_bounds__(1024) void k_validate(DeviceJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const Tables* T = j.tables;
    // replicated slice tables: word i -> rs = i>>14, e = (i>>6)&255, slot = (i>>5)&1, copy = i&31
    for (uint32_t i = threadIdx.x; i < kLdsSliceBytes / 4; i += blockDim.x) {
        const uint32_t rs = i >> 14, e = (i >> 6) & 255, slot = (i >> 5) & 1;
        const uint32_t k = 3 - (rs * 2 + slot);  // A0 = T3, B0 = T2, A1 = T1, B1 = T0
        ((uint32_t*)lds)[i] = T->slice[k][e];
    }
    for (uint32_t i = threadIdx.x; i < kLdsCombineBytes / 4; i += blockDim.x)
        ((uint32_t*)(lds + kLdsCombineOff))[i] = ((const uint32_t*)T->comb)[i];
    __syncthreads();

    const uint32_t l = lane();
    const uint32_t bank = (l & 31) * 4;
    Keys K;
    K.k3 = (0u << 16) | (0u + bank);
    K.k2 = (0u << 16) | (128u + bank);
    K.k1 = (1u << 16) | (0u + bank);
    K.k0 = (1u << 16) | (128u + bank);

    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    const uint32_t waves_per_block = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * waves_per_block;
    const uint64_t gw = (uint64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);

    for (uint64_t b = gw; b < nb; b += nwaves) {
        rpgpu_batch_result* R = &j.batches[b];
        const uint32_t flags0 = uni32(R->flags);
        if (!(flags0 & RPGPU_F_COMPLETE)) {
            if (l == 0) { R->index_base = j.slots[b]; R->decoded_off = j.dcap[b]; R->reserved1 = 0; }
            continue;
        }
        const uint32_t segi = uni32(R->segment);
        const uint64_t seg_base = uni64(j.seg_off[segi]);
        const uint64_t S = seg_base + uni64(R->file_pos) + RPGPU_HEADER_SIZE;
        const uint64_t n = uni32((uint32_t)(R->size_bytes - (int32_t)RPGPU_HEADER_SIZE));
        const uint64_t E = S + n;
        const uint8_t* data = j.data;
#ifdef RPGPU_CHECKED
        {
            bool bad = false;
            RP_CHECK(bad, segi < j.n_segments, "b=%llu segi=%u flags=%u", (unsigned long long)b, segi, flags0);
            if (bad) continue;
            const uint64_t slen = j.seg_off[segi + 1] - j.seg_off[segi];
            RP_CHECK(bad, segi < j.n_segments && uni64(R->file_pos) + RPGPU_HEADER_SIZE + n <= slen && E <= j.data_len,
                     "b=%llu seg=%u file_pos=%llu n=%llu slen=%llu E=%llu data_len=%llu", (unsigned long long)b, segi,
                     (unsigned long long)R->file_pos, (unsigned long long)n, (unsigned long long)slen,
                     (unsigned long long)E, (unsigned long long)j.data_len);
            const uint64_t ib0 = j.slots[b], ib1 = j.slots[b + 1];
            RP_CHECK(bad, ib0 <= ib1 && ib1 <= j.slots[nb], "b=%llu slots %llu %llu total %llu", (unsigned long long)b,
                     (unsigned long long)ib0, (unsigned long long)ib1, (unsigned long long)j.slots[nb]);
            if (bad) continue;
        }
#endif
        // CRC state after the BE40 prefix with init ~0: c40 ^ raw contribution
        // of the prefix bytes (computed by k_emit, parked in reserved1)
        uint32_t Tst = uni32((uint32_t)R->reserved1) ^ T->c40;

        // Lane regions are anchored at E16 = E rounded down to 16 bytes so
        // every vector load is an aligned 16-byte load; chunk c spans
        // [E16 - kStream*(Ntot-c), +kStream), chunk 0 is clipped at S, and
        // the <16-byte tail [E16, E) is folded in after the rounds.
        const uint64_t E16 = (E & ~(uint64_t)15) > S ? (E & ~(uint64_t)15) : S;
        const uint64_t n16 = E16 - S;
        if (n16 > 0) {
            const uint64_t Ntot = (n16 + kStream - 1) / kStream;
            const uint64_t R_ = (Ntot + 127) / 128;
            for (uint64_t r = 0; r < R_; r++) {
                const int64_t c0 = (int64_t)Ntot - (int64_t)(128 * (R_ - r));
                const int64_t ca = c0 + 2 * (int64_t)l;
                // lane region start (bytes), may lie before S in round 0
                const int64_t a = (int64_t)E16 - (int64_t)kStream * ((int64_t)Ntot - ca);
                uint32_t sA = 0, sB = 0;
                if (r == 0) {
                    // the lane holding chunk 0 starts from the prefix state
                    if (ca == 0) sA = Tst;
                    else if (ca + 1 == 0) sB = Tst;
                } else if (l == 0) {
                    sA = Tst;
                }
                if (a >= (int64_t)S) {
                    // full 256-byte region, 16-byte aligned
#ifdef RPGPU_CHECKED
                    if (!(a + 256 <= (int64_t)E16 && (a & 15) == 0))
                        printf("RPGPU_CHECK region b=%llu a=%lld E16=%llu S=%llu\n", (unsigned long long)b, (long long)a,
                               (unsigned long long)E16, (unsigned long long)S);
#endif
                    const uint4* q = (const uint4*)(data + a);
                    uint4 v[16];
#pragma unroll
                    for (int k = 0; k < 16; k++) v[k] = q[k];
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        sA = step4(lds, K, sA, v[k].x);
                        sB = step4(lds, K, sB, v[k + 8].x);
                        sA = step4(lds, K, sA, v[k].y);
                        sB = step4(lds, K, sB, v[k + 8].y);
                        sA = step4(lds, K, sA, v[k].z);
                        sB = step4(lds, K, sB, v[k + 8].z);
                        sA = step4(lds, K, sA, v[k].w);
                        sB = step4(lds, K, sB, v[k + 8].w);
                    }
                } else if (a + (int64_t)kLaneBytes > (int64_t)S) {
                    // region straddles the payload start (round 0 only): bytes
                    // before S are skipped; stream A covers [a, a+128)
                    for (int st = 0; st < 2; st++) {
                        const int64_t sa = a + st * (int64_t)kStream;
                        const int64_t se = sa + (int64_t)kStream;
                        if (se <= (int64_t)S) continue;
                        uint32_t sv = st ? sB : sA;
                        int64_t x = sa > (int64_t)S ? sa : (int64_t)S;
                        for (; ((se - x) & 3) != 0; x++) sv = step1(lds, K, sv, data[x]);
                        for (; x < se; x += 4) sv = step4(lds, K, sv, ldu32(data + x));
                        if (st) sB = sv; else sA = sv;
                    }
                }
                // combine: s = shift(sA, kStream) ^ sB, then a tree over lanes
                uint32_t sv = shift_lvl(lds, sA, 0) ^ sB;
#pragma unroll
                for (uint32_t lv = 1; lv < kCombineLevels; lv++) {
                    const uint32_t d = 1u << (lv - 1);
                    const uint32_t other = __shfl_down(sv, d, 64);
                    sv = shift_lvl(lds, sv, lv) ^ other;
                }
                Tst = uni32(sv);  // lane 0 holds the state after this round
            }
        }
        // tail bytes [E16, E): fewer than 16, uniform
        for (uint64_t x = E16; x < E; x++) Tst = uni32(step1(lds, K, Tst, data[x]));
        const uint32_t crc = ~Tst;
        uint32_t f = flags0;
        if (crc == uni32(R->crc)) f |= RPGPU_F_CRC_OK;

        // plan results
        const uint64_t ib = j.slots[b];
        const uint64_t islots = j.slots[b + 1] - ib;
        const uint32_t codec = (uint32_t)(uint16_t)R->attrs & 7;
        uint32_t parsed = 0, perr = 0;
        if (codec == 0 && (j.flags & RPGPU_JOB_PARSE)) {
            const bool idx_ok = ib + islots <= j.record_capacity;
            WalkResult w = walk_records(data + S, n, R->record_count, (uint32_t)b,
                                        idx_ok ? j.records + ib : nullptr, idx_ok ? islots : 0);
            parsed = w.parsed;
            perr = w.err;
            f |= RPGPU_F_PARSED;
            if (perr == 0) {
                f |= RPGPU_F_PARSE_ASYNC_OK;
                if (w.trailing == 0) f |= RPGPU_F_PARSE_OK;
                else perr = RPGPU_PARSE_ERR_TRAILING;
            }
            if (f & RPGPU_F_PARSE_OK) {
                if (idx_ok) f |= RPGPU_F_INDEX_WRITTEN;
                else { perr = RPGPU_PARSE_ERR_INDEX_CAPACITY; if (l == 0) atomicOr(&j.counters[1], 2u); }
            }
        }
        if (l == 0) {
            R->crc_computed = crc;
            R->flags = f;
            R->index_base = ib;
            R->decoded_off = j.dcap[b];
            R->records_parsed = parsed;
            R->parse_err = (uint8_t)perr;
            R->reserved1 = 0;
        }
    }
}

// ---------------------------------------------------------------------------
// Finalize: per-segment checkpoint (storage/log_replayer.cc:62-79), bytes
// consumed (storage/parser.cc:183-254), bitmap and totals.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize_segments(DeviceJob j) {
    const uint32_t s = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t first = j.chunk_count[j.chunk_base[s]];
    const uint64_t last = j.chunk_count[j.chunk_base[s + 1]];
    const uint64_t cnt = last - first;
    __shared__ uint64_t s_bad;
    __shared__ uint64_t s_bytes, s_phys, s_rec;
    if (tid == 0) { s_bad = cnt; s_bytes = 0; s_phys = 0; s_rec = 0; }
    __syncthreads();
    const bool fits = last <= j.batch_capacity;
    if (fits) {
        for (uint64_t i = tid; i < cnt; i += 256) {
            const uint32_t f = j.batches[first + i].flags;
            if (!((f & RPGPU_F_COMPLETE) && (f & RPGPU_F_CRC_OK))) atomicMin((unsigned long long*)&s_bad, (unsigned long long)i);
        }
    }
    __syncthreads();
    const uint64_t bad = s_bad;
    const uint64_t upto = bad < cnt ? bad + 1 : cnt;
    uint64_t bytes = 0, phys = 0;
    if (fits) {
        for (uint64_t i = tid; i < cnt; i += 256) {
            const uint64_t sz = (uint64_t)(int64_t)j.batches[first + i].size_bytes;
            if (i < upto) bytes += sz;
            if (i < bad) phys += sz;
        }
    }
    atomicAdd((unsigned long long*)&s_bytes, (unsigned long long)bytes);
    atomicAdd((unsigned long long*)&s_phys, (unsigned long long)phys);
    __syncthreads();
    if (tid == 0) {
        rpgpu_segment_summary sm;
        sm.first_batch = first;
        sm.n_batches = cnt;
        const SegTerm t = j.seg_term[s];
        sm.terminal_pos = t.pos;
        sm.terminal_errc = t.errc;
        sm.terminal_eof = t.eof;
        sm.bytes_consumed = fits ? s_bytes : 0;
        sm.first_bad = (uint32_t)bad;
        sm.has_checkpoint = 0;
        sm.ckpt_last_offset = 0;
        sm.ckpt_truncate_pos = 0;
        if (fits && bad > 0) {
            const rpgpu_batch_result& g = j.batches[first + bad - 1];
            sm.has_checkpoint = 1;
            sm.ckpt_last_offset = (int64_t)((uint64_t)g.base_offset + (uint64_t)(int64_t)g.last_offset_delta);
            sm.ckpt_truncate_pos = s_phys;
        }
        const uint64_t sf = first < j.batch_capacity ? first : j.batch_capacity;
        const uint64_t sl = last < j.batch_capacity ? last : j.batch_capacity;
        sm.n_records = j.slots[sl] - j.slots[sf];
        sm.reserved[0] = sm.reserved[1] = 0;
        j.summaries[s] = sm;
        (void)nb_total;
    }
}

DEV bool batch_valid(uint32_t f, uint32_t job_flags) {
    if (!(f & RPGPU_F_HEADER_OK) || !(f & RPGPU_F_COMPLETE) || !(f & RPGPU_F_CRC_OK)) return false;
    if (f & RPGPU_F_CODEC_INVALID) return false;
    if ((f & RPGPU_F_COMPRESSED) && (job_flags & RPGPU_JOB_DECODE) && !(f & RPGPU_F_CODEC_UNSUPPORTED) &&
        !(f & RPGPU_F_CODEC_OK))
        return false;
    if ((f & RPGPU_F_PARSED) && !(f & RPGPU_F_PARSE_OK)) return false;
    return true;
}

__global__ __launch_bounds__(256) void k_finalize_bitmap(DeviceJob j) {
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w * 64 >= nb) return;
    uint64_t word = 0;
    for (uint32_t i = 0; i < 64; i++) {
        const uint64_t b = w * 64 + i;
        if (b < nb && batch_valid(j.batches[b].flags, j.flags)) word |= 1ull << i;
    }
    j.bitmap[w] = word;
}

__global__ void k_finalize_totals(DeviceJob j) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    rpgpu_job_totals t;
    t.n_batches = nb_total;
    t.n_records = j.slots[nb];
    t.decoded_bytes = j.dcap[nb];
    t.batch_capacity_needed = nb_total;
    t.record_capacity_needed = j.slots[nb];
    t.decoded_capacity_needed = j.dcap[nb];
    uint32_t ov = j.counters[1];
    if (nb_total > j.batch_capacity) ov |= 1;
    if (j.slots[nb] > j.record_capacity) ov |= 2;
    if (j.dcap[nb] > j.decoded_capacity) ov |= 4;
    t.overflow = ov;
    t.n_rewalks = j.counters[0];
    t.reserved[0] = t.reserved[1] = 0;
    *j.totals = t;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// chunk_base[s] = sum over earlier segments of max(1, ceil(len / chunk_bytes))
__global__ __launch_bounds__(1024) void k_chunk_base(DeviceJob j) {
    __shared__ uint64_t sh[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < j.n_segments; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        uint64_t v = 0;
        if (i < j.n_segments) {
            const uint64_t len = j.seg_off[i + 1] - j.seg_off[i];
            v = (len + j.chunk_bytes - 1) / j.chunk_bytes;
            if (v == 0) v = 1;
        }
        sh[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            uint64_t x = threadIdx.x >= (uint32_t)o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < j.n_segments) ((uint64_t*)j.chunk_base)[i] = carry + sh[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += sh[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) ((uint64_t*)j.chunk_base)[j.n_segments] = carry;
}

hipError_t launch_chunk_base(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_chunk_base, dim3(1), dim3(1024), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_discover(const DeviceJob& j, hipStream_t s) {
    const uint32_t grid = (j.total_chunks + 3) / 4;
    hipLaunchKernelGGL(k_discover, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_resolve(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_resolve, dim3(j.n_segments), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_emit(const DeviceJob& j, hipStream_t s) {
    const uint32_t grid = (j.total_chunks + 3) / 4;
    hipLaunchKernelGGL(k_emit, dim3(grid), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_validate(const DeviceJob& j, hipStream_t s, uint32_t grid) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_validate, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsValidateBytes);
        attr = true;
    }
    hipLaunchKernelGGL(k_validate, dim3(grid), dim3(1024), kLdsValidateBytes, s, j);
    return hipGetLastError();
}
hipError_t launch_finalize(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize_segments, dim3(j.n_segments), dim3(256), 0, s, j);
    const uint64_t words = (j.batch_capacity + 63) / 64;
    if (j.bitmap) {
        const uint32_t grid = (uint32_t)((words + 255) / 256);
        hipLaunchKernelGGL(k_finalize_bitmap, dim3(grid ? grid : 1), dim3(256), 0, s, j);
    }
    hipLaunchKernelGGL(k_finalize_totals, dim3(1), dim3(64), 0, s, j);
    return hipGetLastError();
}

size_t scan_temp_bytes(uint64_t n) { return ((n + kScanTile - 1) / kScanTile + 1) * sizeof(uint64_t); }

// exclusive scan of data[0..n) in place; data[n] receives the total.
// n is read from *d_n when d_n != nullptr (n_cap bounds the grid).
hipError_t scan_exclusive_dev(uint64_t* data, const uint64_t* d_n, uint64_t n_cap, uint64_t* temp, hipStream_t s) {
    const uint32_t tiles = (uint32_t)((n_cap + kScanTile - 1) / kScanTile);
    const uint32_t g = tiles ? tiles : 1;
    hipLaunchKernelGGL(k_scan_tiles, dim3(g), dim3(256), 0, s, data, d_n, n_cap, temp);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, s, temp, d_n, n_cap, temp + g);
    hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(256), 0, s, data, d_n, n_cap, temp);
    return hipGetLastError();
}

__global__ void k_copy_total(uint64_t* data, const uint64_t* d_n, uint64_t n_host, const uint64_t* total) {
    const uint64_t n = d_n ? (*d_n < n_host ? *d_n : n_host) : n_host;
    data[n] = *total;
}

hipError_t scan_exclusive_u64(uint64_t* data, uint64_t n, void* temp, size_t temp_bytes, hipStream_t s) {
    (void)temp_bytes;
    uint64_t* t = (uint64_t*)temp;
    const uint32_t tiles = (uint32_t)((n + kScanTile - 1) / kScanTile);
    scan_exclusive_dev(data, nullptr, n, t, s);
    hipLaunchKernelGGL(k_copy_total, dim3(1), dim3(1), 0, s, data, (const uint64_t*)nullptr, n, t + (tiles ? tiles : 1));
    return hipGetLastError();
}

hipError_t scan_exclusive_u64_devn(uint64_t* data, const uint64_t* d_n, uint64_t n_cap, void* temp, hipStream_t s) {
    uint64_t* t = (uint64_t*)temp;
    const uint32_t tiles = (uint32_t)((n_cap + kScanTile - 1) / kScanTile);
    scan_exclusive_dev(data, d_n, n_cap, t, s);
    hipLaunchKernelGGL(k_copy_total, dim3(1), dim3(1), 0, s, data, d_n, n_cap, t + (tiles ? tiles : 1));
    return hipGetLastError();
}

}  // namespace rp
