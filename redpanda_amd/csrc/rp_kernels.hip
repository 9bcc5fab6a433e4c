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
#include "rp_device.h"

namespace rp {


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

struct WalkOut {
    uint64_t exit;
    uint64_t tpos;
    uint32_t count;
    int32_t term;
};

// Follow the chain from p while headers start before ce.
DEV WalkOut wave_walk(uint32_t layout, const uint8_t* __restrict__ seg, uint64_t len, uint64_t p, uint64_t ce,
                      const Tables* __restrict__ T) {
    WalkOut w;
    w.count = 0;
    w.term = -1;
    w.tpos = 0;
    while (p < ce) {
        Hdr h = wave_header_of(layout, seg, len, p, T);
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

// Discovery scan (speculation only: a wrong guess is caught by k_resolve,
// so none of this decides a verdict).  A 1 KiB step covers positions
// a + 16 l + i (a 16-aligned, lane l, i < 16) from five coalesced 16-byte
// loads per lane that hold every field a header check reads (bytes i .. i +
// 60); the next step's loads are in flight while a step is tested.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct ScanWin {
    uint32_t w[20];
};

// one 16-byte load per lane; the next 64 bytes come from lanes l + 1 .. l + 4
// (DPP wave_shl:1, four hops), lane 63 loading what lies past the step.
// (Five overlapping loads per lane, or plain instead of non-temporal loads:
// C2 discovery 14.4 / 14.0 ms against 13.5 ms here; the scan is bound by the
// per-position field checks, not by its loads.)
DEV u32x4 scan_ld(const uint8_t* __restrict__ data, uint64_t data_len, uint64_t x) {
    u32x4 v = {0, 0, 0, 0};
    if (x + 16 <= data_len) v = __builtin_nontemporal_load((const u32x4*)(data + x));
    return v;
}
DEV void scan_load(const uint8_t* __restrict__ data, uint64_t data_len, uint64_t a, ScanWin& sw) {
    const uint32_t l = lane();
    const uint64_t la = a + 16ull * l;
    u32x4 v = scan_ld(data, data_len, la), d[4];
#pragma unroll
    for (int k = 1; k < 5; k++) {
        d[k - 1] = (u32x4){0, 0, 0, 0};
        if (l == 63) d[k - 1] = scan_ld(data, data_len, la + 16ull * k);
    }
    sw.w[0] = v.x; sw.w[1] = v.y; sw.w[2] = v.z; sw.w[3] = v.w;
#pragma unroll
    for (int k = 1; k < 5; k++) {
#pragma unroll
        for (int c = 0; c < 4; c++)
            sw.w[4 * k + c] = (uint32_t)__builtin_amdgcn_update_dpp((int)d[k - 1][c], (int)sw.w[4 * (k - 1) + c], 0x130,
                                                                   0xF, 0xF, false);
    }
}

// Plausible header fields (disk or wire) given the 61 header bytes through
// W32(o) / B(o); `rem` = bytes from the header to the segment end.  The
// base_offset sign bit must be clear (offsets are never negative in a real
// log; a real header this misses only costs a re-walk in k_resolve).
#define RP_PLAUSIBLE(layout, W32, B, rem, size_out)                                                          \
    ((layout) == RPGPU_LAYOUT_WIRE                                                                           \
         ? ((size_out) = (int32_t)__builtin_bswap32(W32(8)) + 12,                                            \
            (B(0) & 0x80u) == 0 && (int32_t)__builtin_bswap32(W32(8)) >= (int32_t)RPGPU_HEADER_SIZE - 12 &&  \
                (uint32_t)(size_out) <= (rem) && B(16) == 2u && (B(22) & 7u) <= 4u &&                       \
                (int32_t)__builtin_bswap32(W32(57)) >= 0 && (int32_t)__builtin_bswap32(W32(57)) <= (size_out)) \
         : ((size_out) = (int32_t)W32(4),                                                                    \
            W32(0) != 0u && (size_out) >= (int32_t)RPGPU_HEADER_SIZE && (uint32_t)(size_out) <= (rem) &&     \
                (B(15) & 0x80u) == 0 && B(16) - 1u < 32u && (B(21) & 7u) <= 4u && (int32_t)W32(57) >= 0 &&  \
                (int32_t)W32(57) <= (size_out)))

// the header a candidate's size points at must be plausible too (or lie in
// the last 61 bytes of the segment): random payload bytes pass the field
// checks about once per KiB, both checks about once per GiB
DEV bool follow_ok(uint32_t layout, const uint8_t* __restrict__ seg, uint64_t len, uint64_t q) {
    if (len - q < RPGPU_HEADER_SIZE) return true;
    const uint8_t* h = seg + q;
    const uint32_t f0 = ldu32(h), f4 = ldu32(h + 4), f8 = ldu32(h + 8), f12 = ldu32(h + 12), f16 = ldu32(h + 16),
                   f21 = ldu32(h + 21), f57 = ldu32(h + 57);
#define RP_W32(o) ((o) == 0 ? f0 : (o) == 4 ? f4 : (o) == 8 ? f8 : (o) == 21 ? f21 : f57)
#define RP_B(o) ((o) == 0 ? (f0 & 0xFFu) : (o) == 15 ? (f12 >> 24) : (o) == 16 ? (f16 & 0xFFu) : (o) == 21 ? (f21 & 0xFFu) : ((f21 >> 8) & 0xFFu))
    const uint64_t rem64 = len - q;
    const uint32_t rem = rem64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)rem64;
    int32_t size;
    const bool ok = RP_PLAUSIBLE(layout, RP_W32, RP_B, rem, size);
#undef RP_W32
#undef RP_B
    return ok;
}

// candidate bits of a step (bit i = position a + 16 l + i), with the first
// candidate's follow-up header also checked
DEV uint32_t scan_step(uint32_t layout, const uint8_t* __restrict__ seg, const ScanWin& sw, uint64_t a, uint64_t off,
                       uint64_t len, uint64_t cs, uint64_t ce) {
    const uint64_t la = a + 16ull * lane();
    // 32-bit bounds relative to this lane's first position r = la - off:
    // position i is inside the chunk iff lo <= i < hi, and a size fits iff
    // size <= rem - i (size >= 61 > 0)
    const int64_t r = (int64_t)(la - off);
    const int64_t lo64 = (int64_t)cs - r, hi64 = (int64_t)ce - r, rem64 = (int64_t)len - r;
    const int32_t lo = lo64 < 0 ? 0 : lo64 > 16 ? 16 : (int32_t)lo64;
    const int32_t hi = hi64 < 0 ? 0 : hi64 > 16 ? 16 : (int32_t)hi64;
    const uint32_t rem = rem64 < 0 ? 0u : rem64 > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)rem64;
    uint32_t m = 0, fi = 16, fsize = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
#define RP_W32(o) __builtin_amdgcn_alignbyte(sw.w[((i) + (o)) / 4 + 1], sw.w[((i) + (o)) / 4], ((i) + (o)) & 3)
#define RP_B(o) ((sw.w[((i) + (o)) / 4] >> (8 * (((i) + (o)) & 3))) & 0xFFu)
        const bool in = i >= lo && i < hi && (uint32_t)i + RPGPU_HEADER_SIZE <= rem;
        int32_t size;
        const bool pass = RP_PLAUSIBLE(layout, RP_W32, RP_B, rem - (uint32_t)i, size);
#undef RP_W32
#undef RP_B
        const bool c = in && pass;
        if (c && fi == 16) { fi = i; fsize = (uint32_t)size; }
        m |= (uint32_t)c << i;
    }
    if (fi < 16 && !follow_ok(layout, seg, len, (uint64_t)r + fi + fsize)) m &= ~(1u << fi);
    return m;
}

// Scan budget: a chunk is scanned for its first header over at most its
// first kScanBudget bytes.  A chunk that lies inside a large batch holds no
// header start at all and was scanned to its end (C2: 1 MiB batches over
// 256 KiB chunks, discovery 13.5 ms of a 56 ms step); with the budget such a
// chunk is marked kExhausted instead, and k_chain carries the chain of the
// nearest earlier chunk with an entry through it (storage/parser.cc:139-176
// semantics are unchanged: k_resolve verifies every chunk's entry against
// the true chain and re-walks any it cannot confirm).
// A chunk then holds a header start within its first kScanBudget bytes about
// kScanBudget / (mean batch bytes) of the time: C2's ~420 KB batches leave
// runs of tens of spent chunks between two entries (up to ~150 at 16 KiB),
// each carried by one k_chain lane at ~0.6 header hops per chunk.  (32 KiB:
// C2 discover 3.0 ms, a 32-chunk carry limit made k_resolve re-walk the
// rest of the longer runs serially, 0.86 ms.  Round 6, 16 -> 8 KiB: C2
// discover 1.79 -> 1.28 ms, C5 0.90 -> 0.77 ms, C1 unchanged; 4 KiB: C2 1.17,
// C5 0.82 ms.)
#ifndef RPGPU_SCAN_BUDGET_KIB
#define RPGPU_SCAN_BUDGET_KIB 8
#endif
constexpr uint64_t kScanBudget = (uint64_t)RPGPU_SCAN_BUDGET_KIB << 10;
constexpr uint64_t kExhausted = kNone - 1;
// chunks one k_chain lane carries its chain through: unbounded in practice
// (a run is as long as the gap between two entries); the serial cost is the
// headers in the run, which k_resolve would otherwise re-walk serially
constexpr uint32_t kMaxCarry = 1u << 30;

// One wave per chunk, four chunks per workgroup.  (Four waves per chunk,
// scanning interleaved steps, cut C2's discovery from 14.4 to 9.9 ms but
// cost C1 0.2 ms of its 5 ms step: most C1 chunks find their entry within
// a few steps, and four waves then scan four times the bytes.)
// Output: the default (no entry) ChunkRec, and the discovered entry in
// chunk_entry[g] (a position, kNone: scanned to the chunk end without a
// header, kExhausted: budget spent); k_resolve overwrites chunk_entry later.
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
    bool scan = true;
    if (w == 0) {
        entry = 0;
        scan = false;
    } else if (j.seeds) {
        // index-seeded: follow the chain from the last seed at or before the
        // chunk start (or the segment start) to the first header at or after
        // it; every hop is a verified header, a failed one falls back to the scan
        const uint64_t s0 = uni64(j.seed_off[s]), s1 = uni64(j.seed_off[s + 1]);
        uint64_t lo = s0, hi = s1;  // first seed > cs
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (uni64(j.seeds[m]) <= cs) lo = m + 1;
            else hi = m;
        }
        uint64_t q = lo > s0 ? uni64(j.seeds[lo - 1]) : 0;
        bool ok = q < len;
        for (uint32_t hop = 0; ok && q < cs; hop++) {
            const Hdr h = wave_header_of(j.layout, seg, len, q, j.tables);
            if (hop >= 64 || h.status >= 0 || len - q - RPGPU_HEADER_SIZE < h.need) { ok = false; break; }
            q += RPGPU_HEADER_SIZE + h.need;
        }
        if (ok && q >= cs) {
            if (q < ce) {
                const Hdr h = wave_header_of(j.layout, seg, len, q, j.tables);
                ok = h.status < 0 && len - q - RPGPU_HEADER_SIZE >= h.need;
            }
            if (ok) {
                entry = q < ce ? q : kNone;
                scan = false;
            }
        }
    }
    bool exhausted = false;
    if (scan) {
        // candidates in ascending order: lanes cover consecutive 16-byte
        // spans, bits ascend within a lane
        uint64_t a = (off + cs) & ~15ull;
        const uint64_t se = (cs + kScanBudget < ce) ? cs + kScanBudget : ce;
        ScanWin cur, nxt;
        scan_load(j.data, j.data_len, a, cur);
        for (; a < off + se && entry == kNone; a += 1024) {
            if (a + 1024 < off + se) scan_load(j.data, j.data_len, a + 1024, nxt);
            const uint32_t m = scan_step(j.layout, seg, cur, a, off, len, cs, ce);
            uint64_t lanes = __ballot(m != 0);
            while (lanes && entry == kNone) {
                const uint32_t l = __builtin_ctzll(lanes);
                lanes &= lanes - 1;
                uint32_t bits = rl(m, (int)l);
                while (bits) {
                    const uint32_t i = __builtin_ctz(bits);
                    bits &= bits - 1;
                    const uint64_t qc = a + 16ull * l + i - off;
                    Hdr h = wave_header_of(j.layout, seg, len, qc, j.tables);
                    if (h.status < 0 && len - qc - RPGPU_HEADER_SIZE >= h.need) { entry = qc; break; }
                }
            }
            cur = nxt;
        }
        exhausted = entry == kNone && se < ce;
    }
    if (lane() == 0) {
        ChunkRec r;
        r.entry = kNone;
        r.exit = kNone;
        r.count = 0;
        r.term = -1;
        r.tpos = 0;
        j.chunks[g] = r;
        j.chunk_entry[g] = entry != kNone ? entry : exhausted ? kExhausted : kNone;
    }
}

// Follow the chain from p while headers start before ce, one chain per lane
// (wave_walk's semantics with lane_header).
DEV WalkOut lane_walk(uint32_t layout, const uint8_t* __restrict__ seg, uint64_t len, uint64_t p, uint64_t ce,
                      const uint32_t* __restrict__ th, uint32_t c57) {
    WalkOut w;
    w.count = 0;
    w.term = -1;
    w.tpos = 0;
    while (p < ce) {
        const LHdr h = lane_header(layout, seg, len, p, th, c57);
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

// Speculative chain of every chunk from the entry k_discover found, one chunk
// per LANE: a chunk's headers are a dependent chain, so 64 chains per wave
// keep 64 header reads in flight where a wave-cooperative walk had one.
// The chain then runs on through the following chunks whose scan budget
// was spent (kExhausted, up to kMaxCarry of them), recording each one's
// speculative entry / exit / count as a scan would have: such a chunk is
// written by this lane only (runs of kExhausted chunks after an entry are
// disjoint), and chunk_entry is read-only here.
__global__ __launch_bounds__(256) void k_chain(DeviceJob j) {
    extern __shared__ uint32_t th[];
    init_lds_hdr(th, j.tables);
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= j.total_chunks) return;
    const uint64_t entry = j.chunk_entry[g];
    if (entry >= kExhausted) return;
    const uint32_t s = find_segment(j.chunk_base, j.n_segments, g);
    const uint64_t w = g - j.chunk_base[s];
    const uint64_t W = j.chunk_base[s + 1] - j.chunk_base[s];
    const uint64_t off = j.seg_off[s], len = j.seg_off[s + 1] - off;
    uint64_t p = entry;
    for (uint32_t k = 0;; k++) {
        const uint64_t cs = (w + k) * j.chunk_bytes;
        const uint64_t ce = (cs + j.chunk_bytes < len) ? cs + j.chunk_bytes : len;
        ChunkRec r;
        r.entry = kNone;
        r.exit = kNone;
        r.count = 0;
        r.term = -1;
        r.tpos = 0;
        if (p < ce) {
            // p >= cs: the first chain position at or after the chunk start
            const WalkOut o = lane_walk(j.layout, j.data + off, len, p, ce, th, j.tables->c57);
            r.entry = p;
            r.exit = o.exit;
            r.count = o.count;
            r.term = o.term;
            r.tpos = o.tpos;
            p = o.exit;
        }
        j.chunks[g + k] = r;
        if (r.term >= 0 || k + 1 >= kMaxCarry || w + k + 1 >= W || j.chunk_entry[g + k + 1] != kExhausted) break;
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
                o = wave_walk(j.layout, seg, len, P, ce2, j.tables);
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
__global__ __launch_bounds__(256) void k_emit(DeviceJob j) {
    extern __shared__ uint32_t th[];
    init_lds_hdr(th, j.tables);
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= j.total_chunks) return;
    const uint64_t base_ord = j.chunk_count[g];
    const uint64_t cnt = j.chunk_count[g + 1] - base_ord;
    if (cnt == 0) return;
    const uint32_t s = find_segment(j.chunk_base, j.n_segments, g);
    const uint64_t off = j.seg_off[s], len = j.seg_off[s + 1] - off;
    const uint8_t* seg = j.data + off;
    const uint32_t c57 = j.tables->c57;
    const bool wire = j.layout == RPGPU_LAYOUT_WIRE;
    uint64_t p = j.chunk_entry[g];
    for (uint64_t i = 0; i < cnt; i++) {
#ifdef RPGPU_CHECKED
        if (!(p < len)) {
            printf("RPGPU_CHECK emit g=%llu i=%llu cnt=%llu p=%llu len=%llu\n", (unsigned long long)g,
                   (unsigned long long)i, (unsigned long long)cnt, (unsigned long long)p, (unsigned long long)len);
            break;
        }
#endif
        const LHdr h = lane_header(j.layout, seg, len, p, th, c57);  // known valid (resolved chain)
        const uint64_t ord = base_ord + i;
        const bool complete = (len - p - RPGPU_HEADER_SIZE) >= h.need;
        // prefix state of the batch crc: raw CRC contribution of the BE40
        // prefix (init ~0 is added by k_validate)
        const uint32_t praw = lane_prefix_raw(j.layout, h.w, th);
        const uint32_t attrs = wire ? lbe16(h.w, 21) : l16(h.w, 21);
        const int32_t rc = (int32_t)(wire ? lbe32(h.w, 57) : l32(h.w, 57));
        const uint32_t codec = attrs & 7;
        uint64_t slots = 0, cap = 0;
        const bool decodable = (codec == RPGPU_CODEC_LZ4 || codec == RPGPU_CODEC_SNAPPY) && (j.flags & RPGPU_JOB_DECODE);
        if (complete) {
            if (codec == 0) {
                if ((j.flags & RPGPU_JOB_PARSE) && rc > 0 && (uint64_t)rc <= h.need) slots = (uint64_t)rc;
            } else if (decodable) {
                cap = decode_capacity_dev((int)codec, seg + p + RPGPU_HEADER_SIZE, h.need);
                if ((j.flags & RPGPU_JOB_PARSE) && rc > 0 && (uint64_t)rc <= cap) slots = (uint64_t)rc;
            }
        }
        if (ord < j.batch_capacity) {
            rpgpu_batch_result r;
            r.file_pos = p;
            uint32_t f = RPGPU_F_HEADER_OK;
            if (wire) {
                // kafka_batch_adapter::read_header (kafka_batch_adapter.cc:32-91)
                r.base_offset = (int64_t)lbe64(h.w, 0);
                r.first_timestamp = (int64_t)lbe64(h.w, 27);
                r.max_timestamp = (int64_t)lbe64(h.w, 35);
                r.producer_id = (int64_t)lbe64(h.w, 43);
                r.last_offset_delta = (int32_t)lbe32(h.w, 23);
                r.base_sequence = (int32_t)lbe32(h.w, 53);
                r.header_crc = 0;
                r.crc = lbe32(h.w, 17);
                r.producer_epoch = (int16_t)lbe16(h.w, 51);
                r.type = 1;  // record_batch_type::raft_data
                if (lb(h.w, 16) == 2) f |= RPGPU_F_WIRE_V2;
            } else {
                // storage::header_from_iobuf (storage/parser.cc:36-76)
                r.base_offset = (int64_t)l64(h.w, 8);
                r.first_timestamp = (int64_t)l64(h.w, 27);
                r.max_timestamp = (int64_t)l64(h.w, 35);
                r.producer_id = (int64_t)l64(h.w, 43);
                r.last_offset_delta = (int32_t)l32(h.w, 23);
                r.base_sequence = (int32_t)l32(h.w, 53);
                r.header_crc = h.hcrc;
                r.crc = l32(h.w, 17);
                r.producer_epoch = (int16_t)l16(h.w, 51);
                r.type = (int8_t)lb(h.w, 16);
            }
            r.size_bytes = h.size;
            r.record_count = rc;
            r.crc_computed = 0;
            r.header_crc_computed = h.computed;
            if (complete) f |= RPGPU_F_COMPLETE;
            if (codec) f |= RPGPU_F_COMPRESSED;
            if (codec >= 5) f |= RPGPU_F_CODEC_INVALID;
            const bool host_codec = (j.flags & RPGPU_JOB_DECODE) && (j.flags & RPGPU_JOB_HOST_CODECS);
            if (complete && codec == RPGPU_CODEC_ZSTD && !(j.flags & RPGPU_JOB_DECODE)) f |= RPGPU_F_CODEC_UNSUPPORTED;
            r.flags = f;
            r.segment = s;
            // scratch for k_validate: absolute payload start (overwritten with
            // the record-index base there)
            r.index_base = off + p + RPGPU_HEADER_SIZE;
            r.decoded_off = 0;
            r.records_parsed = 0;
            r.decoded_len = (complete && codec == 0) ? (uint32_t)h.need : 0;
            r.decoded_crc = 0;
            r.decoded_header_crc = 0;
            r.attrs = (int16_t)attrs;
            r.parse_err = 0;
            r.reserved0 = 0;
            // scratch for k_validate: raw CRC contribution of the BE prefix
            r.reserved1 = praw;
            j.batches[ord] = r;
            j.slots[ord] = slots;
            j.dcap[ord] = cap;
            // decode work list for k_decode (order is irrelevant: every item
            // writes only its own batch and its own reserved arena slot)
            if (complete && decodable) j.decode_list[atomicAdd(&j.counters[2], 1u)] = (uint32_t)ord;
            // gzip and zstd members: sized by k_members_first (dcap /
            // slots above are 0 until then)
            if (complete && (j.flags & RPGPU_JOB_DECODE) &&
                (codec == RPGPU_CODEC_GZIP || (codec == RPGPU_CODEC_ZSTD && !host_codec)))
                j.inf_list[atomicAdd(&j.counters[16], 1u)] = (uint32_t)ord;
            // zstd members with RPGPU_JOB_HOST_CODECS: decoded by the host step
            if (complete && codec == RPGPU_CODEC_ZSTD && host_codec)
                j.host_list[atomicAdd(&j.counters[19], 1u)] = (uint32_t)ord;
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
// Finalize: per-segment checkpoint (storage/log_replayer.cc:62-79) and bytes
// consumed (storage/parser.cc:183-254).  The first batch failing
// complete && crc_ok was recorded by k_validate with atomicMin; positions
// accumulate size_bytes (storage/parser.cc:118-128), so the sums are the end
// position of one batch — except in segments >= 4 GiB, where a header with
// size_bytes < 61 can still chain (need wraps as uint32) and the sums are
// taken explicitly.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize_segments(DeviceJob j) {
    const uint32_t s = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const uint64_t first = j.chunk_count[j.chunk_base[s]];
    const uint64_t last = j.chunk_count[j.chunk_base[s + 1]];
    const uint64_t cnt = last - first;
    const bool fits = last <= j.batch_capacity;
    const uint64_t fb = j.seg_first_bad[s];
    const uint64_t bad = (fits && fb < cnt) ? fb : cnt;
    // disk: continuous_batch_parser also counts the batch it stopped in
    // (storage/parser.cc:178-190); wire: batch_reader consumed the accepted
    // prefix (kafka/protocol/batch_reader.cc:122-156)
    const uint64_t upto = bad < cnt ? bad + (j.layout == RPGPU_LAYOUT_WIRE ? 0 : 1) : cnt;
    const uint64_t seg_len = j.seg_off[s + 1] - j.seg_off[s];
    __shared__ unsigned long long s_bytes, s_phys;
    if (tid == 0) { s_bytes = 0; s_phys = 0; }
    __syncthreads();
    if (fits) {
        if (seg_len < (1ull << 32)) {
            if (tid == 0) {
                if (upto > 0) {
                    const rpgpu_batch_result& g = j.batches[first + upto - 1];
                    s_bytes = g.file_pos + (uint64_t)(int64_t)g.size_bytes;
                }
                if (bad > 0) {
                    const rpgpu_batch_result& g = j.batches[first + bad - 1];
                    s_phys = g.file_pos + (uint64_t)(int64_t)g.size_bytes;
                }
            }
        } else {
            uint64_t bytes = 0, phys = 0;
            for (uint64_t i = tid; i < upto; i += 256) {
                const uint64_t sz = (uint64_t)(int64_t)j.batches[first + i].size_bytes;
                bytes += sz;
                if (i < bad) phys += sz;
            }
            atomicAdd(&s_bytes, (unsigned long long)bytes);
            atomicAdd(&s_phys, (unsigned long long)phys);
        }
    }
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
    }
}

DEV bool batch_valid(uint32_t f, uint32_t job_flags, uint32_t layout) {
    if (layout == RPGPU_LAYOUT_WIRE && !(f & RPGPU_F_WIRE_V2)) return false;
    if (!(f & RPGPU_F_HEADER_OK) || !(f & RPGPU_F_COMPLETE) || !(f & RPGPU_F_CRC_OK)) return false;
    if (f & RPGPU_F_CODEC_INVALID) return false;
    if ((f & RPGPU_F_COMPRESSED) && (job_flags & RPGPU_JOB_DECODE) && !(f & RPGPU_F_CODEC_UNSUPPORTED) &&
        !(f & RPGPU_F_CODEC_OK))
        return false;
    if ((f & RPGPU_F_PARSED) && !(f & RPGPU_F_PARSE_OK)) return false;
    return true;
}

// one lane per batch, one wave per bitmap word (a ballot of the lanes)
__global__ __launch_bounds__(256) void k_finalize_bitmap(DeviceJob j) {
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if ((b & ~63ull) >= nb) return;  // whole wave past the end
    const uint64_t word = __ballot(b < nb && batch_valid(j.batches[b].flags, j.flags, j.layout));
    if ((threadIdx.x & 63) == 0) j.bitmap[b >> 6] = word;
}

__global__ void k_finalize_totals(DeviceJob j) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t nb_total = j.chunk_count[j.total_chunks];
    const uint64_t nb = nb_total < j.batch_capacity ? nb_total : j.batch_capacity;
    rpgpu_job_totals t;
    t.n_batches = nb_total;
    t.n_records = j.slots[nb];
    const uint64_t dtot = (j.flags & RPGPU_JOB_DECODE) ? j.dcap[nb] : 0;  // unscanned without DECODE
    t.decoded_bytes = dtot;
    t.batch_capacity_needed = nb_total;
    t.record_capacity_needed = j.slots[nb];
    t.decoded_capacity_needed = dtot;
    uint32_t ov = j.counters[1];
    if (nb_total > j.batch_capacity) ov |= 1;
    if (j.slots[nb] > j.record_capacity) ov |= 2;
    if (dtot > j.decoded_capacity) ov |= 4;
    t.overflow = ov;
    t.n_rewalks = j.counters[0];
    t.reserved[0] = t.reserved[1] = 0;
    *j.totals = t;
}

// ---------------------------------------------------------------------------
// Host-decoded batches (RPGPU_JOB_HOST_CODECS: zstd).  The runtime reads the
// host list's descriptors, gathers the payloads into staging, decodes them
// on the host and hands the results back; these kernels do the device side.
// ---------------------------------------------------------------------------
// descriptor of host item i: payload offset in d_data, bytes, batch ordinal,
// record_count
__global__ __launch_bounds__(256) void k_host_desc(DeviceJob j, HostItem* items) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= j.counters[19]) return;
    const uint32_t b = j.host_list[i];
    const rpgpu_batch_result& R = j.batches[b];
    HostItem it;
    it.src = j.seg_off[R.segment] + R.file_pos + RPGPU_HEADER_SIZE;
    it.n = (uint32_t)(R.size_bytes - (int32_t)RPGPU_HEADER_SIZE);
    it.ord = b;
    it.record_count = R.record_count;
    it.status = 0;
    it.stage = 0;
    it.out_len = 0;
    it.cap = 0;
    items[i] = it;
}

// payload of item i to staging + items[i].stage (one wave per item)
__global__ __launch_bounds__(256) void k_host_gather(DeviceJob j, const HostItem* items, uint32_t n, uint8_t* stage) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint8_t* s = j.data + items[i].src;
    uint8_t* d = stage + items[i].stage;
    for (uint64_t k = threadIdx.x & 63; k < items[i].n; k += 64) d[k] = s[k];
}

// the host's verdicts: arena reservation and index slots, before the scans
__global__ __launch_bounds__(256) void k_host_patch(DeviceJob j, const HostItem* items, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const HostItem it = items[i];
    j.dcap[it.ord] = it.cap;
    j.slots[it.ord] = ((j.flags & RPGPU_JOB_PARSE) && it.record_count > 0 && (uint64_t)it.record_count <= it.cap)
                          ? (uint64_t)it.record_count
                          : 0;
}

// decoded bytes from staging into the arena slots (one wave per item)
__global__ __launch_bounds__(256) void k_host_scatter(DeviceJob j, const HostItem* items, uint32_t n,
                                                      const uint8_t* stage) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const HostItem it = items[i];
    if (it.status != 0) return;
    rpgpu_batch_result* R = &j.batches[it.ord];
    const uint64_t dst = j.dcap[it.ord];
    if (dst + it.cap > j.decoded_capacity) {
        if ((threadIdx.x & 63) == 0) R->flags = R->flags | RPGPU_F_DECODE_OVERFLOW;
        return;
    }
    for (uint64_t k = threadIdx.x & 63; k < it.out_len; k += 64) j.decoded[dst + k] = stage[it.stage + k];
    if ((threadIdx.x & 63) == 0) {
        R->flags = R->flags | RPGPU_F_CODEC_OK;
        R->decoded_len = (uint32_t)it.out_len;
        R->reserved0 = 0;
    }
}

hipError_t launch_host_desc(const DeviceJob& j, HostItem* items, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_host_desc, dim3((n + 255) / 256), dim3(256), 0, s, j, items);
    return hipGetLastError();
}
hipError_t launch_host_gather(const DeviceJob& j, const HostItem* items, uint32_t n, uint8_t* stage, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_host_gather, dim3((n + 3) / 4), dim3(256), 0, s, j, items, n, stage);
    return hipGetLastError();
}
hipError_t launch_host_patch(const DeviceJob& j, const HostItem* items, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_host_patch, dim3((n + 255) / 256), dim3(256), 0, s, j, items, n);
    return hipGetLastError();
}
hipError_t launch_host_scatter(const DeviceJob& j, const HostItem* items, uint32_t n, const uint8_t* stage,
                               hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_host_scatter, dim3((n + 3) / 4), dim3(256), 0, s, j, items, n, stage);
    return hipGetLastError();
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
    hipLaunchKernelGGL(k_discover, dim3((j.total_chunks + 3) / 4), dim3(256), 0, s, j);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_chain, dim3((j.total_chunks + 255) / 256), dim3(256), kLdsHdrBytes, s, j);
    return hipGetLastError();
}
hipError_t launch_resolve(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_resolve, dim3(j.n_segments), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_emit(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_emit, dim3((j.total_chunks + 255) / 256), dim3(256), kLdsHdrBytes, s, j);
    return hipGetLastError();
}
hipError_t launch_finalize(const DeviceJob& j, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize_segments, dim3(j.n_segments), dim3(256), 0, s, j);
    const uint64_t words = (j.batch_capacity + 63) / 64;
    if (j.bitmap) {
        const uint32_t grid = (uint32_t)((words * 64 + 255) / 256);
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
