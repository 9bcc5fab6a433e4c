// rp_index.hip — segment sparse-index rebuild during recovery.
//
// Reference: checksumming_consumer::consume_batch_end calls
// segment_index::maybe_track(hdr, physical_base_offset) for every crc-good
// batch (storage/log_replayer.cc:62-74); maybe_track adds size_bytes to _acc
// and asks index_state::maybe_index whether to add an entry, resetting _acc
// when it did (storage/segment_index.cc:58-72, storage/index_state.cc:48-95).
// An entry is added for the first tracked batch and for every batch at which
// the bytes since the previous entry (inclusive) reach `step` (32 KiB).
//
// The acc reset makes the entry set a serial chain, so the kernel runs one
// wave per segment and walks the segment's batch results 64 at a time:
//   * each lane holds one batch; an inclusive wave scan gives P (bytes of the
//     tile up to and including the lane);
//   * every lane finds its successor entry next(l) = the first lane j > l
//     with P_j >= P_l + step by binary lifting over the lanes (sizes are
//     non-negative on a parser chain, so P is monotone); the tile's first
//     entry is the first lane where the carried bytes reach `step`, and the
//     chain from it is one readlane per entry;
//   * entry lanes write {relative offset, relative time, position} at their
//     rank among the segment's entries.
// The tile loads (the first 64 bytes of each 128-byte rpgpu_batch_result)
// are issued four tiles ahead of the tile being walked so the chain does not
// wait on memory.
#include "rp_device.h"

namespace rp {

namespace {

struct IdxTile {
    uint4 a, b, c, d;  // bytes [0, 64) of rpgpu_batch_result
};

// Unconditional loads (index clamped to the last tracked batch; lanes past n
// are masked out of every use) so the tile loads stay in flight across
// iterations: a load under a divergent branch would make the compiler wait
// for every outstanding load at the join.
DEV IdxTile idx_load(const rpgpu_batch_result* base, uint64_t i, uint64_t n) {
    const uint4* p = reinterpret_cast<const uint4*>(base + (i < n ? i : n - 1));
    IdxTile t;
    t.a = p[0];
    t.b = p[1];
    t.c = p[2];
    t.d = p[3];
    return t;
}

DEV uint64_t u64of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

DEV uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_up((uint32_t)(v >> 32), d, 64);
    return u64of(lo, hi);
}

DEV int64_t shfl_xor_i64(int64_t v, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)(uint64_t)v, m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)((uint64_t)v >> 32), m, 64);
    return (int64_t)u64of(lo, hi);
}

DEV uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64);
    const uint32_t hi = __shfl((uint32_t)(v >> 32), src, 64);
    return u64of(lo, hi);
}

DEV uint64_t rl64(uint64_t v, int l) { return u64of(rl((uint32_t)v, l), rl((uint32_t)(v >> 32), l)); }

}  // namespace

// index_state being rebuilt, uniform across the wave
struct IdxWalk {
    uint64_t a;          // segment_index::_acc (bytes since the last entry)
    uint64_t n_entries;
    uint64_t tracked;
    int64_t base_ts, max_off;
    int64_t lane_max_ts;  // per-lane running max of max(first, last) timestamps, reduced once at the end
    int64_t assert_batch;
};

// One tile of up to 64 tracked batches (lane l = batch tb + l).  Returns true
// when tracking stops inside the tile (the reference's vassert).
DEV bool walk_tile(const IdxTile& cur, uint64_t tb, uint64_t n, uint32_t l, uint64_t lt_mask, uint64_t step,
                   int64_t idx_base, uint64_t first_batch, IdxWalk& w, uint32_t* __restrict__ rel_offset,
                   uint32_t* __restrict__ rel_time, uint64_t* __restrict__ position, uint64_t lo_b = 0,
                   bool write = true) {
    const uint64_t i = tb + l;
    const uint64_t file_pos = u64of(cur.a.x, cur.a.y);
    const int64_t b_off = (int64_t)u64of(cur.a.z, cur.a.w);
    const int64_t first_ts = (int64_t)u64of(cur.b.x, cur.b.y);
    const int64_t last_ts_raw = (int64_t)u64of(cur.b.z, cur.b.w);
    const int64_t size_bytes = (int64_t)(int32_t)cur.c.z;
    const int32_t lod = (int32_t)cur.d.x;
    uint64_t valid = __ballot(i < n && i >= lo_b);
    // vassert(batch_base_offset >= base_offset) (index_state.cc:57-63): the
    // reference aborts there, so tracking ends before that batch
    const uint64_t bad = __ballot(i < n && b_off < idx_base) & valid;
    bool stop = false;
    if (bad) {
        const int f = __builtin_ctzll(bad);
        valid &= (1ull << f) - 1;
        w.assert_batch = (int64_t)(tb + f);
        stop = true;
    }
    if (!valid) return stop;
    const bool mine = (valid >> l) & 1;
    // inclusive scan of size_bytes (segment_index::_acc += hdr.size_bytes)
    uint64_t P = mine ? (uint64_t)size_bytes : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = shfl_up64(P, d);
        if (l >= (uint32_t)d) P += o;
    }
    const int last = 63 - __builtin_clzll(valid);
    uint64_t trig = 0, Pt = 0, a = w.a;
    if (__ballot(mine && size_bytes < 0)) {
        // negative sizes (never on a parser chain): P is not monotone, so
        // find each entry with a ballot: the first lane l > t with
        // a + P_l - P_t >= step
        uint64_t above = ~0ull;
        for (;;) {
            const uint64_t thr = (step - a) + Pt;
            const uint64_t m = __ballot(P >= thr) & valid & above;
            if (!m) break;
            const int t = __builtin_ctzll(m);
            trig |= 1ull << t;
            Pt = rl64(P, t);
            a = 0;
            above = t == 63 ? 0 : (~0ull << (t + 1));
        }
    } else {
        // P is non-decreasing: every lane finds its successor entry in
        // parallel, next(l) = first j > l with P_j >= P_l + step (binary
        // lifting over lanes), then the chain is one readlane per entry
        const uint64_t Pv = mine ? P : ~0ull;
        const uint64_t target = P + step;
        int pos = (int)l;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const int cand = pos + d;
            const uint64_t pc = shfl64(Pv, cand & 63);
            if (cand <= 63 && pc < target) pos = cand;
        }
        const uint32_t nxt = (pos + 1 > last) ? 64u : (uint32_t)(pos + 1);
        // the first entry of the tile continues the carried acc (a <= step)
        const uint64_t m0 = __ballot(P >= step - a) & valid;
        if (m0) {
            int t = __builtin_ctzll(m0);
            for (;;) {
                trig |= 1ull << t;
                const uint32_t nx = uni32(rl(nxt, t));
                if (nx >= 64u) break;
                t = (int)nx;
            }
            Pt = rl64(P, t);
            a = 0;
        }
    }
    w.a = a + (rl64(P, last) - Pt);
    // max_timestamp = max(max_timestamp, max(first, last)) (index_state.cc:77-78);
    // the first batch's max_timestamp = first_timestamp is below its own max
    const int64_t lts = last_ts_raw > first_ts ? last_ts_raw : first_ts;
    if (w.n_entries == 0 && trig) w.base_ts = (int64_t)rl64((uint64_t)first_ts, __builtin_ctzll(trig));
    if (mine && lts > w.lane_max_ts) w.lane_max_ts = lts;
    const int64_t lo = (int64_t)((uint64_t)b_off + (uint64_t)(int64_t)lod);
    w.max_off = (int64_t)rl64((uint64_t)lo, last);
    // add_entry (index_state.h:70-74)
    if (write && ((trig >> l) & 1)) {
        const uint64_t k = first_batch + w.n_entries + __builtin_popcountll(trig & lt_mask);
        rel_offset[k] = (uint32_t)((uint64_t)b_off - (uint64_t)idx_base);
        rel_time[k] = (uint32_t)((uint64_t)lts - (uint64_t)w.base_ts);
        position[k] = file_pos;
    }
    w.n_entries += __builtin_popcountll(trig);
    w.tracked += __builtin_popcountll(valid);
    return stop;
}

__global__ __launch_bounds__(64) void k_segment_index(const rpgpu_batch_result* __restrict__ batches,
                                                      uint64_t cap, const rpgpu_segment_summary* __restrict__ sums,
                                                      uint64_t step, rpgpu_index_state* __restrict__ states,
                                                      uint32_t* __restrict__ rel_offset,
                                                      uint32_t* __restrict__ rel_time,
                                                      uint64_t* __restrict__ position) {
    const uint32_t s = blockIdx.x;
    const uint32_t l = threadIdx.x;
    const rpgpu_segment_summary sm = sums[s];
    const int64_t idx_base = states[s].base_offset;
    // tracked batches: the crc-good prefix [0, first_bad) (log_replayer.cc:62-79)
    uint64_t n = sm.first_bad;
    const uint64_t avail = sm.first_batch < cap ? cap - sm.first_batch : 0;
    IdxWalk w;
    w.assert_batch = -1;
    if (n > avail) {  // the job overflowed its batch capacity
        n = avail;
        w.assert_batch = -2;
    }
    const rpgpu_batch_result* seg = batches + (sm.first_batch < cap ? sm.first_batch : 0);
    const uint64_t lt_mask = (1ull << l) - 1;
    // index_state after reset(): everything zero but base_offset; the empty
    // index makes the first tracked batch an entry (a = step)
    w.a = step;
    w.n_entries = w.tracked = 0;
    w.base_ts = w.max_off = 0;
    w.lane_max_ts = INT64_MIN;

    if (n) {
        // four tiles in flight; unrolled by four so every tile keeps its own
        // registers (no rotation copies, which would wait for the loads)
        IdxTile t0 = idx_load(seg, l, n);
        IdxTile t1 = idx_load(seg, 64 + l, n);
        IdxTile t2 = idx_load(seg, 128 + l, n);
        IdxTile t3 = idx_load(seg, 192 + l, n);
#define RP_IDX_TILE(T, OFF)                                                                                   \
    if (tb + (OFF) >= n ||                                                                                    \
        walk_tile(T, tb + (OFF), n, l, lt_mask, step, idx_base, sm.first_batch, w, rel_offset, rel_time, position)) \
        break;                                                                                                \
    T = idx_load(seg, tb + (OFF) + 256 + l, n);
        for (uint64_t tb = 0;; tb += 256) {
            RP_IDX_TILE(t0, 0)
            RP_IDX_TILE(t1, 64)
            RP_IDX_TILE(t2, 128)
            RP_IDX_TILE(t3, 192)
        }
#undef RP_IDX_TILE
    }
    int64_t max_ts = w.lane_max_ts;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t v = shfl_xor_i64(max_ts, o);
        max_ts = v > max_ts ? v : max_ts;
    }
    if (w.tracked == 0) max_ts = 0;
    if (l == 0) {
        rpgpu_index_state st;
        st.base_offset = idx_base;
        st.max_offset = w.max_off;
        st.base_timestamp = w.base_ts;
        st.max_timestamp = max_ts;
        st.first_entry = sm.first_batch;
        st.n_entries = w.n_entries;
        st.assert_batch = w.assert_batch;
        st.tracked = w.tracked;
        states[s] = st;
    }
}

// ---------------------------------------------------------------------------
// Piece-parallel rebuild.  A segment's tracked batches are cut into pieces of
// kIdxPiece batches.  What a piece contributes depends only on the bytes
// carried into it since the last entry (a_in), and only through which batch
// becomes its first entry: a batch j of the piece can be that only if the
// piece's bytes before j are < step, so the candidates are a prefix of the
// piece (two batches for 16 KiB batches and a 32 KiB step).
//   k_idx_cut      per piece: the first batch below the index base (the
//                  vassert), atomicMin per segment -> tracked count
//   k_idx_cand     per (piece, candidate): walk the piece with its first entry
//                  forced at the candidate -> (entries, carried bytes out)
//   k_idx_resolve  per segment, serial over pieces: a_in -> candidate -> a_out;
//                  writes the state fields that need no walk
//                  (a piece whose first entry lies past the 64 precomputed
//                  candidates is walked here instead)
//   k_idx_emit     per piece: walk from the true a_in writing its entries at
//                  their final ranks; timestamp max per segment
// ---------------------------------------------------------------------------
constexpr uint32_t kIdxPiece = 1024;  // batches per piece (16 tiles)
constexpr uint32_t kIdxCand = 64;     // candidates precomputed per piece

struct IdxCand {
    uint64_t a_out;
    uint32_t count;
    uint32_t valid;
};

// Pieces are laid out densely: segment s owns global pieces
// [pbase[s], pbase[s + 1]), ceil(tracked / 1024) of them, so the workspace and
// the grids grow with the batch capacity plus the segment count (at most
// cap / 1024 + nseg pieces), not with their product.
struct IdxWs {
    uint64_t* cut;      // [nseg]
    uint64_t* pbase;    // [nseg + 1]: exclusive scan of the pieces per segment
    uint64_t* a_in;     // [max_pieces]
    uint64_t* base;     // [max_pieces]
    IdxCand* cand;      // [max_pieces * kIdxCand]
    uint32_t n_segments;
    uint32_t max_pieces;  // bound on the total (grid size)
};

DEV uint64_t idx_tracked(const rpgpu_segment_summary& sm, uint64_t cap, int64_t& assert_batch) {
    uint64_t n = sm.first_bad;
    const uint64_t avail = sm.first_batch < cap ? cap - sm.first_batch : 0;
    assert_batch = -1;
    if (n > avail) {
        n = avail;
        assert_batch = -2;
    }
    return n;
}

// walk [from, end) of a segment starting with carried bytes a; no writes
DEV void idx_walk_range(const rpgpu_batch_result* seg, uint64_t from, uint64_t end, uint64_t lo, uint64_t a,
                        uint64_t step, int64_t idx_base, uint32_t l, uint64_t lt_mask, IdxWalk& w) {
    w.a = a;
    w.n_entries = w.tracked = 0;
    w.base_ts = w.max_off = 0;
    w.lane_max_ts = INT64_MIN;
    w.assert_batch = -1;
    for (uint64_t tb = from; tb < end; tb += 64) {
        const IdxTile t = idx_load(seg, tb + l, end);
        walk_tile(t, tb, end, l, lt_mask, step, idx_base, 0, w, nullptr, nullptr, nullptr, lo, false);
    }
}

// one workgroup: pieces per segment (from the tracked count, which bounds
// every later cut) and their exclusive scan, clamped to the workspace bound
__global__ __launch_bounds__(1024) void k_idx_layout(const rpgpu_segment_summary* __restrict__ sums, uint64_t cap,
                                                     IdxWs ws) {
    __shared__ uint64_t part[1024 / 64];
    __shared__ uint64_t carry;
    const uint32_t t = threadIdx.x, l = t & 63, wv = t >> 6;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < ws.n_segments; b += 1024) {
        const uint32_t s = b + t;
        uint64_t np = 0;
        if (s < ws.n_segments) {
            int64_t ab;
            np = (idx_tracked(sums[s], cap, ab) + kIdxPiece - 1) / kIdxPiece;
        }
        uint64_t P = np;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = shfl_up64(P, d);
            if (l >= (uint32_t)d) P += o;
        }
        if (l == 63) part[wv] = P;
        __syncthreads();
        uint64_t before = carry;
        for (uint32_t k = 0; k < wv; k++) before += part[k];
        const uint64_t lim = ws.max_pieces;
        const uint64_t e0 = before + P - np, e1 = before + P;
        if (s < ws.n_segments) ws.pbase[s] = e0 < lim ? e0 : lim;
        if (s + 1 == ws.n_segments) ws.pbase[s + 1] = e1 < lim ? e1 : lim;
        __syncthreads();
        if (t == 1023) carry = before + P;
        __syncthreads();
    }
}

// global piece g -> (segment, piece within it); false past the last piece
DEV bool idx_piece(const IdxWs& ws, uint64_t g, uint32_t& s, uint64_t& p) {
    if (g >= ws.pbase[ws.n_segments]) return false;
    uint32_t lo = 0, hi = ws.n_segments;  // last s with pbase[s] <= g
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (ws.pbase[m] <= g) lo = m;
        else hi = m;
    }
    s = lo;
    p = g - ws.pbase[lo];
    return true;
}

// grid (max_pieces): the first batch below the index base offset (the
// reference's vassert) per segment, by atomicMin over pieces; ws.cut starts
// at ~0 and every reader takes min(ws.cut, tracked)
__global__ __launch_bounds__(256) void k_idx_cut(const rpgpu_batch_result* __restrict__ batches, uint64_t cap,
                                                 const rpgpu_segment_summary* __restrict__ sums,
                                                 const rpgpu_index_state* __restrict__ states, IdxWs ws) {
    uint32_t s;
    uint64_t p;
    if (!idx_piece(ws, blockIdx.x, s, p)) return;
    const rpgpu_segment_summary sm = sums[s];
    int64_t assert_batch;
    const uint64_t n = idx_tracked(sm, cap, assert_batch);
    const uint64_t from = p * kIdxPiece;
    if (from >= n) return;
    const uint64_t end = from + kIdxPiece < n ? from + kIdxPiece : n;
    const rpgpu_batch_result* seg = batches + sm.first_batch;
    const int64_t idx_base = states[s].base_offset;
    uint64_t mine = ~0ull;
    for (uint64_t i = from + threadIdx.x; i < end; i += 256)
        if (seg[i].base_offset < idx_base) { mine = i; break; }
    const uint64_t m = __ballot(mine != ~0ull);
    if (m) {
        // lowest lane with a hit has the wave's smallest index (lanes stride by 1)
        uint64_t best = mine;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t v = shfl64(best, (int)(threadIdx.x & 63) ^ o);
            best = v < best ? v : best;
        }
        if ((threadIdx.x & 63) == 0) atomicMin((unsigned long long*)&ws.cut[s], (unsigned long long)best);
    }
}

DEV uint64_t idx_cut(const IdxWs& ws, uint32_t s, const rpgpu_segment_summary& sm, uint64_t cap) {
    int64_t ab;
    const uint64_t n = idx_tracked(sm, cap, ab);
    const uint64_t c = ws.cut[s];
    return c < n ? c : n;
}

// grid (max_pieces), 4 waves per block: wave v takes candidates v, v+4, ...
__global__ __launch_bounds__(256) void k_idx_cand(const rpgpu_batch_result* __restrict__ batches, uint64_t cap,
                                                  const rpgpu_segment_summary* __restrict__ sums, uint64_t step,
                                                  const rpgpu_index_state* __restrict__ states, IdxWs ws) {
    uint32_t s;
    uint64_t p;
    if (!idx_piece(ws, blockIdx.x, s, p)) return;
    const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const rpgpu_segment_summary sm = sums[s];
    const uint64_t cut = idx_cut(ws, s, sm, cap);
    const uint64_t from = p * kIdxPiece;
    if (from >= cut || p == 0) return;  // piece 0 starts with the forced first entry: no candidates needed
    const uint64_t end = from + kIdxPiece < cut ? from + kIdxPiece : cut;
    const rpgpu_batch_result* seg = batches + sm.first_batch;
    const int64_t idx_base = states[s].base_offset;
    const uint64_t lt_mask = (1ull << l) - 1;
    // candidates: lanes of the piece's first tile whose preceding piece bytes are < step
    const uint64_t i0 = from + l;
    const uint64_t sz = i0 < end ? (uint64_t)(int64_t)seg[i0].size_bytes : 0;
    uint64_t P = sz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = shfl_up64(P, d);
        if (l >= (uint32_t)d) P += o;
    }
    const uint64_t cmask = __ballot(i0 < end && (P - sz) < step);
    IdxCand* out = ws.cand + (ws.pbase[s] + p) * kIdxCand;
    for (uint32_t k = wv; k < kIdxCand; k += 4) {
        if (!((cmask >> k) & 1)) {
            if (l == 0) out[k].valid = 0;
            continue;
        }
        IdxWalk w;
        idx_walk_range(seg, from, end, from + k, step, step, idx_base, l, lt_mask, w);
        if (l == 0) {
            out[k].a_out = w.a;
            out[k].count = (uint32_t)w.n_entries;
            out[k].valid = 1;
        }
    }
}

// one wave per segment, serial over its pieces.  The loads a piece needs (its
// first 64 sizes and its 64-entry candidate row, one entry per lane) do not
// depend on the carried state, so they are issued eight pieces at a time and
// the serial chain itself is register work.
__global__ __launch_bounds__(64) void k_idx_resolve(const rpgpu_batch_result* __restrict__ batches, uint64_t cap,
                                                    const rpgpu_segment_summary* __restrict__ sums, uint64_t step,
                                                    rpgpu_index_state* __restrict__ states, IdxWs ws) {
    const uint32_t s = blockIdx.x, l = threadIdx.x;
    const rpgpu_segment_summary sm = sums[s];
    int64_t assert_batch;
    const uint64_t n = idx_tracked(sm, cap, assert_batch);
    const uint64_t cut = idx_cut(ws, s, sm, cap);
    const rpgpu_batch_result* seg = batches + (sm.first_batch < cap ? sm.first_batch : 0);
    const int64_t idx_base = states[s].base_offset;
    if (l == 0) {
        // the state fields that need no walk; k_idx_emit folds in the timestamp maxima
        rpgpu_index_state st;
        st.base_offset = idx_base;
        st.max_offset = cut ? (int64_t)((uint64_t)seg[cut - 1].base_offset + (uint64_t)(int64_t)seg[cut - 1].last_offset_delta) : 0;
        st.base_timestamp = cut ? seg[0].first_timestamp : 0;
        st.max_timestamp = cut ? INT64_MIN : 0;
        st.first_entry = sm.first_batch;
        st.n_entries = 0;
        st.assert_batch = cut < n ? (int64_t)cut : assert_batch;
        st.tracked = cut;
        states[s] = st;
    }
    if (cut == 0) return;
    const uint64_t lt_mask = (1ull << l) - 1;
    const uint64_t pb = ws.pbase[s];
    uint64_t np = (cut + kIdxPiece - 1) / kIdxPiece;
    if (np > ws.pbase[s + 1] - pb) np = ws.pbase[s + 1] - pb;  // the layout's clamp (never taken for real jobs)
    const IdxCand* row0 = ws.cand + pb * kIdxCand;
    auto load_size = [&](uint64_t p) {
        const uint64_t i = p * kIdxPiece + l;
        return (int64_t)seg[i < cut ? i : cut - 1].size_bytes;
    };
    uint64_t a = step, entries = 0;
    // eight pieces' loads issued together, then eight serial resolutions
    constexpr int kAhead = 8;
    for (uint64_t p0 = 0; p0 < np; p0 += kAhead) {
        int64_t szv[kAhead];
        IdxCand cv[kAhead];
#pragma unroll
        for (int u = 0; u < kAhead; u++) {
            const uint64_t pp = p0 + u < np ? p0 + u : np - 1;
            szv[u] = load_size(pp);
            cv[u] = row0[pp * kIdxCand + l];
        }
#pragma unroll
        for (int u = 0; u < kAhead; u++) {
            const uint64_t p = p0 + u;
            if (p >= np) break;
            const uint64_t from = p * kIdxPiece;
            const uint64_t end = from + kIdxPiece < cut ? from + kIdxPiece : cut;
            if (l == 0) {
                ws.a_in[pb + p] = a;
                ws.base[pb + p] = entries;
            }
            bool done = false;
            if (p > 0) {
                const uint64_t i0 = from + l;
                uint64_t P = i0 < end ? (uint64_t)szv[u] : 0;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = shfl_up64(P, d);
                    if (l >= (uint32_t)d) P += o;
                }
                const uint64_t m = __ballot(i0 < end && P >= step - a);
                if (m) {
                    const int k = __builtin_ctzll(m);
                    if (rl(cv[u].valid, k)) {
                        a = rl64(cv[u].a_out, k);
                        entries += rl(cv[u].count, k);
                        done = true;
                    }
                }
            }
            if (!done) {
                IdxWalk w;
                idx_walk_range(seg, from, end, from, a, step, idx_base, l, lt_mask, w);
                a = w.a;
                entries += w.n_entries;
            }
        }
    }
    if (l == 0) states[s].n_entries = entries;
}

// grid (max_pieces): one wave per piece writes its entries
__global__ __launch_bounds__(64) void k_idx_emit(const rpgpu_batch_result* __restrict__ batches, uint64_t cap,
                                                 const rpgpu_segment_summary* __restrict__ sums, uint64_t step,
                                                 rpgpu_index_state* __restrict__ states, IdxWs ws,
                                                 uint32_t* __restrict__ rel_offset, uint32_t* __restrict__ rel_time,
                                                 uint64_t* __restrict__ position) {
    uint32_t s;
    uint64_t p;
    if (!idx_piece(ws, blockIdx.x, s, p)) return;
    const uint32_t l = threadIdx.x;
    const rpgpu_segment_summary sm = sums[s];
    const uint64_t cut = idx_cut(ws, s, sm, cap);
    const uint64_t from = p * kIdxPiece;
    if (from >= cut) return;
    const uint64_t end = from + kIdxPiece < cut ? from + kIdxPiece : cut;
    const rpgpu_batch_result* seg = batches + sm.first_batch;
    const int64_t idx_base = states[s].base_offset;
    const uint64_t lt_mask = (1ull << l) - 1;
    IdxWalk w;
    w.a = ws.a_in[ws.pbase[s] + p];
    w.n_entries = ws.base[ws.pbase[s] + p];
    w.tracked = 0;
    w.base_ts = seg[0].first_timestamp;
    w.max_off = 0;
    w.lane_max_ts = INT64_MIN;
    w.assert_batch = -1;
    for (uint64_t tb = from; tb < end; tb += 64) {
        const IdxTile t = idx_load(seg, tb + l, end);
        walk_tile(t, tb, end, l, lt_mask, step, idx_base, sm.first_batch, w, rel_offset, rel_time, position);
    }
    int64_t m = w.lane_max_ts;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t v = shfl_xor_i64(m, o);
        m = v > m ? v : m;
    }
    if (l == 0) atomicMax((long long*)&states[s].max_timestamp, (long long)m);
}

// pieces: sum over segments of ceil(tracked / 1024) <= cap / 1024 + nseg
// (the segments' tracked batches are disjoint ranges of the batch results)
static uint64_t idx_max_pieces(uint32_t n_segments, uint64_t cap) { return cap / kIdxPiece + n_segments + 1; }

size_t segment_index_ws_bytes(uint32_t n_segments, uint64_t cap) {
    const uint64_t mp = idx_max_pieces(n_segments, cap);
    return 256 + ((uint64_t)n_segments * 8 + 256) + ((uint64_t)n_segments * 8 + 8 + 256) + 2 * (mp * 8 + 256) +
           mp * kIdxCand * sizeof(IdxCand) + 1024;
}

hipError_t launch_segment_index_pieces(const rpgpu_batch_result* batches, uint64_t cap,
                                       const rpgpu_segment_summary* sums, uint32_t n_segments, uint64_t step,
                                       rpgpu_index_state* states, uint32_t* rel_offset, uint32_t* rel_time,
                                       uint64_t* position, void* wsp, hipStream_t s) {
    const uint64_t mp = idx_max_pieces(n_segments, cap);
    if (mp > 0x7FFFFFFFull) return hipErrorInvalidValue;
    uint8_t* q = (uint8_t*)(((uintptr_t)wsp + 255) & ~(uintptr_t)255);
    IdxWs ws;
    ws.n_segments = n_segments;
    ws.max_pieces = (uint32_t)mp;
    ws.cut = (uint64_t*)q;
    q += ((uint64_t)n_segments * 8 + 255) & ~255ull;
    ws.pbase = (uint64_t*)q;
    q += ((uint64_t)n_segments * 8 + 8 + 255) & ~255ull;
    ws.a_in = (uint64_t*)q;
    q += (mp * 8 + 255) & ~255ull;
    ws.base = (uint64_t*)q;
    q += (mp * 8 + 255) & ~255ull;
    ws.cand = (IdxCand*)q;
    hipError_t e = hipMemsetAsync(ws.cut, 0xFF, (size_t)n_segments * 8, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_idx_layout, dim3(1), dim3(1024), 0, s, sums, cap, ws);
    hipLaunchKernelGGL(k_idx_cut, dim3((uint32_t)mp), dim3(256), 0, s, batches, cap, sums,
                       (const rpgpu_index_state*)states, ws);
    hipLaunchKernelGGL(k_idx_cand, dim3((uint32_t)mp), dim3(256), 0, s, batches, cap, sums, step,
                       (const rpgpu_index_state*)states, ws);
    hipLaunchKernelGGL(k_idx_resolve, dim3(n_segments), dim3(64), 0, s, batches, cap, sums, step, states, ws);
    hipLaunchKernelGGL(k_idx_emit, dim3((uint32_t)mp), dim3(64), 0, s, batches, cap, sums, step, states, ws,
                       rel_offset, rel_time, position);
    return hipGetLastError();
}

hipError_t launch_segment_index(const rpgpu_batch_result* batches, uint64_t cap, const rpgpu_segment_summary* sums,
                                uint32_t n_segments, uint64_t step, rpgpu_index_state* states, uint32_t* rel_offset,
                                uint32_t* rel_time, uint64_t* position, hipStream_t s) {
    hipLaunchKernelGGL(k_segment_index, dim3(n_segments), dim3(64), 0, s, batches, cap, sums, step, states,
                       rel_offset, rel_time, position);
    return hipGetLastError();
}

}  // namespace rp
