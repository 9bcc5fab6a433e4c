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
                   uint32_t* __restrict__ rel_time, uint64_t* __restrict__ position) {
    const uint64_t i = tb + l;
    const uint64_t file_pos = u64of(cur.a.x, cur.a.y);
    const int64_t b_off = (int64_t)u64of(cur.a.z, cur.a.w);
    const int64_t first_ts = (int64_t)u64of(cur.b.x, cur.b.y);
    const int64_t last_ts_raw = (int64_t)u64of(cur.b.z, cur.b.w);
    const int64_t size_bytes = (int64_t)(int32_t)cur.c.z;
    const int32_t lod = (int32_t)cur.d.x;
    uint64_t valid = __ballot(i < n);
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
    if ((trig >> l) & 1) {
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

hipError_t launch_segment_index(const rpgpu_batch_result* batches, uint64_t cap, const rpgpu_segment_summary* sums,
                                uint32_t n_segments, uint64_t step, rpgpu_index_state* states, uint32_t* rel_offset,
                                uint32_t* rel_time, uint64_t* position, hipStream_t s) {
    hipLaunchKernelGGL(k_segment_index, dim3(n_segments), dim3(64), 0, s, batches, cap, sums, step, states,
                       rel_offset, rel_time, position);
    return hipGetLastError();
}

}  // namespace rp
