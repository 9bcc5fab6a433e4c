// rp_runtime.hip — host side of the C-ABI (include/rpgpu.h): contexts,
// constant tables, the submit pipeline, memory helpers, the host CRC32C
// behind crc::crc32c and the synthetic segment generator.
#include <hip/hip_runtime.h>
#include <nmmintrin.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "rp_device.h"
#include "rp_hostcodec.h"

namespace rp {

// ---------------------------------------------------------------------------
// GF(2) helpers for the CRC tables (reflected CRC32C)
// ---------------------------------------------------------------------------
static uint32_t raw_step_zero(uint32_t c, const uint32_t* t0) { return t0[c & 0xFF] ^ (c >> 8); }

static void build_tables(Tables* T) {
    uint32_t t0[256];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
        t0[i] = c;
    }
    // T_d[b]: raw CRC of byte b followed by d zero bytes
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = t0[b];
        for (uint32_t d = 0; d < 57; d++) {
            T->hdr[d][b] = c;
            if (d < 4) T->slice[d][b] = c;
            c = raw_step_zero(c, t0);
        }
    }
    // braid tables: byte b followed by 1023 - t zero bytes
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = t0[b];
        for (uint32_t z = 0; z < kBraidSkip; z++) c = raw_step_zero(c, t0);
        for (int t = 3; t >= 0; t--) {
            T->braid[t][b] = c;  // t = 3: 1020 zeros ... t = 0: 1023 zeros
            c = raw_step_zero(c, t0);
        }
    }
    // shift tables: state byte j (value b << 8j) advanced over 16 << m zero bytes
    for (uint32_t m = 0; m < kShiftLevels; m++) {
        const uint64_t n = 16ull << m;
        for (uint32_t j = 0; j < 4; j++) {
            for (uint32_t b = 0; b < 256; b++) {
                uint32_t c = b << (8 * j);
                for (uint64_t z = 0; z < n; z++) c = raw_step_zero(c, t0);
                T->shift[m][j][b] = c;
            }
        }
    }
    uint32_t c = 0xFFFFFFFFu;
    for (int z = 0; z < 40; z++) c = raw_step_zero(c, t0);
    T->c40 = c;
    for (int z = 40; z < 57; z++) c = raw_step_zero(c, t0);
    T->c57 = c;
    T->pad[0] = T->pad[1] = 0;
    // x^(8 * 16 k) (reflected, bit 31 = x^0): mulx multiplies by x
    auto mulx = [](uint32_t a) { return (a & 1u) ? (a >> 1) ^ kCrcPoly : a >> 1; };
    auto invx = [](uint32_t a) { return (a & 0x80000000u) ? ((a ^ kCrcPoly) << 1) | 1u : a << 1; };
    uint32_t e = 0x80000000u;
    for (uint32_t k = 0; k < 64; k++) {
        T->lane_rowend[63 - k] = e;
        for (int b = 0; b < 128; b++) e = mulx(e);
    }
    e = 0x80000000u;
    for (uint32_t z = 0; z < 1024; z++) {
        T->inv_shift[z] = e;
        for (int b = 0; b < 8; b++) e = invx(e);
    }
}

// the combine tables take ~2^13 * 1024 zero-steps; build them once per process
static const Tables* host_tables() {
    static Tables* T = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        T = new Tables;
        build_tables(T);
    });
    return T;
}

}  // namespace rp

using namespace rp;

struct rpgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Tables* d_tables = nullptr;
    // growable device workspace
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // pinned staging for small host->device uploads
    void* pin = nullptr;
    size_t pin_bytes = 0;
    bool timing = false;
    // one event set per timed submit: start, discover done, plan done,
    // decode done, validate done, walk done, end; resolved lazily by
    // rpgpu_last_timings
    std::vector<std::array<hipEvent_t, 7>> ev_sets;
    // rpgpu_uncompress staging (device)
    void* uws = nullptr;
    size_t uws_bytes = 0;
    size_t ev_used = 0;
    uint32_t cu_count = 256;
    // rpgpu_query_capacity scratch (summaries, totals, batch results), grow-only
    void* qws = nullptr;
    size_t qws_bytes = 0;
    // rpgpu_uncompress_batch staging: pinned host and device, grow-only
    void* bh = nullptr;
    size_t bh_bytes = 0;
    void* bd = nullptr;
    size_t bd_bytes = 0;
    // rpgpu_stamp workspace (offset steps, scan temporaries, claim cursor)
    void* sws = nullptr;
    size_t sws_bytes = 0;
    // rpgpu_segment_index workspace (piece tables), grow-only
    void* iws = nullptr;
    size_t iws_bytes = 0;
    // k_lz_exec parse records (kRecsPerLane per lane of each resident wave),
    // allocated on the first decode job
    SeqRec* seqs = nullptr;
    uint32_t exec_waves = 0;
    // k_lz_walk record pool (slabs) and its chain links, grow-only
    void* pool = nullptr;
    size_t pool_bytes = 0;
    // k_lzf_walk's 8-byte records (independent-block fast path); without it
    // every piece takes the walk / exec kernels
    void* fpool = nullptr;
    size_t fpool_bytes = 0;
    std::string err;
    // Context scratch (ws, pool, seqs, sws, iws) is shared by every job on
    // the context, whichever stream it is launched on: each async entry
    // point makes its stream wait for the previous job's last event (a
    // device-side wait, no host sync) and records its own at the end, and a
    // scratch buffer is only freed for growth once that event completed.
    hipEvent_t ws_ev = nullptr;
    bool ws_live = false;
    // rpgpu_validate_host: a copy stream and two staging slots (segment
    // bytes in, per-batch results out), used alternately so the H2D copy of
    // group g + 1 runs while group g validates
    hipStream_t copy = nullptr;
    // the zstd members' first pass (k_zparse) runs on a side stream beside
    // k_members_first's gzip members: forked after k_emit, joined before the
    // slot scans
    hipStream_t side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    hipStream_t side2 = nullptr;  // k_raw_copy beside k_lzf_walk and k_lz_walk; the gzip members
                                  // the split decode does not plan, beside it
    hipEvent_t join2_ev = nullptr, mfork_ev = nullptr, mjoin_ev = nullptr;
    struct HostSlot {
        uint8_t* d_data = nullptr;
        uint64_t data_bytes = 0;
        uint64_t* d_offs = nullptr;
        uint64_t offs_n = 0;
        rpgpu_batch_result* d_batches = nullptr;
        uint64_t bcap = 0;
        rpgpu_record_index* d_records = nullptr;
        uint64_t rcap = 0;
        uint8_t* d_decoded = nullptr;
        uint64_t dcap = 0;
        rpgpu_segment_summary* d_sums = nullptr;
        uint64_t sums_n = 0;
        rpgpu_job_totals* d_tot = nullptr;
        rpgpu_job_totals* h_tot = nullptr;  // pinned
        // segment index rebuild (rpgpu_host_job.index_step)
        rpgpu_index_state* d_ist = nullptr;
        uint64_t ist_n = 0;
        uint32_t* d_ro = nullptr;
        uint32_t* d_rt = nullptr;
        uint64_t* d_ps = nullptr;
        uint64_t ix_n = 0;
        hipEvent_t h2d = nullptr, done = nullptr;
        std::vector<uint64_t> h_offs;
        std::vector<rpgpu_index_state> h_ist;
    } hs[2];
    // rpgpu_stamp_host staging (pinned host + device), grow-only
    void* sth = nullptr;
    size_t sth_bytes = 0;
    void* std_ = nullptr;
    size_t std_bytes = 0;
    // RPGPU_JOB_HOST_CODECS: the host step's items and staging (device and
    // pinned host, grow-only); hc_n = items of the job being enqueued
    struct Grow {
        void* p = nullptr;
        size_t bytes = 0;
        bool pinned = false;
    } hc_items, hc_items_h, hc_in, hc_in_h, hc_out, hc_out_h, hc_small;
    uint32_t hc_n = 0;
    // gzip / zstd first-pass output pool (k_members_first), grow-only
    void* gz_pool = nullptr;
    size_t gz_pool_bytes = 0;
    void* gzs_pool = nullptr;  // the gzip split decode's chunk symbols
    size_t gzs_pool_bytes = 0;
};

namespace {

int fail(rpgpu_ctx* c, int code, const char* what, hipError_t e = hipSuccess) {
    if (c) {
        c->err = what;
        if (e != hipSuccess) {
            c->err += ": ";
            c->err += hipGetErrorString(e);
        }
    }
    return code;
}

#define HIPCHK(ctx, call)                                                   \
    do {                                                                    \
        hipError_t _e = (call);                                             \
        if (_e != hipSuccess) return fail((ctx), RPGPU_E_HIP, #call, _e);   \
    } while (0)

// ordering of jobs that share the context scratch (see rpgpu_ctx::ws_ev)
int ws_acquire(rpgpu_ctx* c, hipStream_t s) {
    if (c->ws_live) HIPCHK(c, hipStreamWaitEvent(s, c->ws_ev, 0));
    return RPGPU_OK;
}
int ws_release(rpgpu_ctx* c, hipStream_t s) {
    if (!c->ws_ev) HIPCHK(c, hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ws_ev, s));
    c->ws_live = true;
    return RPGPU_OK;
}
// before freeing scratch for growth: the previous job (any stream) is done
int ws_drain(rpgpu_ctx* c, hipStream_t s) {
    if (c->ws_live) HIPCHK(c, hipEventSynchronize(c->ws_ev));
    HIPCHK(c, hipStreamSynchronize(s));
    return RPGPU_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Environment overrides exist in the diagnostic build only
// (librpgpu_diag.so, -DRPGPU_DIAG, loaded with RPGPU_VARIANT=diag): the
// product library reads no environment.
#ifdef RPGPU_DIAG
const char* diag_env(const char* name) { return getenv(name); }
#else
const char* diag_env(const char*) { return nullptr; }
#endif

// The side stream of a job (the zstd member pass beside the gzip one, the LZ4
// lane walk beside the raw copies and the other pieces' walk): created at the
// device's highest stream priority.  HIP spreads a process's streams over
// GPU_MAX_HW_QUEUES hardware queues (4 here) round robin, and a side stream
// that lands on the caller's queue runs after it instead of beside it (C6's
// member pass measured 64 ms alone, 77 ms after the bench's H2D stanza had
// created its copy streams); a priority of its own gives it a queue of its own.
// RPGPU_SIDE_PRIO=0 (diagnostic build): the default priority (A/B).
hipError_t side_stream_create(hipStream_t* out) {
    static const bool prio = [] { const char* e = diag_env("RPGPU_SIDE_PRIO"); return !(e && *e == '0'); }();
    int least = 0, greatest = 0;
    if (prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least)
        return hipStreamCreateWithPriority(out, hipStreamNonBlocking, greatest);
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
}

// gzip / zstd: the CPU fallback behind compressor::uncompress (rp_hostcodec.cpp)
int host_codec(rpgpu_ctx* c, int codec, const void* in, size_t n, void* out, size_t cap, size_t* out_len) {
    const int rc = host_uncompress(codec, (const uint8_t*)in, n, (uint8_t*)out, cap, out_len);
    if (rc == 0) return RPGPU_OK;
    if (rc == kHostCodecOverflow) return fail(c, RPGPU_E_OVERFLOW, "rpgpu_uncompress: output capacity too small");
    if (rc == kHostCodecMissing) return fail(c, RPGPU_E_UNSUPPORTED, "rpgpu_uncompress: zlib / libzstd not loadable");
    *out_len = 0;
    return fail(c, RPGPU_E_CODEC, codec == RPGPU_CODEC_GZIP ? "gzip uncompress error" : "ZSTD error");
}

}  // namespace

extern "C" {

int rpgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rpgpu_create(int device, rpgpu_ctx** out) {
    if (!out) return RPGPU_E_INVALID;
    *out = nullptr;
    int n = rpgpu_device_count();
    if (n <= 0 || device < 0 || device >= n) return RPGPU_E_NO_DEVICE;
    rpgpu_ctx* c = new rpgpu_ctx;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) { delete c; return RPGPU_E_NO_DEVICE; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = (uint32_t)prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return RPGPU_E_HIP; }
    if (hipMalloc(&c->d_tables, sizeof(Tables)) != hipSuccess) { delete c; return RPGPU_E_NOMEM; }
    if (hipMemcpy(c->d_tables, host_tables(), sizeof(Tables), hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(c->d_tables);
        delete c;
        return RPGPU_E_HIP;
    }
    *out = c;
    return RPGPU_OK;
}

int rpgpu_destroy(rpgpu_ctx* c) {
    if (!c) return RPGPU_E_INVALID;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->ws_live) (void)hipEventSynchronize(c->ws_ev);
    if (c->ws) hipFree(c->ws);
    if (c->uws) hipFree(c->uws);
    if (c->iws) hipFree(c->iws);
    if (c->qws) hipFree(c->qws);
    if (c->sws) hipFree(c->sws);
    if (c->bd) hipFree(c->bd);
    if (c->bh) hipHostFree(c->bh);
    if (c->seqs) hipFree(c->seqs);
    if (c->pool) hipFree(c->pool);
    if (c->fpool) hipFree(c->fpool);
    if (c->pin) hipHostFree(c->pin);
    if (c->sth) hipHostFree(c->sth);
    if (c->std_) hipFree(c->std_);
    if (c->d_tables) hipFree(c->d_tables);
    if (c->gz_pool) hipFree(c->gz_pool);
    if (c->gzs_pool) hipFree(c->gzs_pool);
    for (auto* g : {&c->hc_items, &c->hc_items_h, &c->hc_in, &c->hc_in_h, &c->hc_out, &c->hc_out_h, &c->hc_small})
        if (g->p) (void)(g->pinned ? hipHostFree(g->p) : hipFree(g->p));
    if (c->ws_ev) { (void)hipEventSynchronize(c->ws_ev); (void)hipEventDestroy(c->ws_ev); }
    if (c->side) { (void)hipStreamSynchronize(c->side); (void)hipStreamDestroy(c->side); }
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->join_ev) (void)hipEventDestroy(c->join_ev);
    if (c->side2) { (void)hipStreamSynchronize(c->side2); (void)hipStreamDestroy(c->side2); }
    if (c->join2_ev) (void)hipEventDestroy(c->join2_ev);
    if (c->mfork_ev) (void)hipEventDestroy(c->mfork_ev);
    if (c->mjoin_ev) (void)hipEventDestroy(c->mjoin_ev);
    for (auto& set : c->ev_sets)
        for (auto& e : set) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    if (c->copy) { (void)hipStreamSynchronize(c->copy); (void)hipStreamDestroy(c->copy); }
    for (auto& h : c->hs) {
        (void)hipFree(h.d_data); (void)hipFree(h.d_offs); (void)hipFree(h.d_batches); (void)hipFree(h.d_records);
        (void)hipFree(h.d_decoded);
        (void)hipFree(h.d_sums); (void)hipFree(h.d_tot);
        (void)hipFree(h.d_ist); (void)hipFree(h.d_ro); (void)hipFree(h.d_rt); (void)hipFree(h.d_ps);
        if (h.h_tot) (void)hipHostFree(h.h_tot);
        if (h.h2d) hipEventDestroy(h.h2d);
        if (h.done) hipEventDestroy(h.done);
    }
    delete c;
    return RPGPU_OK;
}

const char* rpgpu_strerror(int s) {
    switch (s) {
    case RPGPU_OK: return "ok";
    case RPGPU_E_INVALID: return "invalid argument";
    case RPGPU_E_NO_DEVICE: return "no HIP device";
    case RPGPU_E_NOMEM: return "out of memory";
    case RPGPU_E_OVERFLOW: return "output capacity too small";
    case RPGPU_E_CODEC: return "uncompress failed";
    case RPGPU_E_UNSUPPORTED: return "codec not supported by the engine";
    case RPGPU_E_HIP: return "HIP runtime error";
    }
    return "unknown";
}

const char* rpgpu_last_error(rpgpu_ctx* c) { return c ? c->err.c_str() : ""; }

int rpgpu_dev_alloc(rpgpu_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return RPGPU_E_INVALID;
    hipSetDevice(c->device);
    if (hipMalloc(out, bytes ? bytes : 1) != hipSuccess) return fail(c, RPGPU_E_NOMEM, "hipMalloc");
    return RPGPU_OK;
}
int rpgpu_dev_free(rpgpu_ctx* c, void* p) {
    if (!c) return RPGPU_E_INVALID;
    hipSetDevice(c->device);
    HIPCHK(c, hipFree(p));
    return RPGPU_OK;
}
int rpgpu_host_alloc(rpgpu_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return RPGPU_E_INVALID;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return fail(c, RPGPU_E_NOMEM, "hipHostMalloc");
    return RPGPU_OK;
}
int rpgpu_host_free(rpgpu_ctx* c, void* p) {
    if (!c) return RPGPU_E_INVALID;
    HIPCHK(c, hipHostFree(p));
    return RPGPU_OK;
}
static hipStream_t pick(rpgpu_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }
int rpgpu_memcpy_h2d(rpgpu_ctx* c, void* dst, const void* src, size_t n, void* s) {
    if (!c) return RPGPU_E_INVALID;
    HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, pick(c, s)));
    return RPGPU_OK;
}
int rpgpu_memcpy_d2h(rpgpu_ctx* c, void* dst, const void* src, size_t n, void* s) {
    if (!c) return RPGPU_E_INVALID;
    HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, pick(c, s)));
    return RPGPU_OK;
}
int rpgpu_memset(rpgpu_ctx* c, void* dst, int v, size_t n, void* s) {
    if (!c) return RPGPU_E_INVALID;
    HIPCHK(c, hipMemsetAsync(dst, v, n, pick(c, s)));
    return RPGPU_OK;
}
int rpgpu_sync(rpgpu_ctx* c, void* s) {
    if (!c) return RPGPU_E_INVALID;
    HIPCHK(c, hipStreamSynchronize(pick(c, s)));
    return RPGPU_OK;
}

int rpgpu_set_timing(rpgpu_ctx* c, int enable) {
    if (!c) return RPGPU_E_INVALID;
    c->timing = enable != 0;
    return RPGPU_OK;
}

// Averages over every timed submit since the previous call (then resets).
// ms[0] whole pipeline, [1] discover, [2] resolve+emit+plan, [3] validate,
// [4] decode, [5] lane record walk.
int rpgpu_last_timings(rpgpu_ctx* c, float* ms, int n) {
    if (!c || !ms) return RPGPU_E_INVALID;
    if (c->ev_used == 0) return fail(c, RPGPU_E_INVALID, "rpgpu_last_timings: no timed submit");
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (size_t i = 0; i < c->ev_used; i++) {
        auto& e = c->ev_sets[i];
        HIPCHK(c, hipEventSynchronize(e[6]));
        const int pairs[6][2] = {{0, 6}, {0, 1}, {1, 2}, {3, 4}, {2, 3}, {4, 5}};
        for (int k = 0; k < 6; k++) {
            float t = 0;
            HIPCHK(c, hipEventElapsedTime(&t, e[pairs[k][0]], e[pairs[k][1]]));
            acc[k] += t;
        }
    }
    for (int i = 0; i < n && i < 6; i++) ms[i] = (float)(acc[i] / (double)c->ev_used);
    c->ev_used = 0;
    return RPGPU_OK;
}

// ---------------------------------------------------------------------------
// submit
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {
// device addresses of the plan a stopped submit leaves in the workspace
struct PlanPtrs {
    const uint64_t* n_batches;  // chunk_count[total_chunks]
    const uint64_t* slots;      // exclusive scan of index slots (batch_capacity + 1)
    const uint64_t* dcap;       // exclusive scan of decode bytes (batch_capacity + 1)
};
enum SubmitStop { kRunAll = 0, kStopAfterCount = 1, kStopAfterPlan = 2 };
int submit_impl(rpgpu_ctx* c, const rpgpu_job* job, void* stream, int stop, PlanPtrs* plan);
}  // namespace

extern "C" {

int rpgpu_submit(rpgpu_ctx* c, const rpgpu_job* job, void* stream) { return submit_impl(c, job, stream, kRunAll, nullptr); }

}  // extern "C"

namespace {
int submit_body(rpgpu_ctx* c, const rpgpu_job* job, hipStream_t s, int stop, PlanPtrs* plan);

// every job on a context is ordered after the previous one (rpgpu_ctx::ws_ev)
int submit_impl(rpgpu_ctx* c, const rpgpu_job* job, void* stream, int stop, PlanPtrs* plan) {
    if (!c) return RPGPU_E_INVALID;
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    if (int rc = ws_acquire(c, s)) return rc;
    const int rc = submit_body(c, job, s, stop, plan);
    const int rr = ws_release(c, s);
    return rc ? rc : rr;
}

// grow-only device pool (drained before it is replaced)
int grow_pool(rpgpu_ctx* c, void*& p, size_t& have, size_t want, hipStream_t s) {
    if (want <= have && p) return RPGPU_OK;
    if (p) {
        if (int rc = ws_drain(c, s)) return rc;
        (void)hipFree(p);
        p = nullptr;
        have = 0;
    }
    if (hipMalloc(&p, want) != hipSuccess) {
        // not an error: without the pool every member is decoded by the
        // second pass, straight into its arena slot
        (void)hipGetLastError();
        p = nullptr;
        return RPGPU_OK;
    }
    have = want;
    return RPGPU_OK;
}

// grow-only device or pinned host buffer (the stream is drained before a
// device buffer is replaced: earlier work on the context may still use it)
int grow_buf(rpgpu_ctx* c, rpgpu_ctx::Grow& g, size_t want, bool pinned, hipStream_t s) {
    if (want <= g.bytes && g.p) return RPGPU_OK;
    if (g.p) {
        if (int rc = ws_drain(c, s)) return rc;
        (void)(g.pinned ? hipHostFree(g.p) : hipFree(g.p));
        g.p = nullptr;
        g.bytes = 0;
    }
    want = std::max<size_t>(align_up(want + want / 4, 4096), 4096);
    const hipError_t e = pinned ? hipHostMalloc(&g.p, want, hipHostMallocDefault) : hipMalloc(&g.p, want);
    if (e != hipSuccess) { g.p = nullptr; return fail(c, RPGPU_E_NOMEM, "host codec staging"); }
    g.bytes = want;
    g.pinned = pinned;
    return RPGPU_OK;
}

// RPGPU_JOB_HOST_CODECS: the batches k_emit put on the host list (zstd) cross
// to the host, are decoded by stream_zstd::do_uncompress's loop over libzstd
// (rp_hostcodec.cpp; compression/stream_zstd.cc:152-178) on a few threads,
// and come back: their arena reservations and index slots are patched in
// before the scans (the same rule as every codec: the decoded size rounded up
// to 16, 0 when the reference throws), the bytes wait in device staging for
// k_host_scatter.  Synchronizes the stream three times.
int host_codec_step(rpgpu_ctx* c, const DeviceJob& j, hipStream_t s) {
    if (int rc = grow_buf(c, c->hc_small, 64, true, s)) return rc;
    uint32_t* cnt = (uint32_t*)c->hc_small.p;
    HIPCHK(c, hipMemcpyAsync(cnt, j.counters + 19, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint32_t n = *cnt;
    if (n == 0) return RPGPU_OK;
    const size_t ib = (size_t)n * sizeof(HostItem);
    if (int rc = grow_buf(c, c->hc_items, ib, false, s)) return rc;
    if (int rc = grow_buf(c, c->hc_items_h, ib, true, s)) return rc;
    HostItem* dit = (HostItem*)c->hc_items.p;
    HostItem* hit = (HostItem*)c->hc_items_h.p;
    HIPCHK(c, launch_host_desc(j, dit, n, s));
    HIPCHK(c, hipMemcpyAsync(hit, dit, ib, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    uint64_t in_total = 0;
    for (uint32_t i = 0; i < n; i++) {
        hit[i].stage = in_total;
        in_total += align_up(hit[i].n, 16);
    }
    if (int rc = grow_buf(c, c->hc_in, in_total + 16, false, s)) return rc;
    if (int rc = grow_buf(c, c->hc_in_h, in_total + 16, true, s)) return rc;
    HIPCHK(c, hipMemcpyAsync(dit, hit, ib, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_host_gather(j, dit, n, (uint8_t*)c->hc_in.p, s));
    HIPCHK(c, hipMemcpyAsync(c->hc_in_h.p, c->hc_in.p, in_total, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    // decode: compressor::uncompress throws on an empty payload
    // (compression/compression.cc:34-55), then the reference loop
    std::vector<std::vector<uint8_t>> outs(n);
    const uint8_t* in = (const uint8_t*)c->hc_in_h.p;
    std::atomic<uint32_t> next{0};
    std::atomic<bool> missing{false};
    // RPGPU_HOST_CODEC_MISSING=1 (diagnostic build): act as if libzstd could
    // not be loaded (tests the unsupported path)
    static const bool force_missing = [] { const char* e = diag_env("RPGPU_HOST_CODEC_MISSING"); return e && *e == '1'; }();
    auto work = [&]() {
        for (uint32_t i; (i = next.fetch_add(1)) < n;) {
            HostItem& it = hit[i];
            it.status = -1;
            it.out_len = 0;
            if (it.n == 0) continue;
            std::vector<uint8_t>& o = outs[i];
            o.resize((size_t)it.n * 4 + 4096);
            size_t len = 0;
            int rc = force_missing ? kHostCodecMissing
                                   : host_uncompress(kHostZstd, in + it.stage, it.n, o.data(), o.size(), &len);
            if (rc == kHostCodecOverflow) {
                o.resize(len);
                rc = host_uncompress(kHostZstd, in + it.stage, it.n, o.data(), o.size(), &len);
            }
            if (rc == kHostCodecMissing) missing = true;
            if (rc == 0) {
                it.status = 0;
                it.out_len = len;
            }
        }
    };
    const uint32_t nt = std::min<uint32_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())), n);
    std::vector<std::thread> pool;
    for (uint32_t t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    // a payload libzstd never saw is not corrupt: the job is unsupported here
    // (rpgpu_uncompress answers RPGPU_E_UNSUPPORTED the same way)
    if (missing) return fail(c, RPGPU_E_UNSUPPORTED, "RPGPU_JOB_HOST_CODECS: libzstd not loadable");
    uint64_t out_total = 0;
    for (uint32_t i = 0; i < n; i++) {
        HostItem& it = hit[i];
        it.cap = it.status == 0 ? align_up(it.out_len, 16) : 0;
        it.stage = out_total;
        out_total += it.cap;
    }
    if (int rc = grow_buf(c, c->hc_out, out_total + 16, false, s)) return rc;
    if (int rc = grow_buf(c, c->hc_out_h, out_total + 16, true, s)) return rc;
    for (uint32_t i = 0; i < n; i++)
        if (hit[i].status == 0) memcpy((uint8_t*)c->hc_out_h.p + hit[i].stage, outs[i].data(), hit[i].out_len);
    HIPCHK(c, hipMemcpyAsync(c->hc_out.p, c->hc_out_h.p, out_total, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(dit, hit, ib, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_host_patch(j, dit, n, s));
    // the pinned copies are read by the copies just queued: done before this
    // context's next host step rewrites them (it syncs the stream first)
    c->hc_n = n;
    return RPGPU_OK;
}

int submit_body(rpgpu_ctx* c, const rpgpu_job* job, hipStream_t s, int stop, PlanPtrs* plan) {
    if (!c || !job || !job->d_data || !job->d_seg_offsets || !job->h_seg_offsets || job->n_segments == 0 ||
        !job->d_batches || !job->d_summaries || !job->d_totals)
        return fail(c, RPGPU_E_INVALID, "rpgpu_submit: missing argument");
    if (((uintptr_t)job->d_data & 15) != 0) return fail(c, RPGPU_E_INVALID, "rpgpu_submit: d_data must be 16-byte aligned");
    if (job->layout != RPGPU_LAYOUT_DISK && job->layout != RPGPU_LAYOUT_WIRE)
        return fail(c, RPGPU_E_INVALID, "rpgpu_submit: unknown layout");
    if ((job->flags & RPGPU_JOB_PARSE) && !job->d_records && job->record_capacity)
        return fail(c, RPGPU_E_INVALID, "rpgpu_submit: PARSE needs d_records");
    const uint32_t nseg = job->n_segments;
    const uint32_t cs = job->chunk_bytes ? job->chunk_bytes : (256u << 10);
    // chunk table from the host offsets
    uint64_t tc = 0;
    for (uint32_t i = 0; i < nseg; i++) {
        const uint64_t len = job->h_seg_offsets[i + 1] - job->h_seg_offsets[i];
        uint64_t nc = (len + cs - 1) / cs;
        tc += nc ? nc : 1;
    }
    if (tc > 0xFFFFFFF0ull) return fail(c, RPGPU_E_INVALID, "rpgpu_submit: too many chunks");
    const uint64_t bcap = job->batch_capacity;
    // workspace layout
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    const size_t o_cbase = take((nseg + 1) * 8);
    const size_t o_chunks = take(tc * sizeof(ChunkRec));
    const size_t o_ccount = take((tc + 1) * 8);
    const size_t o_centry = take(tc * 8);
    const size_t o_segterm = take(nseg * sizeof(SegTerm));
    const size_t o_slots = take((bcap + 1) * 8);
    const size_t o_dcap = take((bcap + 1) * 8);
    const size_t o_counters = take(kCounterBytes);
    const size_t o_dlist = take((bcap + 1) * 4);
    const size_t o_slist = take((bcap + 1) * 4);
    const size_t o_llist = take((bcap + 1) * 4);
    const size_t o_fbad = take((size_t)nseg * 4);
    const bool decode_job = (job->flags & RPGPU_JOB_DECODE) != 0;
    const size_t o_ilist = take(decode_job ? (bcap + 1) * 4 : 0);
    const size_t o_istate = take(decode_job ? (bcap + 1) * 4 : 0);
    const size_t o_ioff = take(decode_job ? (bcap + 1) * 8 : 0);
    const size_t o_itot = take(decode_job ? (bcap + 1) * 8 : 0);
    const bool host_job = decode_job && (job->flags & RPGPU_JOB_HOST_CODECS);
    const size_t o_hlist = take(host_job ? (bcap + 1) * 4 : 0);
    // zstd literal blocks planned ahead (k_zplan -> k_zlits): a 128 KiB block
    // each at most, so the job's bytes / 16 KiB + 8 per batch is ample (past
    // it, blocks decode in place)
    const uint64_t zcap64 = decode_job ? std::min<uint64_t>(job->h_seg_offsets[nseg] / 16384 + 8 * bcap + 64, 0x7FFFFFFFull) : 0;
    const size_t o_zitems = take(zcap64 * 8);
    // gzip split decode: per member its first item and chunk count; items:
    // one per kGzsChunk deflate bytes of the split members, one more each
    const size_t o_gzsmem = take(decode_job ? 2 * (bcap + 1) * 4 : 0);
    const uint64_t gcap64 = decode_job ? std::min<uint64_t>(job->h_seg_offsets[nseg] / kGzsChunk + bcap + 64, 0x7FFFFFFFull) : 0;
    const size_t o_gzsit = take(gcap64 * sizeof(GzsItem));
    // block-parallel decode: one item per LZ4F block / snappy-java chunk
    const bool dec = (job->flags & RPGPU_JOB_DECODE) && job->d_decoded;
    const uint64_t data_len = job->h_seg_offsets[nseg];
    const uint64_t bl_cap64 = dec ? std::min<uint64_t>(data_len / 16384 + 2 * bcap + 64, 0x7FFFFFFFull) : 0;
    const size_t o_blocks = take(bl_cap64 * sizeof(BlockItem));
    const size_t o_plans = take(dec ? (bcap + 1) * sizeof(FramePlan) : 0);
    const size_t o_pstate = take(bl_cap64 * sizeof(PieceState));
    const size_t o_longl = take(bl_cap64 * 4);
    const size_t o_wlong = take(bl_cap64 * 4);
    const size_t o_rawl = take(bl_cap64 * 4);
    const size_t o_lanel = take(bl_cap64 * 4);
    const size_t o_lzfl = take(bl_cap64 * 4);
    const size_t o_lzft = take(bl_cap64 * 4);
    uint64_t split_min = std::max<uint64_t>(kSplitMin, 2 * data_len / ((uint64_t)c->cu_count * kVWaves));
    // RPGPU_SPLIT_MIN_KIB (diagnostic build): override (scripts/bench_skew.py A/B)
    if (const char* e = diag_env("RPGPU_SPLIT_MIN_KIB")) split_min = std::max<uint64_t>(strtoull(e, nullptr, 10) << 10, 64);
    const uint64_t split_cap = std::min<uint64_t>(data_len / split_min + 1, bcap + 1);
    const size_t o_split = take(split_cap * 4);
    const size_t o_spart = take(split_cap * kSplitParts * 4);
    const size_t o_scan = take(scan_temp_bytes(std::max<uint64_t>(tc, bcap)) + 64);
    const size_t need = off;
    if (dec && !c->seqs) {
        const uint32_t waves = c->cu_count * lz_exec_wgs_per_cu();
        if (hipMalloc(&c->seqs, (size_t)waves * kRecsPerLane * sizeof(SeqRec)) != hipSuccess) {
            c->seqs = nullptr;
            return fail(c, RPGPU_E_NOMEM, "decode sequence workspace");
        }
        c->exec_waves = waves;
    }
    // record pool: a compressed LZ4 byte yields at most 1/3 record (16 B),
    // typical data far fewer (C2: 0.33 B of records per stored byte); sized
    // from the job's bytes, clamped; pieces that do not fit are walked by
    // k_lz_exec itself
    const size_t slab_bytes = kSlabRecs * sizeof(SeqRec) + 4;
    const size_t pool_want = dec ? std::min<size_t>(std::max<size_t>(data_len / 2, 256ull << 20), 8ull << 30) : 0;
    if (pool_want > c->pool_bytes) {
        if (c->pool) {
            if (int rc = ws_drain(c, s)) return rc;
            hipFree(c->pool);
            c->pool = nullptr;
            c->pool_bytes = 0;
        }
        if (hipMalloc(&c->pool, pool_want) != hipSuccess) { c->pool = nullptr; return fail(c, RPGPU_E_NOMEM, "decode record pool"); }
        c->pool_bytes = pool_want;
    }
    if (need > c->ws_bytes) {
        if (c->ws) {
            if (int rc = ws_drain(c, s)) return rc;
            hipFree(c->ws);
            c->ws = nullptr;
        }
        if (hipMalloc(&c->ws, need) != hipSuccess) { c->ws_bytes = 0; return fail(c, RPGPU_E_NOMEM, "workspace"); }
        c->ws_bytes = need;
    }
    uint8_t* ws = (uint8_t*)c->ws;

    DeviceJob j;
    j.data = job->d_data;
    j.data_len = job->h_seg_offsets[nseg];
    j.seg_off = job->d_seg_offsets;
    j.chunk_base = (const uint64_t*)(ws + o_cbase);
    j.n_segments = nseg;
    j.flags = job->flags;
    j.layout = job->layout;
    j.chunk_bytes = cs;
    j.total_chunks = (uint32_t)tc;
    j.chunks = (ChunkRec*)(ws + o_chunks);
    j.chunk_count = (uint64_t*)(ws + o_ccount);
    j.chunk_entry = (uint64_t*)(ws + o_centry);
    j.seg_term = (SegTerm*)(ws + o_segterm);
    j.batches = job->d_batches;
    j.batch_capacity = bcap;
    j.slots = (uint64_t*)(ws + o_slots);
    j.dcap = (uint64_t*)(ws + o_dcap);
    j.records = job->d_records;
    j.record_capacity = job->d_records ? job->record_capacity : 0;
    j.decoded = job->d_decoded;
    j.decoded_capacity = job->d_decoded ? job->decoded_capacity : 0;
    j.summaries = job->d_summaries;
    j.totals = job->d_totals;
    j.bitmap = job->d_valid_bitmap;
    j.tables = c->d_tables;
    j.counters = (uint32_t*)(ws + o_counters);
    j.decode_list = (uint32_t*)(ws + o_dlist);
    j.seq_list = (uint32_t*)(ws + o_slist);
    j.link_list = (uint32_t*)(ws + o_llist);
    j.long_list = (uint32_t*)(ws + o_longl);
    j.wlong_list = (uint32_t*)(ws + o_wlong);
    j.raw_list = (dec && stop == kRunAll) ? (uint32_t*)(ws + o_rawl) : nullptr;
    j.lane_list = (uint32_t*)(ws + o_lanel);
    j.split_list = (uint32_t*)(ws + o_split);
    j.split_part = (uint32_t*)(ws + o_spart);
    j.split_capacity = (uint32_t)split_cap;
    j.split_min = split_min;
    j.seqs = c->seqs;
    j.exec_waves = c->exec_waves;
    j.pstate = (PieceState*)(ws + o_pstate);
    j.pool_slabs = (uint32_t)std::min<size_t>(c->pool_bytes / slab_bytes, 0xFFFFFFF0ull);
    // RPGPU_POOL_SLABS (diagnostic build): shrinks the record pool (exercises
    // k_lz_exec's own walk of the pieces the pool cuts short)
    if (const char* e = diag_env("RPGPU_POOL_SLABS")) j.pool_slabs = std::min<uint32_t>(j.pool_slabs, (uint32_t)atoi(e));
    j.pool = (SeqRec*)c->pool;
    // the decoded payloads' record chains (k_dchain) reuse the record pool,
    // idle once decode is done: one u32 per index slot.  RPGPU_DCHAIN=0
    // (diagnostic build): k_validate_decoded chains the records itself (A/B)
    // RPGPU_CRC_COMPOSE=0 (diagnostic build): k_validate streams every stored payload (A/B)
    static const bool compose_on = [] { const char* e = diag_env("RPGPU_CRC_COMPOSE"); return !(e && *e == '0'); }();
    j.crc_compose = compose_on ? 1u : 0u;
    static const bool dchain_on = [] { const char* e = diag_env("RPGPU_DCHAIN"); return !(e && *e == '0'); }();
    j.dchain = (dec && dchain_on && c->pool && (uint64_t)c->pool_bytes / 4 >= j.record_capacity) ? (uint32_t*)c->pool
                                                                                                  : nullptr;
    j.slab_next = (uint32_t*)((uint8_t*)c->pool + (size_t)j.pool_slabs * kSlabRecs * sizeof(SeqRec));
    // fast-path records: the planner reserves csize / 3 + 2 per listed LZ4
    // block (2.7 bytes per compressed byte; C2 uses 0.3 of the job's bytes),
    // 3x the job's bytes (a job of nothing but LZ4 blocks fits whole), 64 MiB
    // .. 16 GiB; a group of blocks that finds no room (and every group after
    // it) takes the walk / exec kernels, with the same results.
    // RPGPU_LZF=0 (diagnostic build): every piece through the walk / exec (A/B);
    // RPGPU_FREC_CAP=n (diagnostic build): at most n records (mixes listed
    // groups with walked ones in small jobs; tests/test_gpu_diag.py)
    j.frecs = nullptr;
    j.frec_cap = 0;
    j.lzf_list = nullptr;
    j.lzf_tail = nullptr;
    static const bool lzf_on = [] { const char* e = diag_env("RPGPU_LZF"); return !(e && *e == '0'); }();
    if (dec && lzf_on && stop == kRunAll) {
        const size_t want = std::min<size_t>(std::max<size_t>(data_len * 3, 64ull << 20), 16ull << 30);
        if (int rc = grow_pool(c, c->fpool, c->fpool_bytes, want, s)) return rc;
        if (c->fpool) {
            j.frecs = (uint2*)c->fpool;
            j.frec_cap = c->fpool_bytes / sizeof(uint2);
            if (const char* e = diag_env("RPGPU_FREC_CAP")) j.frec_cap = std::min<uint64_t>(j.frec_cap, strtoull(e, nullptr, 10));
            j.lzf_list = (uint32_t*)(ws + o_lzfl);
            j.lzf_tail = (uint32_t*)(ws + o_lzft);
        }
    }
    j.seg_first_bad = (uint32_t*)(ws + o_fbad);
    j.seeds = (job->d_seeds && job->d_seed_offsets) ? job->d_seeds : nullptr;
    j.seed_off = j.seeds ? job->d_seed_offsets : nullptr;
    j.inf_list = (uint32_t*)(ws + o_ilist);
    j.inf_state = (uint32_t*)(ws + o_istate);
    j.inf_off = (uint64_t*)(ws + o_ioff);
    j.inf_total = (uint64_t*)(ws + o_itot);
    // gzip first-pass pool: twice the job's bytes, 256 MiB .. 2 GiB (members
    // that do not fit are decoded again, straight into the arena)
    j.inf_scratch = nullptr;
    j.inf_scratch_bytes = 0;
    j.inf_scratch_used = (uint64_t*)(j.counters + 24);  // zeroed with the counters
    // Only a job that writes decoded bytes uses it (a planning run only sizes
    // members); failing to get it costs a second pass, never the job.
    if (dec && stop == kRunAll) {
        size_t want = std::min<size_t>(std::max<size_t>(2 * data_len, 256ull << 20), 2ull << 30);
        // RPGPU_INF_POOL_KIB (diagnostic build): a small pool (exercises members
        // that do not get a scratch slot)
        if (const char* e = diag_env("RPGPU_INF_POOL_KIB")) want = std::max<size_t>(strtoull(e, nullptr, 10) << 10, 4096);
        if (int rc = grow_pool(c, c->gz_pool, c->gz_pool_bytes, want, s)) return rc;
        if (c->gz_pool) {
            j.inf_scratch = (uint8_t*)c->gz_pool;
            j.inf_scratch_bytes = std::min<size_t>(c->gz_pool_bytes, want);
        }
    }
    // RPGPU_ZS_FAST=0 (diagnostic build): every zstd member through the wave decoder (A/B)
    static const uint32_t zs_fast = [] { const char* e = diag_env("RPGPU_ZS_FAST"); return e && *e == '0' ? 0u : 1u; }();
    j.zs_fast = zs_fast;
    j.zs_split = 0;
    j.zs_items = (uint64_t*)(ws + o_zitems);
    j.zs_items_cap = (uint32_t)zcap64;
    j.host_list = (uint32_t*)(ws + o_hlist);
    // the gzip split decode (with the scratch pool only: it writes the
    // members' bytes there); RPGPU_GZS=0 (diagnostic build): every gzip member
    // serial (A/B)
    j.gzs_mem = nullptr;
    j.gzs_items = (GzsItem*)(ws + o_gzsit);
    j.gzs_items_cap = (uint32_t)gcap64;
    j.gzs_pool = nullptr;
    j.gzs_pool_syms = 0;
#ifdef RPGPU_NO_GZS  // A/B variant (scripts/build_exp.py): every gzip member serial
    static const bool gzs_on = false;
#else
    static const bool gzs_on = [] { const char* e = diag_env("RPGPU_GZS"); return !(e && *e == '0'); }();
#endif
    if (j.inf_scratch && gzs_on && gcap64) {
        const size_t want = std::min<size_t>(std::max<size_t>(2 * data_len, 64ull << 20), 4ull << 30);
        if (int rc = grow_pool(c, c->gzs_pool, c->gzs_pool_bytes, want, s)) return rc;
        if (c->gzs_pool) {
            j.gzs_mem = (uint32_t*)(ws + o_gzsmem);
            j.gzs_pool = (uint16_t*)c->gzs_pool;
            j.gzs_pool_syms = c->gzs_pool_bytes / 2;
        }
    }
    c->hc_n = 0;
    j.blocks = (BlockItem*)(ws + o_blocks);
    j.block_capacity = (uint32_t)bl_cap64;
    j.plans = (FramePlan*)(ws + o_plans);
    if (((uintptr_t)job->d_decoded & 15) != 0) return fail(c, RPGPU_E_INVALID, "rpgpu_submit: d_decoded must be 16-byte aligned");
    uint64_t* scan_tmp = (uint64_t*)(ws + o_scan);

    // RPGPU_DEBUG_SYNC=1 (diagnostic build): synchronize after every stage and
    // name the stage that failed (fault localisation)
    static const bool dbg = [] { const char* e = diag_env("RPGPU_DEBUG_SYNC"); return e && *e == '1'; }();
#define STAGE(name, call)                                                                  \
    do {                                                                                   \
        HIPCHK(c, (call));                                                                 \
        if (dbg) {                                                                         \
            fprintf(stderr, "[rpgpu] stage %s\n", name);                                   \
            fflush(stderr);                                                                \
            hipError_t _e = hipStreamSynchronize(s);                                       \
            if (_e == hipSuccess && c->side) _e = hipStreamSynchronize(c->side);           \
            if (_e == hipSuccess && c->side2) _e = hipStreamSynchronize(c->side2);         \
            if (_e != hipSuccess) return fail(c, RPGPU_E_HIP, "stage " name " failed", _e); \
        }                                                                                  \
    } while (0)
    // timed submits only: rpgpu_query_capacity's planning runs stop early
    // and record no timings
    const bool tm = c->timing && stop == kRunAll;
    hipEvent_t* ev = nullptr;
    if (tm) {
        if (c->ev_used == c->ev_sets.size()) {
            std::array<hipEvent_t, 7> set;
            for (auto& e : set) HIPCHK(c, hipEventCreate(&e));
            c->ev_sets.push_back(set);
        }
        ev = c->ev_sets[c->ev_used++].data();
        HIPCHK(c, hipEventRecord(ev[0], s));
    }
    STAGE("chunk_base", launch_chunk_base(j, s));
    HIPCHK(c, hipMemsetAsync(j.counters, 0, kCounterBytes, s));
    HIPCHK(c, hipMemsetAsync(j.seg_first_bad, 0xFF, (size_t)nseg * 4, s));
    STAGE("discover", launch_discover(j, s));
    if (tm) HIPCHK(c, hipEventRecord(ev[1], s));
    STAGE("resolve", launch_resolve(j, s));
    STAGE("scan_chunks", scan_exclusive_u64(j.chunk_count, tc, scan_tmp, 0, s));
    if (plan) {
        plan->n_batches = j.chunk_count + tc;
        plan->slots = j.slots;
        plan->dcap = j.dcap;
    }
    if (stop == kStopAfterCount) return RPGPU_OK;
    STAGE("emit", launch_emit(j, s));
    // gzip members: the first pass (their arena bytes, index slots and, when
    // they fit the pool, their output) before the scans
    if (decode_job) {
        // zstd members on the side stream when the lane parser can run (it
        // needs the scratch pool), gzip members (and, otherwise, zstd ones) here
        const bool split = j.inf_scratch && j.zs_fast;
        STAGE("zstamps", launch_zstamps(s, 0));
        // an error return between the fork and the join still orders `s`
        // after the side stream's kernels (the workspace is released on `s`)
        struct SideJoin {
            hipStream_t s = nullptr, side = nullptr;
            hipEvent_t ev = nullptr;
            ~SideJoin() {
                if (side && hipEventRecord(ev, side) == hipSuccess) hipStreamWaitEvent(s, ev, 0);
            }
        } side_join;
        if (split) {
            if (!c->side) HIPCHK(c, side_stream_create(&c->side));
            if (!c->fork_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
            if (!c->join_ev) HIPCHK(c, hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming));
            j.zs_split = 1;
            HIPCHK(c, hipEventRecord(c->fork_ev, s));
            HIPCHK(c, hipStreamWaitEvent(c->side, c->fork_ev, 0));
            side_join.s = s;
            side_join.ev = c->join_ev;
            side_join.side = c->side;
            STAGE("zplan", launch_zplan(j, c->side, c->cu_count * 4));
            STAGE("zparse", launch_zparse(j, c->side, c->cu_count * 4));
            HIPCHK(c, hipEventRecord(c->join_ev, c->side));
        }
        // the split decode's members first, then the serial first pass over
        // the rest and over the members the split decode did not close
        if (j.gzs_mem) {
            STAGE("gzsplan", launch_gzsplan(j, s));
            // the members it did not plan (below 16 KiB stored, FHCRC: one
            // wave each) beside the split decode's k_gzsdecode, on the
            // raw-copy stream (idle until the decode stage), the rest after
            // it.  (Forked before k_gzsfind instead, they slowed it 14.3 ->
            // 19.9 ms: C6 resolve+plan 58.9 against 56.7 ms.)  Diagnostic build:
            // RPGPU_MEM_SIDE=0 all after the split decode, 1 forked before k_gzsfind
            static const int mem_side = [] { const char* e = diag_env("RPGPU_MEM_SIDE"); return e ? atoi(e) : 2; }();
            if (mem_side == 2) STAGE("gzsfind", launch_gzsplit(j, s, c->cu_count, 1));
            struct MemJoin {
                hipStream_t s = nullptr, side = nullptr;
                hipEvent_t ev = nullptr;
                ~MemJoin() {
                    if (side && hipEventRecord(ev, side) == hipSuccess) hipStreamWaitEvent(s, ev, 0);
                }
            } mem_join;
            if (mem_side) {
                if (!c->side2) HIPCHK(c, side_stream_create(&c->side2));
                if (!c->mfork_ev) HIPCHK(c, hipEventCreateWithFlags(&c->mfork_ev, hipEventDisableTiming));
                if (!c->mjoin_ev) HIPCHK(c, hipEventCreateWithFlags(&c->mjoin_ev, hipEventDisableTiming));
                HIPCHK(c, hipEventRecord(c->mfork_ev, s));
                HIPCHK(c, hipStreamWaitEvent(c->side2, c->mfork_ev, 0));
                mem_join.s = s;
                mem_join.ev = c->mjoin_ev;
                mem_join.side = c->side2;
                STAGE("inflate_plan", launch_inflate_plan(j, c->side2, c->cu_count * 4, 1));
                HIPCHK(c, hipEventRecord(c->mjoin_ev, c->side2));
            }
            STAGE("gzsplit", launch_gzsplit(j, s, c->cu_count, mem_side == 2 ? 2 : 0));
            STAGE("inflate_plan", launch_inflate_plan(j, s, c->cu_count * 4, mem_side ? 2 : 0));
            if (mem_side) {
                HIPCHK(c, hipStreamWaitEvent(s, c->mjoin_ev, 0));
                mem_join.side = nullptr;  // joined
            }
        } else {
            STAGE("inflate_plan", launch_inflate_plan(j, s, c->cu_count * 4));
        }
        if (split) {
            HIPCHK(c, hipStreamWaitEvent(s, c->join_ev, 0));
            side_join.side = nullptr;  // joined
            STAGE("zfallback", launch_zfallback(j, s, c->cu_count * 4));
        }
        // zstd members whose corrupt stream reads ring bytes the current
        // segment has overwritten: decoded again over libzstd's exact buffer
        STAGE("zexact", launch_zexact(j, s, 0));
        STAGE("zstamps", launch_zstamps(s, 1));
    }
    // zstd members (RPGPU_JOB_HOST_CODECS): decoded on the host now, sized
    // before the scans like every other payload
    if (host_job)
        if (int rc = host_codec_step(c, j, s)) return rc;
    const uint64_t* d_nb = j.chunk_count + tc;
    STAGE("scan_slots", scan_exclusive_u64_devn(j.slots, d_nb, bcap, scan_tmp, s));
    // without DECODE every reservation is 0 (k_emit): the scan would write
    // zeros over zeros; k_finalize_totals reads no total then
    if (job->flags & RPGPU_JOB_DECODE) STAGE("scan_dcap", scan_exclusive_u64_devn(j.dcap, d_nb, bcap, scan_tmp, s));
    if (stop == kStopAfterPlan) return RPGPU_OK;
    if (tm) HIPCHK(c, hipEventRecord(ev[2], s));
    // k_content_xxh's side stream (below) joins s on every return, error paths too
    struct SideJoin {
        hipStream_t s = nullptr, side = nullptr;
        hipEvent_t ev = nullptr;
        ~SideJoin() {
            if (side && hipEventRecord(ev, side) == hipSuccess) hipStreamWaitEvent(s, ev, 0);
        }
    } xjoin;
    bool xside = false;
    // decode first: k_validate checksums and walks the decoded payloads
    if ((job->flags & RPGPU_JOB_DECODE) && j.decoded) {
        STAGE("decode", launch_decode(j, s, c->cu_count * 8));
        STAGE("decode_blocks", launch_decode_blocks(j, s, c->cu_count * 8));
        {
            // the listed LZ4 blocks (k_lzf_walk + k_lzf_tail) on the side
            // stream, every other piece (k_lz_walk) here: the planner fixed
            // the two sets (BlockItem.fast), so they run side by side
            struct LzfJoin {
                hipStream_t s = nullptr, side = nullptr;
                hipEvent_t ev = nullptr;
                ~LzfJoin() {
                    if (side && hipEventRecord(ev, side) == hipSuccess) hipStreamWaitEvent(s, ev, 0);
                }
            } lzf_join, raw_join;
            const bool lzf = j.lzf_list != nullptr;
            // RPGPU_WALK_FIRST=1 (diagnostic build): k_lz_walk submitted before
            // the side streams' kernels (dispatch-order A/B)
            static const bool walk_first = [] { const char* e = diag_env("RPGPU_WALK_FIRST"); return e && *e == '1'; }();
            bool walked = false;
            // RPGPU_LZWALK_WGS (diagnostic build): k_lz_walk's grid (workgroups)
            static const uint32_t lzw_env = [] { const char* e = diag_env("RPGPU_LZWALK_WGS"); return e ? (uint32_t)atoi(e) : 0u; }();
            const uint32_t lzw_grid = lzw_env ? lzw_env : c->cu_count * 16;
            if (lzf) {
                if (!c->side) HIPCHK(c, side_stream_create(&c->side));
                if (!c->fork_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
                if (!c->join_ev) HIPCHK(c, hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming));
                HIPCHK(c, hipEventRecord(c->fork_ev, s));
                HIPCHK(c, hipStreamWaitEvent(c->side, c->fork_ev, 0));
                if (walk_first) {
                    STAGE("lz_walk", launch_lz_walk(j, s, lzw_grid));
                    walked = true;
                }
                lzf_join.s = s;
                lzf_join.ev = c->join_ev;
                lzf_join.side = c->side;
                STAGE("lzf_walk", launch_lzf_walk(j, c->side, c->cu_count));
                HIPCHK(c, hipEventRecord(c->join_ev, c->side));
            }
            // the raw copies on a stream of their own, so that neither walk
            // waits for them (C5: the longest raw snappy walk, ~3.7 ms, began
            // after ~0.45 ms of copies).  RPGPU_RAW_SERIAL=1 (diagnostic
            // build): after the join (A/B of the overlap); RPGPU_RAW_STREAM=0:
            // before k_lz_walk on the job's stream (round-5 order)
            static const bool raw_serial = [] { const char* e = diag_env("RPGPU_RAW_SERIAL"); return e && *e == '1'; }();
            static const bool raw_own = [] { const char* e = diag_env("RPGPU_RAW_STREAM"); return !(e && *e == '0'); }();
            if (!raw_serial && lzf && raw_own && j.raw_list) {
                // RPGPU_RAW_PRIO=0 (diagnostic build): the raw-copy stream at the default priority (A/B)
                static const bool raw_prio = [] { const char* e = diag_env("RPGPU_RAW_PRIO"); return !(e && *e == '0'); }();
                if (!c->side2) HIPCHK(c, raw_prio ? side_stream_create(&c->side2) : hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking));
                if (!c->join2_ev) HIPCHK(c, hipEventCreateWithFlags(&c->join2_ev, hipEventDisableTiming));
                HIPCHK(c, hipStreamWaitEvent(c->side2, c->fork_ev, 0));
                raw_join.s = s;
                raw_join.ev = c->join2_ev;
                raw_join.side = c->side2;
                STAGE("raw_copy", launch_raw_copy(j, c->side2, c->cu_count));
                HIPCHK(c, hipEventRecord(c->join2_ev, c->side2));
            } else if (!raw_serial) {
                STAGE("raw_copy", launch_raw_copy(j, s, c->cu_count));
            }
            if (!walked) STAGE("lz_walk", launch_lz_walk(j, s, lzw_grid));
            if (lzf) {
                HIPCHK(c, hipStreamWaitEvent(s, c->join_ev, 0));
                lzf_join.side = nullptr;  // joined
            }
            if (raw_join.side) {
                HIPCHK(c, hipStreamWaitEvent(s, c->join2_ev, 0));
                raw_join.side = nullptr;
            }
            if (raw_serial) STAGE("raw_copy", launch_raw_copy(j, s, c->cu_count));
        }
        STAGE("lz_exec", launch_lz_exec(j, s));
        // RPGPU_XXH_SIDE=0 (diagnostic build): the content checksums inside
        // k_decode_finish, k_crc_compose and k_dchain in the validate stage (A/B)
        static const bool xxh_side = [] { const char* e = diag_env("RPGPU_XXH_SIDE"); return !(e && *e == '0'); }();
        xside = xxh_side;
        // the gzip / zstd members first: k_zexec's workgroups take a CU's
        // registers each and did not fit beside k_content_xxh's waves
        STAGE("inflate", launch_inflate(j, s, c->cu_count * 4));
        STAGE("zexec", launch_zexec(j, s));
        STAGE("zexact", launch_zexact(j, s, 1));
        if (c->hc_n) STAGE("host_scatter", launch_host_scatter(j, (const HostItem*)c->hc_items.p, c->hc_n,
                                                               (const uint8_t*)c->hc_out.p, s));
        if (xside) {
            // k_crc_compose (no dependence on the decoded bytes) before the
            // fork, for the same reason.  Then the LZ4F content checksums
            // (serial XXH32 chains, ~1 ms per MiB on one wave each: the rest
            // of the chip idles) on the side stream beside k_decode_finish
            // and the decoded payloads' record chains, which do not depend on
            // them (k_decode_finish gives a checksummed frame its verdict as
            // if it matched; k_content_apply takes it back after the join)
            // RPGPU_COMPOSE_BESIDE=1 (diagnostic build): k_crc_compose after the
            // fork, 8 waves per workgroup (room for a hashing wave per SIMD) (A/B)
            static const bool compose_beside = [] { const char* e = diag_env("RPGPU_COMPOSE_BESIDE"); return e && *e == '1'; }();
            if (!compose_beside) STAGE("crc_compose", launch_crc_compose(j, s, c->cu_count));
            if (!c->side) HIPCHK(c, side_stream_create(&c->side));
            if (!c->fork_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
            if (!c->join_ev) HIPCHK(c, hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming));
            HIPCHK(c, hipEventRecord(c->fork_ev, s));
            HIPCHK(c, hipStreamWaitEvent(c->side, c->fork_ev, 0));
            xjoin.s = s;
            xjoin.ev = c->join_ev;
            xjoin.side = c->side;
            STAGE("content_xxh", launch_content_xxh(j, c->side, c->cu_count * 2));
            if (compose_beside) STAGE("crc_compose", launch_crc_compose(j, s, c->cu_count, 8));
        }
        STAGE("decode_finish", launch_decode_finish(j, s, c->cu_count * 8, xside));
        if (xside) {
            STAGE("dchain", launch_dchain(j, s, c->cu_count));
            HIPCHK(c, hipEventRecord(c->join_ev, c->side));
            HIPCHK(c, hipStreamWaitEvent(s, c->join_ev, 0));
            xjoin.side = nullptr;  // joined
            STAGE("content_apply", launch_content_apply(j, s, c->cu_count));
        }
    }
    // RPGPU_WALK_WGS (diagnostic build): k_walk's grid (workgroups per CU)
    static const uint32_t walk_wgs = [] { const char* e = diag_env("RPGPU_WALK_WGS"); return e ? (uint32_t)atoi(e) : 8u; }();
    if (tm) HIPCHK(c, hipEventRecord(ev[3], s));
    STAGE("validate", launch_validate(j, s, c->cu_count, !xside));
    // the decoded payloads' record chains, then their walk.  (k_dchain on the
    // side stream beside k_crc_compose / k_validate measured slower than here:
    // C2 validate stage 4.36 against 3.72 ms, the chains' serial loads
    // queueing behind the two streams' HBM traffic)
    if (!xside) STAGE("dchain", launch_dchain(j, s, c->cu_count));
    STAGE("validate_decoded", launch_validate_decoded(j, s, c->cu_count));
    if (tm) HIPCHK(c, hipEventRecord(ev[4], s));
    STAGE("walk", launch_walk(j, s, c->cu_count * walk_wgs));
    if (tm) HIPCHK(c, hipEventRecord(ev[5], s));
    STAGE("finalize", launch_finalize(j, s));
    if (tm) HIPCHK(c, hipEventRecord(ev[6], s));
#undef STAGE
    return RPGPU_OK;
}
}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// output sizing before the run (SURVEY §8(b) segment-engine row: "result
// arrays ... sized by a query call"): the chain is discovered and planned
// (discover -> resolve -> emit -> scans) into context scratch, twice: once to
// count the batches, once with that many result slots to plan the record
// index and the decode arena.  Synchronous.
// ---------------------------------------------------------------------------
int rpgpu_query_capacity(rpgpu_ctx* c, const rpgpu_job* job, void* stream, rpgpu_capacity* out) {
    if (!c || !job || !out) return RPGPU_E_INVALID;
    if (!job->d_data || !job->d_seg_offsets || !job->h_seg_offsets || job->n_segments == 0)
        return fail(c, RPGPU_E_INVALID, "rpgpu_query_capacity: missing argument");
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    const uint32_t nseg = job->n_segments;
    auto grow = [&](void** p, size_t* have, size_t want) -> int {
        if (want <= *have) return RPGPU_OK;
        if (*p) {
            if (int rc = ws_drain(c, s)) return rc;
            HIPCHK(c, hipFree(*p));
            *p = nullptr;
            *have = 0;
        }
        if (hipMalloc(p, want) != hipSuccess) { *p = nullptr; return fail(c, RPGPU_E_NOMEM, "rpgpu_query_capacity: scratch"); }
        *have = want;
        return RPGPU_OK;
    };
    const size_t fixed = align_up((size_t)nseg * sizeof(rpgpu_segment_summary), 256) + align_up(sizeof(rpgpu_job_totals), 256);
    int rc = grow(&c->qws, &c->qws_bytes, fixed + 256);
    if (rc) return rc;
    rpgpu_job q = *job;
    q.d_summaries = (rpgpu_segment_summary*)c->qws;
    q.d_totals = (rpgpu_job_totals*)((uint8_t*)c->qws + align_up((size_t)nseg * sizeof(rpgpu_segment_summary), 256));
    q.d_batches = (rpgpu_batch_result*)((uint8_t*)c->qws + fixed);
    q.batch_capacity = 0;
    q.d_records = nullptr;
    q.record_capacity = 0;
    q.d_decoded = nullptr;
    q.decoded_capacity = 0;
    q.d_valid_bitmap = nullptr;
    PlanPtrs pp;
    rc = submit_impl(c, &q, stream, kStopAfterCount, &pp);
    if (rc) return rc;
    uint64_t nb = 0;
    HIPCHK(c, hipMemcpyAsync(&nb, pp.n_batches, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    rc = grow(&c->qws, &c->qws_bytes, fixed + (size_t)(nb + 1) * sizeof(rpgpu_batch_result));
    if (rc) return rc;
    q.d_summaries = (rpgpu_segment_summary*)c->qws;
    q.d_totals = (rpgpu_job_totals*)((uint8_t*)c->qws + align_up((size_t)nseg * sizeof(rpgpu_segment_summary), 256));
    q.d_batches = (rpgpu_batch_result*)((uint8_t*)c->qws + fixed);
    q.batch_capacity = nb;
    rc = submit_impl(c, &q, stream, kStopAfterPlan, &pp);
    if (rc) return rc;
    uint64_t v[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(&v[0], pp.slots + nb, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&v[1], pp.dcap + nb, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    out->n_batches = nb;
    out->record_capacity = v[0];
    out->decoded_capacity = (job->flags & RPGPU_JOB_DECODE) ? v[1] : 0;
    out->reserved = 0;
    return RPGPU_OK;
}

// ---------------------------------------------------------------------------
// non-blocking completion (rpgpu_poll / rpgpu_wait on a job):
// rpgpu_submit followed by an event on the launch stream
// ---------------------------------------------------------------------------
struct rpgpu_pending {
    rpgpu_ctx* c;
    hipEvent_t ev;
};

int rpgpu_submit_async(rpgpu_ctx* c, const rpgpu_job* job, void* stream, rpgpu_pending** out) {
    if (!c || !out) return RPGPU_E_INVALID;
    *out = nullptr;
    const int rc = submit_impl(c, job, stream, kRunAll, nullptr);
    if (rc) return rc;
    rpgpu_pending* p = new rpgpu_pending{c, nullptr};
    hipError_t e = hipEventCreateWithFlags(&p->ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(p->ev, pick(c, stream));
    if (e != hipSuccess) {
        if (p->ev) (void)hipEventDestroy(p->ev);
        delete p;
        return fail(c, RPGPU_E_HIP, "rpgpu_submit_async: event", e);
    }
    *out = p;
    return RPGPU_OK;
}

int rpgpu_poll(rpgpu_pending* p) {
    if (!p) return RPGPU_E_INVALID;
    const hipError_t e = hipEventQuery(p->ev);
    if (e == hipSuccess) return RPGPU_OK;
    if (e == hipErrorNotReady) return RPGPU_PENDING;
    return fail(p->c, RPGPU_E_HIP, "rpgpu_poll", e);
}

int rpgpu_wait(rpgpu_pending* p) {
    if (!p) return RPGPU_E_INVALID;
    HIPCHK(p->c, hipEventSynchronize(p->ev));
    return RPGPU_OK;
}

int rpgpu_release(rpgpu_pending* p) {
    if (!p) return RPGPU_E_INVALID;
    (void)hipEventDestroy(p->ev);
    delete p;
    return RPGPU_OK;
}

// ---------------------------------------------------------------------------
// crc::crc32c host path (hashing/crc32c.h:19-40).  SSE4.2 crc32 instructions,
// the same arithmetic google crc32c's x86 path uses.
// ---------------------------------------------------------------------------
__attribute__((target("sse4.2"))) uint32_t rpgpu_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
    uint64_t l = crc ^ 0xFFFFFFFFu;
    while (n && ((uintptr_t)p & 7)) { l = _mm_crc32_u8((uint32_t)l, *p++); n--; }
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        l = _mm_crc32_u64(l, v);
        p += 8;
        n -= 8;
    }
    uint32_t s = (uint32_t)l;
    while (n) { s = _mm_crc32_u8(s, *p++); n--; }
    return s ^ 0xFFFFFFFFu;
}

}  // extern "C"

extern "C" {

// compression::compressor::uncompress (compression/compression.h:21-24) for
// one payload: staged to the device, decoded by one wave (rp_codec.hip).
// The reference throws std::runtime_error on empty input, on `none` and on
// any decode failure -> RPGPU_E_CODEC; gzip/zstd are not decoded here.
// segment_index rebuild over a completed job's results (storage/log_replayer.cc:62-74,
// storage/segment_index.cc:58-72, storage/index_state.cc:48-95); kernel in rp_index.hip
int rpgpu_segment_index(rpgpu_ctx* c, const rpgpu_batch_result* d_batches, uint64_t batch_capacity,
                        const rpgpu_segment_summary* d_summaries, uint32_t n_segments, uint64_t step,
                        rpgpu_index_state* d_states, uint32_t* d_rel_offset, uint32_t* d_rel_time,
                        uint64_t* d_position, void* stream) {
    if (!c) return RPGPU_E_INVALID;
    if (n_segments == 0) return RPGPU_OK;
    if (!d_batches || !d_summaries || !d_states || !d_rel_offset || !d_rel_time || !d_position)
        return fail(c, RPGPU_E_INVALID, "rpgpu_segment_index: missing argument");
    if (step >= (1ull << 62)) return fail(c, RPGPU_E_INVALID, "rpgpu_segment_index: step out of range");
    if (n_segments > 0x7FFFFFFFu) return fail(c, RPGPU_E_INVALID, "rpgpu_segment_index: too many segments");
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    // RPGPU_INDEX_SERIAL=1 (diagnostic build): the one-wave-per-segment walk (A/B reference)
    static const bool serial = [] { const char* e = diag_env("RPGPU_INDEX_SERIAL"); return e && e[0] == '1'; }();
    if (serial) {
        HIPCHK(c, launch_segment_index(d_batches, batch_capacity, d_summaries, n_segments, step, d_states, d_rel_offset,
                                       d_rel_time, d_position, s));
        return RPGPU_OK;
    }
    const size_t need = segment_index_ws_bytes(n_segments, batch_capacity);
    if (need > c->iws_bytes) {
        if (c->iws) {
            if (int rc = ws_drain(c, s)) return rc;  // the old tables may still be in use on another stream
            HIPCHK(c, hipFree(c->iws));
            c->iws = nullptr;
            c->iws_bytes = 0;
        }
        HIPCHK(c, hipMalloc(&c->iws, need));
        c->iws_bytes = need;
    }
    if (int rc = ws_acquire(c, s)) return rc;
    HIPCHK(c, launch_segment_index_pieces(d_batches, batch_capacity, d_summaries, n_segments, step, d_states,
                                          d_rel_offset, d_rel_time, d_position, c->iws, s));
    return ws_release(c, s);
}

int rpgpu_uncompress(rpgpu_ctx* c, int codec, const void* in, size_t n, void* out, size_t cap, size_t* out_len) {
    if ((!in && n) || !out_len || (!out && cap)) return RPGPU_E_INVALID;
    // gzip / zstd run on the host: no context needed (ctx may be NULL)
    if (!c && codec != RPGPU_CODEC_GZIP && codec != RPGPU_CODEC_ZSTD) return RPGPU_E_INVALID;
    *out_len = 0;
    if (codec < 0 || codec > RPGPU_CODEC_ZSTD) return fail(c, RPGPU_E_INVALID, "rpgpu_uncompress: unknown codec");
    // compressor::uncompress (compression/compression.cc:34-53): an empty
    // buffer throws before the codec dispatch
    if (n == 0) return fail(c, RPGPU_E_CODEC, "rpgpu_uncompress: asked to decompress an empty buffer");
    if (codec == RPGPU_CODEC_NONE) return fail(c, RPGPU_E_CODEC, "compressor: nothing to uncompress for 'none'");
    if (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD) return host_codec(c, codec, in, n, out, cap, out_len);
    hipSetDevice(c->device);
    const uint64_t dcap = decode_capacity_dev(codec, (const uint8_t*)in, n);
    const size_t in_sz = align_up(n + 16, 256), out_sz = align_up(dcap + 16, 256);
    const size_t need = in_sz + out_sz + 256;
    if (need > c->uws_bytes) {
        if (c->uws) { hipStreamSynchronize(c->stream); hipFree(c->uws); c->uws = nullptr; }
        if (hipMalloc(&c->uws, need) != hipSuccess) { c->uws_bytes = 0; return fail(c, RPGPU_E_NOMEM, "uncompress workspace"); }
        c->uws_bytes = need;
    }
    uint8_t* d_in = (uint8_t*)c->uws;
    uint8_t* d_out = d_in + in_sz;
    int64_t* d_res = (int64_t*)(d_out + out_sz);
    HIPCHK(c, hipMemsetAsync(d_in + n, 0, in_sz - n, c->stream));
    HIPCHK(c, hipMemcpyAsync(d_in, in, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_uncompress_one(codec, d_in, n, d_out, out_sz, d_res, c->stream));
    int64_t res[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(res, d_res, sizeof res, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (res[0] != 0) return fail(c, RPGPU_E_CODEC, "rpgpu_uncompress: payload rejected");
    *out_len = (size_t)res[1];
    if ((size_t)res[1] > cap) return fail(c, RPGPU_E_OVERFLOW, "rpgpu_uncompress: output capacity too small");
    if (res[1]) HIPCHK(c, hipMemcpy(out, d_out, (size_t)res[1], hipMemcpyDeviceToHost));
    return RPGPU_OK;
}

// Write side: stamp the headers of n batches in place (rp_validate.hip
// k_stamp; disk_log_appender.cc:72-74 + parser_utils.cc:114-120).
int rpgpu_stamp(rpgpu_ctx* c, uint8_t* d_data, const uint64_t* d_pos, const uint32_t* d_payload_len, uint32_t n,
                int64_t next_offset, uint32_t flags, void* stream) {
    if (!c) return RPGPU_E_INVALID;
    if (n == 0) return RPGPU_OK;
    if (!d_data || !d_pos || ((flags & RPGPU_STAMP_CRC) && !d_payload_len) ||
        (flags & ~(RPGPU_STAMP_OFFSETS | RPGPU_STAMP_CRC)))
        return fail(c, RPGPU_E_INVALID, "rpgpu_stamp: bad argument");
    if (((uintptr_t)d_data & 15) != 0) return fail(c, RPGPU_E_INVALID, "rpgpu_stamp: d_data must be 16-byte aligned");
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    const size_t o_steps = 0, o_scan = align_up((size_t)(n + 1) * 8, 256);
    const size_t o_cur = align_up(o_scan + scan_temp_bytes(n) + 64, 256), need = o_cur + 256;
    if (need > c->sws_bytes) {
        if (c->sws) {
            if (int rc = ws_drain(c, s)) return rc;
            HIPCHK(c, hipFree(c->sws));
            c->sws = nullptr;
            c->sws_bytes = 0;
        }
        if (hipMalloc(&c->sws, need) != hipSuccess) { c->sws = nullptr; return fail(c, RPGPU_E_NOMEM, "rpgpu_stamp workspace"); }
        c->sws_bytes = need;
    }
    if (int rc = ws_acquire(c, s)) return rc;
    uint8_t* w = (uint8_t*)c->sws;
    uint64_t* steps = (uint64_t*)(w + o_steps);
    uint32_t* cursor = (uint32_t*)(w + o_cur);
    HIPCHK(c, hipMemsetAsync(cursor, 0, 4, s));
    if (flags & RPGPU_STAMP_OFFSETS) {
        HIPCHK(c, launch_stamp_steps(d_data, d_pos, n, steps, s));
        HIPCHK(c, scan_exclusive_u64(steps, n, w + o_scan, scan_temp_bytes(n) + 64, s));
    }
    HIPCHK(c, launch_stamp(d_data, d_pos, d_payload_len, steps, next_offset, n, flags, c->d_tables, cursor, c->cu_count, s));
    return ws_release(c, s);
}

// kafka::writer_serialize_batch over batches [first, first + n) of a
// completed disk-layout job (kafka/protocol/response_writer.h:241-276):
// the Kafka v2 record set, back to back in d_wire; *d_total (device) gets
// its length.  Asynchronous on `stream`.
int rpgpu_serialize_wire(rpgpu_ctx* c, const uint8_t* d_data, const uint64_t* d_seg_offsets,
                         const rpgpu_batch_result* d_batches, uint64_t first, uint32_t n, uint8_t* d_wire,
                         uint64_t* d_total, void* stream) {
    if (!c) return RPGPU_E_INVALID;
    if (!d_data || !d_seg_offsets || !d_batches || !d_wire || !d_total)
        return fail(c, RPGPU_E_INVALID, "rpgpu_serialize_wire: missing argument");
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    const size_t o_dst = align_up((size_t)(n + 1) * 8, 256), o_scan = o_dst + align_up((size_t)(n + 1) * 8, 256);
    const size_t need = o_scan + scan_temp_bytes(n) + 256;
    if (need > c->sws_bytes) {
        if (c->sws) {
            if (int rc = ws_drain(c, s)) return rc;
            HIPCHK(c, hipFree(c->sws));
            c->sws = nullptr;
            c->sws_bytes = 0;
        }
        if (hipMalloc(&c->sws, need) != hipSuccess) { c->sws = nullptr; return fail(c, RPGPU_E_NOMEM, "rpgpu_serialize_wire workspace"); }
        c->sws_bytes = need;
    }
    if (int rc = ws_acquire(c, s)) return rc;
    uint8_t* w = (uint8_t*)c->sws;
    uint64_t* src = (uint64_t*)w;
    uint64_t* dst = (uint64_t*)(w + o_dst);
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(d_total, 0, 8, s));
        return ws_release(c, s);
    }
    HIPCHK(c, launch_to_wire(d_data, d_wire, d_batches, d_seg_offsets, first, n, src, dst, w + o_scan,
                             scan_temp_bytes(n) + 64, c->cu_count * 8, s));
    HIPCHK(c, hipMemcpyAsync(d_total, dst + n, 8, hipMemcpyDeviceToDevice, s));
    return ws_release(c, s);
}

// Many payloads per GPU round trip (the per-batch call sites of
// compressor::uncompress, storage/parser_utils.cc:51 and
// kafka/protocol/kafka_batch_adapter.cc:259, batched): lz4/snappy payloads
// are staged into one pinned buffer, copied once, decoded one per lane, and
// their outputs copied back once; gzip/zstd go to the host fallback; every
// payload gets its own status (the rpgpu_uncompress codes).
int rpgpu_uncompress_batch(rpgpu_ctx* c, uint32_t n, const int* codecs, const void* const* in, const size_t* in_len,
                           void* const* out, const size_t* cap, size_t* out_len, int* status) {
    if (!c || (n && (!codecs || !in || !in_len || !out || !cap || !out_len || !status))) return RPGPU_E_INVALID;
    std::vector<uint32_t> dev;  // payloads decoded on the device
    std::vector<UncItem> items;
    uint64_t in_total = 0, out_total = 0;
    for (uint32_t i = 0; i < n; i++) {
        out_len[i] = 0;
        const int codec = codecs[i];
        if (codec < 0 || codec > RPGPU_CODEC_ZSTD || (!in[i] && in_len[i])) { status[i] = RPGPU_E_INVALID; continue; }
        if (in_len[i] == 0 || codec == RPGPU_CODEC_NONE) { status[i] = RPGPU_E_CODEC; continue; }
        if (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD) {
            status[i] = host_codec(c, codec, in[i], in_len[i], out[i], cap[i], &out_len[i]);
            continue;
        }
        UncItem it;
        it.src = in_total;
        it.n = in_len[i];
        it.dst = out_total;
        it.cap = align_up(decode_capacity_dev(codec, (const uint8_t*)in[i], in_len[i]) + 16, 16);
        it.codec = codec;
        it.pad = 0;
        in_total += align_up(in_len[i], 16);
        out_total += it.cap;
        items.push_back(it);
        dev.push_back(i);
        status[i] = RPGPU_E_CODEC;
    }
    if (items.empty()) return RPGPU_OK;
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const uint32_t m = (uint32_t)items.size();
    // device: [inputs + 16][items][results][outputs]; host (pinned): the same
    // first three parts, then the outputs coming back
    const size_t o_items = align_up(in_total + 16, 256), o_res = align_up(o_items + m * sizeof(UncItem), 256);
    const size_t o_out = align_up(o_res + (size_t)m * 16, 256), total = o_out + out_total;
    if (total > c->bd_bytes) {
        if (c->bd) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipFree(c->bd)); c->bd = nullptr; c->bd_bytes = 0; }
        if (hipMalloc(&c->bd, total) != hipSuccess) { c->bd = nullptr; return fail(c, RPGPU_E_NOMEM, "uncompress batch staging"); }
        c->bd_bytes = total;
    }
    if (total > c->bh_bytes) {
        if (c->bh) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipHostFree(c->bh)); c->bh = nullptr; c->bh_bytes = 0; }
        if (hipHostMalloc(&c->bh, total, hipHostMallocDefault) != hipSuccess) { c->bh = nullptr; return fail(c, RPGPU_E_NOMEM, "uncompress batch pinned staging"); }
        c->bh_bytes = total;
    }
    uint8_t* h = (uint8_t*)c->bh;
    uint8_t* d = (uint8_t*)c->bd;
    std::memset(h + in_total, 0, o_items - in_total);
    for (uint32_t k = 0; k < m; k++) std::memcpy(h + items[k].src, in[dev[k]], items[k].n);
    std::memcpy(h + o_items, items.data(), m * sizeof(UncItem));
    HIPCHK(c, hipMemcpyAsync(d, h, o_res, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_uncompress_many((const UncItem*)(d + o_items), m, d, in_total + 16, d + o_out, (int64_t*)(d + o_res), s));
    HIPCHK(c, hipMemcpyAsync(h + o_res, d + o_res, total - o_res, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const int64_t* res = (const int64_t*)(h + o_res);
    for (uint32_t k = 0; k < m; k++) {
        const uint32_t i = dev[k];
        if (res[2 * k] != 0) { status[i] = RPGPU_E_CODEC; continue; }
        out_len[i] = (size_t)res[2 * k + 1];
        if (out_len[i] > cap[i]) { status[i] = RPGPU_E_OVERFLOW; continue; }
        if (out_len[i]) std::memcpy(out[i], h + o_out + items[k].dst, out_len[i]);
        status[i] = RPGPU_OK;
    }
    return RPGPU_OK;
}

// compressor::compress for lz4 / snappy (rp_compress.hip)
size_t rpgpu_compress_bound(int codec, size_t n, size_t frag) {
    if (codec == RPGPU_CODEC_LZ4) return 15 + ((n + 65535) / 65536) * (4 + 65536) + 4;
    if (codec == RPGPU_CODEC_SNAPPY) {
        if (frag == 0 || frag > n) frag = n ? n : 1;
        const size_t nf = n ? (n + frag - 1) / frag : 0;
        return 16 + nf * (4 + 32 + frag + frag / 6);  // snappy::MaxCompressedLength per fragment
    }
    // deflateBound / ZSTD_compressBound, generously (per-fragment flushes add
    // a few bytes each)
    if (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD) {
        const size_t nf = frag ? (n + frag - 1) / frag : 1;
        return n + n / 64 + 1024 + nf * 16;
    }
    return 0;
}

int rpgpu_compress_batch(rpgpu_ctx* c, uint32_t n, const int* codecs, const void* const* in, const size_t* in_len,
                         const size_t* frag, void* const* out, const size_t* cap, size_t* out_len, int* status) {
    // ctx may be NULL when every payload is gzip / zstd (host work only)
    if (n && (!codecs || !in || !in_len || !out || !cap || !out_len || !status)) return RPGPU_E_INVALID;
    std::vector<uint32_t> dev;
    std::vector<CompPayload> pays;
    std::vector<CompBlock> blocks;
    // staged input pieces: (host bytes, length, staged offset); every snappy
    // fragment (each a RawCompress of its own) starts 16-byte aligned, as
    // the block kernels' dword reads assume
    struct Stage { const uint8_t* src; uint64_t n, off; };
    std::vector<Stage> stage;
    uint64_t in_total = 0, out_total = 0;
    for (uint32_t i = 0; i < n; i++) {
        out_len[i] = 0;
        const int codec = codecs[i];
        if (codec < 0 || codec > RPGPU_CODEC_ZSTD || (!in[i] && in_len[i])) { status[i] = RPGPU_E_INVALID; continue; }
        if (codec == RPGPU_CODEC_NONE) { status[i] = RPGPU_E_CODEC; continue; }
        if (codec == RPGPU_CODEC_GZIP || codec == RPGPU_CODEC_ZSTD) {
            // the CPU fallback: the reference's loops over zlib / libzstd
            const int r = host_compress(codec, (const uint8_t*)in[i], in_len[i], frag ? frag[i] : 0, (uint8_t*)out[i],
                                        cap[i], &out_len[i]);
            status[i] = r == 0 ? RPGPU_OK
                        : r == kHostCodecOverflow ? RPGPU_E_OVERFLOW
                        : r == kHostCodecMissing  ? RPGPU_E_UNSUPPORTED
                                                  : RPGPU_E_CODEC;
            continue;
        }
        // 32-bit frame fields (CompBlock::frag_len, the snappy length varint
        // and BE32 chunk length) hold lengths below 4 GiB only
        if (!c || in_len[i] >= (1ull << 32)) { status[i] = RPGPU_E_INVALID; continue; }
        const uint64_t len = in_len[i];
        uint64_t fr = (codec == RPGPU_CODEC_SNAPPY && frag && frag[i]) ? frag[i] : len;
        if (fr == 0) fr = 1;
        // snappy_java_compressor::compress writes int32_t(omax) per fragment
        // (compression/internal/snappy_java_compressor.cc:58-75): a fragment
        // whose bound does not fit int32 cannot be framed
        if (codec == RPGPU_CODEC_SNAPPY && 32 + std::min<uint64_t>(fr, len) + std::min<uint64_t>(fr, len) / 6 > 0x7FFFFFFFull) {
            status[i] = RPGPU_E_INVALID;
            continue;
        }
        CompPayload p;
        p.n = len;
        p.out = out_total;
        p.first = (uint32_t)blocks.size();
        p.codec = (uint32_t)codec;
        p.pad = 0;
        const uint8_t* src = (const uint8_t*)in[i];
        for (uint64_t f = 0; f < len; f += (codec == RPGPU_CODEC_LZ4 ? len : fr)) {
            // lz4: the frame's 64 KiB blocks whatever the fragmentation;
            // snappy: each fragment is a RawCompress of its own
            const uint64_t flen = codec == RPGPU_CODEC_LZ4 ? len : std::min<uint64_t>(fr, len - f);
            const uint32_t nbk = (uint32_t)((flen + 65535) / 65536);
            for (uint32_t k = 0; k < nbk; k++) {
                CompBlock b;
                b.src = in_total + (uint64_t)k * 65536;
                b.n = (uint32_t)std::min<uint64_t>(65536, flen - (uint64_t)k * 65536);
                b.codec = (uint32_t)codec;
                b.frag_len = k == 0 ? (uint32_t)flen : 0;
                b.frag_blocks = k == 0 ? nbk : 0;
                blocks.push_back(b);
            }
            stage.push_back({src + f, flen, in_total});
            in_total += align_up(flen + 8, 16);
        }
        p.nblocks = (uint32_t)blocks.size() - p.first;
        pays.push_back(p);
        dev.push_back(i);
        out_total += align_up(rpgpu_compress_bound(codec, len, fr), 16);
        status[i] = RPGPU_E_CODEC;
    }
    if (pays.empty()) return RPGPU_OK;
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const uint32_t np = (uint32_t)pays.size(), nb = (uint32_t)blocks.size();
    // device: [inputs][blocks][payloads] | [out_len][sizes][outputs][scratch];
    // host (pinned): the first part, then out_len + outputs coming back
    const size_t o_blk = align_up(in_total + 16, 256), o_pay = align_up(o_blk + (size_t)nb * sizeof(CompBlock), 256);
    const size_t o_len = align_up(o_pay + (size_t)np * sizeof(CompPayload), 256);
    const size_t o_sz = align_up(o_len + (size_t)np * 8, 256), o_out = align_up(o_sz + (size_t)nb * 4, 256);
    const size_t o_scr = align_up(o_out + out_total, 256), total = o_scr + (size_t)nb * kCompSlot;
    if (total > c->bd_bytes) {
        if (c->bd) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipFree(c->bd)); c->bd = nullptr; c->bd_bytes = 0; }
        if (hipMalloc(&c->bd, total) != hipSuccess) { c->bd = nullptr; return fail(c, RPGPU_E_NOMEM, "compress staging"); }
        c->bd_bytes = total;
    }
    if (o_scr > c->bh_bytes) {
        if (c->bh) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipHostFree(c->bh)); c->bh = nullptr; c->bh_bytes = 0; }
        if (hipHostMalloc(&c->bh, o_scr, hipHostMallocDefault) != hipSuccess) { c->bh = nullptr; return fail(c, RPGPU_E_NOMEM, "compress pinned staging"); }
        c->bh_bytes = o_scr;
    }
    uint8_t* h = (uint8_t*)c->bh;
    uint8_t* d = (uint8_t*)c->bd;
    std::memset(h, 0, o_blk);
    for (const Stage& st : stage)
        if (st.n) std::memcpy(h + st.off, st.src, st.n);
    std::memcpy(h + o_blk, blocks.data(), nb * sizeof(CompBlock));
    std::memcpy(h + o_pay, pays.data(), np * sizeof(CompPayload));
    HIPCHK(c, hipMemcpyAsync(d, h, o_len, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_compress(d, (const CompBlock*)(d + o_blk), nb, (const CompPayload*)(d + o_pay), np, d + o_scr,
                              (uint32_t*)(d + o_sz), d + o_out, (uint64_t*)(d + o_len), s));
    HIPCHK(c, hipMemcpyAsync(h + o_len, d + o_len, np * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(h + o_out, d + o_out, out_total, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint64_t* lens = (const uint64_t*)(h + o_len);
    for (uint32_t k = 0; k < np; k++) {
        const uint32_t i = dev[k];
        out_len[i] = (size_t)lens[k];
        if (out_len[i] > cap[i]) { status[i] = RPGPU_E_OVERFLOW; continue; }
        std::memcpy(out[i], h + o_out + pays[k].out, out_len[i]);
        status[i] = RPGPU_OK;
    }
    return RPGPU_OK;
}

// ---------------------------------------------------------------------------
// Host segment path (log_replayer over files, storage/log_replayer.cc:95-114):
// host-resident segments are grouped into staging groups of at most
// kHostGroupBytes (a larger segment is a group of its own), copied H2D with
// hipMemcpyAsync on the context's copy stream into one of two device slots,
// and validated by the same pipeline as rpgpu_submit on the compute stream;
// while group g validates, group g + 1 is being copied and group g - 1's
// per-batch results come back.  Outputs are the caller's host arrays; the
// record index and decoded bytes stay on the device (the verdict bits,
// records_parsed and the decoded crcs are in the batch results).  A group
// whose device outputs overflowed is re-run with the capacities the device
// reported, so the host sees the same results as one big rpgpu_submit.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {
constexpr uint64_t kHostGroupBytes = 256ull << 20;

// staging-group size: rpgpu_host_job.group_kib, 0 = kHostGroupBytes (tests
// use small groups to exercise the double buffering on small inputs)
uint64_t host_group_bytes(const rpgpu_host_job* job) {
    return job->group_kib ? (uint64_t)job->group_kib << 10 : kHostGroupBytes;
}

template <class T>
int grow(rpgpu_ctx* c, T*& p, uint64_t& have, uint64_t need) {
    if (need <= have && p) return RPGPU_OK;
    // hipFree waits for the device work still using the old buffer
    if (p) hipFree(p);
    p = nullptr;
    have = 0;
    if (hipMalloc((void**)&p, (size_t)std::max<uint64_t>(need, 1) * sizeof(T)) != hipSuccess)
        return fail(c, RPGPU_E_NOMEM, "rpgpu_validate_host: device staging");
    have = need;
    return RPGPU_OK;
}

struct HostGroup {
    uint32_t seg0, nseg;
    uint64_t bytes;
};

// issue group g on slot h: H2D on the copy stream, then the pipeline on the
// compute stream (after the copy), then the totals back to pinned memory
int host_issue(rpgpu_ctx* c, rpgpu_ctx::HostSlot& h, const rpgpu_host_job* job, const HostGroup& g) {
    const uint64_t padded = align_up(g.bytes + 64, 256);
    if (int rc = grow(c, h.d_data, h.data_bytes, padded)) return rc;
    if (int rc = grow(c, h.d_offs, h.offs_n, (uint64_t)g.nseg + 1)) return rc;
    if (int rc = grow(c, h.d_sums, h.sums_n, (uint64_t)g.nseg)) return rc;
    // first-try capacities: every batch at least a header, every record at
    // least 7 bytes (length, attributes, three deltas/lengths, header count),
    // decode up to 4x; a group that overflows is re-run
    const uint64_t bneed = g.bytes / RPGPU_HEADER_SIZE + 1;
    if (int rc = grow(c, h.d_batches, h.bcap, bneed)) return rc;
    if (job->flags & RPGPU_JOB_PARSE)
        if (int rc = grow(c, h.d_records, h.rcap, g.bytes / 7 + 1)) return rc;
    if (job->flags & RPGPU_JOB_DECODE)
        if (int rc = grow(c, h.d_decoded, h.dcap, 4 * g.bytes + 4096)) return rc;
    h.h_offs.assign(g.nseg + 1, 0);
    for (uint32_t i = 0; i < g.nseg; i++) h.h_offs[i + 1] = h.h_offs[i] + job->seg_sizes[g.seg0 + i];
    for (uint32_t i = 0; i < g.nseg; i++)
        if (job->seg_sizes[g.seg0 + i])
            HIPCHK(c, hipMemcpyAsync(h.d_data + h.h_offs[i], job->segments[g.seg0 + i], job->seg_sizes[g.seg0 + i],
                                     hipMemcpyHostToDevice, c->copy));
    HIPCHK(c, hipMemcpyAsync(h.d_offs, h.h_offs.data(), (g.nseg + 1) * 8, hipMemcpyHostToDevice, c->copy));
    HIPCHK(c, hipEventRecord(h.h2d, c->copy));
    HIPCHK(c, hipStreamWaitEvent(c->stream, h.h2d, 0));
    rpgpu_job j{};
    j.d_data = h.d_data;
    j.d_seg_offsets = h.d_offs;
    j.h_seg_offsets = h.h_offs.data();
    j.n_segments = g.nseg;
    j.layout = job->layout;
    j.flags = job->flags;
    j.d_batches = h.d_batches;
    j.batch_capacity = h.bcap;
    j.d_records = h.d_records;
    j.record_capacity = (job->flags & RPGPU_JOB_PARSE) ? h.rcap : 0;
    j.d_decoded = h.d_decoded;
    j.decoded_capacity = (job->flags & RPGPU_JOB_DECODE) ? h.dcap : 0;
    j.d_summaries = h.d_sums;
    j.d_totals = h.d_tot;
    if (int rc = rpgpu_submit(c, &j, c->stream)) return rc;
    if (job->index_step && job->layout == RPGPU_LAYOUT_DISK) {
        // segment_index::maybe_track over the group's crc-good prefixes
        // (storage/log_replayer.cc:62-74), base offsets from the caller
        if (int rc = grow(c, h.d_ist, h.ist_n, (uint64_t)g.nseg)) return rc;
        if (h.ix_n < h.bcap || !h.d_ro) {
            uint64_t have = 0;
            if (int rc = grow(c, h.d_ro, have, h.bcap)) return rc;
            have = 0;
            if (int rc = grow(c, h.d_rt, have, h.bcap)) return rc;
            have = 0;
            if (int rc = grow(c, h.d_ps, have, h.bcap)) return rc;
            h.ix_n = h.bcap;
        }
        h.h_ist.assign(g.nseg, rpgpu_index_state{});
        for (uint32_t i = 0; i < g.nseg; i++) h.h_ist[i].base_offset = job->index_states[g.seg0 + i].base_offset;
        HIPCHK(c, hipMemcpyAsync(h.d_ist, h.h_ist.data(), g.nseg * sizeof(rpgpu_index_state), hipMemcpyHostToDevice,
                                 c->stream));
        if (int rc = rpgpu_segment_index(c, h.d_batches, h.bcap, h.d_sums, g.nseg, job->index_step, h.d_ist, h.d_ro, h.d_rt,
                                         h.d_ps, c->stream))
            return rc;
    }
    HIPCHK(c, hipMemcpyAsync(h.h_tot, h.d_tot, sizeof(rpgpu_job_totals), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(h.done, c->stream));
    return RPGPU_OK;
}
}  // namespace

extern "C" {

int rpgpu_validate_host(rpgpu_ctx* c, const rpgpu_host_job* job) {
    if (!c || !job || (job->n_segments && (!job->segments || !job->seg_sizes)) || !job->totals ||
        (job->n_segments && !job->summaries) || (job->batch_capacity && !job->batches) ||
        (job->record_capacity && !job->records) || (job->decoded_capacity && !job->decoded) ||
        (job->index_step && (!job->index_states || (job->batch_capacity && (!job->rel_offset || !job->rel_time ||
                                                                             !job->position)))))
        return fail(c, RPGPU_E_INVALID, "rpgpu_validate_host: missing argument");
    if (job->index_step >= (1ull << 62)) return fail(c, RPGPU_E_INVALID, "rpgpu_validate_host: index step out of range");
    if (job->layout != RPGPU_LAYOUT_DISK && job->layout != RPGPU_LAYOUT_WIRE)
        return fail(c, RPGPU_E_INVALID, "rpgpu_validate_host: unknown layout");
    hipSetDevice(c->device);
    std::memset(job->totals, 0, sizeof(rpgpu_job_totals));
    if (job->n_segments == 0) return RPGPU_OK;
    if (!c->copy) HIPCHK(c, hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
    for (auto& h : c->hs) {
        if (!h.h2d) HIPCHK(c, hipEventCreateWithFlags(&h.h2d, hipEventDisableTiming));
        if (!h.done) HIPCHK(c, hipEventCreateWithFlags(&h.done, hipEventDisableTiming));
        if (!h.h_tot) HIPCHK(c, hipHostMalloc((void**)&h.h_tot, sizeof(rpgpu_job_totals), hipHostMallocDefault));
        if (!h.d_tot) HIPCHK(c, hipMalloc((void**)&h.d_tot, sizeof(rpgpu_job_totals)));
    }
    std::vector<HostGroup> groups;
    const uint64_t gbytes = host_group_bytes(job);
    for (uint32_t i = 0; i < job->n_segments; i++) {
        const uint64_t sz = job->seg_sizes[i];
        if (!job->segments[i] && sz) return fail(c, RPGPU_E_INVALID, "rpgpu_validate_host: null segment");
        if (groups.empty() || groups.back().bytes + sz > gbytes) groups.push_back({i, 0, 0});
        groups.back().nseg++;
        groups.back().bytes += sz;
    }
    rpgpu_job_totals& T = *job->totals;
    uint64_t out_b = 0;
    // collect group gi (slot h): its totals, re-run on overflow, then the
    // batch results and summaries into the caller's arrays
    auto finish = [&](size_t gi) -> int {
        auto& h = c->hs[gi & 1];
        const HostGroup& g = groups[gi];
        HIPCHK(c, hipEventSynchronize(h.done));
        for (int tries = 0; h.h_tot->overflow && tries < 2; tries++) {
            const rpgpu_job_totals t = *h.h_tot;
            if (int rc = grow(c, h.d_batches, h.bcap, t.batch_capacity_needed)) return rc;
            if (job->flags & RPGPU_JOB_PARSE)
                if (int rc = grow(c, h.d_records, h.rcap, t.record_capacity_needed)) return rc;
            if (job->flags & RPGPU_JOB_DECODE)
                if (int rc = grow(c, h.d_decoded, h.dcap, t.decoded_capacity_needed)) return rc;
            if (int rc = host_issue(c, h, job, g)) return rc;
            HIPCHK(c, hipEventSynchronize(h.done));
        }
        const rpgpu_job_totals t = *h.h_tot;
        const uint64_t nb = t.n_batches;
        const uint64_t room = job->batch_capacity > out_b ? job->batch_capacity - out_b : 0;
        const uint64_t take = std::min(nb, room);
        // this group's positions in the job: its records and decoded bytes
        // follow the earlier groups' (the index slots and arena bytes one
        // rpgpu_submit over every segment would have reserved before them)
        const uint64_t rec_base = T.n_records, dec_base = T.decoded_bytes;
        const uint64_t nrec = (job->flags & RPGPU_JOB_PARSE) ? t.n_records : 0;
        const uint64_t ndec = (job->flags & RPGPU_JOB_DECODE) ? t.decoded_bytes : 0;
        const uint64_t rroom = job->record_capacity > rec_base ? job->record_capacity - rec_base : 0;
        const uint64_t droom = job->decoded_capacity > dec_base ? job->decoded_capacity - dec_base : 0;
        const uint64_t rtake = job->records ? std::min(nrec, rroom) : 0;
        const uint64_t dtake = job->decoded ? std::min(ndec, droom) : 0;
        const bool ix = job->index_step && job->layout == RPGPU_LAYOUT_DISK;
        // results back on the copy stream: the compute stream already holds
        // the next group's pipeline, which must not be waited for here
        if (take) {
            HIPCHK(c, hipMemcpyAsync(job->batches + out_b, h.d_batches, take * sizeof(rpgpu_batch_result),
                                     hipMemcpyDeviceToHost, c->copy));
            if (ix) {
                HIPCHK(c, hipMemcpyAsync(job->rel_offset + out_b, h.d_ro, take * 4, hipMemcpyDeviceToHost, c->copy));
                HIPCHK(c, hipMemcpyAsync(job->rel_time + out_b, h.d_rt, take * 4, hipMemcpyDeviceToHost, c->copy));
                HIPCHK(c, hipMemcpyAsync(job->position + out_b, h.d_ps, take * 8, hipMemcpyDeviceToHost, c->copy));
            }
        }
        if (rtake)
            HIPCHK(c, hipMemcpyAsync(job->records + rec_base, h.d_records, rtake * sizeof(rpgpu_record_index),
                                     hipMemcpyDeviceToHost, c->copy));
        if (dtake) HIPCHK(c, hipMemcpyAsync(job->decoded + dec_base, h.d_decoded, dtake, hipMemcpyDeviceToHost, c->copy));
        HIPCHK(c, hipMemcpyAsync(job->summaries + g.seg0, h.d_sums, g.nseg * sizeof(rpgpu_segment_summary),
                                 hipMemcpyDeviceToHost, c->copy));
        if (ix)
            HIPCHK(c, hipMemcpyAsync(job->index_states + g.seg0, h.d_ist, g.nseg * sizeof(rpgpu_index_state),
                                     hipMemcpyDeviceToHost, c->copy));
        HIPCHK(c, hipStreamSynchronize(c->copy));
        // group-relative -> job-wide ordinals and positions
        for (uint64_t i = 0; i < take; i++) {
            rpgpu_batch_result& r = job->batches[out_b + i];
            r.segment += g.seg0;
            r.index_base += rec_base;
            r.decoded_off += dec_base;
        }
        for (uint64_t i = 0; i < rtake; i++) job->records[rec_base + i].batch += (uint32_t)out_b;
        for (uint32_t i = 0; i < g.nseg; i++) job->summaries[g.seg0 + i].first_batch += out_b;
        if (ix)
            for (uint32_t i = 0; i < g.nseg; i++) job->index_states[g.seg0 + i].first_entry += out_b;
        if (nrec > rtake && job->records) T.overflow |= 2u;
        if (ndec > dtake && job->decoded) T.overflow |= 4u;
        T.n_batches += nb;
        T.n_records += t.n_records;
        T.decoded_bytes += t.decoded_bytes;
        T.n_rewalks += t.n_rewalks;
        T.record_capacity_needed += t.record_capacity_needed;
        T.decoded_capacity_needed += t.decoded_capacity_needed;
        T.overflow |= t.overflow;
        if (nb > room) T.overflow |= 1u;
        out_b += nb;
        return RPGPU_OK;
    };
    // issue(g) before finish(g - 1): group g's copy and pipeline are queued
    // while g - 1's results come back; issue(g + 1) reuses g - 1's slot
    for (size_t gi = 0; gi < groups.size(); gi++) {
        if (int rc = host_issue(c, c->hs[gi & 1], job, groups[gi])) return rc;
        if (gi) if (int rc = finish(gi - 1)) return rc;
    }
    if (int rc = finish(groups.size() - 1)) return rc;
    T.batch_capacity_needed = T.n_batches;
    return RPGPU_OK;
}

uint64_t rpgpu_uncompress_bound(int codec, const void* in, size_t n) {
    if (!in || n == 0 || (codec != RPGPU_CODEC_LZ4 && codec != RPGPU_CODEC_SNAPPY)) return 0;
    return decode_capacity_dev(codec, (const uint8_t*)in, n);
}

int rpgpu_stamp_host(rpgpu_ctx* c, uint8_t* buf, size_t len, const uint64_t* pos, const uint32_t* payload_len,
                     uint32_t n, int64_t next_offset, uint32_t flags) {
    if (!c) return RPGPU_E_INVALID;
    if (n == 0) return RPGPU_OK;
    if (!buf || !pos || ((flags & RPGPU_STAMP_CRC) && !payload_len))
        return fail(c, RPGPU_E_INVALID, "rpgpu_stamp_host: missing argument");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    // device: [batches + 16][pos][plen]; host (pinned): the same
    const size_t o_pos = align_up(len + 16, 256), o_len = align_up(o_pos + (size_t)n * 8, 256);
    const size_t total = align_up(o_len + (size_t)n * 4, 256);
    if (total > c->std_bytes) {
        if (c->std_) {
            if (int rc = ws_drain(c, s)) return rc;
            HIPCHK(c, hipFree(c->std_));
            c->std_ = nullptr;
            c->std_bytes = 0;
        }
        if (hipMalloc(&c->std_, total) != hipSuccess) { c->std_ = nullptr; return fail(c, RPGPU_E_NOMEM, "stamp staging"); }
        c->std_bytes = total;
    }
    if (total > c->sth_bytes) {
        if (c->sth) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipHostFree(c->sth)); c->sth = nullptr; c->sth_bytes = 0; }
        if (hipHostMalloc(&c->sth, total, hipHostMallocDefault) != hipSuccess) {
            c->sth = nullptr;
            return fail(c, RPGPU_E_NOMEM, "stamp pinned staging");
        }
        c->sth_bytes = total;
    }
    uint8_t* h = (uint8_t*)c->sth;
    uint8_t* d = (uint8_t*)c->std_;
    std::memcpy(h, buf, len);
    std::memset(h + len, 0, 16);
    std::memcpy(h + o_pos, pos, (size_t)n * 8);
    if (payload_len) std::memcpy(h + o_len, payload_len, (size_t)n * 4);
    HIPCHK(c, hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s));
    if (int rc = rpgpu_stamp(c, d, (const uint64_t*)(d + o_pos), payload_len ? (const uint32_t*)(d + o_len) : nullptr, n,
                             next_offset, flags, s))
        return rc;
    HIPCHK(c, hipMemcpyAsync(h, d, len, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    std::memcpy(buf, h, len);
    return RPGPU_OK;
}

}  // extern "C"
