// C ABI of pairing_amd (include/pairing_amd.h): argument checking, device
// buffers for the host-pointer entry points, error reporting.  No compute
// happens here; every entry point ends in a HIP kernel from
// kernels_field.hip / kernels_pairing.hip.
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/pairing_amd.h"
#include "launch.h"
#include "launch_msm.h"

namespace {

thread_local std::string g_last_error;
// Pairing kernel selection (pa_set_pairing_kernel).  0 (default) by batch
// size, each where it is fastest (round 5, profiles/r05_regimes.txt):
//   n <= pq_min() (768): the cooperative kernels (kernels_coop.hip, a
//      quad-VM workgroup per pairing, ~270 k pairings/s from 1.6 ms);
//   n <= pq_max() (4096; round 6): the lane-group kernels
//      (kernels_pair_quad.hip: one pairing per 32 lanes, rounds of 2048 at
//      ~3.8 ms -- 2048 pairs 3.78 ms, 4096 6.45, where the quad VM took 7.63 /
//      the lane pairs 8.41);
//   n <= pair_max() (32768): the generated kernels with a lane pair per
//      pairing, at most one wave per SIMD: 8.4-9.3 ms whatever n (the
//      cooperative kernels up to coop_max() = 2304 when lane groups are off);
//   n <= pair_max() + tail_max() (34816; round 6): the first 32768 on lane
//      pairs and the tail on a forked stream, on the cooperative kernels up
//      to 832 tail pairings and the lane groups above (split_head below;
//      32769: 10.8 ms, 34816: 13.0, instead of 15.7);
//   n <= one_max() (34048): one lane per pairing (one wave per SIMD at most:
//      ~15.7 ms, where a second lane-pair wave on a few SIMDs costs 15.6-16.7;
//      with the pairing-only lane-pair Miller loop lane pairs win from ~34 000
//      pairs, profiles/r05_regimes_after_ml2p.txt -- 38912 before it, and
//      still 38912 for the Miller-loop-only entries, ml_one_max(), which the
//      tail split leaves alone);
//   larger: lane pairs again, two or more waves per SIMD (2^16: 16.7 ms
//      against 17.2 ms one lane; 2^17: 33.0 vs 34.1 ms).  Round 5 gave the
//      lane-pair final exponentiation the Karabina squarings and the
//      in-kernel binary GCD (8.7 ms at 2^16 instead of 12.3 ms).
// 1 -> lane pairs for every batch size; 2 -> cooperative for every batch
// size; 3 -> one lane per pairing for every batch size; 4 -> cooperative for
// every batch size on the round-2 one-wave VM (A/B against the quad VM).
// written by pa_set_pairing_kernel and read by launches from any host thread
std::atomic<int> g_pairing_variant{0};
int pairing_variant() { return g_pairing_variant.load(std::memory_order_relaxed); }

size_t env_size(const char* name, size_t dflt) {
    const char* e = getenv(name);   // A/B measurements
    return e ? (size_t)strtoull(e, nullptr, 10) : dflt;
}
size_t coop_max() {
    static const size_t v = env_size("PA_COOP_MAX", 2304);
    return v;
}
size_t pair_max() {
    static const size_t v = env_size("PA_PAIR_MAX", 32768);
    return v;
}
size_t one_max() {
    static const size_t v = env_size("PA_ONE_MAX", 34048);
    return v;
}
// the same window's upper edge for the reference-form Miller loop alone (the
// Miller-loop entries: pa_miller_loop_fused_batch_device, pa_multi_miller_loop_affine):
// its lane-pair kernel is slower than the pairing-only one, so one lane per pairing
// wins up to 38912 pairs there (profiles/r05_regimes.txt)
size_t ml_one_max() {
    static const size_t v = env_size("PA_ML_ONE_MAX", 38912);
    return v;
}
bool use_coop(size_t n) {
    const int v = pairing_variant();
    return v == 2 || v == 4 || (v == 0 && n <= coop_max());
}
// the lane-group kernels (kernels_pair_quad.hip, one pairing per 32 lanes):
// variant 5 every size; the default in (PA_PQ_MIN, PA_PQ_MAX] = (768, 4096]:
// a round of them (at most 2048 pairings at one wave per SIMD) takes ~3.8 ms,
// against the quad VM's ~270 k pairings/s (800: 3.70 vs 3.94 ms, 2048: 3.78
// vs 7.63; the quad VM steps up after 768 pairings) and the lane pairs'
// ~8.4 ms (4096: 6.45 vs 8.41, both kernels at two waves per SIMD above 2048);
// profiles/r06_lane_groups.txt
size_t pq_min() {
    static const size_t v = env_size("PA_PQ_MIN", 768);
    return v;
}
size_t pq_max() {
    static const size_t v = env_size("PA_PQ_MAX", 4096);
    return v;
}
bool use_pq(size_t n) {
    const int v = pairing_variant();
    return v == 5 || (v == 0 && n > pq_min() && n <= pq_max());
}
int coop_vm() { return pairing_variant() == 4 ? 1 : 0; }
// lanes per pairing of the generated kernels; ml_only: the reference-form Miller
// loop without a final exponentiation behind it (its own crossover, ml_one_max)
int gen_lanes(size_t n, bool ml_only = false) {
    const int v = pairing_variant();
    if (v == 1) return 2;
    if (v == 3) return 1;
    return n <= pair_max() || n > (ml_only ? ml_one_max() : one_max()) ? 2 : 1;
}
// multi-pairings of at most this many pairs multiply their Miller values inside
// the cooperative final exponentiation (sequential mul12 macros); larger ones
// use the log-depth product tree first
constexpr size_t kCoopProductMax = 16;
// largest wNAF window the explicit-window fixed-base entries accept (the
// reference's heuristics pick 2..16 for G1, 2..15 for G2; its wnaf_form keeps
// a digit mod 2^(w+1) in a u64)
constexpr int kMaxWnafWindow = 62;

// Batches just above pair_max(): n <= pair_max() + tail_max() pairings run as
// the first pair_max() on lane pairs (one wave per SIMD, ~9.3 ms) and the tail
// on the cooperative kernels (a workgroup per pairing, latency-bound), the tail
// on a second stream forked from and joined back into the caller's, so its
// workgroups run beside the lane-pair waves -- instead of a second lane-pair
// wave on a few SIMDs (~15.7 ms whatever the tail).  Values are the same
// whichever kernels run a pairing (final exponentiation output; the
// pairing-only Miller values differ from the cooperative Miller loop's by Fq2
// factors, as pa_pairing_miller_loop_batch_device documents).  Not under
// stream capture (the side stream would join the graph); PA_TAIL_MAX=0 turns
// it off, PA_TAIL_SERIAL=1 runs the tail on the caller's stream (A/B).
size_t tail_max() {
    // profiles/r06_tail/: the forked tail beats a second lane-pair wave (15.6-15.7
    // ms) up to ~2000 tail pairs: 32769 10.8 ms, 33024 10.6, 33792 13.1 (the
    // cooperative kernels), 34048 12.9, 34816 13.0 (the lane groups); 35840
    // 15.7 -- no better than no split
    static const size_t v = env_size("PA_TAIL_MAX", 2048);
    return v;
}
// the tail's kernels: the cooperative ones up to 832 tail pairings, the lane
// groups above (33536: 12.3 vs 13.1 ms; 33664: 13.2 vs 12.9; 34816: 17.1 vs
// 13.0; profiles/r06_tail/); PA_TAIL_KIND=coop / pq forces one (A/B)
bool tail_pq(size_t tail) {
    static const int v = [] {
        const char* e = getenv("PA_TAIL_KIND");
        return !e ? 0 : strcmp(e, "pq") == 0 ? 1 : strcmp(e, "coop") == 0 ? 2 : 0;
    }();
    return v == 1 || (v == 0 && tail > 832);
}
struct TailFork {
    int dev = -1;
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
// a process-wide pool: a call takes a fork, enqueues the fork wait, the tail and
// the join wait, and gives it back (a wait holds the event's state at the time it
// is enqueued, so the next call may record the events again)
std::mutex g_tail_mu;
std::vector<TailFork*> g_tail_free;
size_t split_head(size_t n, hipStream_t s) {
    if (pairing_variant() != 0 || n <= pair_max() || n - pair_max() > tail_max()) return 0;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return 0;
    return pair_max();
}
// a fork whose side stream is ordered after everything enqueued on s (nullptr
// with PA_TAIL_SERIAL: the tail runs on s)
hipError_t tail_begin(hipStream_t s, TailFork** out) {
    static const bool serial = getenv("PA_TAIL_SERIAL") && atoi(getenv("PA_TAIL_SERIAL")) != 0;
    *out = nullptr;
    if (serial) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    TailFork* f = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_tail_mu);
        for (size_t i = 0; i < g_tail_free.size(); i++)
            if (g_tail_free[i]->dev == dev) {
                f = g_tail_free[i];
                g_tail_free.erase(g_tail_free.begin() + i);
                break;
            }
    }
    if (!f) {
        f = new TailFork;
        f->dev = dev;
        if ((e = hipStreamCreateWithFlags(&f->side, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&f->fork, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&f->join, hipEventDisableTiming)) != hipSuccess) {
            if (f->join) (void)hipEventDestroy(f->join);
            if (f->fork) (void)hipEventDestroy(f->fork);
            if (f->side) (void)hipStreamDestroy(f->side);
            delete f;
            return e;
        }
    }
    if ((e = hipEventRecord(f->fork, s)) == hipSuccess) e = hipStreamWaitEvent(f->side, f->fork, 0);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lock(g_tail_mu);
        g_tail_free.push_back(f);
        return e;
    }
    *out = f;
    return hipSuccess;
}
// s waits for the tail; the fork goes back to the pool
hipError_t tail_end(hipStream_t s, TailFork* f) {
    if (!f) return hipSuccess;
    hipError_t e = hipEventRecord(f->join, f->side);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, f->join, 0);
    std::lock_guard<std::mutex> lock(g_tail_mu);
    g_tail_free.push_back(f);
    return e;
}
constexpr size_t kG1Words = sizeof(pa_g1_affine) / 8, kG2Words = sizeof(pa_g2_affine) / 8,
                 kF12Words = sizeof(pa_fq12) / 8;

hipError_t ml_launch(const uint64_t* p, const uint64_t* q, uint64_t* out, size_t n, hipStream_t s) {
    if (use_pq(n)) return pa::launch_pq_miller_loop(p, q, out, n, s);
    if (use_coop(n)) return pa::launch_coop_miller_loop(p, q, out, n, s, coop_vm());
    return pa::launch_miller_loop_gen(gen_lanes(n, true), p, q, out, n, s);
}
// Miller loop of (P_i, G2Prepared_i) pairs: the generated kernel (tools/pgen
// miller_loop_prepared_prog); PA_ML_PREPARED=hipcc selects round 4's HIP C++
// kernel (kernels_pairing.hip) for A/B runs
hipError_t mlp_launch(const uint64_t* p, const uint64_t* q, uint64_t* out, size_t n, hipStream_t s) {
    static const bool hipcc = getenv("PA_ML_PREPARED") && strcmp(getenv("PA_ML_PREPARED"), "hipcc") == 0;
    if (hipcc) return pa::launch_miller_loop_prepared(p, q, out, n, s);
    return pa::launch_miller_loop_prepared_gen(p, q, out, n, s);
}
// The Miller loop in front of a final exponentiation (pa_pairing_batch[_device],
// pa_multi_pairing_device): on lane pairs the pairing-only kernel, whose Miller
// values differ from the reference's by Fq2 factors that the final
// exponentiation removes ((q^12 - 1) / r is a multiple of q^2 - 1) -- 3.5 %
// fewer instructions (tools/pgen/kernels.py doubling_step_h); round 6: one lane
// per pairing too (pa_gen_miller_loop1p).  The Miller-loop entries themselves
// keep ml_launch.  PA_PAIRING_ML=ref: the reference-form kernels (A/B).
hipError_t pairing_ml_launch(const uint64_t* p, const uint64_t* q, uint64_t* out, size_t n, hipStream_t s) {
    static const bool ref = getenv("PA_PAIRING_ML") && strcmp(getenv("PA_PAIRING_ML"), "ref") == 0;
    if (use_coop(n) || use_pq(n)) return ml_launch(p, q, out, n, s);
    if (const size_t h = split_head(n, s)) {
        TailFork* f = nullptr;
        hipError_t e = pa::launch_miller_loop_pairing_gen(2, p, q, out, h, s);
        if (e == hipSuccess) e = tail_begin(s, &f);
        if (e == hipSuccess)
            e = tail_pq(n - h) ? pa::launch_pq_miller_loop(p + h * kG1Words, q + h * kG2Words, out + h * kF12Words, n - h,
                                                      f ? f->side : s)
                          : pa::launch_coop_miller_loop(p + h * kG1Words, q + h * kG2Words, out + h * kF12Words,
                                                        n - h, f ? f->side : s, coop_vm());
        const hipError_t j = tail_end(s, f);
        return e != hipSuccess ? e : j;
    }
    if (ref) return pa::launch_miller_loop_gen(gen_lanes(n), p, q, out, n, s);
    return pa::launch_miller_loop_pairing_gen(gen_lanes(n), p, q, out, n, s);
}
hipError_t fe_launch(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t s) {
    if (use_pq(n)) return pa::launch_pq_final_exp(in, out, ok, n, s);
    if (use_coop(n)) return pa::launch_coop_final_exp(in, out, ok, n, s, coop_vm());
    if (const size_t h = split_head(n, s)) {
        TailFork* f = nullptr;
        hipError_t e = pa::launch_final_exp_gen(2, in, out, ok, h, s);
        if (e == hipSuccess) e = tail_begin(s, &f);
        if (e == hipSuccess)
            e = tail_pq(n - h) ? pa::launch_pq_final_exp(in + h * kF12Words, out + h * kF12Words, ok ? ok + h : nullptr,
                                                    n - h, f ? f->side : s)
                          : pa::launch_coop_final_exp(in + h * kF12Words, out + h * kF12Words, ok ? ok + h : nullptr,
                                                      n - h, f ? f->side : s, coop_vm());
        const hipError_t j = tail_end(s, f);
        return e != hipSuccess ? e : j;
    }
    return pa::launch_final_exp_gen(gen_lanes(n), in, out, ok, n, s);
}

int fail(int code, const char* what, hipError_t e = hipSuccess) {
    char buf[1024];
    const char* detail = pa::gen_error_detail();
    if (e != hipSuccess && detail[0])
        snprintf(buf, sizeof buf, "%s: %s (%d) [%s]", what, hipGetErrorString(e), (int)e, detail);
    else if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    else
        snprintf(buf, sizeof buf, "%s", what);
    g_last_error = buf;
    return code;
}

int hip_code(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return PA_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return PA_ERR_NO_DEVICE;
    return PA_ERR_HIP;
}

#define PA_TRY(expr, what)                                          \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return fail(hip_code(_e), what, _e);  \
    } while (0)

// ---- per-thread device context of the host-pointer entry points ----
// Every host-pointer call runs on its calling thread's own context for the
// current device: a non-blocking compute stream, a copy stream for the
// pipelined pairing path, grow-only device scratch slots and grow-only pinned
// staging buffers.  So a call never hipMallocs in steady state, waits only
// for its own stream (no device-wide synchronize), and calls from different
// host threads run concurrently (the reference traits are Send + Sync,
// lib.rs:120-121).  A thread's contexts go back to a process-wide pool when
// the thread exits (no HIP call at that point) and are reused by new threads.
struct HostCtx {
    int dev = -1;
    hipStream_t compute = nullptr, copy = nullptr, copy_out = nullptr;
    std::vector<std::pair<void*, size_t>> slots;     // device scratch, used as a stack by DevBuf
    size_t depth = 0;
    std::pair<void*, size_t> pinned[4] = {};          // pinned host staging (pipelined pairing)
    std::pair<void*, size_t> pipe[8] = {};            // device buffers of the pipelined pairing
    hipEvent_t ev[16] = {};
    size_t full_batch = 0;                            // pairings that fill the device once (one wave per SIMD)
};

struct CtxPool {
    std::mutex mu;
    std::vector<HostCtx*> free_ctx;
};
CtxPool& ctx_pool() {
    static CtxPool* p = new CtxPool;   // never destroyed: thread exits may return contexts late
    return *p;
}

struct ThreadCtxs {
    HostCtx* by_dev[64] = {};
    ~ThreadCtxs() {
        CtxPool& pool = ctx_pool();
        std::lock_guard<std::mutex> g(pool.mu);
        for (HostCtx* c : by_dev)
            if (c) {
                c->depth = 0;
                pool.free_ctx.push_back(c);
            }
    }
};
thread_local ThreadCtxs t_ctxs;

hipError_t thread_ctx(HostCtx** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (HostCtx* c = t_ctxs.by_dev[dev]) {
        *out = c;
        return hipSuccess;
    }
    {
        CtxPool& pool = ctx_pool();
        std::lock_guard<std::mutex> g(pool.mu);
        for (size_t k = 0; k < pool.free_ctx.size(); k++)
            if (pool.free_ctx[k]->dev == dev) {
                *out = t_ctxs.by_dev[dev] = pool.free_ctx[k];
                pool.free_ctx.erase(pool.free_ctx.begin() + k);
                return hipSuccess;
            }
    }
    HostCtx* c = new HostCtx;
    c->dev = dev;
    if ((e = hipStreamCreateWithFlags(&c->compute, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->copy_out, hipStreamNonBlocking)) != hipSuccess) {
        delete c;   // (a stream created before the failure is leaked: rare, bounded)
        return e;
    }
    for (auto& ev : c->ev)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    *out = t_ctxs.by_dev[dev] = c;
    return hipSuccess;
}

// grow-only buffer: reuse `b` if large enough (its last use has completed --
// every call synchronizes its streams before returning)
hipError_t grow(std::pair<void*, size_t>& b, size_t bytes, bool pinned) {
    if (b.second >= bytes && b.first) return hipSuccess;
    hipError_t e;
    if (b.first && (e = pinned ? hipHostFree(b.first) : hipFree(b.first)) != hipSuccess) return e;
    b = {nullptr, 0};
    bytes = bytes < 4096 ? 4096 : bytes + bytes / 8;   // headroom: fewer regrowths for slowly rising sizes
    if ((e = pinned ? hipHostMalloc(&b.first, bytes, hipHostMallocDefault) : hipMalloc(&b.first, bytes)) !=
        hipSuccess) {
        b.first = nullptr;
        return e;
    }
    b.second = bytes;
    return hipSuccess;
}

// One stream per device for the pipelined pairing kernels of every host
// thread: two batches' kernels running at once on one GPU share its SIMDs
// worse than back to back (each wave holds a whole SIMD), so the kernels of
// concurrent callers queue on this stream while their copies overlap them.
hipError_t pairing_stream(int dev, hipStream_t* out) {
    static std::mutex mu;
    static hipStream_t streams[64] = {};
    std::lock_guard<std::mutex> g(mu);
    if (!streams[dev]) {
        hipError_t e = hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking);
        if (e != hipSuccess) return e;
    }
    *out = streams[dev];
    return hipSuccess;
}

// The calling thread's compute stream on the current device (host entries).
hipStream_t call_stream() {
    HostCtx* c = nullptr;
    return thread_ctx(&c) == hipSuccess ? c->compute : nullptr;
}
hipError_t call_sync() {
    HostCtx* c = nullptr;
    hipError_t e = thread_ctx(&c);
    return e != hipSuccess ? e : hipStreamSynchronize(c->compute);
}

// A device scratch buffer for a host-pointer entry point: the next slot of
// the thread's context, released (not freed) when it goes out of scope.
struct DevBuf {
    void* p = nullptr;
    HostCtx* ctx = nullptr;
    hipError_t alloc(size_t bytes) {
        hipError_t e = thread_ctx(&ctx);
        if (e != hipSuccess) return e;
        if (ctx->slots.size() <= ctx->depth) ctx->slots.resize(ctx->depth + 1, {nullptr, 0});
        if ((e = grow(ctx->slots[ctx->depth], bytes ? bytes : 1, false)) != hipSuccess) {
            ctx = nullptr;
            return e;
        }
        p = ctx->slots[ctx->depth++].first;
        return hipSuccess;
    }
    ~DevBuf() {
        if (ctx) ctx->depth--;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

int upload(DevBuf& d, const void* host, size_t bytes) {
    PA_TRY(d.alloc(bytes), "device scratch");
    if (bytes) PA_TRY(hipMemcpyAsync(d.p, host, bytes, hipMemcpyHostToDevice, d.ctx->compute), "H2D copy");
    return PA_OK;
}
int download(void* host, const DevBuf& d, size_t bytes) {
    if (bytes) {
        PA_TRY(hipMemcpyAsync(host, d.p, bytes, hipMemcpyDeviceToHost, d.ctx->compute), "D2H copy");
        PA_TRY(hipStreamSynchronize(d.ctx->compute), "D2H copy");
    }
    return PA_OK;
}

bool op_needs_b(int op) {
    return op == pa::OP_FQ_MUL || op == pa::OP_FQ_ADD || op == pa::OP_FQ_SUB || op == pa::OP_FQ2_MUL ||
           op == pa::OP_FQ6_MUL || op == pa::OP_FQ12_MUL;
}

// Elementwise field op on host buffers: out = op(a, b).
int host_field_op(int op, const void* a, const void* b, void* out, uint8_t* ok, size_t n, size_t in_bytes,
                  size_t out_bytes, int param) {
    if (n == 0) return PA_OK;
    if (!a || !out || (op_needs_b(op) && !b)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf da, db, dout, dok;
    int rc;
    if ((rc = upload(da, a, in_bytes * n))) return rc;
    if (b && (rc = upload(db, b, in_bytes * n))) return rc;
    PA_TRY(dout.alloc(out_bytes * n), "device scratch");
    if (ok) PA_TRY(dok.alloc(n), "device scratch");
    PA_TRY(pa::launch_field_op(op, da.as<uint64_t>(), db.as<uint64_t>(), dout.as<uint64_t>(), dok.as<uint8_t>(), n,
                               param, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    if ((rc = download(out, dout, out_bytes * n))) return rc;
    if (ok && (rc = download(ok, dok, n))) return rc;
    return PA_OK;
}

}  // namespace

extern "C" {

const char* pa_version(void) { return "pairing_amd 0.1.0 (gfx950)"; }
const char* pa_last_error(void) { return g_last_error.c_str(); }

int pa_device_count(int* count) {
    if (!count) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return fail(PA_ERR_NO_DEVICE, "hipGetDeviceCount", e);
    }
    return PA_OK;
}
int pa_set_device(int device) {
    PA_TRY(hipSetDevice(device), "hipSetDevice");
    return PA_OK;
}
int pa_set_pairing_kernel(int variant) {
    if (variant < 0 || variant > 5) return fail(PA_ERR_INVALID_ARGUMENT, "kernel variant must be 0..5");
    g_pairing_variant.store(variant, std::memory_order_relaxed);
    return PA_OK;
}
int pa_set_decode_kernel(int variant) {
    if (variant < 0 || variant > 2) return fail(PA_ERR_INVALID_ARGUMENT, "decode kernel variant must be 0..2");
    pa::set_decode_variant(variant);
    return PA_OK;
}
int pa_synchronize(void) {
    PA_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return PA_OK;
}

int pa_fq_mul_batch(const pa_fq* a, const pa_fq* b, pa_fq* out, size_t n) {
    return host_field_op(pa::OP_FQ_MUL, a, b, out, nullptr, n, 48, 48, 0);
}
int pa_fq_square_batch(const pa_fq* a, pa_fq* out, size_t n) {
    return host_field_op(pa::OP_FQ_SQR, a, nullptr, out, nullptr, n, 48, 48, 0);
}
int pa_fq_add_batch(const pa_fq* a, const pa_fq* b, pa_fq* out, size_t n) {
    return host_field_op(pa::OP_FQ_ADD, a, b, out, nullptr, n, 48, 48, 0);
}
int pa_fq_sub_batch(const pa_fq* a, const pa_fq* b, pa_fq* out, size_t n) {
    return host_field_op(pa::OP_FQ_SUB, a, b, out, nullptr, n, 48, 48, 0);
}
int pa_fq_inverse_batch(const pa_fq* a, pa_fq* out, uint8_t* ok, size_t n) {
    if (n && !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null ok");
    return host_field_op(pa::OP_FQ_INV, a, nullptr, out, ok, n, 48, 48, 0);
}
int pa_fq_from_repr_batch(const pa_fq_repr* repr, pa_fq* out, uint8_t* ok, size_t n) {
    if (n && !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null ok");
    return host_field_op(pa::OP_FQ_FROM_REPR, repr, nullptr, out, ok, n, 48, 48, 0);
}
int pa_fq_into_repr_batch(const pa_fq* a, pa_fq_repr* out, size_t n) {
    return host_field_op(pa::OP_FQ_INTO_REPR, a, nullptr, out, nullptr, n, 48, 48, 0);
}
int pa_fq2_mul_batch(const pa_fq2* a, const pa_fq2* b, pa_fq2* out, size_t n) {
    return host_field_op(pa::OP_FQ2_MUL, a, b, out, nullptr, n, 96, 96, 0);
}
int pa_fq2_square_batch(const pa_fq2* a, pa_fq2* out, size_t n) {
    return host_field_op(pa::OP_FQ2_SQR, a, nullptr, out, nullptr, n, 96, 96, 0);
}
int pa_fq6_mul_batch(const pa_fq6* a, const pa_fq6* b, pa_fq6* out, size_t n) {
    return host_field_op(pa::OP_FQ6_MUL, a, b, out, nullptr, n, 288, 288, 0);
}
int pa_fq12_mul_batch(const pa_fq12* a, const pa_fq12* b, pa_fq12* out, size_t n) {
    return host_field_op(pa::OP_FQ12_MUL, a, b, out, nullptr, n, 576, 576, 0);
}
int pa_fq12_square_batch(const pa_fq12* a, pa_fq12* out, size_t n) {
    return host_field_op(pa::OP_FQ12_SQR, a, nullptr, out, nullptr, n, 576, 576, 0);
}
int pa_fq12_inverse_batch(const pa_fq12* a, pa_fq12* out, uint8_t* ok, size_t n) {
    if (n && !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null ok");
    return host_field_op(pa::OP_FQ12_INV, a, nullptr, out, ok, n, 576, 576, 0);
}
int pa_fq12_frobenius_map_batch(const pa_fq12* a, pa_fq12* out, size_t n, size_t power) {
    return host_field_op(pa::OP_FQ12_FROB, a, nullptr, out, nullptr, n, 576, 576, (int)(power % 12));
}
int pa_fq2_inverse_batch(const pa_fq2* a, pa_fq2* out, uint8_t* ok, size_t n) {
    if (n && !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null ok");
    return host_field_op(pa::OP_FQ2_INV, a, nullptr, out, ok, n, 96, 96, 0);
}
int pa_fq2_frobenius_map_batch(const pa_fq2* a, pa_fq2* out, size_t n, size_t power) {
    return host_field_op(pa::OP_FQ2_FROB, a, nullptr, out, nullptr, n, 96, 96, (int)(power % 2));
}
int pa_fq6_square_batch(const pa_fq6* a, pa_fq6* out, size_t n) {
    return host_field_op(pa::OP_FQ6_SQR, a, nullptr, out, nullptr, n, 288, 288, 0);
}
int pa_fq6_inverse_batch(const pa_fq6* a, pa_fq6* out, uint8_t* ok, size_t n) {
    if (n && !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null ok");
    return host_field_op(pa::OP_FQ6_INV, a, nullptr, out, ok, n, 288, 288, 0);
}
int pa_fq6_frobenius_map_batch(const pa_fq6* a, pa_fq6* out, size_t n, size_t power) {
    return host_field_op(pa::OP_FQ6_FROB, a, nullptr, out, nullptr, n, 288, 288, (int)(power % 6));
}
namespace {
int host_field_pow(int op, const void* a, const uint64_t* exp, size_t exp_words, void* out, size_t n,
                   size_t bytes) {
    if (n == 0) return PA_OK;
    if (!a || !out || (exp_words && !exp)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (exp_words > (1u << 20)) return fail(PA_ERR_INVALID_ARGUMENT, "exponent too long");
    DevBuf da, de, dout;
    int rc;
    if ((rc = upload(da, a, bytes * n)) || (rc = upload(de, exp, 8 * exp_words))) return rc;
    PA_TRY(dout.alloc(bytes * n), "device scratch");
    PA_TRY(pa::launch_field_op(op, da.as<uint64_t>(), de.as<uint64_t>(), dout.as<uint64_t>(), nullptr, n,
                               (int)exp_words, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, bytes * n);
}
}  // namespace
int pa_fq_pow_batch(const pa_fq* a, const uint64_t* exp, size_t exp_words, pa_fq* out, size_t n) {
    return host_field_pow(pa::OP_FQ_POW, a, exp, exp_words, out, n, 48);
}
int pa_fq12_pow_batch(const pa_fq12* a, const uint64_t* exp, size_t exp_words, pa_fq12* out, size_t n) {
    return host_field_pow(pa::OP_FQ12_POW, a, exp, exp_words, out, n, 576);
}
// not in the public header: cyclotomic squaring, exposed for the parity tests
int pa_fq12_cyclotomic_square_batch(const pa_fq12* a, pa_fq12* out, size_t n) {
    return host_field_op(pa::OP_FQ12_CYC_SQR, a, nullptr, out, nullptr, n, 576, 576, 0);
}

int pa_fq12_mul_by_014_batch(const pa_fq12* a, const pa_fq2* c0, const pa_fq2* c1, const pa_fq2* c4,
                             pa_fq12* out, size_t n) {
    if (n == 0) return PA_OK;
    if (!a || !c0 || !c1 || !c4 || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf da, d0, d1, d4, dout;
    int rc;
    if ((rc = upload(da, a, 576 * n)) || (rc = upload(d0, c0, 96 * n)) || (rc = upload(d1, c1, 96 * n)) ||
        (rc = upload(d4, c4, 96 * n)))
        return rc;
    PA_TRY(dout.alloc(576 * n), "device scratch");
    PA_TRY(pa::launch_fq12_mul_by_014(da.as<uint64_t>(), d0.as<uint64_t>(), d1.as<uint64_t>(), d4.as<uint64_t>(),
                                      dout.as<uint64_t>(), n, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, 576 * n);
}

int pa_g2_prepare_batch(const pa_g2_affine* q, pa_g2_prepared* out, size_t n) {
    if (n == 0) return PA_OK;
    if (!q || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dq, dout;
    int rc;
    if ((rc = upload(dq, q, sizeof(pa_g2_affine) * n))) return rc;
    PA_TRY(dout.alloc(sizeof(pa_g2_prepared) * n), "device scratch");
    PA_TRY(pa::launch_g2_prepare(dq.as<uint64_t>(), dout.as<uint64_t>(), n, call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, sizeof(pa_g2_prepared) * n);
}

int pa_miller_loop_batch(const pa_g1_affine* p, const pa_g2_prepared* q, pa_fq12* out, size_t n) {
    if (n == 0) return PA_OK;
    if (!p || !q || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dp, dq, dout;
    int rc;
    if ((rc = upload(dp, p, sizeof(pa_g1_affine) * n)) || (rc = upload(dq, q, sizeof(pa_g2_prepared) * n)))
        return rc;
    PA_TRY(dout.alloc(576 * n), "device scratch");
    PA_TRY(mlp_launch(dp.as<uint64_t>(), dq.as<uint64_t>(), dout.as<uint64_t>(), n, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, 576 * n);
}

int pa_miller_loop_shared_prepared(const pa_g1_affine* p, size_t n, const pa_g2_prepared* q, pa_fq12* out) {
    if (n == 0) return PA_OK;
    if (!p || !q || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dp, dq, dout;
    int rc;
    if ((rc = upload(dp, p, sizeof(pa_g1_affine) * n)) || (rc = upload(dq, q, sizeof(pa_g2_prepared))))
        return rc;
    PA_TRY(dout.alloc(576 * n), "device scratch");
    PA_TRY(pa::launch_miller_loop_shared_gen(dp.as<uint64_t>(), dq.as<uint64_t>(), dout.as<uint64_t>(), n,
                                             call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, 576 * n);
}

int pa_multi_miller_loop(const pa_g1_affine* p, const pa_g2_prepared* q, size_t n, pa_fq12* out) {
    if (!out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n == 0) {
        // empty product: Fq12::one() (mod.rs:71 with no pairs), conjugated = one
        memset(out, 0, sizeof(pa_fq12));
        const uint64_t r[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                               0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
        memcpy(out->c0.c0.c0.l, r, sizeof r);
        return PA_OK;
    }
    if (!p || !q) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dp, dq, dwork, dout;
    int rc;
    if ((rc = upload(dp, p, sizeof(pa_g1_affine) * n)) || (rc = upload(dq, q, sizeof(pa_g2_prepared) * n)))
        return rc;
    PA_TRY(dwork.alloc(576 * n), "device scratch");
    PA_TRY(dout.alloc(576), "device scratch");
    PA_TRY(mlp_launch(dp.as<uint64_t>(), dq.as<uint64_t>(), dwork.as<uint64_t>(), n, call_stream()),
           "kernel launch");
    PA_TRY(pa::launch_fq12_product(dwork.as<uint64_t>(), n, dout.as<uint64_t>(), call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, 576);
}

int pa_final_exponentiation_batch(const pa_fq12* in, pa_fq12* out, uint8_t* ok, size_t n) {
    if (n == 0) return PA_OK;
    if (!in || !out || !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf din, dout, dok;
    int rc;
    if ((rc = upload(din, in, 576 * n))) return rc;
    PA_TRY(dout.alloc(576 * n), "device scratch");
    PA_TRY(dok.alloc(n), "device scratch");
    PA_TRY(fe_launch(din.as<uint64_t>(), dout.as<uint64_t>(), dok.as<uint8_t>(), n, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    if ((rc = download(out, dout, 576 * n))) return rc;
    return download(ok, dok, n);
}

}  // extern "C"

namespace {

// Host copy into / out of pinned staging, split over up to 8 threads for
// large buffers (a single thread's memcpy would be slower than the DMA it
// feeds).
void pcopy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPiece = 2u << 20;
    unsigned t = std::thread::hardware_concurrency();
    t = t < 1 ? 1 : (t > 8 ? 8 : t);
    if (bytes / kPiece < t) t = (unsigned)(bytes / kPiece);
    if (t <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t per = (bytes + t - 1) / t;
    std::vector<std::thread> th;
    for (unsigned k = 1; k < t; k++) {
        const size_t lo = per * k, len = lo >= bytes ? 0 : (bytes - lo < per ? bytes - lo : per);
        if (len) th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, len); });
    }
    memcpy(dst, src, per < bytes ? per : bytes);
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

// Engine::pairing over host buffers, pipelined: the batch is cut into chunks
// of one device-filling wave count (one pairing per lane, one wave per SIMD:
// multiProcessorCount x 4 x 64 = 65 536 on MI355X); chunk k's inputs are
// staged into pinned memory and copied on the copy stream while chunk k-1
// computes on the compute stream, and chunk k-1's results travel back while
// chunk k computes.  Two pinned / device buffer sets alternate.
int pa_pairing_batch(const pa_g1_affine* p, const pa_g2_affine* q, pa_fq12* out, size_t n) {
    if (n == 0) return PA_OK;
    if (!p || !q || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    HostCtx* c = nullptr;
    PA_TRY(thread_ctx(&c), "device context");
    hipStream_t ks = nullptr;   // kernels: the device's shared pairing stream
    PA_TRY(pairing_stream(c->dev, &ks), "pairing stream");
    if (!c->full_batch) {
        int cus = 0;
        PA_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->dev), "device attribute");
        c->full_batch = (size_t)(cus > 0 ? cus : 1) * 4 * 64;
    }
    size_t chunk = c->full_batch;
    if (const char* e = getenv("PA_PIPELINE_CHUNK")) {   // tests: exercise the pipeline at small n
        const long v = strtol(e, nullptr, 10);
        if (v > 0) chunk = (size_t)v;
    }
    const size_t nchunks = (n + chunk - 1) / chunk;
    const size_t cap = n < chunk ? n : chunk;
    constexpr size_t P1 = sizeof(pa_g1_affine), P2 = sizeof(pa_g2_affine), F12 = sizeof(pa_fq12);
    const int bufs = nchunks > 1 ? 2 : 1;
    for (int k = 0; k < bufs; k++) {
        PA_TRY(grow(c->pinned[2 * k], cap * (P1 + P2), true), "pinned staging");
        PA_TRY(grow(c->pinned[2 * k + 1], cap * F12, true), "pinned staging");
        PA_TRY(grow(c->pipe[4 * k], cap * (P1 + P2), false), "device scratch");   // p | q
        PA_TRY(grow(c->pipe[4 * k + 1], cap * F12, false), "device scratch");     // Miller values
        PA_TRY(grow(c->pipe[4 * k + 2], cap * F12, false), "device scratch");     // e(p, q)
    }
    // PA_PIPELINE_TRACE=1: per-phase host timestamps on stderr (measurement only)
    static const bool trace = getenv("PA_PIPELINE_TRACE") && getenv("PA_PIPELINE_TRACE")[0] == '1';
    const auto t0 = std::chrono::steady_clock::now();
    auto stamp = [&](const char* what, size_t ci) {
        if (trace)
            fprintf(stderr, "[pipeline] chunk %zu %-10s %8.3f ms\n", ci, what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // Within a chunk the staging copies and the DMA run in kPieces pieces
    // (PA_PIPELINE_PIECES, 1..4, default 2), so the host copy of piece j
    // overlaps the DMA of piece j - 1 (in) / j + 1 (out): one caller at 2^16,
    // reused result buffer, 19.19 ms with 1 piece, 18.89 with 2, 18.84 with 4
    // (profiles/r03_host_boundary.txt).
    static const size_t kPieces = [] {
        const char* e = getenv("PA_PIPELINE_PIECES");
        const long v = e ? strtol(e, nullptr, 10) : 2;
        return (size_t)(v < 1 ? 1 : (v > 4 ? 4 : v));
    }();
    hipEvent_t* h2d = c->ev;        // [k]: chunk's inputs copied (pinned in[k] free again)
    hipEvent_t* done = c->ev + 2;   // [k]: chunk's kernels finished (device in[k], ml[k] free)
    hipEvent_t* d2h = c->ev + 4;    // [k * kPieces + j]: piece j of the chunk's results in pinned out[k]
    hipEvent_t* outk = c->ev + 12;  // [k]: every piece of the chunk's results copied (device out[k] free);
                                    // recorded after the piece loop, so an empty last piece cannot leave it stale
    auto piece = [&](size_t cnt, size_t j, size_t* lo) {
        const size_t per = (cnt + kPieces - 1) / kPieces;
        *lo = per * j < cnt ? per * j : cnt;
        return (per * (j + 1) < cnt ? per * (j + 1) : cnt) - *lo;
    };
    auto drain = [&](size_t ci) -> int {
        const int k = (int)(ci & 1);
        const size_t lo = ci * chunk, cnt = n - lo < chunk ? n - lo : chunk;
        for (size_t j = 0; j < kPieces; j++) {
            size_t a;
            const size_t m = piece(cnt, j, &a);
            if (!m) continue;
            PA_TRY(hipEventSynchronize(d2h[k * kPieces + j]), "D2H copy");
            pcopy(out + lo + a, (pa_fq12*)c->pinned[2 * k + 1].first + a, m * F12);
        }
        stamp("copied out", ci);
        return PA_OK;
    };
    for (size_t ci = 0; ci < nchunks; ci++) {
        const int k = (int)(ci & 1);
        const size_t lo = ci * chunk, cnt = n - lo < chunk ? n - lo : chunk;
        char* pin_p = (char*)c->pinned[2 * k].first;
        char* pin_q = pin_p + cnt * P1;
        char* dev_p = (char*)c->pipe[4 * k].first;
        char* dev_q = dev_p + cnt * P1;
        uint64_t* dev_ml = (uint64_t*)c->pipe[4 * k + 1].first;
        uint64_t* dev_out = (uint64_t*)c->pipe[4 * k + 2].first;
        if (ci >= 2) {
            PA_TRY(hipEventSynchronize(h2d[k]), "H2D copy");
            PA_TRY(hipStreamWaitEvent(c->copy, done[k], 0), "stream wait");
        }
        for (size_t j = 0; j < kPieces; j++) {
            size_t a;
            const size_t m = piece(cnt, j, &a);
            if (!m) continue;
            pcopy(pin_p + a * P1, p + lo + a, m * P1);
            pcopy(pin_q + a * P2, q + lo + a, m * P2);
            PA_TRY(hipMemcpyAsync(dev_p + a * P1, pin_p + a * P1, m * P1, hipMemcpyHostToDevice, c->copy), "H2D copy");
            PA_TRY(hipMemcpyAsync(dev_q + a * P2, pin_q + a * P2, m * P2, hipMemcpyHostToDevice, c->copy), "H2D copy");
        }
        PA_TRY(hipEventRecord(h2d[k], c->copy), "event");
        stamp("staged in", ci);
        PA_TRY(hipStreamWaitEvent(ks, h2d[k], 0), "stream wait");
        if (ci >= 2) PA_TRY(hipStreamWaitEvent(ks, outk[k], 0), "stream wait");
        PA_TRY(pairing_ml_launch((const uint64_t*)dev_p, (const uint64_t*)dev_q, dev_ml, cnt, ks), "kernel launch");
        // Engine::pairing unwraps: a Miller-loop value is never zero, ok is not reported
        PA_TRY(fe_launch(dev_ml, dev_out, nullptr, cnt, ks), "kernel launch");
        PA_TRY(hipEventRecord(done[k], ks), "event");
        PA_TRY(hipStreamWaitEvent(c->copy_out, done[k], 0), "stream wait");
        for (size_t j = 0; j < kPieces; j++) {
            size_t a;
            const size_t m = piece(cnt, j, &a);
            if (!m) continue;
            PA_TRY(hipMemcpyAsync((pa_fq12*)c->pinned[2 * k + 1].first + a, (const pa_fq12*)dev_out + a, m * F12,
                                  hipMemcpyDeviceToHost, c->copy_out),
                   "D2H copy");
            PA_TRY(hipEventRecord(d2h[k * kPieces + j], c->copy_out), "event");
        }
        PA_TRY(hipEventRecord(outk[k], c->copy_out), "event");
        stamp("enqueued", ci);
        if (ci >= 1) {
            const int rc = drain(ci - 1);
            if (rc) return rc;
        }
    }
    const int rc = drain(nchunks - 1);
    if (rc) return rc;
    return PA_OK;   // the last chunk's D2H event has completed: so has everything before it
}

int pa_pairing_batch_multi_gpu(const pa_g1_affine* p, const pa_g2_affine* q, pa_fq12* out, size_t n, int ndev) {
    int count = 0;
    PA_TRY(hipGetDeviceCount(&count), "hipGetDeviceCount");
    // shard d runs on device d, or on the d-th entry of PA_DEVICE_MAP (a comma
    // list of device ordinals, e.g. "2,3,6,7" to use a subset of the node, or
    // "0,0" to run two shards' workers on one device)
    std::vector<int> dev_of;
    if (const char* m = getenv("PA_DEVICE_MAP")) {
        for (const char* c = m; *c;) {
            char* end = nullptr;
            const long v = strtol(c, &end, 10);
            if (end == c || v < 0 || v >= count) return fail(PA_ERR_INVALID_ARGUMENT, "bad PA_DEVICE_MAP");
            dev_of.push_back((int)v);
            c = *end == ',' ? end + 1 : end;
            if (*end && *end != ',') return fail(PA_ERR_INVALID_ARGUMENT, "bad PA_DEVICE_MAP");
        }
    } else {
        for (int d = 0; d < count; d++) dev_of.push_back(d);
    }
    if (ndev < 1 || ndev > (int)dev_of.size()) return fail(PA_ERR_INVALID_ARGUMENT, "ndev out of range");
    if (n == 0) return PA_OK;
    if (!p || !q || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    // contiguous shards (SURVEY.md §8 e); each worker thread owns one device
    std::vector<int> rcs(ndev, PA_OK);
    std::vector<std::string> errs(ndev);
    std::vector<std::thread> workers;
    const size_t base = n / ndev, extra = n % ndev;
    size_t lo = 0;
    for (int d = 0; d < ndev; d++) {
        const size_t cnt = base + ((size_t)d < extra ? 1 : 0);
        const int dv = dev_of[d];
        workers.emplace_back([=, &rcs, &errs] {
            hipError_t e = hipSetDevice(dv);
            if (e != hipSuccess) {
                rcs[d] = fail(hip_code(e), "hipSetDevice", e);
            } else {
                rcs[d] = pa_pairing_batch(p + lo, q + lo, out + lo, cnt);
            }
            if (rcs[d] != PA_OK) errs[d] = g_last_error;
        });
        lo += cnt;
    }
    for (auto& t : workers) t.join();
    for (int d = 0; d < ndev; d++)
        if (rcs[d] != PA_OK) {
            g_last_error = "device " + std::to_string(d) + ": " + errs[d];
            return rcs[d];
        }
    return PA_OK;
}

int pa_multi_miller_loop_affine(const pa_g1_affine* p, const pa_g2_affine* q, size_t n, pa_fq12* out) {
    if (!out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n == 0) return pa_multi_miller_loop(nullptr, nullptr, 0, out);
    if (!p || !q) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dp, dq, dwork, dout;
    int rc;
    if ((rc = upload(dp, p, sizeof(pa_g1_affine) * n)) || (rc = upload(dq, q, sizeof(pa_g2_affine) * n)))
        return rc;
    PA_TRY(dwork.alloc(576 * n), "device scratch");
    PA_TRY(dout.alloc(576), "device scratch");
    // per-pair loops (infinity pairs give one, as mod.rs:50-54 skips them), then the product tree
    PA_TRY(ml_launch(dp.as<uint64_t>(), dq.as<uint64_t>(), dwork.as<uint64_t>(), n, call_stream()), "kernel launch");
    PA_TRY(pa::launch_fq12_product(dwork.as<uint64_t>(), n, dout.as<uint64_t>(), call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, 576);
}

int pa_multi_pairing_device(const pa_g1_affine* p, const pa_g2_affine* q, size_t n, pa_fq12* out, uint8_t* ok,
                            pa_fq12* work, void* stream) {
    if (!out || !ok || (n && (!p || !q || !work))) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const hipStream_t s = (hipStream_t)stream;
    if (n == 0) {   // empty product: one, final_exponentiation(one) = one
        pa_fq12 one;
        memset(&one, 0, sizeof one);
        const uint64_t r[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                               0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
        memcpy(one.c0.c0.c0.l, r, sizeof r);
        const uint8_t k = 1;
        PA_TRY(hipMemcpyAsync(out, &one, sizeof one, hipMemcpyHostToDevice, s), "H2D copy");
        PA_TRY(hipMemcpyAsync(ok, &k, 1, hipMemcpyHostToDevice, s), "H2D copy");
        PA_TRY(hipStreamSynchronize(s), "H2D copy");   // the host sources go out of scope
        return PA_OK;
    }
    PA_TRY(pairing_ml_launch((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)work, n, s), "kernel launch");
    if (n <= kCoopProductMax && use_coop(1)) {
        // the product of a few Miller values inside the cooperative final
        // exponentiation (mul12 macros, ~6 us each) instead of the one-lane
        // product-tree kernel (~117 us per level)
        PA_TRY(pa::launch_coop_final_exp((const uint64_t*)work, (uint64_t*)out, ok, 1, s, coop_vm(), n),
               "kernel launch");
        return PA_OK;
    }
    PA_TRY(pa::launch_fq12_product((uint64_t*)work, n, (uint64_t*)work, s), "kernel launch");
    PA_TRY(fe_launch((const uint64_t*)work, (uint64_t*)out, ok, 1, s), "kernel launch");
    return PA_OK;
}

int pa_multi_pairing(const pa_g1_affine* p, const pa_g2_affine* q, size_t n, pa_fq12* out, uint8_t* ok) {
    if (!out || !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n && (!p || !q)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n == 0) {   // the empty product: final_exponentiation(one) = one
        pa_fq12 ml;
        int rc = pa_multi_miller_loop_affine(p, q, 0, &ml);
        if (rc) return rc;
        return pa_final_exponentiation_batch(&ml, out, ok, 1);
    }
    // one stream round trip: the pairs up, the device entry (Miller loops,
    // product, final exponentiation), the result down
    DevBuf dp, dq, dwork, dout, dok;
    int rc;
    if ((rc = upload(dp, p, sizeof(pa_g1_affine) * n)) || (rc = upload(dq, q, sizeof(pa_g2_affine) * n)))
        return rc;
    PA_TRY(dwork.alloc(576 * n), "device scratch");
    PA_TRY(dout.alloc(576), "device scratch");
    PA_TRY(dok.alloc(1), "device scratch");
    if ((rc = pa_multi_pairing_device(dp.as<pa_g1_affine>(), dq.as<pa_g2_affine>(), n, dout.as<pa_fq12>(),
                                      dok.as<uint8_t>(), dwork.as<pa_fq12>(), call_stream())))
        return rc;
    if ((rc = download(out, dout, 576))) return rc;
    return download(ok, dok, 1);
}

// ---- point encodings ----
namespace {
constexpr size_t enc_size(int group, int compressed) { return (group == 1 ? 48 : 96) * (compressed ? 1 : 2); }
int host_decode(int group, const uint8_t* enc, size_t n, int compressed, int checked, void* out, uint8_t* status) {
    if (n == 0) return PA_OK;
    if (!enc || !out || !status) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t rec = group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine);
    DevBuf de, dout, dst;
    int rc;
    if ((rc = upload(de, enc, enc_size(group, compressed) * n))) return rc;
    PA_TRY(dout.alloc(rec * n), "device scratch");
    PA_TRY(dst.alloc(n), "device scratch");
    PA_TRY(pa::launch_decode(group, compressed, checked, de.as<uint8_t>(), n, dout.as<uint64_t>(),
                             dst.as<uint8_t>(), call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    if ((rc = download(out, dout, rec * n))) return rc;
    return download(status, dst, n);
}
int host_subgroup(int group, const void* pts, size_t n, uint8_t* ok) {
    if (n == 0) return PA_OK;
    if (!pts || !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t rec = group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine);
    DevBuf dp, dok;
    int rc;
    if ((rc = upload(dp, pts, rec * n))) return rc;
    PA_TRY(dok.alloc(n), "device scratch");
    PA_TRY(pa::launch_subgroup_check(group, dp.as<uint64_t>(), n, dok.as<uint8_t>(), call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(ok, dok, n);
}
int host_encode(int group, const void* in, size_t n, int compressed, uint8_t* enc) {
    if (n == 0) return PA_OK;
    if (!in || !enc) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t rec = group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine);
    DevBuf din, de;
    int rc;
    if ((rc = upload(din, in, rec * n))) return rc;
    PA_TRY(de.alloc(enc_size(group, compressed) * n), "device scratch");
    PA_TRY(pa::launch_encode(group, compressed, din.as<uint64_t>(), n, de.as<uint8_t>(), call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(enc, de, enc_size(group, compressed) * n);
}
int host_sqrt(int degree, const void* a, void* out, uint8_t* ok, size_t n) {
    if (n == 0) return PA_OK;
    if (!a || !out || !ok) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t bytes = 48 * (size_t)degree * n;
    DevBuf da, dout, dok;
    int rc;
    if ((rc = upload(da, a, bytes))) return rc;
    PA_TRY(dout.alloc(bytes), "device scratch");
    PA_TRY(dok.alloc(n), "device scratch");
    PA_TRY(pa::launch_sqrt(degree, da.as<uint64_t>(), n, dout.as<uint64_t>(), dok.as<uint8_t>(), call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    if ((rc = download(out, dout, bytes))) return rc;
    return download(ok, dok, n);
}
}  // namespace

int pa_g1_decode_batch(const uint8_t* enc, size_t n, int compressed, int checked, pa_g1_affine* out,
                       uint8_t* status) {
    return host_decode(1, enc, n, compressed != 0, checked != 0, out, status);
}
int pa_g2_decode_batch(const uint8_t* enc, size_t n, int compressed, int checked, pa_g2_affine* out,
                       uint8_t* status) {
    return host_decode(2, enc, n, compressed != 0, checked != 0, out, status);
}
int pa_g1_subgroup_check_batch(const pa_g1_affine* p, size_t n, uint8_t* ok) { return host_subgroup(1, p, n, ok); }
int pa_g2_subgroup_check_batch(const pa_g2_affine* p, size_t n, uint8_t* ok) { return host_subgroup(2, p, n, ok); }
int pa_g1_encode_batch(const pa_g1_affine* in, size_t n, int compressed, uint8_t* enc) {
    return host_encode(1, in, n, compressed != 0, enc);
}
int pa_g2_encode_batch(const pa_g2_affine* in, size_t n, int compressed, uint8_t* enc) {
    return host_encode(2, in, n, compressed != 0, enc);
}
int pa_fq_sqrt_batch(const pa_fq* a, pa_fq* out, uint8_t* ok, size_t n) { return host_sqrt(1, a, out, ok, n); }
int pa_fq2_sqrt_batch(const pa_fq2* a, pa_fq2* out, uint8_t* ok, size_t n) { return host_sqrt(2, a, out, ok, n); }

int pa_g1_batch_normalization(pa_g1* v, size_t n) {
    if (n == 0) return PA_OK;
    if (!v) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dv;
    int rc;
    if ((rc = upload(dv, v, sizeof(pa_g1) * n))) return rc;
    PA_TRY(pa::launch_g1_batch_normalize(dv.as<uint64_t>(), n, call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(v, dv, sizeof(pa_g1) * n);
}

int pa_g1_wnaf_fixed_base(const pa_g1* base, const pa_fr_repr* scalars, size_t n, pa_g1* out) {
    return pa_g1_wnaf_fixed_base_window(base, scalars, n, pa_g1_recommended_wnaf_for_num_scalars(n), out);
}
int pa_g1_wnaf_fixed_base_window(const pa_g1* base, const pa_fr_repr* scalars, size_t n, int window, pa_g1* out) {
    if (n == 0) return PA_OK;
    if (!base || !scalars || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (window < 1 || window > kMaxWnafWindow) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range");
    DevBuf db, ds, dt, dw, dout;
    int rc;
    if ((rc = upload(db, base, sizeof(pa_g1))) || (rc = upload(ds, scalars, sizeof(pa_fr_repr) * n))) return rc;
    PA_TRY(dt.alloc(8 * pa::g1_comb_table_words()), "device scratch");
    PA_TRY(dw.alloc(8 * pa::g1_comb_workspace_words()), "device scratch");
    PA_TRY(dout.alloc(sizeof(pa_g1) * n), "device scratch");
    PA_TRY(pa::launch_g1_fixed_base(db.as<uint64_t>(), ds.as<uint64_t>(), dout.as<uint64_t>(), n, dt.as<uint64_t>(),
                                    dw.as<uint64_t>(), window, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, sizeof(pa_g1) * n);
}

// ---- bit-exact Wnaf (kernels_wnaf_exact.hip) ----
namespace {
// window 0 -> the reference's recommendation; else checked against the limit
int wx_window(int window, int dflt, int max) { return window == 0 ? dflt : (window < 1 || window > max ? -1 : window); }

int wx_host(int group, bool fixed_scalar, const void* base_or_bases, size_t n, const pa_fr_repr* s, size_t ns,
            int window, void* out) {
    if (n == 0) return PA_OK;
    const size_t jb = group == 1 ? sizeof(pa_g1) : sizeof(pa_g2);
    DevBuf db, ds, dw, dout;
    int rc;
    if ((rc = upload(db, base_or_bases, jb * (fixed_scalar ? n : 1))) ||
        (rc = upload(ds, s, sizeof(pa_fr_repr) * ns)))
        return rc;
    const size_t bytes = fixed_scalar ? pa::wx_scalar_layout(group, n, window).bytes
                                      : pa::wx_layout(group, n, window).bytes;
    PA_TRY(dw.alloc(bytes), "device scratch");
    PA_TRY(dout.alloc(jb * n), "device scratch");
    if (fixed_scalar)
        PA_TRY(pa::launch_wnaf_exact_fixed_scalar(group, db.as<uint64_t>(), n, ds.as<uint64_t>(), dout.as<uint64_t>(),
                                                  window, dw.p, call_stream()),
               "kernel launch");
    else
        PA_TRY(pa::launch_wnaf_exact_fixed_base(group, db.as<uint64_t>(), ds.as<uint64_t>(), dout.as<uint64_t>(), n,
                                                window, dw.p, call_stream()),
               "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, jb * n);
}
int wx_device(int group, bool fixed_scalar, const void* base_or_bases, size_t n, const pa_fr_repr* s, int window,
              void* out, void* workspace, size_t workspace_bytes, void* stream) {
    if (n == 0) return PA_OK;
    if (!base_or_bases || !s || !out || !workspace) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t need = fixed_scalar ? pa::wx_scalar_layout(group, n, window).bytes
                                     : pa::wx_layout(group, n, window).bytes;
    if (workspace_bytes < need) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf exact workspace too small");
    if (fixed_scalar)
        PA_TRY(pa::launch_wnaf_exact_fixed_scalar(group, (const uint64_t*)base_or_bases, n, (const uint64_t*)s,
                                                  (uint64_t*)out, window, workspace, (hipStream_t)stream),
               "kernel launch");
    else
        PA_TRY(pa::launch_wnaf_exact_fixed_base(group, (const uint64_t*)base_or_bases, (const uint64_t*)s,
                                                (uint64_t*)out, n, window, workspace, (hipStream_t)stream),
               "kernel launch");
    return PA_OK;
}
}  // namespace

int pa_g1_wnaf_fixed_base_exact(const pa_g1* base, const pa_fr_repr* scalars, size_t n, int window, pa_g1* out) {
    if (n && (!base || !scalars || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int w = wx_window(window, pa_g1_recommended_wnaf_for_num_scalars(n), pa::kWxMaxWindow);
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact: 1..20)");
    return wx_host(1, false, base, n, scalars, n, w, out);
}
int pa_g2_wnaf_fixed_base_exact(const pa_g2* base, const pa_fr_repr* scalars, size_t n, int window, pa_g2* out) {
    if (n && (!base || !scalars || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int w = wx_window(window, pa_g2_recommended_wnaf_for_num_scalars(n), pa::kWxMaxWindow);
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact: 1..20)");
    return wx_host(2, false, base, n, scalars, n, w, out);
}
int pa_g1_wnaf_fixed_scalar_exact(const pa_g1* bases, size_t n, const pa_fr_repr* scalar, int window, pa_g1* out) {
    if (n && (!bases || !scalar || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int w = n ? wx_window(window, pa_g1_recommended_wnaf_for_scalar(scalar), pa::kWxMaxScalarWindow) : 1;
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact fixed scalar: 1..12)");
    return wx_host(1, true, bases, n, scalar, 1, w, out);
}
int pa_g2_wnaf_fixed_scalar_exact(const pa_g2* bases, size_t n, const pa_fr_repr* scalar, int window, pa_g2* out) {
    if (n && (!bases || !scalar || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int w = n ? wx_window(window, pa_g2_recommended_wnaf_for_scalar(scalar), pa::kWxMaxScalarWindow) : 1;
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact fixed scalar: 1..12)");
    return wx_host(2, true, bases, n, scalar, 1, w, out);
}
size_t pa_wnaf_exact_workspace_bytes(int group, size_t n, int window, int fixed_scalar) {
    const int max = fixed_scalar ? pa::kWxMaxScalarWindow : pa::kWxMaxWindow;
    if ((group != 1 && group != 2) || window < 1 || window > max) return 0;
    return fixed_scalar ? pa::wx_scalar_layout(group, n, window).bytes : pa::wx_layout(group, n, window).bytes;
}
int pa_g1_wnaf_fixed_base_exact_device(const pa_g1* base, const pa_fr_repr* scalars, pa_g1* out, size_t n,
                                       int window, void* workspace, size_t workspace_bytes, void* stream) {
    const int w = wx_window(window, pa_g1_recommended_wnaf_for_num_scalars(n), pa::kWxMaxWindow);
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact: 1..20)");
    return wx_device(1, false, base, n, scalars, w, out, workspace, workspace_bytes, stream);
}
int pa_g2_wnaf_fixed_base_exact_device(const pa_g2* base, const pa_fr_repr* scalars, pa_g2* out, size_t n,
                                       int window, void* workspace, size_t workspace_bytes, void* stream) {
    const int w = wx_window(window, pa_g2_recommended_wnaf_for_num_scalars(n), pa::kWxMaxWindow);
    if (w < 0) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact: 1..20)");
    return wx_device(2, false, base, n, scalars, w, out, workspace, workspace_bytes, stream);
}
// the scalar is device memory here: the window must be given (1..12)
int pa_g1_wnaf_fixed_scalar_exact_device(const pa_g1* bases, size_t n, const pa_fr_repr* scalar, pa_g1* out,
                                         int window, void* workspace, size_t workspace_bytes, void* stream) {
    if (window < 1 || window > pa::kWxMaxScalarWindow)
        return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact fixed scalar, device: 1..12)");
    return wx_device(1, true, bases, n, scalar, window, out, workspace, workspace_bytes, stream);
}
int pa_g2_wnaf_fixed_scalar_exact_device(const pa_g2* bases, size_t n, const pa_fr_repr* scalar, pa_g2* out,
                                         int window, void* workspace, size_t workspace_bytes, void* stream) {
    if (window < 1 || window > pa::kWxMaxScalarWindow)
        return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range (exact fixed scalar, device: 1..12)");
    return wx_device(2, true, bases, n, scalar, window, out, workspace, workspace_bytes, stream);
}

// ---- device-resident variants ----
int pa_g1_subgroup_check_batch_device(const pa_g1_affine* p, size_t n, uint8_t* ok, void* stream) {
    if (n && (!p || !ok)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_subgroup_check(1, (const uint64_t*)p, n, ok, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_g2_subgroup_check_batch_device(const pa_g2_affine* p, size_t n, uint8_t* ok, void* stream) {
    if (n && (!p || !ok)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_subgroup_check(2, (const uint64_t*)p, n, ok, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_g1_decode_batch_device(const uint8_t* enc, size_t n, int compressed, int checked, pa_g1_affine* out,
                              uint8_t* status, void* stream) {
    if (n && (!enc || !out || !status)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_decode(1, compressed != 0, checked != 0, enc, n, (uint64_t*)out, status, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g2_decode_batch_device(const uint8_t* enc, size_t n, int compressed, int checked, pa_g2_affine* out,
                              uint8_t* status, void* stream) {
    if (n && (!enc || !out || !status)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_decode(2, compressed != 0, checked != 0, enc, n, (uint64_t*)out, status, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g1_batch_normalization_device(pa_g1* v, size_t n, void* stream) {
    if (n && !v) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g1_batch_normalize((uint64_t*)v, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
size_t pa_g1_fixed_base_table_words(void) { return pa::g1_comb_table_words(); }
size_t pa_g1_fixed_base_workspace_words(void) { return pa::g1_comb_workspace_words(); }
int pa_g1_fixed_base_table_device(const pa_g1* base, uint64_t* table, uint64_t* workspace, void* stream) {
    if (!base || !table || !workspace) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g1_comb_table((const uint64_t*)base, table, workspace, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_g1_fixed_base_mul_device(const uint64_t* table, const pa_fr_repr* scalars, pa_g1* out, size_t n,
                                void* stream) {
    if (n && (!table || !scalars || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g1_comb_mul(table, (const uint64_t*)scalars, (uint64_t*)out, n,
                                  pa_g1_recommended_wnaf_for_num_scalars(n), (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g1_fixed_base_glv_table_device(const pa_g1* base, uint64_t* table, uint64_t* workspace, void* stream) {
    if (!base || !table || !workspace) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g1_glv_table((const uint64_t*)base, table, workspace, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_g1_fixed_base_glv_mul_device(const pa_g1* base, const uint64_t* table, const uint64_t* workspace,
                                    const pa_fr_repr* scalars, pa_g1* out, size_t n, void* stream) {
    if (n && (!base || !table || !workspace || !scalars || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g1_glv_mul((const uint64_t*)base, table, workspace,
                                 (const uint64_t*)scalars, (uint64_t*)out, n, pa_g1_recommended_wnaf_for_num_scalars(n),
                                 (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g1_wnaf_fixed_base_device(const pa_g1* base, const pa_fr_repr* scalars, pa_g1* out, size_t n,
                                 uint64_t* table, uint64_t* workspace, void* stream) {
    return pa_g1_wnaf_fixed_base_window_device(base, scalars, out, n, pa_g1_recommended_wnaf_for_num_scalars(n), table,
                                               workspace, stream);
}
int pa_g1_wnaf_fixed_base_window_device(const pa_g1* base, const pa_fr_repr* scalars, pa_g1* out, size_t n,
                                        int window, uint64_t* table, uint64_t* workspace, void* stream) {
    if (n && (!base || !scalars || !out || !table || !workspace)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (window < 1 || window > kMaxWnafWindow) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range");
    PA_TRY(pa::launch_g1_fixed_base((const uint64_t*)base, (const uint64_t*)scalars, (uint64_t*)out, n, table,
                                    workspace, window, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_fq_mul_batch_device(const pa_fq* a, const pa_fq* b, pa_fq* out, size_t n, void* stream) {
    if (n && (!a || !b || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_fq_mul_batch((const uint64_t*)a, (const uint64_t*)b, (uint64_t*)out, n, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_fq_mul_batch_soa_device(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, void* stream) {
    if (n && (!a || !b || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_fq_mul_batch_soa(a, b, out, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_miller_loop_fused_batch_device(const pa_g1_affine* p, const pa_g2_affine* q, pa_fq12* out, size_t n,
                                      void* stream) {
    if (n && (!p || !q || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(ml_launch((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)out, n, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_pairing_miller_loop_batch_device(const pa_g1_affine* p, const pa_g2_affine* q, pa_fq12* out, size_t n,
                                        void* stream) {
    if (n && (!p || !q || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pairing_ml_launch((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)out, n, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_final_exponentiation_batch_device(const pa_fq12* in, pa_fq12* out, uint8_t* ok, size_t n, void* stream) {
    if (n && (!in || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(fe_launch((const uint64_t*)in, (uint64_t*)out, ok, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_g2_prepare_batch_device(const pa_g2_affine* q, pa_g2_prepared* out, size_t n, void* stream) {
    if (n && (!q || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g2_prepare((const uint64_t*)q, (uint64_t*)out, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
int pa_miller_loop_batch_device(const pa_g1_affine* p, const pa_g2_prepared* q, pa_fq12* out, size_t n,
                                void* stream) {
    if (n && (!p || !q || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(mlp_launch((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)out, n,
                                           (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_miller_loop_shared_prepared_device(const pa_g1_affine* p, size_t n, const pa_g2_prepared* q, pa_fq12* out,
                                          void* stream) {
    if (n && (!p || !q || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_miller_loop_shared_gen((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)out, n,
                                             (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_pairing_batch_device(const pa_g1_affine* p, const pa_g2_affine* q, pa_fq12* out, pa_fq12* scratch,
                            size_t n, void* stream) {
    if (n && (!p || !q || !out || !scratch)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pairing_ml_launch((const uint64_t*)p, (const uint64_t*)q, (uint64_t*)scratch, n, (hipStream_t)stream),
           "kernel launch");
    PA_TRY(fe_launch((const uint64_t*)scratch, (uint64_t*)out, nullptr, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}

// ---- scalar field Fr (fr.rs) ----
namespace {
bool fr_op_needs_b(int op) { return op == pa::FR_MUL || op == pa::FR_ADD || op == pa::FR_SUB; }
int host_fr_op(int op, const void* a, const void* b, void* out, uint8_t* flag, const uint64_t* exp, size_t exp_words,
               size_t n) {
    if (n == 0) return PA_OK;
    const bool has_out = op != pa::FR_LEGENDRE;
    const bool has_flag = op == pa::FR_INV || op == pa::FR_FROM_REPR || op == pa::FR_SQRT || op == pa::FR_LEGENDRE;
    if (!a || (has_out && !out) || (fr_op_needs_b(op) && !b) || (has_flag && !flag) ||
        (op == pa::FR_POW && exp_words && !exp))
        return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (exp_words > (1u << 20)) return fail(PA_ERR_INVALID_ARGUMENT, "exponent too long");
    DevBuf da, db, dout, dflag, dexp;
    int rc;
    const size_t bytes = 32 * n;
    if ((rc = upload(da, a, bytes))) return rc;
    if (fr_op_needs_b(op) && (rc = upload(db, b, bytes))) return rc;
    if (op == pa::FR_POW && (rc = upload(dexp, exp, 8 * exp_words))) return rc;
    PA_TRY(dout.alloc(bytes), "device scratch");
    if (has_flag) PA_TRY(dflag.alloc(n), "device scratch");
    PA_TRY(pa::launch_fr_op(op, da.as<uint64_t>(), db.as<uint64_t>(), dout.as<uint64_t>(), dflag.as<uint8_t>(),
                            dexp.as<uint64_t>(), (int)exp_words, n, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    if (has_out && (rc = download(out, dout, bytes))) return rc;
    if (has_flag && (rc = download(flag, dflag, n))) return rc;
    return PA_OK;
}
}  // namespace

int pa_fr_mul_batch(const pa_fr* a, const pa_fr* b, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_MUL, a, b, out, nullptr, nullptr, 0, n);
}
int pa_fr_square_batch(const pa_fr* a, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_SQR, a, nullptr, out, nullptr, nullptr, 0, n);
}
int pa_fr_add_batch(const pa_fr* a, const pa_fr* b, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_ADD, a, b, out, nullptr, nullptr, 0, n);
}
int pa_fr_sub_batch(const pa_fr* a, const pa_fr* b, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_SUB, a, b, out, nullptr, nullptr, 0, n);
}
int pa_fr_double_batch(const pa_fr* a, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_DBL, a, nullptr, out, nullptr, nullptr, 0, n);
}
int pa_fr_negate_batch(const pa_fr* a, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_NEG, a, nullptr, out, nullptr, nullptr, 0, n);
}
int pa_fr_inverse_batch(const pa_fr* a, pa_fr* out, uint8_t* ok, size_t n) {
    return host_fr_op(pa::FR_INV, a, nullptr, out, ok, nullptr, 0, n);
}
int pa_fr_from_repr_batch(const pa_fr_repr* repr, pa_fr* out, uint8_t* ok, size_t n) {
    return host_fr_op(pa::FR_FROM_REPR, repr, nullptr, out, ok, nullptr, 0, n);
}
int pa_fr_into_repr_batch(const pa_fr* a, pa_fr_repr* out, size_t n) {
    return host_fr_op(pa::FR_INTO_REPR, a, nullptr, out, nullptr, nullptr, 0, n);
}
int pa_fr_pow_batch(const pa_fr* a, const uint64_t* exp, size_t exp_words, pa_fr* out, size_t n) {
    return host_fr_op(pa::FR_POW, a, nullptr, out, nullptr, exp, exp_words, n);
}
int pa_fr_legendre_batch(const pa_fr* a, int8_t* out, size_t n) {
    return host_fr_op(pa::FR_LEGENDRE, a, nullptr, nullptr, (uint8_t*)out, nullptr, 0, n);
}
int pa_fr_sqrt_batch(const pa_fr* a, pa_fr* out, uint8_t* ok, size_t n) {
    return host_fr_op(pa::FR_SQRT, a, nullptr, out, ok, nullptr, 0, n);
}
int pa_fr_mul_batch_device(const pa_fr* a, const pa_fr* b, pa_fr* out, size_t n, void* stream) {
    if (n && (!a || !b || !out)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_fr_mul_batch((const uint64_t*)a, (const uint64_t*)b, (uint64_t*)out, n, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}

// ---- variable-base scalar multiplication and MSM (kernels_msm.hip) ----
namespace {
int host_scalar_mul(int group, int projective, const void* p, const pa_fr_repr* s, void* out, size_t n) {
    if (n == 0) return PA_OK;
    if (!p || !s || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t in_rec = projective ? (group == 1 ? sizeof(pa_g1) : sizeof(pa_g2))
                                     : (group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine));
    const size_t out_rec = group == 1 ? sizeof(pa_g1) : sizeof(pa_g2);
    DevBuf dp, ds, dout;
    int rc;
    if ((rc = upload(dp, p, in_rec * n)) || (rc = upload(ds, s, sizeof(pa_fr_repr) * n))) return rc;
    PA_TRY(dout.alloc(out_rec * n), "device scratch");
    PA_TRY(pa::launch_scalar_mul(group, projective, dp.as<uint64_t>(), ds.as<uint64_t>(), n, dout.as<uint64_t>(),
                                 call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, out_rec * n);
}
int host_multiexp(int group, const void* bases, const pa_fr_repr* s, size_t n, void* out) {
    if (!out || (n && (!bases || !s))) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n >= 0x80000000ull) return fail(PA_ERR_INVALID_ARGUMENT, "multiexp supports n < 2^31");
    const size_t in_rec = group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine);
    const size_t out_rec = group == 1 ? sizeof(pa_g1) : sizeof(pa_g2);
    DevBuf db, ds, dout, dws;
    int rc;
    if ((rc = upload(db, bases, in_rec * n)) || (rc = upload(ds, s, sizeof(pa_fr_repr) * n))) return rc;
    PA_TRY(dout.alloc(out_rec), "device scratch");
    const size_t ws = pa::msm_workspace_bytes(group, n);
    PA_TRY(dws.alloc(ws), "device scratch");
    PA_TRY(pa::launch_msm(group, db.as<uint64_t>(), ds.as<uint64_t>(), n, dout.as<uint64_t>(), dws.p, ws, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, out_rec);
}
}  // namespace

int pa_g1_affine_mul_batch(const pa_g1_affine* p, const pa_fr_repr* s, pa_g1* out, size_t n) {
    return host_scalar_mul(1, 0, p, s, out, n);
}
int pa_g2_affine_mul_batch(const pa_g2_affine* p, const pa_fr_repr* s, pa_g2* out, size_t n) {
    return host_scalar_mul(2, 0, p, s, out, n);
}
int pa_g1_mul_assign_batch(const pa_g1* p, const pa_fr_repr* s, pa_g1* out, size_t n) {
    return host_scalar_mul(1, 1, p, s, out, n);
}
int pa_g2_mul_assign_batch(const pa_g2* p, const pa_fr_repr* s, pa_g2* out, size_t n) {
    return host_scalar_mul(2, 1, p, s, out, n);
}
int pa_g1_multiexp(const pa_g1_affine* bases, const pa_fr_repr* scalars, size_t n, pa_g1* out) {
    return host_multiexp(1, bases, scalars, n, out);
}
int pa_g2_multiexp(const pa_g2_affine* bases, const pa_fr_repr* scalars, size_t n, pa_g2* out) {
    return host_multiexp(2, bases, scalars, n, out);
}
size_t pa_multiexp_workspace_bytes(int group, size_t n) {
    return (group == 1 || group == 2) ? pa::msm_workspace_bytes(group, n) : 0;
}
int pa_g1_multiexp_device(const pa_g1_affine* bases, const pa_fr_repr* scalars, size_t n, pa_g1* out,
                          void* workspace, size_t workspace_bytes, void* stream) {
    if (!out || (n && (!bases || !scalars || !workspace))) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n && workspace_bytes < pa::msm_workspace_bytes(1, n))
        return fail(PA_ERR_INVALID_ARGUMENT, "workspace smaller than pa_multiexp_workspace_bytes");
    PA_TRY(pa::launch_msm(1, (const uint64_t*)bases, (const uint64_t*)scalars, n, (uint64_t*)out, workspace,
                          workspace_bytes, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g2_multiexp_device(const pa_g2_affine* bases, const pa_fr_repr* scalars, size_t n, pa_g2* out,
                          void* workspace, size_t workspace_bytes, void* stream) {
    if (!out || (n && (!bases || !scalars || !workspace))) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (n && workspace_bytes < pa::msm_workspace_bytes(2, n))
        return fail(PA_ERR_INVALID_ARGUMENT, "workspace smaller than pa_multiexp_workspace_bytes");
    PA_TRY(pa::launch_msm(2, (const uint64_t*)bases, (const uint64_t*)scalars, n, (uint64_t*)out, workspace,
                          workspace_bytes, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}

// ---- CurveProjective / CurveAffine surface, G1 and G2 (kernels_group.hip) ----
namespace {
constexpr size_t jac_bytes(int group) { return group == 1 ? sizeof(pa_g1) : sizeof(pa_g2); }
constexpr size_t aff_bytes(int group) { return group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine); }
size_t op_in_bytes(int group, int op) { return op == pa::GROUP_FROM_AFFINE ? aff_bytes(group) : jac_bytes(group); }
size_t op_b_bytes(int group, int op) {
    if (op == pa::GROUP_ADD || op == pa::GROUP_SUB || op == pa::GROUP_EQ) return jac_bytes(group);
    return op == pa::GROUP_ADD_MIXED ? aff_bytes(group) : 0;
}
size_t op_out_bytes(int group, int op) {
    if (op == pa::GROUP_EQ) return 1;
    return op == pa::GROUP_INTO_AFFINE ? aff_bytes(group) : jac_bytes(group);
}

int host_group_op(int group, int op, const void* a, const void* b, void* out, size_t n) {
    if (n == 0) return PA_OK;
    const size_t ib = op_in_bytes(group, op), bb = op_b_bytes(group, op), ob = op_out_bytes(group, op);
    if (!a || !out || (bb && !b)) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf da, db, dout;
    int rc;
    if ((rc = upload(da, a, ib * n))) return rc;
    if (bb && (rc = upload(db, b, bb * n))) return rc;
    PA_TRY(dout.alloc(ob * n), "device scratch");
    PA_TRY(pa::launch_group_op(group, op, da.as<uint64_t>(), db.as<uint64_t>(), dout.as<uint64_t>(), n, call_stream()),
           "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, ob * n);
}
int device_group_op(int group, int op, const void* a, const void* b, void* out, size_t n, void* stream) {
    if (n && (!a || !out || (op_b_bytes(group, op) && !b))) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_group_op(group, op, (const uint64_t*)a, (const uint64_t*)b, (uint64_t*)out, n,
                               (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}

// FrRepr::num_bits (fr.rs:58 via the repr macro): 256 minus leading zeros
int repr_num_bits(const pa_fr_repr* s) {
    for (int w = 3; w >= 0; w--)
        if (s->l[w]) return 64 * w + 64 - __builtin_clzll(s->l[w]);
    return 0;
}
int window_for_count(size_t n, const size_t* rec, int m) {
    int ret = 4;
    for (int k = 0; k < m && n > rec[k]; k++) ret++;
    return ret;
}
}  // namespace

#define PA_GROUP_ENTRIES(G, JAC, AFF)                                                                            \
    int pa_g##G##_double_batch(const JAC* a, JAC* out, size_t n) {                                              \
        return host_group_op(G, pa::GROUP_DOUBLE, a, nullptr, out, n);                                          \
    }                                                                                                           \
    int pa_g##G##_add_batch(const JAC* a, const JAC* b, JAC* out, size_t n) {                                    \
        return host_group_op(G, pa::GROUP_ADD, a, b, out, n);                                                   \
    }                                                                                                           \
    int pa_g##G##_add_mixed_batch(const JAC* a, const AFF* b, JAC* out, size_t n) {                              \
        return host_group_op(G, pa::GROUP_ADD_MIXED, a, b, out, n);                                             \
    }                                                                                                           \
    int pa_g##G##_negate_batch(const JAC* a, JAC* out, size_t n) {                                              \
        return host_group_op(G, pa::GROUP_NEGATE, a, nullptr, out, n);                                          \
    }                                                                                                           \
    int pa_g##G##_sub_batch(const JAC* a, const JAC* b, JAC* out, size_t n) {                                    \
        return host_group_op(G, pa::GROUP_SUB, a, b, out, n);                                                   \
    }                                                                                                           \
    int pa_g##G##_into_affine_batch(const JAC* a, AFF* out, size_t n) {                                         \
        return host_group_op(G, pa::GROUP_INTO_AFFINE, a, nullptr, out, n);                                     \
    }                                                                                                           \
    int pa_g##G##_into_projective_batch(const AFF* a, JAC* out, size_t n) {                                     \
        return host_group_op(G, pa::GROUP_FROM_AFFINE, a, nullptr, out, n);                                     \
    }                                                                                                           \
    int pa_g##G##_double_batch_device(const JAC* a, JAC* out, size_t n, void* stream) {                         \
        return device_group_op(G, pa::GROUP_DOUBLE, a, nullptr, out, n, stream);                                \
    }                                                                                                           \
    int pa_g##G##_add_batch_device(const JAC* a, const JAC* b, JAC* out, size_t n, void* stream) {              \
        return device_group_op(G, pa::GROUP_ADD, a, b, out, n, stream);                                         \
    }                                                                                                           \
    int pa_g##G##_add_mixed_batch_device(const JAC* a, const AFF* b, JAC* out, size_t n, void* stream) {        \
        return device_group_op(G, pa::GROUP_ADD_MIXED, a, b, out, n, stream);                                   \
    }                                                                                                           \
    int pa_g##G##_into_affine_batch_device(const JAC* a, AFF* out, size_t n, void* stream) {                    \
        return device_group_op(G, pa::GROUP_INTO_AFFINE, a, nullptr, out, n, stream);                           \
    }                                                                                                           \
    int pa_g##G##_eq_batch(const JAC* a, const JAC* b, uint8_t* eq, size_t n) {                                 \
        return host_group_op(G, pa::GROUP_EQ, a, b, eq, n);                                                     \
    }                                                                                                           \
    int pa_g##G##_eq_batch_device(const JAC* a, const JAC* b, uint8_t* eq, size_t n, void* stream) {            \
        return device_group_op(G, pa::GROUP_EQ, a, b, eq, n, stream);                                           \
    }

PA_GROUP_ENTRIES(1, pa_g1, pa_g1_affine)
PA_GROUP_ENTRIES(2, pa_g2, pa_g2_affine)
#undef PA_GROUP_ENTRIES

int pa_g2_batch_normalization(pa_g2* v, size_t n) {
    if (n == 0) return PA_OK;
    if (!v) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    DevBuf dv;
    int rc;
    if ((rc = upload(dv, v, sizeof(pa_g2) * n))) return rc;
    PA_TRY(pa::launch_g2_batch_normalize(dv.as<uint64_t>(), n, call_stream()), "kernel launch");
    PA_TRY(call_sync(), "kernel execution");
    return download(v, dv, sizeof(pa_g2) * n);
}
int pa_g2_batch_normalization_device(pa_g2* v, size_t n, void* stream) {
    if (n && !v) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    PA_TRY(pa::launch_g2_batch_normalize((uint64_t*)v, n, (hipStream_t)stream), "kernel launch");
    return PA_OK;
}
size_t pa_g2_fixed_base_table_words(void) { return pa::g2_comb_table_words(); }
size_t pa_g2_fixed_base_workspace_words(void) { return pa::g2_comb_workspace_words(); }
int pa_g2_wnaf_fixed_base_device(const pa_g2* base, const pa_fr_repr* scalars, pa_g2* out, size_t n,
                                 uint64_t* table, uint64_t* workspace, void* stream) {
    return pa_g2_wnaf_fixed_base_window_device(base, scalars, out, n, pa_g2_recommended_wnaf_for_num_scalars(n), table,
                                               workspace, stream);
}
int pa_g2_wnaf_fixed_base_window_device(const pa_g2* base, const pa_fr_repr* scalars, pa_g2* out, size_t n,
                                        int window, uint64_t* table, uint64_t* workspace, void* stream) {
    if (n == 0) return PA_OK;
    if (!base || !scalars || !out || !table || !workspace) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (window < 1 || window > kMaxWnafWindow) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range");
    PA_TRY(pa::launch_g2_comb_table((const uint64_t*)base, table, workspace, (hipStream_t)stream), "kernel launch");
    PA_TRY(pa::launch_g2_comb_mul(table, (const uint64_t*)scalars, (uint64_t*)out, n, window, (hipStream_t)stream),
           "kernel launch");
    return PA_OK;
}
int pa_g2_wnaf_fixed_base(const pa_g2* base, const pa_fr_repr* scalars, size_t n, pa_g2* out) {
    return pa_g2_wnaf_fixed_base_window(base, scalars, n, pa_g2_recommended_wnaf_for_num_scalars(n), out);
}
int pa_g2_wnaf_fixed_base_window(const pa_g2* base, const pa_fr_repr* scalars, size_t n, int window, pa_g2* out) {
    if (n == 0) return PA_OK;
    if (!base || !scalars || !out) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    if (window < 1 || window > kMaxWnafWindow) return fail(PA_ERR_INVALID_ARGUMENT, "wnaf window out of range");
    DevBuf db, ds, dt, dw, dout;
    int rc;
    if ((rc = upload(db, base, sizeof(pa_g2))) || (rc = upload(ds, scalars, sizeof(pa_fr_repr) * n))) return rc;
    PA_TRY(dt.alloc(8 * pa::g2_comb_table_words()), "device scratch");
    PA_TRY(dw.alloc(8 * pa::g2_comb_workspace_words()), "device scratch");
    PA_TRY(dout.alloc(sizeof(pa_g2) * n), "device scratch");
    if ((rc = pa_g2_wnaf_fixed_base_window_device(db.as<pa_g2>(), ds.as<pa_fr_repr>(), dout.as<pa_g2>(), n, window,
                                                  dt.as<uint64_t>(), dw.as<uint64_t>(), call_stream())))
        return rc;
    PA_TRY(call_sync(), "kernel execution");
    return download(out, dout, sizeof(pa_g2) * n);
}

// window heuristics (ec.rs:895-921 for G1, 1586-1612 for G2)
int pa_g1_recommended_wnaf_for_scalar(const pa_fr_repr* s) {
    if (!s) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int b = repr_num_bits(s);
    return b >= 130 ? 4 : b >= 34 ? 3 : 2;
}
int pa_g2_recommended_wnaf_for_scalar(const pa_fr_repr* s) {
    if (!s) return fail(PA_ERR_INVALID_ARGUMENT, "null pointer");
    const int b = repr_num_bits(s);
    return b >= 103 ? 4 : b >= 37 ? 3 : 2;
}
int pa_g1_recommended_wnaf_for_num_scalars(size_t num_scalars) {
    static const size_t rec[12] = {1, 3, 7, 20, 43, 120, 273, 563, 1630, 3128, 7933, 62569};
    return window_for_count(num_scalars, rec, 12);
}
int pa_g2_recommended_wnaf_for_num_scalars(size_t num_scalars) {
    static const size_t rec[11] = {1, 3, 8, 20, 47, 126, 260, 826, 1501, 4555, 84071};
    return window_for_count(num_scalars, rec, 11);
}

}  // extern "C"
