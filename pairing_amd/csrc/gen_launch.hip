// Host side of the generated pairing kernels (tools/pgen): the code objects
// pairing_amd/lib/pa_gen_*.hsaco sit next to libpairing_amd.so and are
// loaded once per device through the HIP module API; each launch passes the
// five kernel arguments of tools/pgen/kcfg.py and a per-wave spill
// workspace (pa_gen_meta.h gives its size).  A missing code object is an
// error, never a fallback.
//
// Spill workspaces.  A launch's waves index their workspace from its base by
// block, so two launches that run at the same time must not share one.  Each
// device keeps a pool of workspaces; a workspace records the stream and an
// event of its last launch and is handed to a new launch only if that launch
// is on the same stream (stream order serializes them) or the event has
// completed (acquire() below).  Otherwise a new workspace is allocated, so
// concurrent callers on different streams (pairing_amd.h: every entry point is
// reentrant) each get their own.  The pool only grows to the number of
// launches in flight at once.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "launch.h"
#include "pa_gen_meta.h"

namespace pa {
namespace {

constexpr int kKernels = 8;
constexpr size_t kSlotBytes = 3584;  // one 14-limb spill slot for a 64-lane wave

struct Workspace {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t last = nullptr;
    hipEvent_t done = nullptr;
};

struct GenDevice {
    bool loaded[kKernels] = {};
    hipModule_t mod[kKernels] = {};
    hipFunction_t fn[kKernels] = {};
    std::vector<Workspace> pool;
    // a non-blocking stream of the library's own for the load-time symbol read:
    // a copy on the legacy stream would join a caller's stream capture
    // (hipStreamCaptureModeRelaxed) and invalidate it
    hipStream_t load_stream = nullptr;
    std::vector<void*> graph_ws;   // workspaces of captured launches (never reused)
};

std::mutex g_mu;
GenDevice g_dev[64];
thread_local std::string g_detail;   // the code object that failed to load, for pa_last_error

// 0, 1: one lane per pairing; 2, 3: a lane pair per pairing; 4: the Miller
// loop of a batch against one shared G2Prepared (a line table in place of a1);
// 5: the Miller loop of (P_i, G2Prepared_i) pairs, a1 = the prepared records;
// 6: the pairing-only lane-pair Miller loop (e(P, Q) paths: its Miller values
// differ from the reference's by Fq2 factors the final exponentiation removes);
// 7: the same one lane per pairing
const char* const kFile[kKernels] = {"pa_gen_miller_loop.hsaco", "pa_gen_final_exp.hsaco",
                                     "pa_gen_miller_loop2.hsaco", "pa_gen_final_exp2.hsaco",
                                     "pa_gen_miller_loop_shared.hsaco", "pa_gen_miller_loop_prepared.hsaco",
                                     "pa_gen_miller_loop2p.hsaco", "pa_gen_miller_loop1p.hsaco"};
const char* const kName[kKernels] = {"pa_gen_miller_loop", "pa_gen_final_exp", "pa_gen_miller_loop2",
                                     "pa_gen_final_exp2", "pa_gen_miller_loop_shared",
                                     "pa_gen_miller_loop_prepared", "pa_gen_miller_loop2p", "pa_gen_miller_loop1p"};
const size_t kWaveBytes[kKernels] = {PA_GEN_MILLER_LOOP_MEM_SLOTS * kSlotBytes, PA_GEN_FINAL_EXP_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_MILLER_LOOP2_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_FINAL_EXP2_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_MILLER_LOOP_SHARED_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_MILLER_LOOP_PREPARED_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_MILLER_LOOP2P_MEM_SLOTS * kSlotBytes,
                                     PA_GEN_MILLER_LOOP1P_MEM_SLOTS * kSlotBytes};
const int kLanes[kKernels] = {1, 1, 2, 2, 1, 1, 2, 1};

// PA_GEN_DIR (A/B experiments with alternative generated code objects) overrides
// the directory of libpairing_amd.so; PA_GEN_WS_SLOTS raises the workspace size
// to fit their spill slots.
std::string lib_dir() {
    if (const char* e = getenv("PA_GEN_DIR")) return e;
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&lib_dir), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t k = p.rfind('/');
        if (k != std::string::npos) return p.substr(0, k);
    }
    return ".";
}

size_t wave_bytes();

// Loads the one code object a launch needs, on first use.  Each object loads
// on its own: a missing or refused file fails only the entries that launch it
// (the others keep working), and a failed load is retried by the next launch.
hipError_t load(GenDevice& d, int k) {
    if (d.loaded[k]) return hipSuccess;
    const std::string path = lib_dir() + "/" + kFile[k];
    hipError_t e;
    if ((e = hipModuleLoad(&d.mod[k], path.c_str())) != hipSuccess) {
        d.mod[k] = nullptr;
        g_detail = "generated kernel " + path;
        return e;
    }
    if ((e = hipModuleGetFunction(&d.fn[k], d.mod[k], kName[k])) != hipSuccess) {
        g_detail = "kernel " + std::string(kName[k]) + " in " + path;
    } else {
        // the code object states its spill slots per wave: one that needs more
        // workspace than this library allocates (a stale or swapped file,
        // PA_GEN_DIR) would write past its wave's slice -- refuse it
        hipDeviceptr_t gp = nullptr;
        size_t gb = 0;
        uint32_t need = 0;
        const std::string sym = std::string(kName[k]) + "_mem_slots";
        if ((e = hipModuleGetGlobal(&gp, &gb, d.mod[k], sym.c_str())) != hipSuccess || gb != 4 ||
            (!d.load_stream && (e = hipStreamCreateWithFlags(&d.load_stream, hipStreamNonBlocking)) != hipSuccess) ||
            (e = hipMemcpyDtoHAsync(&need, gp, 4, d.load_stream)) != hipSuccess ||
            (e = hipStreamSynchronize(d.load_stream)) != hipSuccess) {
            if (e == hipSuccess) e = hipErrorInvalidImage;
            g_detail = "workspace size symbol " + sym + " in " + path;
        } else if ((size_t)need * kSlotBytes > wave_bytes()) {
            e = hipErrorInvalidImage;
            g_detail = path + " needs " + std::to_string(need) + " workspace slots per wave, the library allocates " +
                       std::to_string(wave_bytes() / kSlotBytes) + " (rebuild, or PA_GEN_WS_SLOTS)";
        }
    }
    if (e != hipSuccess) {
        (void)hipModuleUnload(d.mod[k]);
        d.mod[k] = nullptr;
        d.fn[k] = nullptr;
        return e;
    }
    d.loaded[k] = true;
    return hipSuccess;
}

size_t wave_bytes() {
    size_t b = 0;
    for (int k = 0; k < kKernels; k++) b = kWaveBytes[k] > b ? kWaveBytes[k] : b;
    if (const char* e = getenv("PA_GEN_WS_SLOTS")) {
        const size_t x = strtoull(e, nullptr, 10) * kSlotBytes;
        b = x > b ? x : b;
    }
    return b;
}

// A workspace of at least `need` bytes that no unfinished launch on another
// stream uses (caller holds g_mu).  Reuse is decided by the completion event;
// an unfinished workspace of the same stream handle is also reused, with the
// new launch made to wait for that event: on the same stream the wait changes
// nothing (stream order), and if the handle now names another stream (a
// destroyed stream's handle reused, hipStreamPerThread from two threads) it
// keeps the two launches apart.  A finished workspace that is too small is
// grown in place, whatever stream used it.
hipError_t acquire(GenDevice& d, size_t need, hipStream_t stream, Workspace** out) {
    Workspace* idle_small = nullptr;
    Workspace* same = nullptr;
    for (auto& w : d.pool) {
        if (hipEventQuery(w.done) == hipSuccess) {
            if (w.bytes >= need) {
                *out = &w;
                return hipSuccess;
            }
            if (!idle_small) idle_small = &w;
        } else if (w.last == stream && w.bytes >= need && !same) {
            same = &w;
        }
    }
    hipError_t e;
    if (same) {
        if ((e = hipStreamWaitEvent(stream, same->done, 0)) != hipSuccess) return e;
        *out = same;
        return hipSuccess;
    }
    if (idle_small) {  // its last launch has finished: grow it in place
        if ((e = hipFree(idle_small->p)) != hipSuccess) return e;
        idle_small->p = nullptr;
        idle_small->bytes = 0;
        if ((e = hipMalloc(&idle_small->p, need)) != hipSuccess) return e;
        idle_small->bytes = need;
        *out = idle_small;
        return hipSuccess;
    }
    Workspace w;
    if ((e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipMalloc(&w.p, need)) != hipSuccess) {
        (void)hipEventDestroy(w.done);
        return e;
    }
    w.bytes = need;
    d.pool.push_back(w);
    *out = &d.pool.back();
    return hipSuccess;
}

// which == 4 (shared G2Prepared): a1 is the prepared record; its line table
// is built in the workspace behind the waves' spill slices first
hipError_t launch(int which, const void* a0, const void* a1, const void* a2, size_t n, hipStream_t stream) {
    g_detail.clear();
    if (n == 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(g_mu);
    GenDevice& d = g_dev[dev];
    if ((e = load(d, which)) != hipSuccess) {
        if (g_detail.empty()) g_detail = std::string("generated kernel ") + kFile[which] + " in " + lib_dir();
        return e;
    }
    const size_t blocks = (n * kLanes[which] + 63) / 64;
    if (blocks > 0xffffffffull) return hipErrorInvalidValue;
    const size_t table_at = (blocks * wave_bytes() + 255) & ~(size_t)255;
    const size_t need = which == 4 ? table_at + kSharedTableAlloc : blocks * wave_bytes();
    // under stream capture the workspace goes into the caller's graph, which may
    // replay it at any later time: a dedicated allocation that the pool never
    // hands out again (kept for the process's lifetime), and no event query or
    // record on the capturing stream
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if ((e = hipStreamIsCapturing(stream, &cs)) != hipSuccess) return e;
    const bool captured = cs != hipStreamCaptureStatusNone;
    Workspace* ws = nullptr;
    void* wsp = nullptr;
    if (captured) {
        if ((e = hipMalloc(&wsp, need)) != hipSuccess) return e;
        d.graph_ws.push_back(wsp);
    } else {
        if ((e = acquire(d, need, stream, &ws)) != hipSuccess) return e;
        wsp = ws->p;
    }
    if (which == 4) {
        uint32_t* table = reinterpret_cast<uint32_t*>(static_cast<char*>(wsp) + table_at);
        if ((e = launch_shared_line_table(static_cast<const uint64_t*>(a1), table, stream)) != hipSuccess) return e;
        a1 = table;
    }
    struct {
        const void* a0;
        const void* a1;
        const void* a2;
        uint64_t n;
        void* ws;
    } args{a0, a1, a2, (uint64_t)n, wsp};
    size_t size = sizeof(args);
    void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                      HIP_LAUNCH_PARAM_END};
    if ((e = hipModuleLaunchKernel(d.fn[which], (unsigned)blocks, 1, 1, 64, 1, 1, 0, stream, nullptr, config)) !=
        hipSuccess)
        return e;
    if (captured) return hipSuccess;
    ws->last = stream;
    return hipEventRecord(ws->done, stream);
}

}  // namespace

const char* gen_error_detail() { return g_detail.c_str(); }

hipError_t launch_miller_loop_gen(int lanes, const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                  hipStream_t stream) {
    return launch(lanes == 2 ? 2 : 0, p_aff, q_aff, out, n, stream);
}
// One kernel per final exponentiation, in place or not (round 3: its
// inversions run in the kernel by binary GCD and exp_by_x squares compressed,
// Karabina; tools/pgen/kernels.py).  Round 2's form split around a separate
// inversion kernel was removed in round 4.
hipError_t launch_final_exp_gen(int lanes, const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n,
                                hipStream_t stream) {
    return launch(lanes == 2 ? 3 : 1, in, out, ok, n, stream);
}
hipError_t launch_miller_loop_shared_gen(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out, size_t n,
                                         hipStream_t stream) {
    return launch(4, p_aff, prepared, out, n, stream);
}
hipError_t launch_miller_loop_pairing_gen(int lanes, const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out,
                                          size_t n, hipStream_t stream) {
    return launch(lanes == 2 ? 6 : 7, p_aff, q_aff, out, n, stream);
}
hipError_t launch_miller_loop_prepared_gen(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out,
                                           size_t n, hipStream_t stream) {
    return launch(5, p_aff, prepared, out, n, stream);
}

}  // namespace pa
