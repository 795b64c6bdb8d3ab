// Host side of the generated pairing kernels (tools/pgen): the code objects
// pairing_amd/lib/pa_gen_*.hsaco sit next to libpairing_amd.so and are
// loaded once per device through the HIP module API; each launch passes the
// five kernel arguments of tools/pgen/kcfg.py and a per-wave spill
// workspace (pa_gen_meta.h gives its size).  A missing code object is an
// error, never a fallback.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>

#include "launch.h"
#include "pa_gen_meta.h"

namespace pa {
namespace {

constexpr int kKernels = 6;

struct GenDevice {
    bool loaded = false;
    hipError_t err = hipSuccess;
    hipModule_t mod[kKernels] = {};
    hipFunction_t fn[kKernels] = {};
    void* ws = nullptr;
    size_t ws_bytes = 0;
};

std::mutex g_mu;
GenDevice g_dev[64];
thread_local std::string g_detail;   // the code object that failed to load, for pa_last_error

// 0, 1: one lane per pairing; 2, 3: a lane pair per pairing; 4, 5: one lane,
// lazy reduction (tower.TowerLazy)
const char* const kFile[kKernels] = {"pa_gen_miller_loop.hsaco", "pa_gen_final_exp.hsaco",
                                     "pa_gen_miller_loop2.hsaco", "pa_gen_final_exp2.hsaco",
                                     "pa_gen_miller_loop_lazy.hsaco", "pa_gen_final_exp_lazy.hsaco"};
const char* const kName[kKernels] = {"pa_gen_miller_loop", "pa_gen_final_exp", "pa_gen_miller_loop2",
                                     "pa_gen_final_exp2", "pa_gen_miller_loop_lazy", "pa_gen_final_exp_lazy"};
const size_t kWaveBytes[kKernels] = {
    PA_GEN_MILLER_LOOP_MEM_SLOTS * 3584ull, PA_GEN_FINAL_EXP_MEM_SLOTS * 3584ull,
    PA_GEN_MILLER_LOOP2_MEM_SLOTS * 3584ull, PA_GEN_FINAL_EXP2_MEM_SLOTS * 3584ull,
    PA_GEN_MILLER_LOOP_LAZY_MEM_SLOTS * 3584ull, PA_GEN_FINAL_EXP_LAZY_MEM_SLOTS * 3584ull};
const int kLanes[kKernels] = {1, 1, 2, 2, 1, 1};

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

hipError_t load(GenDevice& d) {
    if (d.loaded) return d.err;
    d.loaded = true;
    const std::string dir = lib_dir();
    for (int k = 0; k < kKernels; k++) {
        const std::string path = dir + "/" + kFile[k];
        if ((d.err = hipModuleLoad(&d.mod[k], path.c_str())) != hipSuccess ||
            (d.err = hipModuleGetFunction(&d.fn[k], d.mod[k], kName[k])) != hipSuccess) {
            g_detail = "generated kernel " + path;
            return d.err;
        }
    }
    return hipSuccess;
}

hipError_t launch(int which, const void* a0, const void* a1, const void* a2, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(g_mu);
    GenDevice& d = g_dev[dev];
    if ((e = load(d)) != hipSuccess) {
        if (g_detail.empty()) g_detail = "generated kernels in " + lib_dir();
        return e;
    }
    const size_t blocks = (n * kLanes[which] + 63) / 64;
    size_t wave_bytes = 0;
    for (int k = 0; k < kKernels; k++) wave_bytes = kWaveBytes[k] > wave_bytes ? kWaveBytes[k] : wave_bytes;
    if (const char* e = getenv("PA_GEN_WS_SLOTS")) {
        const size_t b = strtoull(e, nullptr, 10) * 3584ull;
        wave_bytes = b > wave_bytes ? b : wave_bytes;
    }
    const size_t need = blocks * wave_bytes;
    if (need > d.ws_bytes) {
        if (d.ws) (void)hipFree(d.ws);
        d.ws = nullptr;
        d.ws_bytes = 0;
        if ((e = hipMalloc(&d.ws, need)) != hipSuccess) return e;
        d.ws_bytes = need;
    }
    struct {
        const void* a0;
        const void* a1;
        const void* a2;
        uint64_t n;
        void* ws;
    } args{a0, a1, a2, (uint64_t)n, d.ws};
    size_t size = sizeof(args);
    void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                      HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(d.fn[which], (unsigned)blocks, 1, 1, 64, 1, 1, 0, stream, nullptr, config);
}

}  // namespace

const char* gen_error_detail() { return g_detail.c_str(); }

hipError_t launch_miller_loop_gen(const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                  hipStream_t stream) {
    return launch(0, p_aff, q_aff, out, n, stream);
}
hipError_t launch_final_exp_gen(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t stream) {
    return launch(1, in, out, ok, n, stream);
}
hipError_t launch_miller_loop_gen2(const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                   hipStream_t stream) {
    return launch(2, p_aff, q_aff, out, n, stream);
}
hipError_t launch_final_exp_gen2(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t stream) {
    return launch(3, in, out, ok, n, stream);
}
hipError_t launch_miller_loop_gen_lazy(const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                       hipStream_t stream) {
    return launch(4, p_aff, q_aff, out, n, stream);
}
hipError_t launch_final_exp_gen_lazy(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n,
                                     hipStream_t stream) {
    return launch(5, in, out, ok, n, stream);
}

}  // namespace pa
