// Prototype harness for the Fl leaves (tools/gen_fl.py): raw-limb products for
// bound checks from Python, and an in-register throughput loop against the
// 32-bit-word multiply.  Build: hipcc -O3 --offload-arch=gfx950 -fPIC -shared
#include "../pairing_amd/csrc/fl.h"
#include "../pairing_amd/csrc/fq_mul_gen.h"

using namespace pa;

__global__ void k_raw(int op, const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d,
                      uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fl x, y, z, w, r;
    for (int j = 0; j < 14; j++) {
        x.w[j] = a[i * 14 + j]; y.w[j] = b[i * 14 + j];
        z.w[j] = c[i * 14 + j]; w.w[j] = d[i * 14 + j];
    }
    if (op == 0) fl_mul_leaf(r, x, y);
    else if (op == 1) fl_sop2_leaf(r, x, y, z, w);
    else fl_sqr_leaf(r, x);
    for (int j = 0; j < 14; j++) out[i * 14 + j] = r.w[j];
}

__global__ void k_abi(const uint64_t* a, const uint64_t* b, uint64_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq x, y, r;
    fq_load(x, a + 6 * i);
    fq_load(y, b + 6 * i);
    Fl X, Y, Z;
    fl_from_abi(X, x);
    fl_from_abi(Y, y);
    fl_mul_leaf(Z, X, Y);
    fl_to_abi(r, Z);
    fq_store(out + 6 * i, r);
}

template <int OP>
__global__ void __launch_bounds__(256) k_loop(const uint64_t* a, uint64_t* out, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    Fq x, y;
    fq_load(x, a + 6 * i);
    fq_load(y, a + 6 * (i ^ 1));
    if constexpr (OP == 0) {
        for (int it = 0; it < iters; it++) fq_mul(x, x, y);
    } else {
        Fl X, Y;
        fl_split(X, x);
        fl_split(Y, y);
        for (int it = 0; it < iters; it++) {
            if constexpr (OP == 1) fl_mul_leaf(X, X, Y);
            else fl_sqr_leaf(X, X);
        }
        fl_canon(X, X);
        fl_pack(x, X);
    }
    fq_store(out + 6 * i, x);
}

extern "C" {
int flp_raw(int op, const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d, uint32_t* out,
            int n) {
    uint32_t* dv;
    size_t sz = (size_t)n * 14 * 4;
    hipMalloc(&dv, 5 * sz);
    hipMemcpy(dv, a, sz, hipMemcpyHostToDevice);
    hipMemcpy(dv + n * 14, b, sz, hipMemcpyHostToDevice);
    hipMemcpy(dv + 2 * n * 14, c, sz, hipMemcpyHostToDevice);
    hipMemcpy(dv + 3 * n * 14, d, sz, hipMemcpyHostToDevice);
    k_raw<<<(n + 255) / 256, 256>>>(op, dv, dv + n * 14, dv + 2 * n * 14, dv + 3 * n * 14, dv + 4 * n * 14, n);
    hipMemcpy(out, dv + 4 * n * 14, sz, hipMemcpyDeviceToHost);
    hipFree(dv);
    return (int)hipGetLastError();
}

int flp_abi(const uint64_t* a, const uint64_t* b, uint64_t* out, int n) {
    uint64_t* dv;
    size_t sz = (size_t)n * 48;
    hipMalloc(&dv, 3 * sz);
    hipMemcpy(dv, a, sz, hipMemcpyHostToDevice);
    hipMemcpy(dv + n * 6, b, sz, hipMemcpyHostToDevice);
    k_abi<<<(n + 255) / 256, 256>>>(dv, dv + n * 6, dv + 2 * n * 6, n);
    hipMemcpy(out, dv + 2 * n * 6, sz, hipMemcpyDeviceToHost);
    hipFree(dv);
    return (int)hipGetLastError();
}

// ms for `iters` dependent products per lane over n lanes
float flp_time(int op, const uint64_t* a, int n, int iters) {
    uint64_t* dv;
    hipMalloc(&dv, (size_t)n * 96);
    hipMemcpy(dv, a, (size_t)n * 48, hipMemcpyHostToDevice);
    auto launch = [&]() {
        if (op == 0) k_loop<0><<<n / 256, 256>>>(dv, dv + n * 6, iters);
        else if (op == 1) k_loop<1><<<n / 256, 256>>>(dv, dv + n * 6, iters);
        else k_loop<2><<<n / 256, 256>>>(dv, dv + n * 6, iters);
    };
    launch();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(dv);
    return ms;
}
}
