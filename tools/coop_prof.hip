// Per-step-kind cycle profile of the cooperative kernels (one wave, one item):
// builds kernels_coop.hip with PA_COOP_PROFILE, runs one Miller loop and one
// final exponentiation, prints cycles per step kind.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I pairing_amd/csrc tools/coop_prof.hip -o tools/coop_prof
#define PA_COOP_PROFILE 1
#include "../pairing_amd/csrc/kernels_coop.hip"
#include <cstdio>
#include <vector>

static void report(const char* what, float ms) {
    unsigned long long h[8][3], wk[8];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(pa::g_coop_prof), sizeof h);
    (void)hipMemcpyFromSymbol(wk, HIP_SYMBOL(pa::g_coop_prof_work), sizeof wk);
    const char* names[8] = {"LIN", "P1", "P2", "SQ", "INV", "LC", "k6", "k7"};
    unsigned long long tot = 0;
    for (int k = 0; k < 8; k++) tot += h[k][0];
    printf("%s: %.3f ms, %llu profiled cycles\n", what, ms, tot);
    for (int k = 0; k < 8; k++)
        if (h[k][1])
            printf("  %-4s steps %6llu  cycles/step %8.0f  (lane 0's own work %6.0f)  lanes/step %5.1f  share %5.1f%%\n",
                   names[k], h[k][1], (double)h[k][0] / h[k][1], (double)wk[k] / h[k][1], (double)h[k][2] / h[k][1],
                   100.0 * h[k][0] / tot);
    unsigned long long z[8][3] = {}, zw[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_coop_prof), z, sizeof z);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_coop_prof_work), zw, sizeof zw);
}

int main() {
    std::vector<uint64_t> p(13, 0), q(25, 0), f(72, 0);
    for (int i = 0; i < 6; i++) { p[i] = 0x0123456789abcdefull * (i + 1) >> 8; q[i] = p[i] ^ 0x55; q[6 + i] = p[i] ^ 0x77; }
    for (int i = 0; i < 72; i++) f[i] = (0x9e3779b97f4a7c15ull * (i + 3)) >> 8;
    uint64_t *dp, *dq, *df, *dout;
    uint8_t* dok;
    (void)hipMalloc(&dp, 13 * 8); (void)hipMalloc(&dq, 25 * 8); (void)hipMalloc(&df, 72 * 8);
    (void)hipMalloc(&dout, 72 * 8); (void)hipMalloc(&dok, 8);
    (void)hipMemcpy(dp, p.data(), 13 * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dq, q.data(), 25 * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(df, f.data(), 72 * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float ms;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(e0);
        (void)pa::launch_coop_miller_loop(dp, dq, dout, 1, nullptr);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        report("miller loop", ms);
        (void)hipEventRecord(e0);
        (void)pa::launch_coop_final_exp(df, dout, dok, 1, nullptr);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        report("final exp", ms);
    }
    return 0;
}
