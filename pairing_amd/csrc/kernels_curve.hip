// G1 kernels for the parameter-generation path (BASELINE config 3):
//   Wnaf::new().base(g, n).scalar(s_i) for n scalars   (wnaf.rs:93-107, 169-178)
//   G1::batch_normalization(&mut out)                    (ec.rs:246-294)
//
// Fixed-base multiplication.  The reference recodes each scalar in wNAF with
// window recommended_wnaf_for_num_scalars(n) (16 at n = 2^18, ec.rs:907-921)
// against a 2^15-entry Jacobian table built by a serial add chain, then runs
// ~255 doublings + ~16 additions per scalar.  Only the *point* s*g is
// observable (CurveProjective's PartialEq is representation-independent,
// ec.rs:45-85, and batch_normalization makes it canonical), so the GPU uses
// the fixed-base algorithm that suits a wide machine: a signed base-256 comb.
//   T[i][d] = d * 2^(8i) * g  (affine), i = 0..32, d = 1..128      (420 KB,
//   read-only, resident in every XCD's L2)
//   s*g = sum_i sign(d_i) T[i][|d_i|], digits d_i in [-127, 128]
// = at most 33 mixed additions (madd-2007-bl) per scalar and no doublings,
// against ~255 doublings + 16 additions for wNAF.
//
// batch_normalization.  Montgomery's trick over chunks of CHUNK points per
// lane with one Fermat inversion per chunk; zero and already-normalized points
// are left bit-for-bit untouched, as in the reference (ec.rs:255-257, 271, 285).
#include <mutex>

#include "curve_fl.h"
#include "launch.h"
#include "pairing.h"

namespace pa {

constexpr int kCombWindows = 33;      // 8-bit digits of a 255-bit scalar + final carry
constexpr int kCombEntries = 128;     // |d| in 1..128
constexpr int kG1Jac = 18;            // u64 words per Jacobian G1
constexpr uint32_t kFlInfinity = 0xffffffffu;  // table entry marker: no lazy limb has all 32 bits set
constexpr int kFlPair = 14;           // u64 words per table entry: x, y as 14 x 28-bit limbs (lazy core)
constexpr int kNormChunk = 8;         // points per lane in batch_normalization (4 measured slower at 2^18)

// ---------------- batch_normalization ----------------
__global__ void __launch_bounds__(64) k_g1_batch_normalize(uint64_t* __restrict__ v, size_t n) {
    __builtin_amdgcn_s_setprio(2);   // latency-bound: ahead of a concurrent comb multiply's waves
    const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t begin = lane * kNormChunk;
    if (begin >= n) return;
    const int cnt = (int)((n - begin) < (size_t)kNormChunk ? (n - begin) : (size_t)kNormChunk);
    uint64_t* base = v + begin * kG1Jac;
    // forward pass: prod[k] = z_0 * ... * z_k over non-normalized points
    Fq prod[kNormChunk];
    bool skip[kNormChunk];
    Fq acc;
    fq_one(acc);
#pragma unroll
    for (int k = 0; k < kNormChunk; k++) {
        if (k < cnt) {
            Fq z;
            fq_load(z, base + k * kG1Jac + 12);
            skip[k] = fq_is_zero(z) || fq_is_one(z);
            Fq t;
            fq_mul(t, acc, z);
            if (!skip[k]) acc = t;
            prod[k] = acc;
        } else {
            skip[k] = true;
        }
    }
    Fq inv;
    fq_inv(inv, acc);  // acc != 0: product of nonzero z's (or one)
    // backward pass: z_k^-1 = inv * prod[k-1]; inv *= z_k
#pragma unroll
    for (int k = kNormChunk - 1; k >= 0; k--) {
        if (k < cnt && !skip[k]) {
            Fq z, zinv, prev;
            fq_load(z, base + k * kG1Jac + 12);
            fq_one(prev);
#pragma unroll
            for (int j = 0; j < kNormChunk; j++)
                if (j == k - 1) prev = prod[j];
            // prod[j] for the last non-skipped j < k equals prod[k-1] (skipped entries carry acc)
            fq_mul_x2(zinv, inv, prev, inv, inv, z);
            Fq zz, x, y;
            fq_sqr(zz, zinv);
            fq_load(x, base + k * kG1Jac);
            fq_load(y, base + k * kG1Jac + 6);
            Fq zzz;
            fq_mul_x2(x, x, zz, zzz, zz, zinv);
            fq_mul(y, y, zzz);
            Fq one;
            fq_one(one);
            fq_store(base + k * kG1Jac, x);
            fq_store(base + k * kG1Jac + 6, y);
            fq_store(base + k * kG1Jac + 12, one);
        }
    }
}

// ---------------- fixed-base comb ----------------
// T[i][d-1] = d * B_i (Jacobian), one lane per entry: double-and-add over d's 8 bits.
__global__ void __launch_bounds__(64) k_g1_comb_fill(const uint64_t* __restrict__ bases, uint64_t* __restrict__ table_jac,
                                                     int e0, int e1) {
    __builtin_amdgcn_s_setprio(2);   // table work of a later part runs beside the multiply
    const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= e1) return;
    const int i = e / kCombEntries, d = e % kCombEntries + 1;
    Jac<Fq> b, acc;
    load_jac(b, bases + kG1Jac * i);
    jac_zero(acc);
#pragma unroll 1
    for (int bit = 7; bit >= 0; bit--) {
        jac_double(acc);
        if ((d >> bit) & 1) jac_add(acc, b);
    }
    store_jac(table_jac + (size_t)kG1Jac * e, acc);
}

// normalized Jacobian table -> affine (x, y) in the lazy 28-bit core's
// representation (fl.h: 14 limbs, R = 2^392), 28 u32 per entry
__global__ void __launch_bounds__(64) k_g1_comb_pack(const uint64_t* __restrict__ table_jac, uint64_t* __restrict__ table_fl,
                                                     int e0, int e1) {
    __builtin_amdgcn_s_setprio(2);   // table work of a later part runs beside the multiply
    const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= e1) return;
    const F<1> x = fl_load(table_jac + (size_t)kG1Jac * e);
    const F<1> y = fl_load(table_jac + (size_t)kG1Jac * e + 6);
    Fq z;
    fq_load(z, table_jac + (size_t)kG1Jac * e + 12);
    const bool zero = fq_is_zero(z);  // e.g. every entry of a zero base: marked, skipped by the multiply
    uint32_t* d = reinterpret_cast<uint32_t*>(table_fl + (size_t)kFlPair * e);
#pragma unroll
    for (int i = 0; i < 14; i++) {
        d[i] = zero ? kFlInfinity : x.w[i];
        d[14 + i] = zero ? kFlInfinity : y.w[i];
    }
}

// B_i = 2^(8i) g for i in [w0, w1) (Jacobian): one wave, 8 sequential
// doublings per base on the lazy core, three lanes per doubling, starting from
// g (w0 = 0) or from B_(w0-1) already in `bases`.  A zero point stays zero
// (ec.rs:299-301); a nonzero point never doubles to zero (#E(Fq) is odd).
__global__ void __launch_bounds__(64) k_g1_comb_bases(const uint64_t* __restrict__ base, uint64_t* __restrict__ bases,
                                                      int w0, int w1) {
    if (blockIdx.x != 0) return;
    // the serial chain runs beside the (chip-filling) comb multiply of earlier
    // parts: top issue priority on its SIMD, or it gets the multiply waves' leftovers
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x;
    Jac<Fq> p0;
    load_jac(p0, w0 == 0 ? base : bases + kG1Jac * (w0 - 1));
    if (fq_is_zero(p0.z)) {
        if (lane == 0)
            for (int i = w0; i < w1; i++) store_jac(bases + kG1Jac * i, p0);
        return;
    }
    FlJac p;
    p.x = fl_from_abi(p0.x);
    p.y = fl_from_abi(p0.y);
    p.z = fl_from_abi(p0.z);
#pragma unroll 1
    for (int i = w0; i < w1; i++) {
        if (i > 0) {
#pragma unroll 1
            for (int k = 0; k < 8; k++) fl_jac_double_3lane(p, lane);
        }
        if (lane == 0) {
            uint64_t* o = bases + kG1Jac * i;
            fl_store(o, p.x);
            fl_store(o + 6, p.y);
            fl_store(o + 12, p.z);
        }
    }
}

// s*g for n scalars (FrRepr, 4 x u64 canonical): out Jacobian.  Runs on the
// lazy 28-bit core (fl.h): the mixed additions are the reference's formulas,
// so the stored coordinates are the bits the 12-word core would produce.
// Windows [w0, w1) only; `first` = the accumulator starts at zero, else it
// continues from `out` (the previous window range's result, stored only if
// this range added something -- so the bits match one full-range pass).
__global__ void __launch_bounds__(64) k_g1_comb_mul(const uint64_t* __restrict__ table_fl,
                                                    const uint64_t* __restrict__ scalars,
                                                    uint64_t* __restrict__ out, size_t n, int w0, int w1,
                                                    int first) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[4];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    uint64_t* o = out + (size_t)kG1Jac * i;
    FlJac acc;
    bool untouched = true, changed = false;
    if (first) {
        acc.x = fl_zero();
        acc.y = fl_one();
        acc.z = fl_zero();
    } else {
        acc.x = fl_load(o);
        acc.y = fl_load(o + 6);
        acc.z = fl_load(o + 12);
        untouched = false;  // a zero (z == 0) is caught by fl_jac_add_mixed
    }
    int carry = 0;
#pragma unroll 1
    for (int win = 0; win < w1; win++) {
        int d = carry;
        if (win < 32) d += (int)((s[win >> 3] >> (8 * (win & 7))) & 0xff);
        carry = d > 128 ? 1 : 0;
        if (d > 128) d -= 256;
        if (d != 0 && win >= w0) {
            const int ad = d < 0 ? -d : d;
            const uint2* src = reinterpret_cast<const uint2*>(table_fl + (size_t)kFlPair * (win * kCombEntries + ad - 1));
            F<1> tx, ty;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                const uint2 a = src[k], b = src[7 + k];
                tx.w[2 * k] = a.x;
                tx.w[2 * k + 1] = a.y;
                ty.w[2 * k] = b.x;
                ty.w[2 * k + 1] = b.y;
            }
            if (tx.w[0] != kFlInfinity) {  // adding the identity is add_assign_mixed's no-op
                const F<2> oy = d < 0 ? neg(ty) : relax<2>(ty);
                fl_jac_add_mixed(acc, untouched, tx, oy);
                changed = true;
            }
        }
    }
    if (!first && !changed) return;
    if (untouched) {
        Jac<Fq> z;
        jac_zero(z);
        store_jac(o, z);
    } else {
        fl_store(o, acc.x);
        fl_store(o + 6, acc.y);
        fl_store(o + 12, acc.z);
    }
}

static inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_g1_batch_normalize(uint64_t* v, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t lanes = (n + kNormChunk - 1) / kNormChunk;
    hipLaunchKernelGGL(k_g1_batch_normalize, dim3(blocks_for(lanes, 64)), dim3(64), 0, stream, v, n);
    return hipGetLastError();
}

size_t g1_comb_workspace_words() {
    return (size_t)kG1Jac * kCombWindows + (size_t)kG1Jac * kCombWindows * kCombEntries;
}
size_t g1_comb_table_words() { return (size_t)kFlPair * kCombWindows * kCombEntries; }

static hipError_t comb_table_range(const uint64_t* base, uint64_t* table_fl, uint64_t* workspace, int w0, int w1,
                                   hipStream_t stream) {
    uint64_t* bases = workspace;
    uint64_t* table_jac = workspace + (size_t)kG1Jac * kCombWindows;
    const int e0 = w0 * kCombEntries, e1 = w1 * kCombEntries;
    hipLaunchKernelGGL(k_g1_comb_bases, dim3(1), dim3(64), 0, stream, base, bases, w0, w1);
    hipLaunchKernelGGL(k_g1_comb_fill, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, stream, bases, table_jac, e0, e1);
    const hipError_t e = launch_g1_batch_normalize(table_jac + (size_t)kG1Jac * e0, e1 - e0, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_g1_comb_pack, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, stream, table_jac, table_fl, e0,
                       e1);
    return hipGetLastError();
}

hipError_t launch_g1_comb_table(const uint64_t* base, uint64_t* table_fl, uint64_t* workspace, hipStream_t stream) {
    return comb_table_range(base, table_fl, workspace, 0, kCombWindows, stream);
}

hipError_t launch_g1_comb_mul(const uint64_t* table_fl, const uint64_t* scalars, uint64_t* out, size_t n,
                              hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_g1_comb_mul, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table_fl, scalars, out, n, 0,
                       kCombWindows, 1);
    return hipGetLastError();
}

// Table + multiply with the serial base chain overlapped, in window parts: the
// multiply over part p (accumulating into `out`) runs on `stream` while the
// chain doubles toward later parts' bases and their table entries are built.
// Same result bits as launch_g1_comb_table + launch_g1_comb_mul.
hipError_t launch_g1_fixed_base(const uint64_t* base, const uint64_t* scalars, uint64_t* out, size_t n,
                                uint64_t* table_fl, uint64_t* workspace, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    // two per-device side streams: `chain` runs the serial base chain part by
    // part; `fill` turns each finished part's bases into its table entries
    // (double-and-add, batch normalization, packing); the caller's stream
    // multiplies part p while the chain and the table work on parts > p.
    static std::mutex mu;
    static hipStream_t side[64][2] = {};
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> g(mu);
        for (int k = 0; k < 2; k++)
            if (!side[dev][k] && (e = hipStreamCreateWithFlags(&side[dev][k], hipStreamNonBlocking)) != hipSuccess)
                return e;
    }
    hipStream_t chain = side[dev][0], fill = side[dev][1], mul = stream;
    // parts of the 33 windows (PA_COMB_PARTS, 1..8): 3 measured best; more parts
    // lose, each later chain part waiting for wave slots behind the previous
    // part's multiply (profiles/r02_comb_parts.txt; a CU-masked chain stream and
    // raised wave priorities did not change that)
    static const int parts = [] {
        const char* v = getenv("PA_COMB_PARTS");
        const int k = v ? atoi(v) : 3;
        return k < 1 ? 1 : (k > 8 ? 8 : k);
    }();
    int wb[9];
    for (int p = 0; p <= parts; p++) wb[p] = (kCombWindows * p + parts - 1) / parts;
    wb[parts] = kCombWindows;
    hipEvent_t ev[2 + 2 * 8] = {};
    int made = 0;
    hipError_t err = hipSuccess;
    auto ck = [&](hipError_t x) {
        if (err == hipSuccess) err = x;
        return err == hipSuccess;
    };
    for (; made < 2 + 2 * parts; made++)
        if (!ck(hipEventCreateWithFlags(&ev[made], hipEventDisableTiming))) break;
    uint64_t* bases = workspace;
    uint64_t* table_jac = workspace + (size_t)kG1Jac * kCombWindows;
    if (ck(hipEventRecord(ev[0], stream)) && ck(hipStreamWaitEvent(chain, ev[0], 0)) &&
        ck(hipStreamWaitEvent(fill, ev[0], 0)) && (mul == stream || ck(hipStreamWaitEvent(mul, ev[0], 0)))) {
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            hipLaunchKernelGGL(k_g1_comb_bases, dim3(1), dim3(64), 0, chain, base, bases, wb[p], wb[p + 1]);
            ck(hipGetLastError()) && ck(hipEventRecord(ev[1 + 2 * p], chain));
        }
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            const int e0 = wb[p] * kCombEntries, e1 = wb[p + 1] * kCombEntries;
            if (!ck(hipStreamWaitEvent(fill, ev[1 + 2 * p], 0))) break;
            hipLaunchKernelGGL(k_g1_comb_fill, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, fill, bases, table_jac, e0,
                               e1);
            if (!ck(hipGetLastError()) || !ck(launch_g1_batch_normalize(table_jac + (size_t)kG1Jac * e0, e1 - e0, fill)))
                break;
            hipLaunchKernelGGL(k_g1_comb_pack, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, fill, table_jac, table_fl,
                               e0, e1);
            ck(hipGetLastError()) && ck(hipEventRecord(ev[2 + 2 * p], fill));
        }
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            if (!ck(hipStreamWaitEvent(mul, ev[2 + 2 * p], 0))) break;
            hipLaunchKernelGGL(k_g1_comb_mul, dim3(blocks_for(n, 64)), dim3(64), 0, mul, table_fl, scalars, out, n,
                               wb[p], wb[p + 1], p == 0 ? 1 : 0);
            ck(hipGetLastError());
        }
        // the caller's stream resumes after the last multiply
        if (err == hipSuccess && mul != stream)
            ck(hipEventRecord(ev[1 + 2 * parts], mul)) && ck(hipStreamWaitEvent(stream, ev[1 + 2 * parts], 0));
    }
    for (int k = 0; k < made; k++) (void)hipEventDestroy(ev[k]);
    return err;
}

}  // namespace pa
