// The CurveProjective / CurveAffine surface for G1 and G2 as batch kernels
// (src/lib.rs:114-234, the `curve_impl!` macro ec.rs:1-621 instantiated for
// both groups):
//   k_group_op          double / add_assign / add_assign_mixed / negate /
//                       sub_assign / into_affine / into_projective /
//                       PartialEq (a byte per item), one item
//                       per lane, the reference's exact formula sequence
//                       (curve.h) so Jacobian words are bit-identical
//   k_batch_normalize   batch_normalization (ec.rs:246-294) for G2:
//                       Montgomery's trick over chunks of points per lane
//   k_comb_*            fixed-base Wnaf::base(g, n).scalar(s_i) for G2
//                       (wnaf.rs:93-107, 169-178): the signed base-256 comb of
//                       kernels_curve.hip on the 12-word core, G2 affine table
//                       (33 x 128 entries, 845 KB) -- equal as points to the
//                       reference's wNAF (representation-independent
//                       PartialEq, ec.rs:45-85).
#include <mutex>

#include "curve.h"
#include "launch.h"

namespace pa {
namespace {

template <int G> struct Grp;
template <> struct Grp<1> {
    using F = Fq;
    static constexpr int AW = 13;  // u64 words per affine record (pa_g1_affine)
    static constexpr int JW = 18;  // u64 words per Jacobian record (pa_g1)
};
template <> struct Grp<2> {
    using F = Fq2;
    static constexpr int AW = 25;
    static constexpr int JW = 36;
};

inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// ---------------- per-op batches ----------------
template <int G, int OP>
__global__ void __launch_bounds__(64) k_group_op(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                 uint64_t* __restrict__ out, size_t n) {
    using F = typename Grp<G>::F;
    constexpr int AW = Grp<G>::AW, JW = Grp<G>::JW;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if constexpr (OP == GROUP_INTO_AFFINE) {
        Jac<F> p;
        load_jac(p, a + JW * i);
        Aff<F> r;
        jac_to_affine(r, p);
        store_aff(out + AW * i, r);
    } else if constexpr (OP == GROUP_EQ) {
        // ec.rs:45-85: X1 Z2^2 == X2 Z1^2 and Y1 Z2^3 == Y2 Z1^3; zero equals only zero
        Jac<F> p, q;
        load_jac(p, a + JW * i);
        load_jac(q, b + JW * i);
        bool eqv;
        if (jac_is_zero(p) || jac_is_zero(q)) {
            eqv = jac_is_zero(p) && jac_is_zero(q);
        } else {
            F z1, z2, t1, t2;
            sqr(z1, p.z);
            sqr(z2, q.z);
            mul(t1, p.x, z2);
            mul(t2, q.x, z1);
            eqv = eq(t1, t2);
            mul(z1, z1, p.z);
            mul(z2, z2, q.z);
            mul(z2, z2, p.y);
            mul(z1, z1, q.y);
            eqv = eqv && eq(z1, z2);
        }
        reinterpret_cast<uint8_t*>(out)[i] = eqv ? 1 : 0;
    } else if constexpr (OP == GROUP_FROM_AFFINE) {
        Aff<F> p;
        load_aff(p, a + AW * i);
        Jac<F> r;
        jac_from_affine(r, p);
        store_jac(out + JW * i, r);
    } else {
        Jac<F> s;
        load_jac(s, a + JW * i);
        if constexpr (OP == GROUP_DOUBLE) {
            jac_double(s);
        } else if constexpr (OP == GROUP_NEGATE) {
            jac_negate(s);
        } else if constexpr (OP == GROUP_ADD_MIXED) {
            Aff<F> o;
            load_aff(o, b + AW * i);
            jac_add_mixed(s, o);
        } else {
            Jac<F> o;
            load_jac(o, b + JW * i);
            if constexpr (OP == GROUP_SUB) jac_sub(s, o);
            else jac_add(s, o);
        }
        store_jac(out + JW * i, s);
    }
}

template <int G>
hipError_t group_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t s) {
    const dim3 g(blocks_for(n, 64)), bl(64);
    switch (op) {
        case GROUP_DOUBLE: hipLaunchKernelGGL((k_group_op<G, GROUP_DOUBLE>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_ADD: hipLaunchKernelGGL((k_group_op<G, GROUP_ADD>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_ADD_MIXED: hipLaunchKernelGGL((k_group_op<G, GROUP_ADD_MIXED>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_NEGATE: hipLaunchKernelGGL((k_group_op<G, GROUP_NEGATE>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_SUB: hipLaunchKernelGGL((k_group_op<G, GROUP_SUB>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_INTO_AFFINE: hipLaunchKernelGGL((k_group_op<G, GROUP_INTO_AFFINE>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_FROM_AFFINE: hipLaunchKernelGGL((k_group_op<G, GROUP_FROM_AFFINE>), g, bl, 0, s, a, b, out, n); break;
        case GROUP_EQ: hipLaunchKernelGGL((k_group_op<G, GROUP_EQ>), g, bl, 0, s, a, b, out, n); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------- batch_normalization (ec.rs:246-294) ----------------
// One lane owns CHUNK consecutive points: prefix products of the z's of the
// points that are neither zero nor normalized (ec.rs:253-261), one inversion
// (264), the backward pass (267-281), then x z^-2, y z^-3, z = 1 (284-293).
// Zero and normalized points are left bit-for-bit untouched.
template <int G, int CHUNK>
__global__ void __launch_bounds__(64) k_batch_normalize(uint64_t* __restrict__ v, size_t n) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW, W = FieldWords<F>::n;
    const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t begin = lane * CHUNK;
    if (begin >= n) return;
    const int cnt = (int)((n - begin) < (size_t)CHUNK ? (n - begin) : (size_t)CHUNK);
    uint64_t* base = v + begin * JW;
    F prod[CHUNK];
    bool skip[CHUNK];
    F acc;
    one(acc);
#pragma unroll
    for (int k = 0; k < CHUNK; k++) {
        skip[k] = true;
        if (k < cnt) {
            F z;
            load(z, base + k * JW + 2 * W);
            skip[k] = is_zero(z) || is_one(z);
            if (!skip[k]) mul(acc, acc, z);
        }
        prod[k] = acc;
    }
    F inv;
    inverse(inv, acc);  // acc is a product of nonzero z's (or one)
#pragma unroll
    for (int k = CHUNK - 1; k >= 0; k--) {
        if (k < cnt && !skip[k]) {
            F z, zinv, prev;
            load(z, base + k * JW + 2 * W);
            one(prev);
#pragma unroll
            for (int j = 0; j < CHUNK; j++)
                if (j == k - 1) prev = prod[j];
            mul(zinv, inv, prev);
            mul(inv, inv, z);
            F zz, zzz, x, y;
            sqr(zz, zinv);
            mul(zzz, zz, zinv);
            load(x, base + k * JW);
            load(y, base + k * JW + W);
            mul(x, x, zz);
            mul(y, y, zzz);
            F o;
            one(o);
            store(base + k * JW, x);
            store(base + k * JW + W, y);
            store(base + k * JW + 2 * W, o);
        }
    }
}

constexpr int kG2NormChunk = 4;

// ---------------- fixed-base comb (G2) ----------------
constexpr int kCombWindows = 33;   // 8-bit digits of a 256-bit scalar + the final carry
constexpr int kCombEntries = 128;  // |d| in 1..128

// B_i = 2^(8i) g, i in [0, 33): one wave, eight doublings per base, the seven
// products of each doubling over three lanes (jac_double_3lane).
template <int G>
__global__ void __launch_bounds__(64) k_comb_bases(const uint64_t* __restrict__ base, uint64_t* __restrict__ bases) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    const int lane = threadIdx.x;
    Jac<F> p;
    load_jac(p, base);
#pragma unroll 1
    for (int i = 0; i < kCombWindows; i++) {
        if (i > 0) {
#pragma unroll 1
            for (int k = 0; k < 8; k++) jac_double_3lane(p, lane);
        }
        if (lane == 0) store_jac(bases + JW * i, p);
    }
}

// T[i][d-1] = d B_i (Jacobian), one lane per entry: double-and-add over d's 8 bits
template <int G>
__global__ void __launch_bounds__(64) k_comb_fill(const uint64_t* __restrict__ bases, uint64_t* __restrict__ table_jac) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCombWindows * kCombEntries) return;
    const int i = e / kCombEntries, d = e % kCombEntries + 1;
    Jac<F> b, acc;
    load_jac(b, bases + JW * i);
    jac_zero(acc);
#pragma unroll 1
    for (int bit = 7; bit >= 0; bit--) {
        jac_double(acc);
        if ((d >> bit) & 1) jac_add(acc, b);
    }
    store_jac(table_jac + (size_t)JW * e, acc);
}

// normalized Jacobian entries -> affine records (zero -> infinity flag)
template <int G>
__global__ void __launch_bounds__(64) k_comb_pack(const uint64_t* __restrict__ table_jac, uint64_t* __restrict__ table) {
    using F = typename Grp<G>::F;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCombWindows * kCombEntries) return;
    Jac<F> p;
    load_jac(p, table_jac + (size_t)Grp<G>::JW * e);
    Aff<F> a;
    a.inf = jac_is_zero(p);
    a.x = p.x;
    a.y = p.y;
    store_aff(table + (size_t)Grp<G>::AW * e, a);
}

// s g = sum_i sign(d_i) T[i][|d_i|], digits d_i in [-127, 128] (carry into the
// next window), mixed additions from zero (madd-2007-bl, ec.rs:446-526)
template <int G>
__global__ void __launch_bounds__(64) k_comb_mul(const uint64_t* __restrict__ table, const uint64_t* __restrict__ scalars,
                                                 uint64_t* __restrict__ out, size_t n, int window) {
    using F = typename Grp<G>::F;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[4];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    const bool flip = wnaf_wrap(s, window);   // the reference's digits spell -(2^256 - s)
    Jac<F> acc;
    jac_zero(acc);
    int carry = 0;
#pragma unroll 1
    for (int win = 0; win < kCombWindows; win++) {
        int d = carry;
        if (win < 32) d += (int)((s[win >> 3] >> (8 * (win & 7))) & 0xff);
        carry = d > 128 ? 1 : 0;
        if (d > 128) d -= 256;
        if (d == 0) continue;
        Aff<F> t;
        load_aff(t, table + (size_t)Grp<G>::AW * (win * kCombEntries + (d < 0 ? -d : d) - 1));
        if ((d < 0) != flip && !t.inf) neg(t.y, t.y);
        jac_add_mixed(acc, t);
    }
    store_jac(out + (size_t)Grp<G>::JW * i, acc);
}

}  // namespace

hipError_t launch_group_op(int group, int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n,
                           hipStream_t stream) {
    if (n == 0) return hipSuccess;
    return group == 1 ? group_op<1>(op, a, b, out, n, stream) : group_op<2>(op, a, b, out, n, stream);
}

hipError_t launch_g2_batch_normalize(uint64_t* v, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t lanes = (n + kG2NormChunk - 1) / kG2NormChunk;
    hipLaunchKernelGGL((k_batch_normalize<2, kG2NormChunk>), dim3(blocks_for(lanes, 64)), dim3(64), 0, stream, v, n);
    return hipGetLastError();
}

size_t g2_comb_table_words() { return (size_t)Grp<2>::AW * kCombWindows * kCombEntries; }
size_t g2_comb_workspace_words() { return (size_t)Grp<2>::JW * kCombWindows * (1 + kCombEntries); }

hipError_t launch_g2_comb_table(const uint64_t* base, uint64_t* table, uint64_t* workspace, hipStream_t stream) {
    uint64_t* bases = workspace;
    uint64_t* table_jac = workspace + (size_t)Grp<2>::JW * kCombWindows;
    const unsigned entries = kCombWindows * kCombEntries;
    hipLaunchKernelGGL(k_comb_bases<2>, dim3(1), dim3(64), 0, stream, base, bases);
    hipLaunchKernelGGL(k_comb_fill<2>, dim3(blocks_for(entries, 64)), dim3(64), 0, stream, bases, table_jac);
    hipError_t e = launch_g2_batch_normalize(table_jac, entries, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_comb_pack<2>, dim3(blocks_for(entries, 64)), dim3(64), 0, stream, table_jac, table);
    return hipGetLastError();
}

hipError_t launch_g2_comb_mul(const uint64_t* table, const uint64_t* scalars, uint64_t* out, size_t n,
                              int window, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_comb_mul<2>, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table, scalars, out, n, window);
    return hipGetLastError();
}

}  // namespace pa
