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
//                       kernels_curve.hip, G2 affine table (33 x 128 entries)
//                       -- equal as points to the reference's wNAF
//                       (representation-independent PartialEq, ec.rs:45-85).
//                       Round 4: the base chain on lane-quad groups, the
//                       entries and the multiply on the lazy Fq2 (curve_fl2.h),
//                       the table in the lazy core's limbs (224 B per entry);
//                       the batch normalization stays on the 12-word core.
#include <mutex>

#include "curve.h"
#include "curve_fl2.h"
#include "dec_quad.h"
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

// B_i = 2^(8i) g, i in [0, 33), on a group of eight lane quads (dec_quad.h, as
// k_g1_comb_bases: each doubling three levels of side-by-side products, one Fq2
// coordinate per quad; round 4, was three lanes on the 12-word core) -- the
// 256-doubling chain is the G2 table's latency; canonical at the store
__global__ void __launch_bounds__(64) k_comb_bases_g2q(const uint64_t* __restrict__ base, uint64_t* __restrict__ bases) {
    constexpr int JW = Grp<2>::JW;
    if (blockIdx.x != 0) return;
    const int lane = threadIdx.x;
    Jac<Fq2> p0;
    load_jac(p0, base);
    if (jac_is_zero(p0)) {
        if (lane == 0)
            for (int i = 0; i < kCombWindows; i++) store_jac(bases + JW * i, p0);
        return;
    }
    if (lane >= 32) return;
    const dq::Lc l = dq::lctx(lane, 8);
    dq::Jq<dq::Q2> p;
    p.x = {dq::from_abi(p0.x.c0, l), dq::from_abi(p0.x.c1, l)};
    p.y = {dq::from_abi(p0.y.c0, l), dq::from_abi(p0.y.c1, l)};
    p.z = {dq::from_abi(p0.z.c0, l), dq::from_abi(p0.z.c1, l)};
#pragma unroll 1
    for (int i = 0; i < kCombWindows; i++) {
        if (i > 0) {
#pragma unroll 1
            for (int k = 0; k < 8; k++) dq::jdbl<8>(p, l);
        }
        const Fq v[6] = {dq::to_abi(p.x.c0), dq::to_abi(p.x.c1), dq::to_abi(p.y.c0),
                         dq::to_abi(p.y.c1), dq::to_abi(p.z.c0), dq::to_abi(p.z.c1)};
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 6; k++) fq_store(bases + JW * i + 6 * k, v[k]);
    }
}

// T[i][d-1] = d B_i (Jacobian), one lane per entry: double-and-add over d's 8
// bits on the lazy core's Fq2 (dbl-2009-l / add-2007-bl, curve_fl2.h; round 4),
// canonical at the store
__global__ void __launch_bounds__(64) k_comb_fill_fl2(const uint64_t* __restrict__ bases,
                                                      uint64_t* __restrict__ table_jac) {
    constexpr int JW = Grp<2>::JW;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCombWindows * kCombEntries) return;
    const int i = e / kCombEntries, d = e % kCombEntries + 1;
    const FlJac2 b = fl2_load_jac(bases + JW * i);
    FlJac2 acc = fl2_jac_zero();
#pragma unroll 1
    for (int bit = 7; bit >= 0; bit--) {
        if (!f2_is_zero(acc.z)) fl2_jac_double(acc);
        if ((d >> bit) & 1) fl2_jac_add(acc, b);
    }
    if (f2_is_zero(acc.z)) {
        Jac<Fq2> z;
        jac_zero(z);
        store_jac(table_jac + (size_t)JW * e, z);
    } else {
        fl2_store_jac(table_jac + (size_t)JW * e, acc);
    }
}

// G2 table entries in the lazy core's limbs: x.c0, x.c1, y.c0, y.c1 as 14 u32
// each, the infinity flag in bit 31 of x.c0's top limb (below 2^18 for F<1>)
constexpr int kFl2Words = 28;   // u64 per entry
__global__ void __launch_bounds__(64) k_comb_pack_fl2(const uint64_t* __restrict__ table_jac,
                                                      uint64_t* __restrict__ table) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCombWindows * kCombEntries) return;
    Jac<Fq2> p;
    load_jac(p, table_jac + (size_t)Grp<2>::JW * e);
    const bool inf = jac_is_zero(p);
    const F<1> v[4] = {fl_from_abi(p.x.c0), fl_from_abi(p.x.c1), fl_from_abi(p.y.c0), fl_from_abi(p.y.c1)};
    uint32_t* d = reinterpret_cast<uint32_t*>(table + (size_t)kFl2Words * e);
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < 14; k++) d[14 * c + k] = v[c].w[k] | (c == 0 && k == 13 && inf ? 0x80000000u : 0u);
}

// s g = sum_i sign(d_i) T[i][|d_i|], digits d_i in [-127, 128] (carry into the
// next window), mixed additions from zero (madd-2007-bl, ec.rs:446-526) on the
// lazy core's Fq2 (curve_fl2.h), canonical at the store
__global__ void __launch_bounds__(64) k_comb_mul_fl2(const uint64_t* __restrict__ table,
                                                     const uint64_t* __restrict__ scalars, uint64_t* __restrict__ out,
                                                     size_t n, int window) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[4];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    const bool flip = wnaf_wrap(s, window);   // the reference's digits spell -(2^256 - s)
    FlJac2 acc = fl2_jac_zero();
    bool untouched = true;
    int carry = 0;
#pragma unroll 1
    for (int win = 0; win < kCombWindows; win++) {
        int d = carry;
        if (win < 32) d += (int)((s[win >> 3] >> (8 * (win & 7))) & 0xff);
        carry = d > 128 ? 1 : 0;
        if (d > 128) d -= 256;
        if (d == 0) continue;
        const uint2* src = reinterpret_cast<const uint2*>(table + (size_t)kFl2Words *
                                                                     (win * kCombEntries + (d < 0 ? -d : d) - 1));
        F<1> c[4];
#pragma unroll
        for (int q = 0; q < 28; q++) {
            const uint2 t = src[q];
            c[q / 7].w[2 * (q % 7)] = t.x;
            c[q / 7].w[2 * (q % 7) + 1] = t.y;
        }
        if ((c[0].w[13] >> 31) != 0) continue;   // an infinity entry: add_assign_mixed's no-op
        const F2<1> y = {c[2], c[3]};
        const F2<2> oy = ((d < 0) != flip) ? neg(y) : relax<2>(y);
        fl2_jac_add_mixed(acc, untouched, F2<1>{c[0], c[1]}, oy);
    }
    uint64_t* o = out + (size_t)Grp<2>::JW * i;
    if (untouched) {
        Jac<Fq2> z;
        jac_zero(z);
        store_jac(o, z);
    } else {
        fl2_store_jac(o, acc);
    }
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

size_t g2_comb_table_words() { return (size_t)kFl2Words * kCombWindows * kCombEntries; }
size_t g2_comb_workspace_words() { return (size_t)Grp<2>::JW * kCombWindows * (1 + kCombEntries); }

hipError_t launch_g2_comb_table(const uint64_t* base, uint64_t* table, uint64_t* workspace, hipStream_t stream) {
    uint64_t* bases = workspace;
    uint64_t* table_jac = workspace + (size_t)Grp<2>::JW * kCombWindows;
    const unsigned entries = kCombWindows * kCombEntries;
    hipLaunchKernelGGL(k_comb_bases_g2q, dim3(1), dim3(64), 0, stream, base, bases);
    hipLaunchKernelGGL(k_comb_fill_fl2, dim3(blocks_for(entries, 64)), dim3(64), 0, stream, bases, table_jac);
    hipError_t e = launch_g2_batch_normalize(table_jac, entries, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_comb_pack_fl2, dim3(blocks_for(entries, 64)), dim3(64), 0, stream, table_jac, table);
    return hipGetLastError();
}

hipError_t launch_g2_comb_mul(const uint64_t* table, const uint64_t* scalars, uint64_t* out, size_t n,
                              int window, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_comb_mul_fl2, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table, scalars, out, n, window);
    return hipGetLastError();
}

}  // namespace pa
