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
// batch_normalization.  Montgomery's trick over chunks of kNormChunk points per
// lane with one binary-GCD inversion per chunk (bgcd.h); zero and already-normalized points
// are left bit-for-bit untouched, as in the reference (ec.rs:255-257, 271, 285).
#include <mutex>

#include "curve_fl.h"
#include "dec_quad.h"
#include "launch.h"
#include "pairing.h"

namespace pa {

constexpr int kCombWindows = 33;      // 8-bit digits of a 255-bit scalar + final carry
constexpr int kCombEntries = 128;     // |d| in 1..128
constexpr int kG1Jac = 18;            // u64 words per Jacobian G1
constexpr uint32_t kFlInfinity = 0xffffffffu;  // table entry marker: no lazy limb has all 32 bits set
constexpr int kFlPair = 14;           // u64 words per table entry: x, y as 14 x 28-bit limbs (lazy core)
constexpr int kNormChunk = 8;         // points per lane in batch_normalization (4 measured slower at 2^18)
// GLV (endomorphism) form of the comb, used when the base passes the G1
// membership test phi(P) == -[x^2] P (Scott, eprint 2021/1130; the decode
// kernel's test): phi(x, y) = (beta x, y) acts on G1 as multiplication by
// -x^2, so with s = q x^2 + rem (integer division, any 256-bit s)
//   s P = rem P + q (x^2 P) = rem P + q psi(P),  psi(x, y) = (beta x, -y),
// rem < 2^128, q < 2^129: 17 windows of each over rows T[0..16] and their
// psi images T[17..33], after a base chain of 128 doublings instead of 256.
// A base outside G1 (or off the curve) takes a 256-bit double-and-add ladder
// (k_g1_fixed_base_ladder); both paths are launched, each kernel reading the
// membership flag and returning at once when it is not its path's.
constexpr int kGlvWindows = 17;
constexpr int kTableRows = 2 * kGlvWindows;   // >= kCombWindows
static_assert(kTableRows >= kCombWindows, "table rows");
constexpr uint64_t kX2Lo = 0x0000000100000000ull, kX2Hi = 0xac45a4010001a402ull;   // x^2 = 0xd201000000010000^2
// beta (a primitive cube root of unity in Fq, Montgomery R = 2^384), the decode kernel's kBeta
__constant__ const uint64_t kGlvBeta[6] = {0x30f1361b798a64e8ULL, 0xf3b8ddab7ece5a2aULL, 0x16a8ca3ac61577f7ULL,
                                           0xc26a2ff874fd029bULL, 0x3636b76660701c6eULL, 0x051ba4ab241b6160ULL};
constexpr uint32_t kGateGlv = 1, kGatePlain = 0;   // membership flag values

// ---------------- batch_normalization ----------------
template <int kNormChunk>
PA_DEV void g1_batch_normalize_chunk(uint64_t* __restrict__ v, size_t n) {
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
__global__ void __launch_bounds__(64) k_g1_batch_normalize(uint64_t* __restrict__ v, size_t n) {
    g1_batch_normalize_chunk<kNormChunk>(v, n);
}
// ---------------- fixed-base comb ----------------
// T[i][d-1] = d * B_i as affine (x, y) in the lazy 28-bit core's
// representation (fl.h: 14 limbs, R = 2^392, 28 u32 per entry), one lane per
// entry: double-and-add over d's bits on the lazy core, then the lane's own
// inversion of z (binary GCD) -- one launch instead of double-and-add, batch
// normalization and packing (the table's rows sit on the multiply's critical
// path, and every lane's inversion runs at once).  The entries are other
// representatives (< 2q) of the same affine values; the multiply's outputs are
// canonical at the store, so its bits do not change.  `phi_rows`: the GLV
// table, row 17 + i also gets phi(T[i]) = (beta x, y).
__global__ void __launch_bounds__(64) k_g1_comb_entries(const uint64_t* __restrict__ bases,
                                                        uint64_t* __restrict__ table_fl, int e0, int e1,
                                                        int phi_rows) {
    __builtin_amdgcn_s_setprio(2);   // table work of a later part runs beside the multiply
    const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= e1) return;
    const int i = e / kCombEntries, d = e % kCombEntries + 1;
    Jac<Fq> b0;
    load_jac(b0, bases + kG1Jac * i);
    uint32_t* o = reinterpret_cast<uint32_t*>(table_fl + (size_t)kFlPair * e);
    uint32_t* op = o + 2 * kFlPair * kGlvWindows * kCombEntries;
    if (fq_is_zero(b0.z)) {  // zero base: every entry marked, skipped by the multiply
#pragma unroll
        for (int k = 0; k < 28; k++) {
            o[k] = kFlInfinity;
            if (phi_rows) op[k] = kFlInfinity;
        }
        return;
    }
    // from d's top bit (d < 2^8 < the order: no intermediate is zero)
    const FlJac b = {fl_from_abi(b0.x), fl_from_abi(b0.y), fl_from_abi(b0.z)};
    FlJac acc = b;
    const int top = 31 - __builtin_clz(d);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; bit--) {
        fl_jac_double(acc);
        if ((d >> bit) & 1) fl_jac_add(acc, b);
    }
    Fq zi;
    fq_inv(zi, fl_to_abi(acc.z));
    const F<1> zf = fl_from_abi(zi);
    const F<1> zz = sqr(zf);
    const F<1> x = mul(acc.x, zz);
    const F<1> y = mul(acc.y, mul(zz, zf));
#pragma unroll
    for (int k = 0; k < 14; k++) {
        o[k] = x.w[k];
        o[14 + k] = y.w[k];
    }
    if (phi_rows) {
        Fq beta;
        fq_load(beta, kGlvBeta);
        const F<1> bx = mul(x, fl_from_abi(beta));
#pragma unroll
        for (int k = 0; k < 14; k++) {
            op[k] = bx.w[k];
            op[14 + k] = y.w[k];
        }
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
    // the doublings on a group of four lane quads (dec_quad.h: three levels of
    // side-by-side quad products per doubling); lanes 16..63 idle
    if (lane >= 16) return;
    const dq::Lc l = dq::lctx(lane, 4);
    dq::Jq<dq::Q> p{dq::from_abi(p0.x, l), dq::from_abi(p0.y, l), dq::from_abi(p0.z, l)};
#pragma unroll 1
    for (int i = w0; i < w1; i++) {
        if (i > 0) {
#pragma unroll 1
            for (int k = 0; k < 8; k++) dq::jdbl<4>(p, l);
        }
        const Fq x = dq::to_abi(p.x), y = dq::to_abi(p.y), z = dq::to_abi(p.z);
        if (lane == 0) {
            uint64_t* o = bases + kG1Jac * i;
            fq_store(o, x);
            fq_store(o + 6, y);
            fq_store(o + 12, z);
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
                                                    int first, int window) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[4];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    const bool flip = wnaf_wrap(s, window);   // the reference's digits spell -(2^256 - s)
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
                const F<2> oy = (d < 0) != flip ? neg(ty) : relax<2>(ty);
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

// GLV membership flag: *flag = kGateGlv iff phi(P) == -[x^2] P (or P is
// zero: every path gives zero), computed as [|x|]([|x|] P) by two 64-bit
// double-and-add chains on the lazy core (three lanes per doubling), then
// compared in Jacobian coordinates.  One wave; runs beside the GLV table
// build and multiply, and only the fallback's launches wait for it.
__global__ void __launch_bounds__(64) k_g1_glv_check(const uint64_t* __restrict__ base, uint32_t* __restrict__ flag) {
    if (blockIdx.x != 0) return;
    const int lane = threadIdx.x;
    Jac<Fq> p0;
    load_jac(p0, base);
    uint32_t glv = kGateGlv;
    if (!fq_is_zero(p0.z)) {
        FlJac p;
        p.x = fl_from_abi(p0.x);
        p.y = fl_from_abi(p0.y);
        p.z = fl_from_abi(p0.z);
        constexpr uint64_t kX = 0xd201000000010000ull;   // |x|, the BLS parameter (x < 0)
        FlJac a = p, b = p;
#pragma unroll 1
        for (int round = 0; round < 2; round++) {   // a = |x| b, then b = a
#pragma unroll 1
            for (int bit = 62; bit >= 0; bit--) {
                if (!fl_is_zero(a.z)) fl_jac_double_3lane(a, lane);
                if ((kX >> bit) & 1) fl_jac_add(a, b);
            }
            b = a;
        }
        // phi(P) = (beta X_P, Y_P, Z_P) == -(X_A, Y_A, Z_A), A = [x^2] P
        Fq beta;
        fq_load(beta, kGlvBeta);
        const F<1> za2 = sqr(a.z), zp2 = sqr(p.z);
        const bool xs = fl_eq(mul(mul(p.x, fl_from_abi(beta)), za2), mul(a.x, zp2));
        const bool ys = fl_is_zero(add(mul(mul(p.y, a.z), za2), mul(mul(a.y, p.z), zp2)));
        glv = (!fl_is_zero(a.z) && xs && ys) ? kGateGlv : kGatePlain;
    }
    if (lane == 0) *flag = glv;
}

// s = q x^2 + rem for a 256-bit s (Barrett, HAC 14.42 without the final
// corrections): q = floor(floor(s / 2^127) m / 2^129), m = floor(2^256 / x^2),
// never above floor(s / x^2), so rem = s - q x^2 is in [0, 2 x^2) < 2^129
// (one correction short at most) and q < 2^129: 17 signed base-256 digits each.
PA_DEV void glv_split(const uint64_t s[4], uint64_t rem[3], uint64_t q[3]) {
    constexpr uint64_t m[3] = {0x63f6e522f6cfee2eull, 0x7c6becf1e01faaddull, 1};
    const uint64_t t[3] = {(s[1] >> 63) | (s[2] << 1), (s[2] >> 63) | (s[3] << 1), s[3] >> 63};
    uint64_t pr[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const unsigned __int128 v = (unsigned __int128)t[i] * m[j] + pr[i + j] + c;
            pr[i + j] = (uint64_t)v;
            c = (uint64_t)(v >> 64);
        }
        pr[i + 3] = c;
    }
    q[0] = (pr[2] >> 1) | (pr[3] << 63);
    q[1] = (pr[3] >> 1) | (pr[4] << 63);
    q[2] = (pr[4] >> 1) | (pr[5] << 63);
    // q x^2 mod 2^192
    const unsigned __int128 a0 = (unsigned __int128)q[0] * kX2Lo;
    const unsigned __int128 a1 = (unsigned __int128)q[0] * kX2Hi + (uint64_t)(a0 >> 64);
    const unsigned __int128 b1 = (unsigned __int128)q[1] * kX2Lo + (uint64_t)a1;
    const uint64_t w0 = (uint64_t)a0, w1 = (uint64_t)b1;
    const uint64_t w2 = (uint64_t)(a1 >> 64) + (uint64_t)(b1 >> 64) + q[1] * kX2Hi + q[2] * kX2Lo;
    unsigned __int128 d = (unsigned __int128)s[0] - w0;
    rem[0] = (uint64_t)d;
    d = (unsigned __int128)s[1] - w1 - (uint64_t)((d >> 64) & 1);
    rem[1] = (uint64_t)d;
    rem[2] = s[2] - w2 - (uint64_t)((d >> 64) & 1);
}

// next signed base-256 digit of a little-endian 3-word value (window `win`)
PA_DEV int glv_digit(const uint64_t v[3], int win, int& carry) {
    int d = carry + (int)((v[win >> 3] >> (8 * (win & 7))) & 0xff);
    carry = d > 128 ? 1 : 0;
    if (d > 128) d -= 256;
    return d;
}

PA_DEV void comb_add_entry(FlJac& acc, bool& untouched, bool& changed, const uint64_t* table_fl, int row, int d,
                           bool flip) {
    const int ad = d < 0 ? -d : d;
    const uint2* src = reinterpret_cast<const uint2*>(table_fl + (size_t)kFlPair * (row * kCombEntries + ad - 1));
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
        const F<2> oy = ((d < 0) != flip) ? neg(ty) : relax<2>(ty);
        fl_jac_add_mixed(acc, untouched, tx, oy);
        changed = true;
    }
}

// GLV comb multiply, windows [w0, w1) of both halves: s g = rem g + q psi(g)
// with psi(g) = -phi(g), so a q digit d adds -d phi(T[win][|d|]) from row 17 + win.
// Same accumulate/store protocol as k_g1_comb_mul.
// (4 waves per SIMD via launch bounds, <= 128 VGPRs, spills: 1.57 -> 2.75 ms)
__global__ void __launch_bounds__(64) k_g1_glv_mul(const uint64_t* __restrict__ table_fl,
                                                   const uint64_t* __restrict__ scalars, uint64_t* __restrict__ out,
                                                   size_t n, int w0, int w1, int first,
                                                   const uint32_t* __restrict__ gate, int window) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (gate && *gate != kGateGlv)) return;
    uint64_t s[4], rem[3], q[3];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    const int neg = wnaf_wrap(s, window) ? 1 : 0;   // -(2^256 - s): every digit negated
    glv_split(s, rem, q);
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
        untouched = false;
    }
    int cr = 0, cq = 0;
    for (int win = 0; win < w0; win++) {
        glv_digit(rem, win, cr);
        glv_digit(q, win, cq);
    }
    // one add site for both halves (two inlined copies of the mixed addition
    // outgrow the instruction cache): step 2 win + h, h = 1 the q digit
    int dq = 0;
#pragma unroll 1
    for (int step = 2 * w0; step < 2 * w1; step++) {
        const int win = step >> 1;
        int d;
        if ((step & 1) == 0) {
            d = glv_digit(rem, win, cr);
            dq = glv_digit(q, win, cq);
        } else {
            d = dq;
        }
        if (d != 0)
            comb_add_entry(acc, untouched, changed, table_fl, (step & 1) * kGlvWindows + win, d, (step & 1) ^ neg);
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

// s * P by double-and-add over the 256 scalar bits with full Jacobian
// additions (add-2007-bl, ec.rs:356-444, doubling and zero cases inside), one
// lane per scalar, for the GLV path's fallback (*gate == kGatePlain)
__global__ void __launch_bounds__(64) k_g1_fixed_base_ladder(const uint64_t* __restrict__ base,
                                                             const uint64_t* __restrict__ scalars,
                                                             uint64_t* __restrict__ out, size_t n,
                                                             const uint32_t* __restrict__ gate, int window) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || *gate != kGatePlain) return;
    uint64_t s[4];
#pragma unroll
    for (int w = 0; w < 4; w++) s[w] = scalars[4 * i + w];
    FlJac p = fl_load_jac(base);
    if (wnaf_wrap(s, window)) p.y = red(neg(p.y));   // (2^256 - s) (-P)
    FlJac acc = {fl_zero(), fl_one(), fl_zero()};
#pragma unroll 1
    for (int bit = 255; bit >= 0; bit--) {
        if (!fl_is_zero(acc.z)) fl_jac_double(acc);
        if ((s[bit >> 6] >> (bit & 63)) & 1) fl_jac_add(acc, p);
    }
    uint64_t* o = out + (size_t)kG1Jac * i;
    if (fl_is_zero(acc.z)) {
        Jac<Fq> z;
        jac_zero(z);
        store_jac(o, z);
    } else {
        fl_store_jac(o, acc);
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
    // the chain's bases, then one u64 holding the GLV membership flag
    return (size_t)kG1Jac * kCombWindows + 1;
}
size_t g1_comb_table_words() { return (size_t)kFlPair * kTableRows * kCombEntries; }

static uint32_t* glv_flag(const uint64_t* workspace) {
    const uint64_t* f = workspace + (size_t)kG1Jac * kCombWindows;
    return reinterpret_cast<uint32_t*>(const_cast<uint64_t*>(f));
}

// bases + table rows [w0, w1) on one stream; `phi_rows` also writes the GLV rows 17 + i
static hipError_t comb_table_range(const uint64_t* base, uint64_t* table_fl, uint64_t* workspace, int w0, int w1,
                                   int phi_rows, hipStream_t stream) {
    uint64_t* bases = workspace;
    const int e0 = w0 * kCombEntries, e1 = w1 * kCombEntries;
    hipLaunchKernelGGL(k_g1_comb_bases, dim3(1), dim3(64), 0, stream, base, bases, w0, w1);
    hipLaunchKernelGGL(k_g1_comb_entries, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, stream, bases, table_fl, e0, e1,
                       phi_rows);
    return hipGetLastError();
}

hipError_t launch_g1_comb_table(const uint64_t* base, uint64_t* table_fl, uint64_t* workspace, hipStream_t stream) {
    return comb_table_range(base, table_fl, workspace, 0, kCombWindows, 0, stream);
}

hipError_t launch_g1_comb_mul(const uint64_t* table_fl, const uint64_t* scalars, uint64_t* out, size_t n,
                              int window, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_g1_comb_mul, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table_fl, scalars, out, n, 0,
                       kCombWindows, 1, window);
    return hipGetLastError();
}

// the GLV path's fallback, one launch that returns at once unless the base
// failed the membership check (a base outside G1: the reference's types never
// hold one, so throughput does not matter there, the launch count does)
static hipError_t glv_fallback(const uint64_t* base, const uint64_t* workspace, const uint64_t* scalars, uint64_t* out,
                               size_t n, int window, hipStream_t stream) {
    hipLaunchKernelGGL(k_g1_fixed_base_ladder, dim3(blocks_for(n, 64)), dim3(64), 0, stream, base, scalars, out, n,
                       glv_flag(workspace), window);
    return hipGetLastError();
}

hipError_t launch_g1_glv_table(const uint64_t* base, uint64_t* table_fl, uint64_t* workspace, hipStream_t stream) {
    hipLaunchKernelGGL(k_g1_glv_check, dim3(1), dim3(64), 0, stream, base, glv_flag(workspace));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return comb_table_range(base, table_fl, workspace, 0, kGlvWindows, 1, stream);
}

hipError_t launch_g1_glv_mul(const uint64_t* base, const uint64_t* table_fl, const uint64_t* workspace, const uint64_t* scalars,
                             uint64_t* out, size_t n, int window, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_g1_glv_mul, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table_fl, scalars, out, n, 0,
                       kGlvWindows, 1, glv_flag(workspace), window);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return glv_fallback(base, workspace, scalars, out, n, window, stream);
}

// Table + multiply in one call, GLV form with the serial base chain
// overlapped, in window parts of the 17 GLV windows: the chain (side stream 0)
// doubles toward part p + 1's bases while side stream 1 builds part p's rows
// and their phi images and the caller's stream multiplies part p.  Side
// stream 2 runs the membership check from the start; after the last GLV
// multiply the caller's stream waits for it and runs the double-and-add ladder
// (k_g1_fixed_base_ladder), which returns at once unless the check failed.
// Equal as points to launch_g1_comb_table + launch_g1_comb_mul.
hipError_t launch_g1_fixed_base(const uint64_t* base, const uint64_t* scalars, uint64_t* out, size_t n,
                                uint64_t* table_fl, uint64_t* workspace, int window, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    static std::mutex mu;
    static hipStream_t side[64][3] = {};
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> g(mu);
        for (int k = 0; k < 3; k++)
            if (!side[dev][k] && (e = hipStreamCreateWithFlags(&side[dev][k], hipStreamNonBlocking)) != hipSuccess)
                return e;
    }
    hipStream_t chain = side[dev][0], fill = side[dev][1], check = side[dev][2], mul = stream;
    static const bool serial = getenv("PA_COMB_SERIAL") && atoi(getenv("PA_COMB_SERIAL")) != 0;
    if (serial) chain = fill = check = stream;   // measurement only: every kernel in order on the caller's stream
    // window boundaries of the parts (PA_COMB_SPLIT, e.g. "5" or "2,7": the
    // first window of every part after the first); "5" (5 + 12 windows)
    // measured best of the even and two-part splits (profiles/r02_glv_comb.txt)
    // -- a short first part starts the multiply early, a long second one hides
    // the rest of the chain and its rows behind the first part's multiply
    struct Split {
        int parts = 1, wb[9] = {0};
    };
    static const Split split = [] {
        Split r;
        const char* v = getenv("PA_COMB_SPLIT");
        const char* t = v ? v : "5";
        while (*t && r.parts < 8) {
            char* end = nullptr;
            const long w = strtol(t, &end, 10);
            if (end == t) break;
            if (w > r.wb[r.parts - 1] && w < kGlvWindows) r.wb[r.parts++] = (int)w;
            t = *end == ',' ? end + 1 : end;
        }
        r.wb[r.parts] = kGlvWindows;
        return r;
    }();
    const int parts = split.parts;
    const int* wb = split.wb;
    // ev[0]: start; ev[1 + 2p]: chain part p done; ev[2 + 2p]: rows of part p done; ev[1 + 2 parts]: check done
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
    uint32_t* flag = glv_flag(workspace);
    if (ck(hipEventRecord(ev[0], stream)) && ck(hipStreamWaitEvent(chain, ev[0], 0)) &&
        ck(hipStreamWaitEvent(fill, ev[0], 0)) && ck(hipStreamWaitEvent(check, ev[0], 0))) {
        hipLaunchKernelGGL(k_g1_glv_check, dim3(1), dim3(64), 0, check, base, flag);
        ck(hipGetLastError()) && ck(hipEventRecord(ev[1 + 2 * parts], check));
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            hipLaunchKernelGGL(k_g1_comb_bases, dim3(1), dim3(64), 0, chain, base, bases, wb[p], wb[p + 1]);
            ck(hipGetLastError()) && ck(hipEventRecord(ev[1 + 2 * p], chain));
        }
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            const int e0 = wb[p] * kCombEntries, e1 = wb[p + 1] * kCombEntries;
            if (!ck(hipStreamWaitEvent(fill, ev[1 + 2 * p], 0))) break;
            hipLaunchKernelGGL(k_g1_comb_entries, dim3(blocks_for(e1 - e0, 64)), dim3(64), 0, fill, bases, table_fl,
                               e0, e1, 1);
            ck(hipGetLastError()) && ck(hipEventRecord(ev[2 + 2 * p], fill));
        }
        for (int p = 0; p < parts && err == hipSuccess; p++) {
            if (!ck(hipStreamWaitEvent(mul, ev[2 + 2 * p], 0))) break;
            hipLaunchKernelGGL(k_g1_glv_mul, dim3(blocks_for(n, 64)), dim3(64), 0, mul, table_fl, scalars, out, n,
                               wb[p], wb[p + 1], p == 0 ? 1 : 0, nullptr, window);
            ck(hipGetLastError());
        }
        // fallback: the double-and-add ladder, live only when the base failed the check
        if (err == hipSuccess && ck(hipStreamWaitEvent(mul, ev[1 + 2 * parts], 0)))
            ck(glv_fallback(base, workspace, scalars, out, n, window, mul));
    }
    for (int k = 0; k < made; k++) (void)hipEventDestroy(ev[k]);
    return err;
}

}  // namespace pa
