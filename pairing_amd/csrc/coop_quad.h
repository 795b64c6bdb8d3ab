// Quad-cooperative base-field operations for the cooperative verifier VM
// (kernels_coop.hip, Vm4): FOUR lanes share one Fq value.  Lane r = lane & 3
// holds limbs 4r .. 4r+3 of the lazy 14 x 28-bit representation (fl.h);
// lane 3 holds limbs 12, 13 and two zero pads, so a quad's four 16-byte
// pieces are exactly one 64-byte VM slot.  Limbs and carries move between the
// lanes of a quad with DPP quad_perm (broadcast of one lane, shift by one
// lane) -- the wavefront shuffle for limb / carry exchange, no LDS round trip.
//
// Every routine returns exactly the limbs of its one-lane counterpart, so the
// quad VM is bit-identical to the one-lane VM (and tools/pgen/coop.py's replay
// of the schedules stays the model of both):
//   * mont<TWO>: a*b (+ c*d) by CIOS Montgomery over 14 digit rows.  Row i
//     adds a_i * b (the quad holds b spread, a whole), takes the digit
//     m_i = (t_0 (-q^-1)) mod 2^28 from lane 0's low accumulator -- the unique
//     digit, as in the leaves' column scan (fl_gen.h) -- broadcasts it, adds
//     m_i * q and drops one limb (the dropped limb is 0 mod 2^28, its carry
//     stays in the lane).  The result (T + m q) / 2^392 is the leaves' value;
//     `norm` writes its exact base-2^28 digits (the leaves' output limbs).
//     Column bounds are the leaves': sum U_x U_y <= 17 keeps every 64-bit
//     accumulator below 2^64.
//   * red: fl.h red() -- the same quotient estimate k from limbs 12, 13 (lane
//     3, broadcast) and the exact digits of x - k q.
#pragma once
#include "fl.h"

namespace pa {
namespace quad {

constexpr int kB0 = 0x00, kB1 = 0x55, kB2 = 0xaa, kB3 = 0xff;  // quad_perm: every lane reads lane 0 / 1 / 2 / 3
constexpr int kDown = 0x39;   // quad_perm [1,2,3,0]: lane r reads lane r+1 (lane 3 reads lane 0)
constexpr int kUp = 0x93;     // quad_perm [3,0,1,2]: lane r reads lane r-1 (lane 0 reads lane 3)

template <int C>
PA_DEV uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, C, 0xf, 0xf, false);
}
PA_DEV uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// per-lane constants: r and this lane's four limbs of q (pads 0)
struct Ctx {
    int r;
    bool lead;   // r == 0: receives no carry from below
    uint32_t q[4];
};
PA_DEV Ctx ctx(int lane) {
    Ctx c;
    c.r = lane & 3;
    c.lead = c.r == 0;
#pragma unroll
    for (int j = 0; j < 4; j++) c.q[j] = 4 * c.r + j < 14 ? FL_Q[4 * c.r + j] : 0u;
    return c;
}

// whole value in every lane of the quad from the spread pieces
PA_DEV void gather(uint32_t* full, const uint32_t* v) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        full[j] = dpp<kB0>(v[j]);
        full[4 + j] = dpp<kB1>(v[j]);
        full[8 + j] = dpp<kB2>(v[j]);
    }
    full[12] = dpp<kB3>(v[0]);
    full[13] = dpp<kB3>(v[1]);
}

// exact base-2^28 digits of sum t_k 2^(28 (4r + k)) over the quad (value
// < 2^392, t_k < 2^64): a lane-local ripple, then three rounds that each move
// the carries one lane up (lane 1 is final after the first, lane 3 after the
// third); the first round's carries are up to 36 bits
PA_DEV void norm(uint32_t* o, uint64_t t0, uint64_t t1, uint64_t t2, uint64_t t3, const Ctx& c) {
    t1 += t0 >> 28;
    t2 += t1 >> 28;
    t3 += t2 >> 28;
    uint32_t o0 = (uint32_t)t0 & FL_MASK, o1 = (uint32_t)t1 & FL_MASK, o2 = (uint32_t)t2 & FL_MASK,
             o3 = (uint32_t)t3 & FL_MASK;
    const uint64_t cy = t3 >> 28;
    const uint32_t lo = dpp<kUp>((uint32_t)cy), hi = dpp<kUp>((uint32_t)(cy >> 32));
    const uint64_t v = (uint64_t)o0 + (c.lead ? 0ull : ((uint64_t)hi << 32 | lo));
    o0 = (uint32_t)v & FL_MASK;
    uint32_t k = (uint32_t)(v >> 28);
    o1 += k; k = o1 >> 28; o1 &= FL_MASK;
    o2 += k; k = o2 >> 28; o2 &= FL_MASK;
    o3 += k; k = o3 >> 28; o3 &= FL_MASK;
#pragma unroll
    for (int round = 0; round < 2; round++) {
        const uint32_t in = dpp<kUp>(k);
        o0 += c.lead ? 0u : in;
        k = o0 >> 28; o0 &= FL_MASK;
        o1 += k; k = o1 >> 28; o1 &= FL_MASK;
        o2 += k; k = o2 >> 28; o2 &= FL_MASK;
        o3 += k; k = o3 >> 28; o3 &= FL_MASK;
    }
    o[0] = o0; o[1] = o1; o[2] = o2; o[3] = o3;
}

// a b (+ c d) R'^-1, R' = 2^392: a, c whole (14 limbs), b, d this lane's
// pieces; o = this lane's piece of the leaves' output
template <bool TWO>
PA_DEV void mont(uint32_t* o, const uint32_t* a, const uint32_t* b, const uint32_t* cc, const uint32_t* d,
                 const Ctx& c) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        t0 = mad(a[i], b[0], t0);
        t1 = mad(a[i], b[1], t1);
        t2 = mad(a[i], b[2], t2);
        t3 = mad(a[i], b[3], t3);
        if (TWO) {
            t0 = mad(cc[i], d[0], t0);
            t1 = mad(cc[i], d[1], t1);
            t2 = mad(cc[i], d[2], t2);
            t3 = mad(cc[i], d[3], t3);
        }
        const uint32_t m = dpp<kB0>(((uint32_t)t0 * FL_QINV) & FL_MASK);
        t0 = mad(m, c.q[0], t0);
        t1 = mad(m, c.q[1], t1);
        t2 = mad(m, c.q[2], t2);
        t3 = mad(m, c.q[3], t3);
        // lane 0's t0 is now 0 mod 2^28: lane 3 receives 0 as its new top limb
        const uint32_t nx = dpp<kDown>((uint32_t)t0 & FL_MASK);
        t1 += t0 >> 28;
        t0 = t1;
        t1 = t2;
        t2 = t3;
        t3 = nx;
    }
    norm(o, t0, t1, t2, t3, c);
}

// fl.h red() on a spread value: x (this lane's piece, U <= 16) -> F<1> piece
PA_DEV void red(uint32_t* x, const Ctx& c) {
    const uint32_t x12 = dpp<kB3>(x[0]), x13 = dpp<kB3>(x[1]);
    const uint64_t p1 = (uint64_t)x12 * FL_KQ, p2 = (uint64_t)x13 * FL_KQ;
    const uint32_t k = (uint32_t)((p2 + (p1 >> 28)) >> 36);
    int64_t v0 = (int64_t)x[0] - (int64_t)((uint64_t)k * c.q[0]);
    int64_t v1 = (int64_t)x[1] - (int64_t)((uint64_t)k * c.q[1]);
    int64_t v2 = (int64_t)x[2] - (int64_t)((uint64_t)k * c.q[2]);
    int64_t v3 = (int64_t)x[3] - (int64_t)((uint64_t)k * c.q[3]);
    v1 += v0 >> 28;
    v2 += v1 >> 28;
    v3 += v2 >> 28;
    int32_t o0 = (int32_t)(v0 & FL_MASK), o1 = (int32_t)(v1 & FL_MASK), o2 = (int32_t)(v2 & FL_MASK),
            o3 = (int32_t)(v3 & FL_MASK);
    int32_t cy = (int32_t)(v3 >> 28);
    // signed carries one lane up per round; the value is in [0, 2q), so the
    // digits end in [0, 2^28) with zero pads and no carry out of lane 3
#pragma unroll
    for (int round = 0; round < 3; round++) {
        const int32_t in = (int32_t)dpp<kUp>((uint32_t)cy);
        int32_t w = o0 + (c.lead ? 0 : in);
        o0 = w & (int32_t)FL_MASK;
        w = o1 + (w >> 28); o1 = w & (int32_t)FL_MASK;
        w = o2 + (w >> 28); o2 = w & (int32_t)FL_MASK;
        w = o3 + (w >> 28); o3 = w & (int32_t)FL_MASK;
        cy = w >> 28;
    }
    x[0] = (uint32_t)o0; x[1] = (uint32_t)o1; x[2] = (uint32_t)o2; x[3] = (uint32_t)o3;
}

}  // namespace quad
}  // namespace pa
