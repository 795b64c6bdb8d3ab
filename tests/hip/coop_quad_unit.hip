// Test-only code object (built into pairing_amd/lib/test/coop_quad_unit.hsaco,
// never loaded by the product): the quad-cooperative field operations of
// coop_quad.h side by side with the one-lane code they must reproduce bit for
// bit (fl_gen.h leaves, fl.h red).  One case per quad of lanes:
//   in  [case][4][16] u32: operands a, b, c, d as 14 limbs + 2 zero pads
//   out [case][2][16] u32: quad result, one-lane result
//   op 0 = a*b (P1), 1 = a*b + c*d (P2), 2 = a^2 (SQ), 3 = red(a),
//   4 = gather(a) then a*b with a spread (the prologue path)
#include "../../pairing_amd/csrc/coop_quad.h"

using namespace pa;

extern "C" __global__ void __launch_bounds__(256) coop_quad_unit(const uint32_t* __restrict__ in,
                                                                 uint32_t* __restrict__ out, uint32_t n,
                                                                 uint32_t op) {
    const int tid = threadIdx.x;
    const uint32_t item = blockIdx.x * 64 + (tid >> 2);
    const quad::Ctx c = quad::ctx(tid);
    if (item >= n) return;   // whole quads leave together
    const uint32_t* x = in + (size_t)item * 64;
    uint32_t af[14], cf[14], b[4], d[4], a[4], o[4];
    for (int i = 0; i < 14; i++) {
        af[i] = x[i];
        cf[i] = x[32 + i];
    }
    for (int j = 0; j < 4; j++) {
        a[j] = x[4 * c.r + j];
        b[j] = x[16 + 4 * c.r + j];
        d[j] = x[48 + 4 * c.r + j];
    }
    if (op == 0) {
        quad::mont<false>(o, af, b, af, b, c);
    } else if (op == 1) {
        quad::mont<true>(o, af, b, cf, d, c);
    } else if (op == 2) {
        quad::mont<false>(o, af, a, af, a, c);
    } else if (op == 3) {
        for (int j = 0; j < 4; j++) o[j] = a[j];
        quad::red(o, c);
    } else {
        uint32_t g[14];
        quad::gather(g, a);
        quad::mont<false>(o, g, b, g, b, c);
    }
    uint32_t* y = out + (size_t)item * 32;
    for (int j = 0; j < 4; j++) y[4 * c.r + j] = o[j];
    if (c.lead) {
        uint32_t r[14], bf[14], df[14];
        for (int i = 0; i < 14; i++) {
            bf[i] = x[16 + i];
            df[i] = x[48 + i];
        }
        if (op == 0 || op == 4) {
            fl_mul_leaf(r, af, bf);
        } else if (op == 1) {
            fl_sop2_leaf(r, af, bf, cf, df);
        } else if (op == 2) {
            fl_sqr_leaf(r, af);
        } else {
            F<16> v;
            for (int i = 0; i < 14; i++) v.w[i] = af[i];
            const F<1> t = red(v);
            for (int i = 0; i < 14; i++) r[i] = t.w[i];
        }
        for (int i = 0; i < 14; i++) y[16 + i] = r[i];
        y[30] = y[31] = 0;
    }
}
