// Internal host-side launchers shared between the kernel translation units
// and the C ABI (capi.hip).  All pointers are device pointers; all launches
// are asynchronous on `stream`.  Sizes are element counts.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

namespace pa {

enum FieldOp : int {
    OP_FQ_MUL = 0,
    OP_FQ_SQR,
    OP_FQ_ADD,
    OP_FQ_SUB,
    OP_FQ_INV,
    OP_FQ2_MUL,
    OP_FQ2_SQR,
    OP_FQ6_MUL,
    OP_FQ12_MUL,
    OP_FQ12_SQR,
    OP_FQ12_INV,
    OP_FQ12_FROB,
    OP_FQ12_CYC_SQR,
    OP_FQ2_INV,
    OP_FQ2_FROB,
    OP_FQ6_SQR,
    OP_FQ6_INV,
    OP_FQ6_FROB,
    OP_FQ_POW,     // b = exponent words (device), param = their count
    OP_FQ12_POW,
    OP_FQ_FROM_REPR,   // ok = 0 (Err(NotInField)) and out = 0 for a repr >= q
    OP_FQ_INTO_REPR,
};

// Generic elementwise field op: out[i] = op(a[i], b[i]); `ok` (may be null)
// receives the Option flag of inversions; `param` is the Frobenius power.
hipError_t launch_field_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, uint8_t* ok,
                           size_t n, int param, hipStream_t stream);
hipError_t launch_fq12_mul_by_014(const uint64_t* a, const uint64_t* c0, const uint64_t* c1,
                                  const uint64_t* c4, uint64_t* out, size_t n, hipStream_t stream);
// Launch shape of the HBM-streaming batch multiplies (Fq, Fr): grid cap in
// 256-thread blocks and whether the grid-stride loop prefetches.  Read once;
// PA_STREAM_BLOCKS / PA_STREAM_PREFETCH override for A/B measurements.
struct StreamCfg {
    size_t max_blocks;
    int prefetch;
};
inline StreamCfg stream_cfg() {
    static const StreamCfg c = [] {
        StreamCfg r{4096, 1};
        if (const char* e = getenv("PA_STREAM_BLOCKS")) {
            const long v = strtol(e, nullptr, 10);
            if (v > 0) r.max_blocks = (size_t)v;
        }
        if (const char* e = getenv("PA_STREAM_PREFETCH")) r.prefetch = atoi(e) != 0;
        return r;
    }();
    return c;
}

// Fq::mul_assign batch, 6 x u64 AoS in and out (config 2 kernel)
// config 2 on the SoA device layout: word j of element i at a[j n + i]
hipError_t launch_fq_mul_batch_soa(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t stream);
hipError_t launch_fq_mul_batch(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n,
                               hipStream_t stream);

hipError_t launch_g2_prepare(const uint64_t* q_aff, uint64_t* prepared, size_t n, hipStream_t stream);
hipError_t launch_miller_loop_prepared(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out,
                                       size_t n, hipStream_t stream);
// one G2Prepared (`prepared`, one record) for every G1 point of the batch:
// the line table (kernels_pairing.hip) and the generated Miller loop over it
constexpr int kSharedLineWords = 6 * 14;
constexpr int kSharedTableLines = 64;   // byte offset of line 0 (word 0: infinity flag)
constexpr size_t kSharedTableBytes = kSharedTableLines + 68 * kSharedLineWords * 4;
// what the generated shared kernel may read: it stages the lines into LDS as
// 45 rows of 512 bytes (tools/pgen/kcfg.py MillerLoopSharedCfg.pre_exec)
constexpr size_t kSharedTableAlloc = kSharedTableLines + 45 * 512;
static_assert(kSharedTableAlloc >= kSharedTableBytes, "staging rows cover the table");
hipError_t launch_shared_line_table(const uint64_t* prepared, uint32_t* table, hipStream_t stream);
hipError_t launch_miller_loop_shared_gen(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out, size_t n,
                                         hipStream_t stream);
// the pairing-only lane-pair Miller loop (homogeneous G2 steps, own line
// scaling): for e(P, Q) paths only -- its values equal the reference's Miller
// values up to Fq2 factors, which the final exponentiation removes
hipError_t launch_miller_loop_pairing_gen(int lanes, const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                          hipStream_t stream);
// the generated Miller loop of (P_i, G2Prepared_i) pairs (tools/pgen
// MillerLoopPreparedCfg): each lane reads its own record's lines
hipError_t launch_miller_loop_prepared_gen(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out,
                                           size_t n, hipStream_t stream);
// non-empty after a generated code object failed to load (names the file)
const char* gen_error_detail();
// The generated Miller-loop / final-exponentiation kernels (tools/pgen,
// gen_launch.hip).  `lanes` = 1: one pairing per lane (default); 2: a lane
// pair per pairing (A/B alternative, same results).  Each launch draws its
// spill workspace from a per-device pool keyed by stream and completion
// event, so concurrent launches on different streams never share one.
hipError_t launch_miller_loop_gen(int lanes, const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                  hipStream_t stream);
hipError_t launch_final_exp_gen(int lanes, const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n,
                                hipStream_t stream);
// Cooperative kernels (kernels_coop.hip): a workgroup per pairing, for small
// batches -- miller_loop with fused prepare / final_exponentiation, same
// results as the one-lane kernels at a fraction of their latency.  vm: 0 =
// by batch size (the four-wave quad VM up to PA_COOP_QUAD_MAX items, else the
// one-wave VM; PA_COOP_VM=1 / 4 overrides), 1 = one-wave VM, 4 = quad VM
// pairings on lane groups (kernels_pair_quad.hip, pair_quad.h): one pairing per
// 32 lanes; the Miller values are the reference's, the final exponentiation
// gives ok = 0 / zero for in == 0
hipError_t launch_pq_miller_loop(const uint64_t* p, const uint64_t* q, uint64_t* out, size_t n, hipStream_t s);
hipError_t launch_pq_final_exp(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t s);
hipError_t launch_coop_miller_loop(const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                   hipStream_t stream, int vm = 0);
// nin > 1 (with n = 1): the final exponentiation of in[0] * ... * in[nin - 1]
// (a multi-pairing's per-pair Miller values), the product on the same VM
hipError_t launch_coop_final_exp(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t stream,
                                 int vm = 0, size_t nin = 1);
// out = work[0] * ... * work[n - 1] by levels of 16-value products on the
// cooperative VM (mul12 macros, one workgroup per 16 values; `work` clobbered)
hipError_t launch_coop_fq12_product(uint64_t* work, size_t n, uint64_t* out, hipStream_t stream);
// out[0] = prod_i in[i] (Fq12), in-place tree reduction over `work` (n entries, clobbered)
hipError_t launch_fq12_product(uint64_t* work, size_t n, uint64_t* out, hipStream_t stream);

// point decoding / encoding (group 1 or 2; records in the wire format) and
// square roots (degree 1: Fq, 2: Fq2), kernels_decode.hip
// is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144) over affine records: ok = 1 / 0
hipError_t launch_subgroup_check(int group, const uint64_t* pts, size_t n, uint8_t* ok, hipStream_t stream);
hipError_t launch_decode(int group, int compressed, int checked, const uint8_t* enc, size_t n, uint64_t* out,
                         uint8_t* status, hipStream_t stream);
// 0: by batch size (<= PA_DECODE_QUAD_MAX records: the quad-group latency
// kernel), 1: one lane per record, 2: quad groups for every size
void set_decode_variant(int v);
hipError_t launch_encode(int group, int compressed, const uint64_t* in, size_t n, uint8_t* enc, hipStream_t stream);
hipError_t launch_sqrt(int degree, const uint64_t* in, size_t n, uint64_t* out, uint8_t* ok, hipStream_t stream);

// G1 batch_normalization in place (n Jacobian records of 18 u64)
hipError_t launch_g1_batch_normalize(uint64_t* v, size_t n, hipStream_t stream);
// fixed-base comb: table (g1_comb_table_words() u64) built from `base` using
// `workspace` (g1_comb_workspace_words() u64); then out[i] = scalars[i] * base
// -- the wNAF point of window `window` (wnaf_wrap in curve.h; 0 = exact s * base)
size_t g1_comb_table_words();
size_t g1_comb_workspace_words();
hipError_t launch_g1_comb_table(const uint64_t* base, uint64_t* table_aff, uint64_t* workspace, hipStream_t stream);
hipError_t launch_g1_comb_mul(const uint64_t* table_aff, const uint64_t* scalars, uint64_t* out, size_t n,
                              int window, hipStream_t stream);
// GLV form as two stages on one stream (table rows + phi rows + membership
// flag; multiply, with a double-and-add fallback for a base that failed the check)
hipError_t launch_g1_glv_table(const uint64_t* base, uint64_t* table, uint64_t* workspace, hipStream_t stream);
hipError_t launch_g1_glv_mul(const uint64_t* base, const uint64_t* table, const uint64_t* workspace, const uint64_t* scalars,
                             uint64_t* out, size_t n, int window, hipStream_t stream);
// both in one call, the GLV table's serial base chain overlapped with the
// multiply (side streams per device; equal as points)
hipError_t launch_g1_fixed_base(const uint64_t* base, const uint64_t* scalars, uint64_t* out, size_t n,
                                uint64_t* table, uint64_t* workspace, int window, hipStream_t stream);

// CurveProjective / CurveAffine per-op batches for G1 (group 1) and G2
// (group 2), kernels_group.hip.  Records: Jacobian 18 / 36 u64, affine
// 13 / 25 u64.  `b` is Jacobian for ADD / SUB, affine for ADD_MIXED, unused
// otherwise; INTO_AFFINE writes affine records, FROM_AFFINE reads them.
enum GroupOp : int {
    GROUP_DOUBLE = 0,
    GROUP_ADD,
    GROUP_ADD_MIXED,
    GROUP_NEGATE,
    GROUP_SUB,
    GROUP_INTO_AFFINE,
    GROUP_FROM_AFFINE,
    GROUP_EQ,   // PartialEq (ec.rs:45-85): `out` is one byte per item, 1 = equal
};
hipError_t launch_group_op(int group, int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n,
                           hipStream_t stream);
// G2 batch_normalization in place (n Jacobian records of 36 u64)
hipError_t launch_g2_batch_normalize(uint64_t* v, size_t n, hipStream_t stream);
// G2 fixed-base comb: table (g2_comb_table_words() u64, affine records)
// built from `base` using `workspace` (g2_comb_workspace_words() u64), then
// out[i] = scalars[i] * base (Jacobian)
size_t g2_comb_table_words();
size_t g2_comb_workspace_words();
hipError_t launch_g2_comb_table(const uint64_t* base, uint64_t* table, uint64_t* workspace, hipStream_t stream);
hipError_t launch_g2_comb_mul(const uint64_t* table, const uint64_t* scalars, uint64_t* out, size_t n,
                              int window, hipStream_t stream);

// Scalar field Fr (kernels_fr.hip).  `flag` receives the Option / Result byte
// (inverse, from_repr, sqrt) or the LegendreSymbol as int8 (0, 1, -1);
// `exp` / `exp_words` is the device-resident exponent of FR_POW.
enum FrOp : int {
    FR_MUL = 0,
    FR_SQR,
    FR_ADD,
    FR_SUB,
    FR_DBL,
    FR_NEG,
    FR_INV,
    FR_FROM_REPR,
    FR_INTO_REPR,
    FR_POW,
    FR_LEGENDRE,
    FR_SQRT,
};
hipError_t launch_fr_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, uint8_t* flag,
                        const uint64_t* exp, int exp_words, size_t n, hipStream_t stream);
hipError_t launch_fr_mul_batch(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t stream);

// ---- bit-exact Wnaf (kernels_wnaf_exact.hip) ----
constexpr int kWxMaxWindow = 20;         // fixed base: 2^19 table entries, int32 digits
constexpr int kWxMaxScalarWindow = 12;   // fixed scalar: a table per base
constexpr int kWxMaxDigits = 260;        // wnaf_form of a 256-bit repr: at most 257 digits
struct WxLayout {
    size_t meta, table, aff, c0, c1, digits, tfl, keys, perm, cnts, sort_tmp, sort_tmp_bytes, bytes;
};
// nonzero wNAF digits of one scalar at window w: nonzero digits sit at least
// w + 1 positions apart among the < kWxMaxDigits positions
constexpr int wx_max_nonzero(int w) { return kWxMaxDigits / (w + 1) + 1; }
WxLayout wx_layout(int group, size_t n, int window);
WxLayout wx_scalar_layout(int group, size_t n, int window);
hipError_t launch_wnaf_exact_fixed_base(int group, const uint64_t* base, const uint64_t* scalars, uint64_t* out,
                                        size_t n, int window, void* workspace, hipStream_t stream);
hipError_t launch_wnaf_exact_fixed_scalar(int group, const uint64_t* bases, size_t n, const uint64_t* scalar,
                                          uint64_t* out, int window, void* workspace, hipStream_t stream);

}  // namespace pa
