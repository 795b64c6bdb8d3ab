// Host-side launchers of kernels_msm.hip (variable-base scalar multiplication
// and MSM, SURVEY.md §8 f rank 3).  Device pointers, asynchronous on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pa {

// out[i] = scalars[i] * p[i] (group 1: G1, 2: G2), Jacobian, bit-exact with
// CurveAffine::mul (projective = 0, p = affine records, ec.rs:174-177, 88-95)
// or CurveProjective::mul_assign (projective = 1, p = Jacobian, ec.rs:534-553).
hipError_t launch_scalar_mul(int group, int projective, const uint64_t* p, const uint64_t* scalars, size_t n,
                             uint64_t* out, hipStream_t stream);
// out[0] = sum_i scalars[i] * bases[i] (Jacobian; equal as a point to the
// reference's sum).  `ws` must hold msm_workspace_bytes(group, n) bytes.
size_t msm_workspace_bytes(int group, size_t n);
hipError_t launch_msm(int group, const uint64_t* bases, const uint64_t* scalars, size_t n, uint64_t* out, void* ws,
                      size_t ws_bytes, hipStream_t stream);

}  // namespace pa
