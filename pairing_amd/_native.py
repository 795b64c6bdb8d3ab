"""ctypes binding of the HIP library pairing_amd/lib/libpairing_amd.so.

This is the only way the Python package reaches compute: every function
below ends in a HIP kernel on the current device.  There is no CPU fallback;
if the library is missing or fails to load, import raises.

Array convention (numpy uint64, C-contiguous, the ABI layout of
include/pairing_amd.h):
  Fq (n,6)  Fq2 (n,12)  Fq6 (n,36)  Fq12 (n,72)
  G1Affine (n,13)  G2Affine (n,25)  G1 (n,18)  G2 (n,36)  G2Prepared (n,2449)
  Fr / FrRepr (n,4)
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PA_LIB_PATH: an A/B build of the same sources (tools/curve_variants.sh); default the in-tree library
LIB_PATH = os.environ.get("PA_LIB_PATH") or os.path.join(HERE, "lib", "libpairing_amd.so")

W_FQ, W_FQ2, W_FQ6, W_FQ12 = 6, 12, 36, 72
W_G1A, W_G1, W_G2A, W_G2 = 13, 18, 25, 36
W_G2P = 68 * 3 * 12 + 1
W_FR = 4

PA_OK = 0


class PairingError(RuntimeError):
    """A negative status code from the C ABI (see include/pairing_amd.h)."""


def _share_torch_hip_runtime():
    """Make this library and torch use ONE HIP runtime in the process.

    The torch wheel ships its own libamdhip64.so (soname libamdhip64.so.7,
    loaded by torch's libc10_hip through RPATH $ORIGIN), while
    libpairing_amd.so needs libamdhip64.so.7 from /opt/rocm.  Imported after
    torch, this library binds to torch's runtime by soname; imported before
    it, two runtimes would end up in the process and torch's would find no
    device.  So torch's runtime file is loaded first (without importing
    torch): a later `import torch` then reuses it (same file), and the
    stream handles and device pointers of the device.py layer belong to the
    runtime that launches our kernels.  PA_SYSTEM_HIP=1 keeps /opt/rocm's."""
    if "torch" in sys.modules or os.environ.get("PA_SYSTEM_HIP") == "1":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def _load():
    _share_torch_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "pairing_amd: HIP library %s is missing -- build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)" % LIB_PATH)
    return ctypes.CDLL(LIB_PATH)


_lib = _load()
_P = ctypes.c_void_p
_N = ctypes.c_size_t

# Every exported entry point with its argument types (all return int).
_SIGS = {
    "pa_device_count": [ctypes.POINTER(ctypes.c_int)],
    "pa_set_device": [ctypes.c_int],
    "pa_synchronize": [],
    "pa_set_pairing_kernel": [ctypes.c_int],
    "pa_set_decode_kernel": [ctypes.c_int],
    "pa_fq_mul_batch": [_P, _P, _P, _N],
    "pa_fq_square_batch": [_P, _P, _N],
    "pa_fq_add_batch": [_P, _P, _P, _N],
    "pa_fq_sub_batch": [_P, _P, _P, _N],
    "pa_fq_inverse_batch": [_P, _P, _P, _N],
    "pa_fq_from_repr_batch": [_P, _P, _P, _N],
    "pa_fq_into_repr_batch": [_P, _P, _N],
    "pa_fq2_mul_batch": [_P, _P, _P, _N],
    "pa_fq2_square_batch": [_P, _P, _N],
    "pa_fq6_mul_batch": [_P, _P, _P, _N],
    "pa_fq12_mul_batch": [_P, _P, _P, _N],
    "pa_fq12_square_batch": [_P, _P, _N],
    "pa_fq12_inverse_batch": [_P, _P, _P, _N],
    "pa_fq12_frobenius_map_batch": [_P, _P, _N, _N],
    "pa_fq12_cyclotomic_square_batch": [_P, _P, _N],
    "pa_fq12_mul_by_014_batch": [_P, _P, _P, _P, _P, _N],
    "pa_g2_prepare_batch": [_P, _P, _N],
    "pa_miller_loop_batch": [_P, _P, _P, _N],
    "pa_miller_loop_shared_prepared": [_P, _N, _P, _P],
    "pa_multi_miller_loop": [_P, _P, _N, _P],
    "pa_final_exponentiation_batch": [_P, _P, _P, _N],
    "pa_pairing_batch": [_P, _P, _P, _N],
    "pa_g1_batch_normalization": [_P, _N],
    "pa_g1_wnaf_fixed_base": [_P, _P, _N, _P],
    "pa_g1_wnaf_fixed_base_window": [_P, _P, _N, ctypes.c_int, _P],
    "pa_g1_batch_normalization_device": [_P, _N, _P],
    "pa_g1_fixed_base_table_device": [_P, _P, _P, _P],
    "pa_g1_fixed_base_mul_device": [_P, _P, _P, _N, _P],
    "pa_g1_wnaf_fixed_base_device": [_P, _P, _P, _N, _P, _P, _P],
    "pa_g1_wnaf_fixed_base_window_device": [_P, _P, _P, _N, ctypes.c_int, _P, _P, _P],
    "pa_g1_fixed_base_glv_table_device": [_P, _P, _P, _P],
    "pa_g1_fixed_base_glv_mul_device": [_P, _P, _P, _P, _P, _N, _P],
    "pa_fq_mul_batch_device": [_P, _P, _P, _N, _P],
    "pa_fq_mul_batch_soa_device": [_P, _P, _P, _N, _P],
    "pa_miller_loop_fused_batch_device": [_P, _P, _P, _N, _P],
    "pa_pairing_miller_loop_batch_device": [_P, _P, _P, _N, _P],
    "pa_g2_prepare_batch_device": [_P, _P, _N, _P],
    "pa_miller_loop_batch_device": [_P, _P, _P, _N, _P],
    "pa_miller_loop_shared_prepared_device": [_P, _N, _P, _P, _P],
    "pa_final_exponentiation_batch_device": [_P, _P, _P, _N, _P],
    "pa_pairing_batch_device": [_P, _P, _P, _P, _N, _P],
    "pa_g1_decode_batch": [_P, _N, ctypes.c_int, ctypes.c_int, _P, _P],
    "pa_g2_decode_batch": [_P, _N, ctypes.c_int, ctypes.c_int, _P, _P],
    "pa_g1_encode_batch": [_P, _N, ctypes.c_int, _P],
    "pa_g2_encode_batch": [_P, _N, ctypes.c_int, _P],
    "pa_fq_sqrt_batch": [_P, _P, _P, _N],
    "pa_fq2_sqrt_batch": [_P, _P, _P, _N],
    "pa_multi_miller_loop_affine": [_P, _P, _N, _P],
    "pa_multi_pairing": [_P, _P, _N, _P, _P],
    "pa_pairing_batch_multi_gpu": [_P, _P, _P, _N, ctypes.c_int],
    "pa_g1_decode_batch_device": [_P, _N, ctypes.c_int, ctypes.c_int, _P, _P, _P],
    "pa_g2_decode_batch_device": [_P, _N, ctypes.c_int, ctypes.c_int, _P, _P, _P],
    "pa_fr_mul_batch": [_P, _P, _P, _N],
    "pa_fr_square_batch": [_P, _P, _N],
    "pa_fr_add_batch": [_P, _P, _P, _N],
    "pa_fr_sub_batch": [_P, _P, _P, _N],
    "pa_fr_double_batch": [_P, _P, _N],
    "pa_fr_negate_batch": [_P, _P, _N],
    "pa_fr_inverse_batch": [_P, _P, _P, _N],
    "pa_fr_from_repr_batch": [_P, _P, _P, _N],
    "pa_fr_into_repr_batch": [_P, _P, _N],
    "pa_fr_pow_batch": [_P, _P, _N, _P, _N],
    "pa_fr_legendre_batch": [_P, _P, _N],
    "pa_fr_sqrt_batch": [_P, _P, _P, _N],
    "pa_fr_mul_batch_device": [_P, _P, _P, _N, _P],
    "pa_g1_affine_mul_batch": [_P, _P, _P, _N],
    "pa_g2_affine_mul_batch": [_P, _P, _P, _N],
    "pa_g1_mul_assign_batch": [_P, _P, _P, _N],
    "pa_g2_mul_assign_batch": [_P, _P, _P, _N],
    "pa_g1_multiexp": [_P, _P, _N, _P],
    "pa_g2_multiexp": [_P, _P, _N, _P],
    "pa_g1_multiexp_device": [_P, _P, _N, _P, _P, _N, _P],
    "pa_g2_multiexp_device": [_P, _P, _N, _P, _P, _N, _P],
}
for _g in (1, 2):
    for _op in ("double", "negate", "into_affine", "into_projective"):
        _SIGS["pa_g%d_%s_batch" % (_g, _op)] = [_P, _P, _N]
    for _op in ("add", "add_mixed", "sub", "eq"):
        _SIGS["pa_g%d_%s_batch" % (_g, _op)] = [_P, _P, _P, _N]
    for _op in ("double", "into_affine"):
        _SIGS["pa_g%d_%s_batch_device" % (_g, _op)] = [_P, _P, _N, _P]
    for _op in ("add", "add_mixed", "eq"):
        _SIGS["pa_g%d_%s_batch_device" % (_g, _op)] = [_P, _P, _P, _N, _P]
    _SIGS["pa_g%d_recommended_wnaf_for_scalar" % _g] = [_P]
    _SIGS["pa_g%d_wnaf_fixed_base_exact" % _g] = [_P, _P, _N, ctypes.c_int, _P]
    _SIGS["pa_g%d_wnaf_fixed_scalar_exact" % _g] = [_P, _N, _P, ctypes.c_int, _P]
    _SIGS["pa_g%d_wnaf_fixed_base_exact_device" % _g] = [_P, _P, _P, _N, ctypes.c_int, _P, _N, _P]
    _SIGS["pa_g%d_wnaf_fixed_scalar_exact_device" % _g] = [_P, _N, _P, _P, ctypes.c_int, _P, _N, _P]
    _SIGS["pa_g%d_recommended_wnaf_for_num_scalars" % _g] = [_N]
_SIGS.update({
    "pa_fq2_inverse_batch": [_P, _P, _P, _N],
    "pa_multi_pairing_device": [_P, _P, _N, _P, _P, _P, _P],
    "pa_fq2_frobenius_map_batch": [_P, _P, _N, _N],
    "pa_fq6_square_batch": [_P, _P, _N],
    "pa_fq6_inverse_batch": [_P, _P, _P, _N],
    "pa_fq6_frobenius_map_batch": [_P, _P, _N, _N],
    "pa_fq_pow_batch": [_P, _P, _N, _P, _N],
    "pa_fq12_pow_batch": [_P, _P, _N, _P, _N],
    "pa_g2_batch_normalization": [_P, _N],
    "pa_g2_batch_normalization_device": [_P, _N, _P],
    "pa_g2_wnaf_fixed_base": [_P, _P, _N, _P],
    "pa_g2_wnaf_fixed_base_window": [_P, _P, _N, ctypes.c_int, _P],
    "pa_g2_wnaf_fixed_base_device": [_P, _P, _P, _N, _P, _P, _P],
    "pa_g2_wnaf_fixed_base_window_device": [_P, _P, _P, _N, ctypes.c_int, _P, _P, _P],
})
for _name, _args in _SIGS.items():
    _fn = getattr(_lib, _name)
    _fn.argtypes = _args
    _fn.restype = ctypes.c_int
_lib.pa_version.restype = ctypes.c_char_p
_lib.pa_g1_fixed_base_table_words.restype = ctypes.c_size_t
_lib.pa_g1_fixed_base_workspace_words.restype = ctypes.c_size_t
_lib.pa_g2_fixed_base_table_words.restype = ctypes.c_size_t
_lib.pa_g2_fixed_base_workspace_words.restype = ctypes.c_size_t
_lib.pa_last_error.restype = ctypes.c_char_p
_lib.pa_multiexp_workspace_bytes.argtypes = [ctypes.c_int, _N]
_lib.pa_multiexp_workspace_bytes.restype = ctypes.c_size_t
_lib.pa_wnaf_exact_workspace_bytes.argtypes = [ctypes.c_int, _N, ctypes.c_int, ctypes.c_int]
_lib.pa_wnaf_exact_workspace_bytes.restype = ctypes.c_size_t


def version():
    return _lib.pa_version().decode()


def _check(rc, what):
    if rc != PA_OK:
        raise PairingError("%s failed (%d): %s" % (what, rc, _lib.pa_last_error().decode()))


def call(name, *args):
    _check(getattr(_lib, name)(*args), name)


def device_count():
    c = ctypes.c_int(0)
    rc = _lib.pa_device_count(ctypes.byref(c))
    return c.value if rc == PA_OK else 0


def set_pairing_kernel(variant):
    """Pairing kernels: 0 default by batch size (<= 2304 pairs on the
    cooperative kernels: a four-wave quad VM per pairing; <= 32768 a lane pair
    per pairing; <= 34048 one lane per pairing; larger lane pairs), 1 lane pairs, 2
    cooperative for every size, 3 one lane per pairing for every size, 4
    cooperative for every size on the round-2 one-wave VM.  Identical results."""
    call("pa_set_pairing_kernel", int(variant))


def set_decode_kernel(variant):
    """Point-decoding kernels: 0 default by batch size (<= PA_DECODE_QUAD_MAX
    records: one record per group of lane quads, the latency form), 1 one lane
    per record, 2 quad groups for every size.  Identical results."""
    call("pa_set_decode_kernel", int(variant))


def set_device(dev):
    call("pa_set_device", dev)


def ptr(a):
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("arrays must be C-contiguous")
    return a.ctypes.data_as(ctypes.c_void_p)


def as_rows(a, width, name="array"):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if a.ndim == 1:
        a = a.reshape(1, -1)
    if a.ndim != 2 or a.shape[1] != width:
        raise ValueError("%s must have shape (n, %d), got %s" % (name, width, a.shape))
    return a
