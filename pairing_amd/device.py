"""Device-resident entry points over torch tensors (HBM in, HBM out).

torch is plumbing here: it owns the device allocations and the stream; the
work is the C ABI's `_device` functions (HIP kernels) enqueued on that
stream.  Tensors hold the raw ABI records as int64 words (torch has no full
uint64 support), shape (n, words) exactly as the numpy layer.
"""
import ctypes

import torch

from ._native import W_FQ, W_FQ12, W_G1, W_G1A, W_G2, W_G2A, W_G2P, _lib, call


def _stream_ptr(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dptr(t, width, name):
    if not t.is_cuda or not t.is_contiguous() or t.dtype != torch.int64:
        raise ValueError("%s must be a contiguous int64 CUDA tensor" % name)
    if t.dim() != 2 or t.shape[1] != width:
        raise ValueError("%s must have shape (n, %d), got %s" % (name, width, tuple(t.shape)))
    return ctypes.c_void_p(t.data_ptr())


def _rows(t, n, name):
    """t holds at least the n records the call writes or reads"""
    if t.shape[0] < n:
        raise ValueError("%s has %d rows, the call needs %d" % (name, t.shape[0], n))


def _flags(ok, n, name="ok"):
    """a contiguous uint8 CUDA tensor of at least n flags, or None"""
    if ok is None:
        return ctypes.c_void_p(0)
    if not ok.is_cuda or not ok.is_contiguous() or ok.dtype != torch.uint8 or ok.numel() < n:
        raise ValueError("%s must be a contiguous uint8 CUDA tensor of >= %d elements" % (name, n))
    return ctypes.c_void_p(ok.data_ptr())


def _words(t, need, name):
    """a contiguous int64 CUDA buffer of at least `need` 8-byte words"""
    if not t.is_cuda or not t.is_contiguous() or t.dtype != torch.int64 or t.numel() < need:
        raise ValueError("%s must be a contiguous int64 CUDA tensor of >= %d words" % (name, need))
    return ctypes.c_void_p(t.data_ptr())


def _fb_table(table, ws):
    return (_words(table, int(_lib.pa_g1_fixed_base_table_words()), "table"),
            _words(ws, int(_lib.pa_g1_fixed_base_workspace_words()), "ws"))


def empty_records(n, width, device):
    return torch.empty((n, width), dtype=torch.int64, device=device)


def fq_mul(a, b, out, stream=None):
    """Fq::mul_assign over a batch resident in HBM (BASELINE config 2)."""
    n = a.shape[0]
    args = (_dptr(a, W_FQ, "a"), _dptr(b, W_FQ, "b"), _dptr(out, W_FQ, "out"))
    _rows(b, n, "b")
    _rows(out, n, "out")
    call("pa_fq_mul_batch_device", *args, n, _stream_ptr(stream))


def fq_mul_soa(a, b, out, stream=None):
    """Fq::mul_assign on the SoA device layout: (6, n) int64 planes, word j of
    element i at [j, i]."""
    for t, name in ((a, "a"), (b, "b"), (out, "out")):
        if not t.is_cuda or not t.is_contiguous() or t.dtype != torch.int64 or t.dim() != 2 or t.shape[0] != 6:
            raise ValueError("%s must be a contiguous (6, n) int64 CUDA tensor" % name)
    n = a.shape[1]
    if b.shape[1] != n or out.shape[1] != n:
        raise ValueError("operand lengths differ")
    call("pa_fq_mul_batch_soa_device", ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
         ctypes.c_void_p(out.data_ptr()), n, _stream_ptr(stream))


def miller_loop(p, q, out, stream=None):
    """Fused-prepare single-pair Miller loops: out[i] = miller_loop([(p[i], q[i].prepare())])."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(q, W_G2A, "q"), _dptr(out, W_FQ12, "out"))
    _rows(q, n, "q")
    _rows(out, n, "out")
    call("pa_miller_loop_fused_batch_device", *args, n, _stream_ptr(stream))


def pairing_miller_loop(p, q, out, stream=None):
    """The Miller-loop stage of pairing(): final_exponentiation(out) = e(p[i], q[i]);
    out equals the reference's Miller values only up to Fq2 factors (see
    pa_pairing_miller_loop_batch_device)."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(q, W_G2A, "q"), _dptr(out, W_FQ12, "out"))
    _rows(q, n, "q")
    _rows(out, n, "out")
    call("pa_pairing_miller_loop_batch_device", *args, n, _stream_ptr(stream))


def g2_prepare(q, out, stream=None):
    """G2Prepared::from_affine over a batch (mod.rs:168-358): out (n, W_G2P) int64 records."""
    n = q.shape[0]
    args = (_dptr(q, W_G2A, "q"), _dptr(out, W_G2P, "out"))
    _rows(out, n, "out")
    call("pa_g2_prepare_batch_device", *args, n, _stream_ptr(stream))


def miller_loop_prepared(p, qp, out, stream=None):
    """out[i] = miller_loop([(p[i], qp[i])]) over materialized G2Prepared records (mod.rs:40-102)."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(qp, W_G2P, "qp"), _dptr(out, W_FQ12, "out"))
    _rows(qp, n, "qp")
    _rows(out, n, "out")
    call("pa_miller_loop_batch_device", *args, n, _stream_ptr(stream))


def miller_loop_shared_prepared(p, qp, out, stream=None):
    """out[i] = miller_loop([(p[i], qp[0])]): one G2Prepared record shared by the
    batch, its lines staged once (lib.rs:88-96, mod.rs:40-102)."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(qp, W_G2P, "qp"), _dptr(out, W_FQ12, "out"))
    _rows(qp, 1, "qp")
    _rows(out, n, "out")
    call("pa_miller_loop_shared_prepared_device", args[0], n, args[1], args[2], _stream_ptr(stream))


def final_exponentiation(f, out, ok=None, stream=None):
    n = f.shape[0]
    args = (_dptr(f, W_FQ12, "f"), _dptr(out, W_FQ12, "out"), _flags(ok, n))
    _rows(out, n, "out")
    call("pa_final_exponentiation_batch_device", *args, n, _stream_ptr(stream))


def pairing(p, q, out, scratch, stream=None):
    """out[i] = e(p[i], q[i]) for a batch resident in HBM (BASELINE config 4)."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(q, W_G2A, "q"), _dptr(out, W_FQ12, "out"), _dptr(scratch, W_FQ12, "scratch"))
    for t, name in ((q, "q"), (out, "out"), (scratch, "scratch")):
        _rows(t, n, name)
    call("pa_pairing_batch_device", *args, n, _stream_ptr(stream))


def multi_pairing(p, q, out, ok, work, stream=None):
    """final_exponentiation(miller_loop(pairs)) over pairs resident in HBM (the verifier's
    batch check, mod.rs:40-160): out (1, 72), ok (1,) uint8, work (n, 72) scratch."""
    n = p.shape[0]
    args = (_dptr(p, W_G1A, "p"), _dptr(q, W_G2A, "q"))
    _rows(q, n, "q")
    _rows(out, 1, "out")
    _rows(work, n, "work")   # the per-pair Miller values and the product tree
    call("pa_multi_pairing_device", *args, n, _dptr(out, W_FQ12, "out"), _flags(ok, 1),
         _dptr(work, W_FQ12, "work"), _stream_ptr(stream))


def g1_fixed_base_table(base, stream=None):
    """Build the fixed-base table for `base` (a (1,18) Jacobian record) in HBM."""
    dev = base.device
    table = torch.empty(int(_lib.pa_g1_fixed_base_table_words()), dtype=torch.int64, device=dev)
    ws = torch.empty(int(_lib.pa_g1_fixed_base_workspace_words()), dtype=torch.int64, device=dev)
    call("pa_g1_fixed_base_table_device", _dptr(base, W_G1, "base"), ctypes.c_void_p(table.data_ptr()),
         ctypes.c_void_p(ws.data_ptr()), _stream_ptr(stream))
    return table, ws


def g1_fixed_base_mul(table, scalars, out, stream=None):
    """out[i] = scalars[i] * base (config 3), scalars (n,4) int64 FrRepr."""
    n = scalars.shape[0]
    args = (_words(table, int(_lib.pa_g1_fixed_base_table_words()), "table"), _dptr(scalars, 4, "scalars"),
            _dptr(out, W_G1, "out"))
    _rows(out, n, "out")
    call("pa_g1_fixed_base_mul_device", *args, n, _stream_ptr(stream))


def g1_fixed_base_glv_table(base, table, ws, stream=None):
    """GLV stage 1: table rows, their phi images and the membership flag (ws)."""
    call("pa_g1_fixed_base_glv_table_device", _dptr(base, W_G1, "base"), *_fb_table(table, ws),
         _stream_ptr(stream))


def g1_fixed_base_glv_mul(base, table, ws, scalars, out, stream=None):
    """GLV stage 2: out[i] = scalars[i] * base (for a base outside G1 the
    double-and-add ladder k_g1_fixed_base_ladder takes over inside)."""
    n = scalars.shape[0]
    args = (_dptr(base, W_G1, "base"), *_fb_table(table, ws), _dptr(scalars, 4, "scalars"), _dptr(out, W_G1, "out"))
    _rows(out, n, "out")
    call("pa_g1_fixed_base_glv_mul_device", *args, n, _stream_ptr(stream))


def g1_wnaf_fixed_base(base, scalars, out, table, ws, stream=None, window=None):
    """out[i] = the reference's wNAF product scalars[i] * base (its wnaf_form
    wrap included; `window` default recommended_wnaf_for_num_scalars(n)) with
    the table built in the same call (its serial base chain overlapped with the
    multiply); table / ws as returned by fixed_base_buffers()."""
    n = scalars.shape[0]
    args = (_dptr(base, W_G1, "base"), _dptr(scalars, 4, "scalars"), _dptr(out, W_G1, "out"))
    _rows(out, n, "out")
    if window is None:
        call("pa_g1_wnaf_fixed_base_device", *args, n, *_fb_table(table, ws), _stream_ptr(stream))
    else:
        call("pa_g1_wnaf_fixed_base_window_device", *args, n, int(window), *_fb_table(table, ws),
             _stream_ptr(stream))


def fixed_base_buffers(dev):
    """(table, workspace) device buffers for g1_wnaf_fixed_base."""
    table = torch.empty(int(_lib.pa_g1_fixed_base_table_words()), dtype=torch.int64, device=dev)
    ws = torch.empty(int(_lib.pa_g1_fixed_base_workspace_words()), dtype=torch.int64, device=dev)
    return table, ws


def g1_batch_normalization(v, stream=None):
    call("pa_g1_batch_normalization_device", _dptr(v, W_G1, "v"), v.shape[0], _stream_ptr(stream))


def g2_batch_normalization(v, stream=None):
    call("pa_g2_batch_normalization_device", _dptr(v, W_G2, "v"), v.shape[0], _stream_ptr(stream))


def g2_fixed_base_buffers(dev):
    """(table, workspace) device buffers for g2_wnaf_fixed_base."""
    table = torch.empty(int(_lib.pa_g2_fixed_base_table_words()), dtype=torch.int64, device=dev)
    ws = torch.empty(int(_lib.pa_g2_fixed_base_workspace_words()), dtype=torch.int64, device=dev)
    return table, ws


def g2_wnaf_fixed_base(base, scalars, out, table, ws, stream=None, window=None):
    """out[i] = the reference's wNAF product scalars[i] * base for G2 (base a
    (1,36) Jacobian record; `window` as in g1_wnaf_fixed_base)."""
    n = scalars.shape[0]
    args = (_dptr(base, W_G2, "base"), _dptr(scalars, 4, "scalars"), _dptr(out, W_G2, "out"))
    _rows(out, n, "out")
    tw = (_words(table, int(_lib.pa_g2_fixed_base_table_words()), "table"),
          _words(ws, int(_lib.pa_g2_fixed_base_workspace_words()), "ws"))
    if window is None:
        call("pa_g2_wnaf_fixed_base_device", *args, n, *tw, _stream_ptr(stream))
    else:
        call("pa_g2_wnaf_fixed_base_window_device", *args, n, int(window), *tw, _stream_ptr(stream))


def group_add(group, a, b, out, stream=None):
    """CurveProjective::add_assign over Jacobian rows in HBM: out = a + b (group 1 or 2)."""
    w = W_G1 if group == 1 else W_G2
    args = (_dptr(a, w, "a"), _dptr(b, w, "b"), _dptr(out, w, "out"))
    _rows(b, a.shape[0], "b")
    _rows(out, a.shape[0], "out")
    call("pa_g%d_add_batch_device" % group, *args, a.shape[0], _stream_ptr(stream))


def subgroup_check(group, pts, ok, stream=None):
    """is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144) over affine rows in HBM
    (n, 13|25) int64: ok (n,) uint8 = 1 in the subgroup (infinity included), 0 not."""
    n = pts.shape[0]
    args = (_dptr(pts, W_G1A if group == 1 else W_G2A, "pts"),)
    call("pa_g%d_subgroup_check_batch_device" % group, *args, n, _flags(ok, n), _stream_ptr(stream))


def decode(group, enc, compressed, checked, out, status, stream=None):
    """EncodedPoint::into_affine[_unchecked] over records resident in HBM:
    enc (n, 48|96|192) uint8, out (n, 13|25) int64 affine records, status (n,) uint8."""
    size = (48 if group == 1 else 96) * (1 if compressed else 2)
    if not enc.is_cuda or not enc.is_contiguous() or enc.dtype != torch.uint8 or enc.dim() != 2 \
            or enc.shape[1] != size:
        raise ValueError("enc must be a contiguous (n, %d) uint8 CUDA tensor" % size)
    if not status.is_cuda or status.dtype != torch.uint8 or status.numel() != enc.shape[0]:
        raise ValueError("status must be an (n,) uint8 CUDA tensor")
    width = W_G1A if group == 1 else W_G2A
    call("pa_g%d_decode_batch_device" % group, ctypes.c_void_p(enc.data_ptr()), enc.shape[0],
         int(bool(compressed)), int(bool(checked)), _dptr(out, width, "out"), ctypes.c_void_p(status.data_ptr()),
         _stream_ptr(stream))



def fr_mul(a, b, out, stream=None):
    """Fr::mul_assign (fr.rs:438-465) over a batch resident in HBM, rows (n, 4)."""
    args = (_dptr(a, 4, "a"), _dptr(b, 4, "b"), _dptr(out, 4, "out"))
    _rows(b, a.shape[0], "b")
    _rows(out, a.shape[0], "out")
    call("pa_fr_mul_batch_device", *args, a.shape[0], _stream_ptr(stream))


def multiexp_workspace(group, n, device):
    """A device workspace sized for pa_g{group}_multiexp_device over n terms."""
    nbytes = int(_lib.pa_multiexp_workspace_bytes(int(group), int(n)))
    return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)


def multiexp(group, bases, scalars, out, workspace, stream=None):
    """out (1, 18|36) = sum_i scalars[i] * bases[i] (affine records (n, 13|25), FrRepr (n, 4))."""
    aw, jw = (W_G1A, W_G1) if group == 1 else (W_G2A, 36)
    call("pa_g%d_multiexp_device" % group, _dptr(bases, aw, "bases"), _dptr(scalars, 4, "scalars"),
         bases.shape[0], _dptr(out, jw, "out"), ctypes.c_void_p(workspace.data_ptr()), workspace.numel(),
         _stream_ptr(stream))


def wnaf_exact_workspace(group, n, window, fixed_scalar, device):
    """A device workspace for the bit-exact Wnaf device entries (window as resolved)."""
    nbytes = int(_lib.pa_wnaf_exact_workspace_bytes(int(group), int(n), int(window), int(bool(fixed_scalar))))
    if nbytes == 0:
        raise ValueError("wnaf exact: group %r / window %r out of range" % (group, window))
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def wnaf_fixed_base_exact(group, base, scalars, out, window, workspace, stream=None):
    """Wnaf::new().base(base, n).scalar(s_i) with the reference's Jacobian words
    (pa_g{1,2}_wnaf_fixed_base_exact_device); base (1, 18|36), scalars (n, 4)."""
    jw = W_G1 if group == 1 else W_G2
    n = scalars.shape[0]
    _rows(out, n, "out")
    _rows(base, 1, "base")
    if base.shape[0] != 1:
        raise ValueError("base: expected exactly one record, got %d" % base.shape[0])
    call("pa_g%d_wnaf_fixed_base_exact_device" % group, _dptr(base, jw, "base"), _dptr(scalars, 4, "scalars"),
         _dptr(out, jw, "out"), n, int(window), ctypes.c_void_p(workspace.data_ptr()), workspace.numel(),
         _stream_ptr(stream))


def wnaf_fixed_scalar_exact(group, bases, scalar, out, window, workspace, stream=None):
    """Wnaf::new().scalar(s).base(g_i) with the reference's Jacobian words
    (pa_g{1,2}_wnaf_fixed_scalar_exact_device); bases (n, 18|36), scalar (1, 4)."""
    jw = W_G1 if group == 1 else W_G2
    n = bases.shape[0]
    _rows(out, n, "out")
    _rows(scalar, 1, "scalar")
    if scalar.shape[0] != 1:
        raise ValueError("scalar: expected exactly one record, got %d" % scalar.shape[0])
    call("pa_g%d_wnaf_fixed_scalar_exact_device" % group, _dptr(bases, jw, "bases"), n,
         _dptr(scalar, 4, "scalar"), _dptr(out, jw, "out"), int(window), ctypes.c_void_p(workspace.data_ptr()),
         workspace.numel(), _stream_ptr(stream))
