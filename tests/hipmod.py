"""Test-only launcher for generated TEST code objects (pairing_amd/lib/test/,
tools/pgen/unit_progs.py) through the HIP module API via ctypes, on buffers
torch allocated (torch is plumbing here).  The product library never loads
these kernels."""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_LIB = os.path.join(ROOT, "pairing_amd", "lib", "test")
SLOT_BYTES = 3584


def _hip():
    """the HIP runtime this process already uses (torch's / libpairing_amd's)"""
    path = None
    with open("/proc/self/maps") as fh:
        for line in fh:
            if "libamdhip64.so" in line:
                path = line.split()[-1]
                break
    return ctypes.CDLL(path or "libamdhip64.so", mode=ctypes.RTLD_GLOBAL)


def launch(name, a0, a1, a2, n, ws_slots=1, lanes=1):
    """run kernel pa_gen_<name> from lib/test/pa_gen_<name>.hsaco over n lanes
    with the generated kernels' five arguments (a0, a1, a2: torch CUDA tensors
    or None; a per-wave spill workspace of ws_slots slots)"""
    import torch
    hip = _hip()
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    path = os.path.join(TEST_LIB, "pa_gen_%s.hsaco" % name)
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    assert hip.hipModuleLoad(ctypes.byref(mod), path.encode()) == 0, "hipModuleLoad " + path
    try:
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, ("pa_gen_" + name).encode()) == 0
        blocks = (n * lanes + 63) // 64
        ws = torch.zeros(blocks * ws_slots * SLOT_BYTES, dtype=torch.uint8, device="cuda")

        class Args(ctypes.Structure):
            _fields_ = [("a0", ctypes.c_uint64), ("a1", ctypes.c_uint64), ("a2", ctypes.c_uint64),
                        ("n", ctypes.c_uint64), ("ws", ctypes.c_uint64)]
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        args = Args(ptr(a0), ptr(a1), ptr(a2), n, ws.data_ptr())
        size = ctypes.c_size_t(ctypes.sizeof(args))
        extra = (ctypes.c_void_p * 5)(ctypes.c_void_p(1), ctypes.cast(ctypes.pointer(args), ctypes.c_void_p),
                                      ctypes.c_void_p(2), ctypes.cast(ctypes.pointer(size), ctypes.c_void_p),
                                      ctypes.c_void_p(3))
        torch.cuda.synchronize()
        rc = hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 64, 1, 1, 0, None, None, extra)
        assert rc == 0, "hipModuleLaunchKernel %d" % rc
        torch.cuda.synchronize()
    finally:
        hip.hipModuleUnload(mod)


def launch_kernel(path, name, args, grid, block):
    """run extern "C" kernel `name` of the code object at `path` with args =
    [(ctypes type, value), ...] packed as its kernel-argument struct"""
    import torch
    hip = _hip()
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    assert hip.hipModuleLoad(ctypes.byref(mod), path.encode()) == 0, "hipModuleLoad " + path
    try:
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, name.encode()) == 0, name

        class Args(ctypes.Structure):
            _fields_ = [("a%d" % i, t) for i, (t, _) in enumerate(args)]
        packed = Args(*[v for _, v in args])
        size = ctypes.c_size_t(ctypes.sizeof(packed))
        extra = (ctypes.c_void_p * 5)(ctypes.c_void_p(1), ctypes.cast(ctypes.pointer(packed), ctypes.c_void_p),
                                      ctypes.c_void_p(2), ctypes.cast(ctypes.pointer(size), ctypes.c_void_p),
                                      ctypes.c_void_p(3))
        torch.cuda.synchronize()
        rc = hip.hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, None, None, extra)
        assert rc == 0, "hipModuleLaunchKernel %d" % rc
        torch.cuda.synchronize()
    finally:
        hip.hipModuleUnload(mod)
