"""ctypes binding of libgmat_hip.so (the C ABI declared in include/gmat_hip.h).

The product path has no CPU fallback: if the library or a GPU is missing, every compute
entry point raises ``GmatNativeError``.  (cffi is not importable in this image; the C ABI is
plain ``extern "C"`` with POD arguments, so cffi ABI mode would bind it unchanged -- see
INTEGRATION.md.)
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMAT_HIP_LIB", os.path.join(_HERE, "libgmat_hip.so"))

GMAT_AA, GMAT_AD, GMAT_DD = 0, 1, 2
GMAT_GRM_ADD, GMAT_GRM_DOM = 0, 1
GMAT_SCREEN_NONE = -9  # gmat_epi_scan level: no screen, every pair refined exactly

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_D = ctypes.c_double
_INT = ctypes.c_int

_PROTOS = {
    "gmat_last_error": (ctypes.c_char_p, []),
    "gmat_version": (_INT, []),
    "gmat_device_count": (_INT, [_P]),
    "gmat_set_device": (_INT, [_INT]),
    "gmat_device_synchronize": (_INT, []),
    "gmat_empty_cache": (_INT, []),
    "gmat_reml_stats": (_INT, [_P]),
    "gmat_reml_trace": (_INT, [_INT, _P, _P, _P, _P]),
    "gmat_epi_setup_stats": (_INT, [_P, _P]),
    "gmat_geno_create": (_INT, [_P, _P, _I64, _I64, _I64]),
    "gmat_geno_counts": (_INT, [_P, _P, _P, _P]),
    "gmat_geno_destroy": (_INT, [_P]),
    "gmat_grm": (_INT, [_P, _INT, _D, _P, _P]),
    "gmat_grm_stats": (_INT, [_P]),
    "gmat_spd_inverse": (_INT, [_I64, _P, _P, _P]),
    "gmat_reml": (_INT, [_I64, _I64, _I64, _INT, _P, _P, _P, _P, _P, _INT, _D, _D, _P, _P, _P]),
    "gmat_projection": (_INT, [_I64, _I64, _I64, _INT, _P, _P, _P, _P, _P, _P, _P]),
    "gmat_epi_create": (_INT, [_P, _P, _P, _P, _INT]),
    "gmat_epi_create_with": (_INT, [_P, _P, _P, _P, _INT, _P, _I64]),
    "gmat_epi_export": (_INT, [_P, _P, _I64, _P]),
    "gmat_epi_scan": (_INT, [_P, _INT, _P, _I64, _D, _D, _INT, _P]),
    "gmat_epi_hits": (_INT, [_P, _I64, _P, _P, _P, _P, _P, _P]),
    "gmat_epi_pairs": (_INT, [_P, _INT, _P, _I64, _P, _P, _P, _P]),
    "gmat_epi_stats": (_INT, [_P, _P]),
    "gmat_epi_audit": (_INT, [_P, _INT, _P, _I64, _P]),
    "gmat_epi_kernel_stats": (_INT, [_P, _P]),
    "gmat_epi_kernel_stats_ext": (_INT, [_P, _P, _INT, _P]),
    "gmat_epi_info": (_INT, [_P, _P]),
    "gmat_epi_layout": (_INT, [_P, _P]),
    "gmat_epi_destroy": (_INT, [_P]),
    "gmat_eff_scan": (_INT, [_P, _INT, _P, _P, _I64, _P, _P, _P, ctypes.c_char_p, _P]),
    "gmat_eff_stats": (_INT, [_P]),
    "gmat_geno_decode": (_INT, [_P, _P]),
    "gmat_blup": (_INT, [_I64, _I64, _I64, _INT, _P, _P, _P, _P, _P, _P]),
    "gmat_write_grm_text": (_INT, [ctypes.c_char_p, _P, _I64, _INT, ctypes.c_char_p, _INT]),
    "gmat_float_repr": (_INT, [_D, ctypes.c_char_p, _INT]),
    "gmat_append_hit_rows": (_INT, [ctypes.c_char_p, _I64, _P, _P, _INT, _P, _P, _P, _P]),
    "gmat_snp_test": (_INT, [_P, _INT, _P, _P, _P, _P]),
    "gmat_probe_mx_accum": (_INT, [_INT, _P, _P, _P]),
    "gmat_probe_eig_bottom": (_INT, [_I64, _P, _INT, _D, _INT, _P, _P, _P, _P]),
    "gmat_comm_unique_id": (_INT, [_P]),
    "gmat_comm_init": (_INT, [_P, _INT, _INT, _P]),
    "gmat_comm_destroy": (_INT, [_P]),
    "gmat_comm_allgather": (_INT, [_P, _P, _P, _I64]),
    "gmat_comm_broadcast": (_INT, [_P, _P, _I64, _INT]),
    "gmat_comm_allreduce_f64": (_INT, [_P, _P, _I64, _INT]),
    "gmat_comm_gatherv": (_INT, [_P, _P, _I64, _INT, _P, _P, _I64, _P]),
    "gmat_comm_barrier": (_INT, [_P]),
    # include/gmat_remma_eff.h: the reference's cffi prototypes (char*, long long, ...)
    "read_plink_bed": (_INT, [ctypes.c_char_p, _I64, _I64, _P]),
    "remma_epiAA_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _D, ctypes.c_char_p]),
    "remma_epiAD_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _D, ctypes.c_char_p]),
    "remma_epiDD_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _D, ctypes.c_char_p]),
    "remma_epiAA_maf_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _P, _P, ctypes.c_char_p]),
    "remma_epiDD_maf_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _P, _P, ctypes.c_char_p]),
    "remma_epiAD_maf_eff_cpu": (_INT, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _P, _P, _P, ctypes.c_char_p]),
}


class GmatNativeError(RuntimeError):
    pass


_lib = None
_device_set = False


def load(required=True):
    """Load the library (once).  Raises GmatNativeError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not required:
            return None
        raise GmatNativeError("libgmat_hip.so not found at %s -- build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return sorted(_PROTOS)


def check(rc, what=""):
    if rc != 0:
        msg = _lib.gmat_last_error().decode(errors="replace") if _lib else ""
        raise GmatNativeError("%s failed (rc=%d): %s" % (what, rc, msg))


def device_count():
    lib = load()
    n = ctypes.c_int(0)
    check(lib.gmat_device_count(ctypes.byref(n)), "gmat_device_count")
    return n.value


def shared_gpu_allowed():
    """Several ranks on one device (the gloo rehearsals of the multi-GPU path on a one-GPU box)."""
    return os.environ.get("GMAT_ALLOW_SHARED_GPU", "") not in ("", "0")


def ensure_device():
    """Bind this process to its GPU (LOCAL_RANK / GMAT_DEVICE, default 0); raise when
    there is none -- the product path never falls back to the CPU."""
    global _device_set
    lib = load()
    if _device_set:
        return lib
    if device_count() < 1:
        raise GmatNativeError("no HIP device visible: the gmat_amd product path needs an MI355X")
    dev = int(os.environ.get("GMAT_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    n_dev = device_count()
    if dev >= n_dev and not shared_gpu_allowed():
        # one process per GPU: a rank without a device of its own would silently share one and the
        # job would report more GPUs than it used (GMAT_ALLOW_SHARED_GPU=1: test rehearsals only)
        raise GmatNativeError("device %d requested (LOCAL_RANK / GMAT_DEVICE) but only %d visible; set "
                              "GMAT_ALLOW_SHARED_GPU=1 to share devices (tests only)" % (dev, n_dev))
    check(lib.gmat_set_device(dev % n_dev), "gmat_set_device")
    _device_set = True
    return lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)
