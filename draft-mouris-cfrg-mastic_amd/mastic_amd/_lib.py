"""ctypes binding of libmastic_hip.so (the C ABI declared in include/mastic_hip.h).

There is no fallback: if the shared library is missing or no gfx950 device is
present, every entry point raises.  ``build()`` compiles the library in-tree
with hipcc for gfx950.
"""
import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(PKG_DIR)
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
LIB_PATH = os.path.join(PKG_DIR, "libmastic_hip.so")
# The library lib() loads: always the shipped in-tree build, unless an A/B tool
# calls load(path) explicitly (no process variable can swap it).
LOAD_PATH = LIB_PATH
ABI_VERSION = 6  # include/mastic_hip.h MASTIC_ABI_VERSION

MASTIC_OK = 0
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -19: "ENODEV", -5: "EHIP", -110: "ETIMEDOUT"}

# Every symbol include/mastic_hip.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "mastic_ctx_create", "mastic_ctx_destroy", "mastic_last_error", "mastic_get_sizes",
    "mastic_set_memory_budget", "mastic_reports_create", "mastic_reports_destroy",
    "mastic_reports_count", "mastic_reports_upload", "mastic_reports_download",
    "mastic_reports_shard", "mastic_prep_init", "mastic_prep_result", "mastic_aggregate",
    "mastic_synchronize", "mastic_prep_init_batch", "mastic_decide_batch",
    "mastic_shard_batch", "mastic_last_timing", "mastic_tree_stats", "mastic_fold_shares",
    "mastic_work_bytes", "mastic_last_timing3", "mastic_proof_tree", "mastic_set_frontier_cache",
    "mastic_reports_view", "mastic_decide_results",
    "mastic_aggregate_device_on_stream", "mastic_abi_version", "mastic_set_test_hooks",
    "mastic_set_test_sponge_delay", "mastic_set_serial_sponges",
    "mastic_comm_unique_id", "mastic_comm_init", "mastic_comm_init_timeout", "mastic_comm_info",
    "mastic_comm_destroy",
    "mastic_allgather_fold", "mastic_aggregate_merged", "mastic_merge_host",
]
COMM_ID_BYTES = 128  # MASTIC_COMM_ID_BYTES (= RCCL's NCCL_UNIQUE_ID_BYTES)
ROCM_PATH = "/opt/rocm"  # the image's ROCm (the library dlopens librccl.so.1 from its lib/ on first comm use)


class MasticParams(ctypes.Structure):
    _fields_ = [
        ("circuit", ctypes.c_uint32),
        ("bits", ctypes.c_uint32),
        ("length", ctypes.c_uint32),
        ("sum_vec_bits", ctypes.c_uint32),
        ("max_measurement", ctypes.c_uint64),
        ("chunk_length", ctypes.c_uint32),
        ("device", ctypes.c_int32),
    ]


class MasticSizes(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint32) for name in (
        "field_bytes", "value_len", "meas_len", "output_len", "proof_len", "verifier_len",
        "joint_rand_len", "query_rand_len", "prove_rand_len", "rand_size", "public_share_size")] + [
        ("input_share_size", ctypes.c_uint32 * 2),
        ("prep_share_size", ctypes.c_uint32 * 2),
        ("algorithm_id", ctypes.c_uint32),
    ]


class MasticError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%s)" % (msg, ERRORS.get(code, code)))
        self.code = code


def build(verbose=False, force=False, out=None, defines=()) -> str:
    """Compile csrc/mastic_hip.hip for gfx950 into the package directory.
    ``out`` / ``defines``: another build of the same source (e.g.
    ``defines=("MASTIC_EXPERIMENT_KNOBS",)`` for the A/B tools, which load it
    through ``load(path)``); the shipped library is the default one."""
    out = out or LIB_PATH
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    srcs.append(os.path.join(INCLUDE, "mastic_hip.h"))
    newest = max(os.path.getmtime(s) for s in srcs)
    if not force and os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    tmp = out + ".%d.tmp" % os.getpid()
    rocm_lib = os.path.join(ROCM_PATH, "lib")
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + INCLUDE] + ["-D" + d for d in defines] + ["-o", tmp, os.path.join(CSRC, "mastic_hip.hip"),
                                                         "-Wl,-rpath," + rocm_lib]
    if verbose:
        print(" ".join(cmd))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(cmd)
    os.replace(tmp, out)
    return out


_lib = None
_lock = threading.Lock()


def load(path: str):
    """A/B and timing tools only: bind another build of the library (e.g. a
    -DMASTIC_EXPERIMENT_KNOBS build) instead of the shipped one.  Must be
    called before the first lib() call of the process."""
    global LOAD_PATH
    with _lock:
        if _lib is not None and os.path.abspath(path) != os.path.abspath(LOAD_PATH):
            raise RuntimeError("libmastic_hip is already loaded from %s" % LOAD_PATH)
        LOAD_PATH = os.path.abspath(path)


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LOAD_PATH):
                    raise ImportError("libmastic_hip.so is not built (run __graft_entry__.build()); "
                                      "the HIP path has no CPU fallback")
                l = ctypes.CDLL(LOAD_PATH)
                P = ctypes.c_void_p
                u8p = ctypes.c_char_p
                sz = ctypes.c_size_t
                i32 = ctypes.c_int
                sig = {
                    "mastic_ctx_create": (i32, [ctypes.POINTER(MasticParams), ctypes.POINTER(P)]),
                    "mastic_ctx_destroy": (None, [P]),
                    "mastic_last_error": (ctypes.c_char_p, [P]),
                    "mastic_get_sizes": (i32, [P, ctypes.POINTER(MasticSizes)]),
                    "mastic_set_memory_budget": (i32, [P, ctypes.c_uint64]),
                    "mastic_reports_create": (i32, [P, sz, ctypes.POINTER(P)]),
                    "mastic_reports_destroy": (None, [P]),
                    "mastic_reports_count": (sz, [P]),
                    "mastic_reports_upload": (i32, [P, P, P, P, P]),
                    "mastic_reports_download": (i32, [P, P, P, P, P]),
                    "mastic_reports_shard": (i32, [P, u8p, sz, P, P, P, P]),
                    "mastic_prep_init": (i32, [P, P, u8p, sz, u8p, sz, i32, u8p, sz]),
                    "mastic_prep_result": (i32, [P, i32, P, P, P, P]),
                    "mastic_aggregate": (i32, [P, i32, P, P]),
                    "mastic_synchronize": (i32, [P]),
                    "mastic_prep_init_batch": (i32, [P, u8p, sz, u8p, sz, i32, u8p, sz, sz, P, P, P, P, P, P, P]),
                    "mastic_decide_batch": (i32, [P, u8p, sz, u8p, sz, sz, P, P, P, P]),
                    "mastic_shard_batch": (i32, [P, u8p, sz, sz, P, P, P, P, P, P, P]),
                    "mastic_last_timing": (i32, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_double)]),
                    "mastic_fold_shares": (i32, [P, P, sz, sz, P, P]),
                    "mastic_comm_unique_id": (i32, [P]),
                    "mastic_comm_init": (i32, [P, i32, i32, P]),
                    "mastic_comm_init_timeout": (i32, [P, i32, i32, P, i32]),
                    "mastic_comm_info": (i32, [P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
                    "mastic_comm_destroy": (i32, [P]),
                    "mastic_allgather_fold": (i32, [P, P, sz, sz, P, P]),
                    "mastic_aggregate_merged": (i32, [P, ctypes.c_uint32, P, sz, P]),
                    "mastic_merge_host": (i32, [P, P, sz, sz, P]),
                    "mastic_aggregate_device_on_stream": (i32, [P, i32, P, P, P]),
                    "mastic_abi_version": (i32, []),
                    "mastic_set_test_hooks": (i32, [P, i32, i32]),
                    "mastic_set_test_sponge_delay": (i32, [P, i32]),
                    "mastic_set_serial_sponges": (i32, [P, i32]),
                    "mastic_reports_view": (i32, [P, sz, sz, ctypes.POINTER(P)]),
                    "mastic_decide_results": (i32, [P, u8p, sz, P, P]),
                    "mastic_last_timing3": (i32, [P] + [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)] * 3
                                            + [ctypes.POINTER(ctypes.c_double)]),
                    "mastic_work_bytes": (i32, [P, u8p, sz, ctypes.POINTER(ctypes.c_uint64)]),
                    "mastic_proof_tree": (i32, [P, ctypes.c_int, u8p, sz, P, sz]),
                    "mastic_set_frontier_cache": (i32, [P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
                    "mastic_tree_stats": (i32, [P, u8p, sz, ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
                }
                for name, (res, args) in sig.items():
                    fn = getattr(l, name)
                    fn.restype = res
                    fn.argtypes = args
                if l.mastic_abi_version() != ABI_VERSION:
                    raise ImportError("%s has ABI version %d, this binding expects %d (rebuild it)"
                                      % (LOAD_PATH, l.mastic_abi_version(), ABI_VERSION))
                _lib = l
    return _lib


def buf(data) -> ctypes.c_void_p:
    """Pointer to the bytes of a bytes/bytearray/numpy array (None -> NULL)."""
    if data is None:
        return None
    import numpy as np
    if isinstance(data, np.ndarray):
        assert data.flags["C_CONTIGUOUS"]
        return ctypes.c_void_p(data.ctypes.data)
    if isinstance(data, bytearray):
        return ctypes.c_void_p(ctypes.addressof((ctypes.c_char * len(data)).from_buffer(data)))
    if isinstance(data, bytes):
        return ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p)
    raise TypeError(type(data))
