"""ctypes binding of libmog_air.so (the C ABI declared in include/mog_air.h).

The product path has no fallback: if the HIP library is missing or fails to
load, every op raises.  Build it with ``make -C mog-asr_amd`` (or
``__graft_entry__.build()``)."""
from __future__ import annotations

import ctypes
import os
import re
from typing import List

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOG_AIR_LIB: another build of the library (A/B timing scripts only)
LIB_PATH = os.environ.get("MOG_AIR_LIB") or os.path.join(_HERE, "_lib", "libmog_air.so")
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "mog_air.h"))

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
L = ctypes.c_long
ULL = ctypes.c_ulonglong
LL = ctypes.c_longlong

# argtypes per entry point (mirrors include/mog_air.h)
_SIGS = {
    "mog_gemm_f32": [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, F, I, P],
    "mog_gemm_f32_kseg": [I, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "mog_gemm_f32_x3_tn": [P, P, P, P, I, I, I, I, I, I, I, P, L, P],
    "mog_split3_bf16": [P, I, I, I, P, I, L, P],
    "mog_split3_sum_bf16": [P, I, L, I, I, I, P, I, L, P],
    "mog_gemm_x3p_tn": [P, L, P, L, P, P, I, I, I, I, I, I, I, I, P, L, P],
    "mog_gemm_f32_wgrad_group": [P, I, P],
    "mog_wgrad_tn_work_elems": [I, P, I],
    "mog_wgrad_tn_bf16": [I, P, P, P, P, P, I, I, P, L, P],
    "mog_wgrad_tn_x3": [I, P, P, P, P, P, I, I, P, L, P],
    "mog_build_id": [P, I],
    "mog_gemm_x3_nt": [P, P, L, P, P, I, I, I, I, I, I, I, I, P],
    "mog_gemm_f32_sigmoid_philox": [P, P, P, P, I, I, I, I, I, I, F, ULL, ULL, P],
    "mog_stn_forward": [P, I, I, I, P, I, I, P, P, P, I, P],
    "mog_stn_forward_periodic": [P, I, I, I, I, P, I, I, P, P, P, I, P],
    "mog_stn_backward": [P, I, I, I, P, I, I, P, P, P, P, P, I, I, P],
    "mog_stn_backward_sigmoid_bf16": [P, I, I, I, P, I, I, P, P, P, P, P, I, I, P],
    "mog_stn_backward_sigmoid_f32": [P, I, I, I, P, I, I, P, P, P, P, P, I, I, P],
    "mog_lstm_cell_forward": [P, P, P, P, P, I, I, P],
    "mog_lstm_cell_backward": [P, P, P, P, P, P, P, P, P, I, I, P],
    "mog_lstm_cell_backward_parts": [P, P, P, P, P, P, I, L, P, P, P, P, I, I, P],
    "mog_gemm_f32_kseg_group": [I, P, P, P, P, P, I, I, I, I, I, I, I, P],
    "mog_lstm_cell_forward_pair": [P, I, I, P],
    "mog_lstm_cell_backward_pair": [P, I, I, P],
    "mog_air_step_forward": [I, I, I, I, I, I, F, F, F, F, F, F, F, F, F, F, P, P, P, P, P, P,
                             P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "mog_air_step_forward_steps": [I, I, I, I, I, I, F, F, F, P, F, F, F, F, F, F, P, L, P, P, P,
                                   P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "mog_air_step_backward": [I, I, I, I, F, F, F, F, F, F, F, F, P, P, P, P, P, P, P, P, P,
                              P, L, P, L, P],
    "mog_air_step_backward_steps": [I, I, I, I, I, F, F, F, F, F, F, F, F, P, P, P, P, P, P, P,
                                    P, P, P, L, P, L, P],
    "mog_vae_sample_forward": [I, I, F, F, F, P, P, P, P, P, I, P, P, P, P],
    "mog_stn_vae_step_forward": ([I] * 8 + [P] * 7 + [I, ULL, ULL] + [P] * 2 + [F] * 4 + [P] * 14
                                 + [I, P]),
    "mog_pack_frag_f32": [I, P, P, P, P, P],
    "mog_stn_vae_step_forward_f32": ([I, I] + [P] * 7 + [I, ULL, ULL] + [P] * 2 + [F] * 4
                                     + [P] * 19 + [I, P]),
    "mog_air_runloss": [I, I, P, L, P, P, P, P, P, P],
    "mog_stn_write_parts": [P, I, I, I, P, I, I, P, P, P, P, P],
    "mog_vae_sample_backward": [I, I, F, F, F, P, P, P, P, P, P, P, P, P, I, P],
    "mog_sigmoid_backward": [P, P, P, L, I, P],
    "mog_gemm_bf16": [I, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, F, I, P],
    "mog_cvt_bf16": [P, I, I, I, P, I, I, I, I, P],
    "mog_cvt_bf16_batch": [I, P, P, P, P],
    "mog_recon_loss": [P, P, P, I, L, P, I, P, P, P, I, I, F, P, P, P, P, P, P, P],
    "mog_batch_mean": [P, P, P, P, I, P, P],
    "mog_colsum_add": [P, I, I, I, P, P],
    "mog_heads_output_wgrad_work_elems": [I, I, I],
    "mog_heads_output_wgrad": [I, P, P, P, P, P, I, I, P, L, P],
    "mog_add": [P, P, P, L, P],
    "mog_optim_chunk_elems": [],
    "mog_clip_adam": [P, P, P, P, P, P, P, P, I, P, F, F, F, F, F, P],
    "mog_rng_fill": [P, L, ULL, ULL, I, P],
    "mog_rng_fill_batch": [I, P, P, ULL, P, P, P],
    "mog_fill32_batch": [I, P, P, P, P],
    "mog_copy32_batch": [I, P, P, P, P],
    "mog_transpose32_batch": [I, P, P, P, P, P],
    "mog_copy_f4": [P, P, L, P],
    "mog_generation_prior": [I, I, F, F, F, F, F, F, P, P, P, P, P, P, P, P],
    "mog_asr_pack": [I, I, I, I, P, P, P, P, P, P, P],
    "mog_asr_unpack": [I, I, I, I, P, P, P, P, P, P, I, P],
    "mog_asr_unpack_parts": [I, I, I, I, P, P, I, L, P, P, P, P, I, P],
    "mog_asr_step_forward": [I, I, I, I, F, F, F, F, F, F, P, P, P, P, P, P, P, P, P, P, P, P,
                             P, P, P, P, P, P, P],
    "mog_asr_terms": [I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "mog_asr_finalize": [I, I, I, I, P, P, F, P, P, P, P, P, P, P, P],
    "mog_asr_terms_backward": [I, I, I, I, P, P, F, F, P, P, P, P, P],
    "mog_asr_step_backward": [I, I, I, F, F, F, F, P, P, P, P, P, P, P, P, P, P, P, P, P],
}

# entry points that do not return an int status
_RESTYPE = {"mog_wgrad_tn_work_elems": L, "mog_heads_output_wgrad_work_elems": L}

_lib = None


class MogError(RuntimeError):
    pass


def header_symbols() -> List[str]:
    """Entry points declared in include/mog_air.h."""
    with open(HEADER_PATH) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|long)\s+(mog_\w+)\s*\(", src)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MogError(
            f"HIP library not found at {LIB_PATH}; build it with `make -C mog-asr_amd` "
            "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, I)
    built, src = library_build_id(lib), source_build_id()
    if src is not None and built != src:
        raise MogError(f"{LIB_PATH} was built from other sources (library {built}, sources "
                       f"{src}); rebuild it with `make -C mog-asr_amd`")
    _lib = lib
    return lib


# test-only instruments (include/mog_air_test.h): their own library
TEST_LIB_PATH = os.path.join(_HERE, "_lib", "libmog_air_test.so")
_TEST_SIGS = {"mog_spin": [LL, P], "mog_lds_poison": [ctypes.c_uint, P]}
_test_lib = None


def load_test():
    """libmog_air_test.so (mog_spin, mog_lds_poison): the stream-ordering and
    LDS-hygiene test instruments, kept out of the product library."""
    global _test_lib
    if _test_lib is None:
        if not os.path.exists(TEST_LIB_PATH):
            raise MogError(f"{TEST_LIB_PATH} not built (make -C mog-asr_amd)")
        lib = ctypes.CDLL(TEST_LIB_PATH)
        for name, args in _TEST_SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = I
        _test_lib = lib
    return _test_lib


def library_build_id(lib=None) -> str:
    """The source hash compiled into libmog_air.so (mog_build_id)."""
    buf = ctypes.create_string_buffer(32)
    if (lib or load()).mog_build_id(buf, 32) != 0:
        raise MogError("mog_build_id failed")
    return buf.value.decode()


def source_build_id():
    """The Makefile's hash of the sources beside the library (None when they
    are not there)."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    csrc, inc = os.path.join(pkg, "csrc"), os.path.join(os.path.dirname(pkg), "include")
    files = (sorted(glob.glob(os.path.join(csrc, "*.hip"))) +
             sorted(glob.glob(os.path.join(csrc, "*.h"))) +
             sorted(glob.glob(os.path.join(inc, "*.h"))))
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        what = "invalid argument" if rc == 1001 else f"hipError {rc}"
        raise MogError(f"{name} failed: {what}")


def ptr_array(ptrs) -> ctypes.Array:
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


# ---- PyTorch custom operators (csrc/torch_ops.cpp) --------------------------
TORCH_OPS_PATH = os.path.join(_HERE, "_lib", "libmog_air_torch.so")
_torch_ops_loaded = False


def build_torch_ops(verbose: bool = False) -> str:
    """Compile csrc/torch_ops.cpp (TORCH_LIBRARY_FRAGMENT(mog_air) over the C
    ABI) against this torch and libmog_air.so into mog_air/_lib/
    libmog_air_torch.so (in-tree, so it travels with the tree)."""
    import shutil

    import torch
    from torch.utils import cpp_extension
    load()  # libmog_air.so mapped first (the extension links it by soname)
    pkg = os.path.normpath(os.path.join(_HERE, ".."))
    bdir = os.path.join(pkg, "build", "torch_ops")
    os.makedirs(bdir, exist_ok=True)
    cpp_extension.load(
        name="libmog_air_torch", sources=[os.path.join(pkg, "csrc", "torch_ops.cpp")],
        extra_include_paths=[os.path.dirname(HEADER_PATH), "/opt/rocm/include"],
        extra_cflags=["-O2", "-D__HIP_PLATFORM_AMD__"],
        # libmog_air.so: resolved by its soname once load() has mapped it
        # (runpath kept as a fallback); c10_hip for the current-stream query
        extra_ldflags=["-L" + os.path.dirname(LIB_PATH), "-lmog_air",
                       "-L" + os.path.join(os.path.dirname(torch.__file__), "lib"), "-lc10_hip", "-ltorch_hip",
                       "-Wl,-rpath," + os.path.dirname(LIB_PATH)],
        build_directory=bdir, is_python_module=False, verbose=verbose)
    # cpp_extension.load registered the ops from the build copy already
    global _torch_ops_loaded
    _torch_ops_loaded = True
    shutil.copy2(os.path.join(bdir, "libmog_air_torch.so"), TORCH_OPS_PATH)
    return TORCH_OPS_PATH


def load_torch_ops() -> None:
    """Register torch.ops.mog_air.* (fails loudly when the extension is
    missing: there is no fallback path)."""
    global _torch_ops_loaded
    if _torch_ops_loaded:
        return
    load()
    if not os.path.exists(TORCH_OPS_PATH):
        raise MogError(f"{TORCH_OPS_PATH} not built (run __graft_entry__.build())")
    import torch
    torch.ops.load_library(TORCH_OPS_PATH)
    _torch_ops_loaded = True
