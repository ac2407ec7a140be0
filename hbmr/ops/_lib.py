"""ctypes binding of ``hbmr/lib/libhbmr.so`` (the native HIP/C++ kernels).

PyTorch is imported first so its bundled ``libamdhip64.so.7`` is the HIP
runtime in the process; libhbmr.so names the same soname and therefore shares
that runtime (streams and device pointers are interchangeable with torch's).

On a machine with a GPU the library MUST load: a missing or stale build raises
instead of silently falling back to a PyTorch path.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen below)

_LIB_PATH = Path(__file__).resolve().parent.parent / "lib" / "libhbmr.so"
_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
c_long = ctypes.c_long
c_int = ctypes.c_int
c_uint = ctypes.c_uint
c_uint64 = ctypes.c_uint64
c_double_p = ctypes.POINTER(ctypes.c_double)

_SIGS = {
    "hbmr_kmeans_assign_bf16": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int,
                                        c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_accum_bf16": (c_int, [c_void_p, c_long, c_int, c_void_p, c_int, c_void_p,
                                       c_void_p, c_int, c_void_p, c_long, c_int, c_void_p]),
    "hbmr_kmeans_accum_f32": (c_int, [c_void_p, c_long, c_int, c_void_p, c_int, c_void_p,
                                      c_void_p, c_int, c_void_p, c_long, c_int, c_void_p]),
    "hbmr_kmeans_assign_top3_bf16": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_assign_top3_f16": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_exact_prep": (c_int, [c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_assign_top3_q1_grouped": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int,
                                                   c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                                   c_void_p, c_void_p, c_void_p, c_int, c_int,
                                                   c_void_p, c_void_p, c_void_p, c_void_p,
                                                   c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_kmeans_centroid_nbr": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "hbmr_kmeans_image16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_image16_tiled": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "hbmr_kmeans_set_exact_kernel": (c_int, [c_int]),
    "hbmr_kmeans_refine_f32": (c_int, [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                       c_void_p]),
    "hbmr_kmeans_refine_batch_bytes": (c_long, [c_int, c_void_p]),
    "hbmr_kmeans_assign_top3_grouped": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int,
                                                c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                                c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_refine_batch_q1g": (c_int, [c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_kmeans_refine_batch_q1": (c_int, [c_int, c_void_p, c_int, c_int, c_int, c_int,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_long, c_int,
                                            c_void_p, c_void_p]),
    "hbmr_kmeans_refine_batch_finish": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int,
                                                c_int, c_void_p, c_int, c_int, c_void_p,
                                                c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                                c_int, c_void_p, c_long, c_void_p]),
    "hbmr_kmeans_accum_workspace_bytes": (c_long, [c_long, c_int]),
    "hbmr_kmeans_batch_workspace_bytes": (c_long, [c_long, c_int, c_int]),
    "hbmr_kmeans_map_batch": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                      c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p,
                                      c_int, c_int, c_void_p]),
    "hbmr_kmeans_delta_workspace_bytes": (c_long, [c_long, c_int, c_int]),
    "hbmr_kmeans_delta_combine": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                          c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_int,
                                          c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_map_batch_delta": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                            c_int, c_int, c_void_p, c_void_p, c_long, c_void_p,
                                            c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                            c_void_p]),
    "hbmr_kmeans_update": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_kmeans_padded_k": (c_int, [c_int]),
    "hbmr_kmeans_map_cpu_f32": (c_int, [c_void_p, c_long, c_int, c_void_p, c_int, c_void_p,
                                        c_void_p, c_void_p, c_double_p, c_int, c_int]),
    "hbmr_kmeans_map_cpu_f32_ex": (c_int, [c_void_p, c_long, c_int, c_void_p, c_int, c_void_p,
                                           c_void_p, c_void_p, c_double_p, c_int, c_int, c_int,
                                           c_void_p]),
    "hbmr_kmeans_padded_dim": (c_int, [c_int]),
    "hbmr_f32_to_bf16_pad": (c_int, [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p]),
    # sort / shuffle (native/kernels/sort.hip)
    "hbmr_radix_sort_workspace_bytes": (c_long, [c_long]),
    "hbmr_radix_onesweep_workspace_bytes": (c_long, [c_long]),
    "hbmr_radix_onesweep_status_bytes": (c_long, [c_long]),
    "hbmr_radix_sort_keys_u64": (c_int, [c_void_p, c_void_p, c_long, c_int, c_int, c_void_p,
                                         c_long, c_void_p, c_long, c_void_p, c_void_p, c_int,
                                         c_void_p]),
    "hbmr_radix_sort_pairs_u64": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int,
                                          c_int, c_void_p, c_long, c_void_p]),
    "hbmr_teragen": (c_int, [c_long, c_long, c_void_p, c_void_p]),
    "hbmr_tera_keys": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p]),
    "hbmr_gather_u64": (c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_gather_records": (c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p]),
    "hbmr_split_offsets": (c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_int,
                                   c_void_p, c_void_p]),
    "hbmr_check_sorted": (c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_tera_keys_part": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "hbmr_tera_collect": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_tera_collect_slots": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_long,
                                        c_void_p, c_void_p, c_void_p]),
    "hbmr_gather_records_multi": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int,
                                          c_void_p, c_void_p]),
    "hbmr_tera_partition_workspace_bytes": (c_long, [c_long, c_int]),
    "hbmr_tera_collect_gid": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long,
                                      c_int, c_uint64, c_uint, c_uint, c_int, c_void_p, c_void_p,
                                      c_void_p]),
    "hbmr_gather_records_gid": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_tera_group_stats": (c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                                      c_void_p]),
    "hbmr_radix_set_onesweep_waves": (c_int, [c_int]),
    "hbmr_gather_set_unroll": (c_int, [c_int]),
    "hbmr_tera_tie_fix_scratch_bytes": (c_long, [c_long, c_int]),
    "hbmr_tera_tie_fix_records": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_uint64,
                                          c_uint, c_uint, c_int, c_void_p, c_void_p, c_void_p,
                                          c_long, c_void_p]),
    "hbmr_merge_path": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                                c_long, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_tera_tie_fix": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_tera_partition": (c_int, [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long,
                                    c_void_p]),
    # text / WordCount (native/kernels/text.hip)
    "hbmr_wc_tiles": (c_long, [c_long]),
    "hbmr_wc_tokenize_count": (c_int, [c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_wc_tokenize_write": (c_int, [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_wc_insert": (c_int, [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                               c_void_p, c_long, c_void_p, c_void_p]),
    "hbmr_wc_compact": (c_int, [c_void_p, c_long, c_void_p, c_void_p, c_long, c_int, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hbmr_wc_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p,
                             c_void_p]),
    # PiEstimator (native/kernels/pi.hip)
    "hbmr_pi_halton": (c_int, [ctypes.c_longlong, ctypes.c_longlong, c_void_p, c_void_p]),
    # GEMM (native/kernels/gemm.hip)
    "hbmr_gemm_bf16_tn": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_long, c_long,
                                  ctypes.c_float, c_int, c_void_p]),
    "hbmr_gemm_set_kernel": (c_int, [c_int]),
    "hbmr_gemm_bf16_tn_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_long, c_long,
                                     ctypes.c_float, c_int, c_void_p, c_void_p]),
}


class NativeLibraryError(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB_PATH


def available() -> bool:
    try:
        load()
        return True
    except NativeLibraryError:
        return False


def load():
    """Load (once) and return the ctypes handle, building in-tree if needed."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists() and os.environ.get("HBMR_AUTOBUILD", "1") == "1":
            try:
                import importlib.util
                spec = importlib.util.spec_from_file_location(
                    "hbmr_native_build", _LIB_PATH.parent.parent.parent / "native" / "build.py")
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                mod.build()
            except Exception as e:  # pragma: no cover - surfaced below
                raise NativeLibraryError(f"libhbmr.so missing and build failed: {e}") from e
        if not _LIB_PATH.exists():
            raise NativeLibraryError(f"native library not found at {_LIB_PATH}; run native/build.py")
        try:
            lib = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {_LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with native error code {rc}")


def stream_handle(stream=None) -> int:
    """hipStream_t of the given (or current) torch stream as an int."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)
