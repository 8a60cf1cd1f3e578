"""ctypes binding of the C ABI in include/walrus_rs2.h (libwalrus_rs2.so, built in-tree).

There is no CPU fallback: if the shared library is missing or no GPU is visible, every
entry point that computes raises.  The library is built by ``build_library()`` (make -j in
walrus_amd/csrc) and travels with the repository snapshot.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
LIB_PATH = Path(os.environ.get("WALRUS_RS2_LIB", PKG_DIR / "libwalrus_rs2.so"))

RS2_OK = 0
RS2_E_DATA_TOO_LARGE = -1
RS2_E_EMPTY_DATA = -2
RS2_E_INCORRECT_DATA_LENGTH = -3
RS2_E_INCOMPATIBLE_PARAMETERS = -4
RS2_E_NOT_ENOUGH_SHARDS = -5
RS2_E_DECODING_UNSUCCESSFUL = -6
RS2_E_VERIFICATION = -7
RS2_E_INVALID_ARGUMENT = -8
RS2_E_UNSUPPORTED = -9
RS2_E_DEVICE = -10
RS2_E_INTERNAL = -11

AXIS_PRIMARY = 0
AXIS_SECONDARY = 1
CHECK_SKIP, CHECK_DEFAULT, CHECK_STRICT = 0, 1, 2

# (name, restype, argtypes) for every function declared in include/walrus_rs2.h
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("n_shards", ctypes.c_uint16),
        ("n_primary", ctypes.c_uint16),
        ("n_secondary", ctypes.c_uint16),
        ("symbol_size", ctypes.c_uint16),
        ("blob_len", ctypes.c_uint64),
        ("primary_sliver_len", ctypes.c_uint64),
        ("secondary_sliver_len", ctypes.c_uint64),
    ]


SIGNATURES = {
    "rs2_source_symbols_for_n_shards": (ctypes.c_int, [ctypes.c_uint16, _u16p, _u16p]),
    "rs2_symbol_size_for_blob": (ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint64, _u16p]),
    "rs2_encoded_blob_length": (ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint64, _u64p]),
    "rs2_set_device": (ctypes.c_int, [ctypes.c_int]),
    "rs2_last_error": (ctypes.c_char_p, []),
    "rs2_device_available": (ctypes.c_int, []),
    "rs2_set_block_limit": (ctypes.c_int, [ctypes.c_uint32]),
    "rs2_plan_create": (ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint64, ctypes.POINTER(_vp)]),
    "rs2_plan_info_get": (ctypes.c_int, [_vp, ctypes.POINTER(PlanInfo)]),
    "rs2_plan_destroy": (None, [_vp]),
    "rs2_plan_rebind": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "rs2_device_memory_stats": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    "rs2_device_memory_trim": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    "rs2_upload_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "rs2_host_register": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "rs2_host_unregister": (ctypes.c_int, [_vp]),
    "rs2_encode_with_metadata": (
        ctypes.c_int, [_vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp]),
    "rs2_compute_metadata": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "rs2_decode_blob": (
        ctypes.c_int,
        [_vp, ctypes.c_int, ctypes.c_uint32, _u16p, ctypes.POINTER(_vp), _u64p, _u16p, _vp]),
    "rs2_decode_and_verify": (
        ctypes.c_int,
        [_vp, ctypes.c_int, ctypes.c_uint32, _u16p, ctypes.POINTER(_vp), _u64p, _u16p, _vp, _vp,
         ctypes.c_int, _vp]),
    "rs2_encode_device_async": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rs2_compute_metadata_device_async": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "rs2_encode_device_split_async": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "rs2_encode_batch_device_async": (
        ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint64, _u64p, _vp, ctypes.c_uint64,
                       _vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "rs2_encode_batch_with_metadata": (
        ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(_vp), _u64p, ctypes.POINTER(_vp),
                       ctypes.POINTER(_vp), _vp, _vp]),
    "rs2_quilt_layout_device_async": (ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint16,
                                                     ctypes.c_uint16, _vp, _vp, _vp, _vp, _vp]),
    "rs2_decode_device_async": (
        ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_uint32, _u16p, _vp, _u64p, _vp, _vp]),
    "rs2_decode_and_verify_device": (
        ctypes.c_int,
        [_vp, ctypes.c_int, ctypes.c_uint32, _u16p, _vp, _u64p, _vp, _vp, ctypes.c_int, _vp, _vp]),
    "rs2_sync": (ctypes.c_int, [_vp, _vp]),
    "rs2_profile_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rs2_profile_read": (
        ctypes.c_int,
        [_vp, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "rs2_encode_1d": (
        ctypes.c_int,
        [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint32, _vp, _vp]),
    "rs2_decode_1d": (
        ctypes.c_int,
        [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint32, _u16p,
         ctypes.POINTER(_vp), _vp]),
    "rs2_sliver_merkle_root": (
        ctypes.c_int,
        [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_int, _vp, ctypes.c_uint64, _vp]),
    "rs2_sliver_merkle_roots": (
        ctypes.c_int,
        [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_vp),
         _u64p, _vp]),
    "rs2_verifier_create": (
        ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_int, ctypes.POINTER(_vp)]),
    "rs2_verifier_roots_device_async": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp]),
    "rs2_verifier_destroy": (None, [_vp]),
    "rs2_recovery_symbols": (
        ctypes.c_int,
        [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_vp),
         _u64p, _u16p, _vp, _vp]),
    "rs2_verifier_recovery_symbols_device_async": (
        ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _u16p, _vp, _vp, _vp, _vp]),
    "rs2_merkle_tree_shape": (
        ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), _u64p]),
    "rs2_merkle_proof_roots": (
        ctypes.c_int,
        [ctypes.c_uint32, _vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), _vp,
         ctypes.c_uint32, _vp]),
    "rs2_merkle_root": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    "rs2_blob_id_from_hashes": (
        ctypes.c_int, [_vp, ctypes.c_uint16, ctypes.c_uint64, _vp]),
    "rs2_codec_create": (
        ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16, ctypes.POINTER(_vp)]),
    "rs2_codec_destroy": (None, [_vp]),
    "rs2_codec_encode_device_async": (
        ctypes.c_int,
        [_vp, ctypes.c_uint32, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, ctypes.c_uint64,
         ctypes.c_uint64, _vp]),
    "rs2_codec_decode_device_async": (
        ctypes.c_int,
        [_vp, ctypes.c_uint32, ctypes.c_uint32, _u16p, _vp, _u64p, ctypes.c_uint64, _vp,
         ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    "rs2_copy_segments_device_async": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_uint32, ctypes.c_uint32, _vp]),
    "rs2_leaf_hashes_device_async": (
        ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint16, _vp, _vp]),
    "rs2_merkle_roots_device_async": (
        ctypes.c_int,
        [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, _vp,
         ctypes.c_uint64, _vp]),
    "rs2_blob_id_device_async": (
        ctypes.c_int, [_vp, ctypes.c_uint16, ctypes.c_uint64, _vp, _vp]),
}


def build_library(jobs: int = 16, quiet: bool = True) -> Path:
    """Compile libwalrus_rs2.so for gfx950 in place (make -j)."""
    cmd = ["make", f"-j{jobs}", "-C", str(CSRC)]
    out = subprocess.run(cmd, capture_output=quiet, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"building libwalrus_rs2.so failed:\n{out.stdout}\n{out.stderr}")
    return LIB_PATH


_LIB = None


def lib():
    """The loaded shared library (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with walrus_amd._lib.build_library() "
                "(there is no CPU fallback)")
        # PyTorch's wheel bundles its own HIP runtime (libamdhip64.so) beside the system one this
        # library links (libamdhip64.so.7).  If the engine's runtime is loaded and initialises
        # the GPU before torch is imported, torch's later CUDA init reports "No HIP GPUs are
        # available" (seen on the MI355X box); importing torch first lets both runtimes share
        # the device, which is the order bench.py and callers that pass torch streams use.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def last_error() -> str:
    return lib().rs2_last_error().decode(errors="replace")


def device_available() -> bool:
    return bool(lib().rs2_device_available())


def exported_symbols():
    return list(SIGNATURES)


def header_symbols():
    """Function names declared in include/walrus_rs2.h."""
    import re
    hdr = (PKG_DIR.parent / "include" / "walrus_rs2.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(rs2_\w+)\(", hdr, re.M)))


def buf(data) -> ctypes.c_void_p:
    """Pointer to a bytes-like / numpy buffer (kept alive by the caller)."""
    import numpy as np
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return ctypes.c_void_p(arr.ctypes.data)


if os.environ.get("WALRUS_AMD_DEVICE"):
    try:
        lib().rs2_set_device(int(os.environ["WALRUS_AMD_DEVICE"]))
    except RuntimeError:
        pass
