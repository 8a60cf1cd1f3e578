"""CPU tests of the C ABI: the library loads, exports every symbol include/walrus_rs2.h
declares, and its parameter functions agree with the oracle.  No GPU compute (every hash and
codec entry point runs on the device; those are tested in tests/test_gpu_*.py)."""
import ctypes
import subprocess

import numpy as np
import pytest

import rs2_oracle as O
from walrus_amd import _lib


def test_library_exports_every_header_symbol():
    hdr = _lib.header_symbols()
    assert len(hdr) >= 20
    assert sorted(_lib.exported_symbols()) == hdr
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in hdr if s not in exported]
    assert not missing, missing
    lib = _lib.lib()
    for s in hdr:
        assert getattr(lib, s) is not None


@pytest.mark.parametrize("n", [1, 3, 4, 7, 9, 10, 31, 51, 100, 101, 301, 1000, 65535])
def test_source_symbols(n):
    kp, ks = ctypes.c_uint16(), ctypes.c_uint16()
    assert _lib.lib().rs2_source_symbols_for_n_shards(n, ctypes.byref(kp), ctypes.byref(ks)) == 0
    assert (kp.value, ks.value) == O.source_symbols_for_n_shards(n)


@pytest.mark.parametrize("n,length", [(10, 0), (10, 1), (10, 33), (1000, 1 << 28),
                                      (1000, 334 * 667 * 65534), (102, 31415)])
def test_symbol_size_and_encoded_length(n, length):
    s = ctypes.c_uint16()
    assert _lib.lib().rs2_symbol_size_for_blob(n, length, ctypes.byref(s)) == 0
    kp, ks = O.source_symbols_for_n_shards(n)
    assert s.value == O.compute_symbol_size(length, kp * ks)
    enc = ctypes.c_uint64()
    assert _lib.lib().rs2_encoded_blob_length(n, length, ctypes.byref(enc)) == 0
    assert enc.value == n * (kp + ks) * s.value + n * (n * 64 + 32)


def test_encoded_length_table():
    """config.rs:858-882 (mirrored by the Move tests)."""
    enc = ctypes.c_uint64()
    for length, n, expected in [(0, 10, 10 * (2 * (4 + 7) + 10 * 2 * 32 + 32)),
                                (1, 10, 10 * (2 * (4 + 7) + 10 * 2 * 32 + 32)),
                                ((4 * 7) * 100, 10, 10 * ((4 + 7) * 100 + 10 * 2 * 32 + 32)),
                                (1, 1000, 1000 * (2 * (334 + 667) + 1000 * 2 * 32 + 32))]:
        assert _lib.lib().rs2_encoded_blob_length(n, length, ctypes.byref(enc)) == 0
        assert enc.value == expected


def test_encoded_length_reference_publisher_example():
    """docs/content/http-api/storing-blobs.mdx:114-139: the 17-byte "some other string" blob at
    mainnet's n = 1000 reports encodedLength = storageSize = 66,034,000."""
    enc = ctypes.c_uint64()
    assert _lib.lib().rs2_encoded_blob_length(1000, 17, ctypes.byref(enc)) == 0
    assert enc.value == 66_034_000


def test_data_too_large_error():
    s = ctypes.c_uint16()
    rc = _lib.lib().rs2_symbol_size_for_blob(1000, 334 * 667 * 65535 + 1, ctypes.byref(s))
    assert rc == _lib.RS2_E_DATA_TOO_LARGE
