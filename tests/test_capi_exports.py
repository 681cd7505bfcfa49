"""The C-ABI library loads and exports every entry point its public headers declare (no GPU:
no compute call is made)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fec_[a-z0-9_]+)\s*\(", src)))


def test_headers_declare_entry_points():
    names = declared("fec_hip.h")
    for want in ["fec_ctx_create", "fec_rs_encode_batch", "fec_rs_reconstruct_batch",
                 "fec_xor_encode_batch", "fec_xor_reconstruct_batch", "fec_sync", "fec_strerror"]:
        assert want in names


def test_library_exports_every_declared_symbol(fec):
    lib = ctypes.CDLL(fec._LIB_PATH)
    headers = [h for h in os.listdir(os.path.join(ROOT, "include")) if h.endswith(".h")]
    missing = []
    for h in headers:
        for name in declared(h):
            if not hasattr(lib, name):
                missing.append((h, name))
    assert not missing, missing


def test_no_device_needed_for_host_helpers(fec):
    assert fec.version().startswith("0xfec")
    assert fec.lib.fec_strerror(fec.FEC_ERR_TOO_FEW_SHARDS) == b"too few shards given"
    m = fec.rs_matrix(8, 4)
    assert bytes(m[8]).hex() == "1a84ba33e710c627"
    assert (m[:8] == np.eye(8, dtype=np.uint8)).all()


def test_matrix_matches_oracle(fec, oracle):
    for k, m in [(1, 1), (2, 1), (6, 2), (8, 4), (16, 8), (20, 10), (3, 29), (100, 156)]:
        assert np.array_equal(fec.rs_matrix(k, m), oracle.build_matrix(k, k + m)), (k, m)


def test_shard_count_errors_without_device(fec):
    import pytest
    with pytest.raises(fec.FecError) as e:
        fec.rs_matrix(0, 1)
    assert e.value.code == fec.FEC_ERR_INV_SHARD_NUM
    with pytest.raises(fec.FecError) as e:
        fec.rs_matrix(200, 57)
    assert e.value.code == fec.FEC_ERR_MAX_SHARD_NUM


def test_context_fails_loudly_without_gpu(fec):
    """No CPU fallback: with no HIP device the context cannot be created."""
    import pytest
    if fec.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(fec.FecError) as e:
        fec.Codec(0)
    assert e.value.code == fec.FEC_ERR_NO_DEVICE


def test_lane_permtab_builder_matches_bytewise(fec):
    # the rebuild kernels expand coefficient rows with gf::make_permtab_fast (32-bit lane
    # arithmetic, v_perm byte moves restated on the host); it must equal the byte-wise table
    # builder for all 256 coefficients
    lib = ctypes.CDLL(fec._LIB_PATH)
    assert lib.fec__selftest_permtab() == 0


def test_copy_workers_cover_every_index_once(fec):
    # FEC_HOST's staging / scatter copies run through parallel_for on persistent copy workers
    # (fec_capi.cpp CopyPool) or on threads made per call: every index exactly once, for sizes
    # around the part boundaries, 2..16 parts, four callers at once (no device needed; the
    # sanitized CPU run repeats it under ASan / UBSan)
    lib = ctypes.CDLL(fec._LIB_PATH)
    assert lib.fec__selftest_copypool() == 0
