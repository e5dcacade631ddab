"""CPU: libmsdsp.so loads (no GPU needed) and exports every function include/msdsp.h declares,
and the ctypes binding covers exactly that set.  No compute calls here."""
import ctypes
import os
import re

from meteorgpu import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "msdsp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(msd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    names = _declared()
    assert "msd_stft_psd_dev" in names and "msd_detect_dev" in names and "msd_block_delta_dev" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_matches_header():
    assert sorted(_lib.SYMBOLS) == _declared()


def test_abi_version_and_error_string():
    lib = _lib.load()
    assert lib.msd_abi_version() == 1
    assert isinstance(lib.msd_last_error(), bytes)


def test_struct_layouts():
    # msd_det {i64,i64,f64}; msd_det_cfg {i32,i32,f64,4*i64}; msd_hist_cfg {ptr,i64,i64,i32,i32,f64,ptr}
    assert ctypes.sizeof(_lib.MsdDet) == 24 == _lib.DET_DTYPE.itemsize
    assert ctypes.sizeof(_lib.MsdDetCfg) == 48
    assert ctypes.sizeof(_lib.MsdHistCfg) == 48
    # msd_stream_state {i64 freeze_until, i64 last_stop, f64 thr, i64 src, f64 thr_err}
    assert ctypes.sizeof(_lib.MsdStreamState) == 40


def test_invalid_args_fail_without_gpu():
    lib = _lib.load()
    assert lib.msd_create(0, None) == _lib.MSD_ERR_INVALID
    assert b"null" in lib.msd_last_error()
    assert lib.msd_stream_wait(None, None) == _lib.MSD_ERR_INVALID
    assert b"msd_stream_wait" in lib.msd_last_error()
