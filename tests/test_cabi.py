"""CPU checks of the C-ABI boundary: the library loads without a GPU and exports every
symbol include/td3.h declares, with argument checking that fails loudly."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "td3.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void|void\*|double|const char\*)\s*\**\s*(\w+)\s*\(",
                                 txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from td3_amd.build import build_library
    build_library()
    from td3_amd import _lib
    return _lib.load()


def test_header_symbols_exported(lib):
    from td3_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/td3.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} not bound in td3_amd/_lib.py"


def test_no_cpu_fallback_symbols(lib):
    # the product library must not reference the oracle
    data = open(os.path.join(ROOT, "td3_amd", "libtd3hip.so"), "rb").read()
    assert b"td3_oracle" not in data


def test_default_config(lib):
    from td3_amd import _lib
    cfg = _lib.td3_config()
    lib.td3_default_config(C.byref(cfg))
    assert list(cfg.actor_hidden) == [500, 400, 300]      # TD3_featured.py:19
    assert list(cfg.critic_hidden) == [500, 400, 200]     # TD3_featured.py:54
    assert cfg.policy_freq == 2 and abs(cfg.tau - 0.005) < 1e-12
    assert abs(cfg.discount - 0.99) < 1e-12 and abs(cfg.lr - 1e-4) < 1e-15
    assert abs(cfg.policy_noise - 0.2) < 1e-12 and abs(cfg.noise_clip - 0.5) < 1e-12


def test_argument_errors_are_reported(lib):
    from td3_amd import _lib
    h = C.c_void_p()
    assert lib.rb_create(0, 1, 10, 0, 0, C.byref(h)) == -1
    assert b"dims" in lib.td3_last_error()
    cfg = _lib.td3_config()
    lib.td3_default_config(C.byref(cfg))
    cfg.state_dim, cfg.action_dim = 17, 40
    assert lib.td3_create(C.byref(cfg), C.byref(h)) == -1
    assert b"action_dim" in lib.td3_last_error()
    with pytest.raises(_lib.TD3Error):
        _lib.check(-1, "x")


def test_product_modules_import_without_gpu():
    import td3_amd.TD3_featured as tf
    import td3_amd.my_replay_buffer as mrb
    assert tf.TD3 and mrb.ReplayBuffer_featured
